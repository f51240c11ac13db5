"""Fully-sharded data parallel (ZeRO-3 style) with flat parameters, from scratch.

Reference: ``torch.distributed.fsdp.FullyShardedDataParallel`` with ``FULL_SHARD``,
``size_based_auto_wrap_policy(min_num_params=100_000)`` and ``MixedPrecision(bf16, bf16, bf16)``
for the LM (``02_development/distributed_utils.py:318-332``), and a custom policy for Llama
(:479-499) that never recursed, leaving the whole 6.7B model as ONE unit.  Gradient
clipping there used the local shard norm (C25) and the full-state-dict save was entered by rank 0
only, a mismatched collective (K13).

Design (MI355X-first, not a wrapper tree):

* **Units.**  A wrap policy picks submodules (``transformer_auto_wrap_policy`` — layer-class
  semantics that recurse everywhere; ``size_based_auto_wrap_policy``).  Each unit's own
  parameters (minus nested units') become one flat fp32 *master shard* per rank (padded to a
  multiple of the world size); the remaining parameters form the root unit.  Module attribute
  names are untouched, so ``state_dict`` keys stay the reference's (no ``_fsdp_wrapped_module``).
* **Gather.**  Before a unit runs (forward pre-hook, and again before its backward via a grad
  hook on its outputs) its shard is cast to ``param_dtype`` and all-gathered (RCCL over xGMI) into
  a persistent full buffer; the module's parameters are views of that buffer.  After the unit's
  forward / backward the buffer's *storage* is released (``resize_(0)``) — the autograd graph keeps
  the same view objects, which become valid again when the next gather refills the storage.
  The next unit's gather is issued asynchronously as soon as the current one starts (forward and
  backward prefetch), so the all-gather of unit i±1 overlaps compute of unit i.
* **Reduce.**  Each parameter's gradient accumulates in place into a flat ``reduce_dtype``
  gradient buffer; when a unit's last gradient lands (post-accumulate-grad hooks), one
  ``reduce_scatter`` produces this rank's shard gradient (async, overlapped with the rest of
  backward) which is converted into the fp32 master shard's ``.grad``.
* **Optimizer** sees only the flat fp32 shards (``fsdp.parameters()``): a handful of large
  tensors — ideal for the multi-tensor fused Adam.
* **Clipping** is global (``clip_grad_norm_`` all-reduces the squared norm over shards).
* **State dicts** are collective on every rank: ``full_state_dict()`` all-gathers every unit's
  fp32 shard (all ranks participate; rank 0 keeps the result, optionally on CPU), and
  ``sharded_state_dict()`` / ``load_sharded_state_dict()`` save/restore the flat shards per rank.

With 288 GB of HBM per MI355X the default is to keep units coarse (one transformer layer per
unit) so every all-gather / reduce-scatter moves tens to hundreds of MB — the regime where ring
collectives over the 7 xGMI links reach their bus bandwidth.
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Sequence, Set, Tuple, Type

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import streams as _streams
from ..ops.conv import flush_wgrad as _flush_wgrad
from ..ops.optim import clip_grad_norm_
from ..train import segments as _seg
from .comm import NativeComm, get_comm

log = logging.getLogger("hyperion.fsdp")


# ------------------------------------------------------------------------------------ policies
def transformer_auto_wrap_policy(layer_classes: Iterable[Type[nn.Module]]) -> Callable[[nn.Module, int], bool]:
    """Wrap every module whose class is in ``layer_classes`` (recursing into all children)."""
    cls = tuple(layer_classes)

    def policy(module: nn.Module, unwrapped_numel: int) -> bool:
        return isinstance(module, cls)

    policy.layer_classes = cls  # type: ignore[attr-defined]
    return policy


def size_based_auto_wrap_policy(min_num_params: int = 100_000) -> Callable[[nn.Module, int], bool]:
    """Wrap a module once the parameters not yet claimed by a nested unit reach ``min_num_params``."""

    def policy(module: nn.Module, unwrapped_numel: int) -> bool:
        return unwrapped_numel >= min_num_params

    return policy


def _group_rank0(group) -> int:
    """GLOBAL rank of the group's rank 0 (``dist.broadcast``'s ``src`` is a global rank; the
    sharded state dict elects group-rank 0, which is not global rank 0 in a subgroup)."""
    if group is None or group is dist.group.WORLD:
        return 0
    return dist.get_global_rank(group, 0)


@dataclass
class MixedPrecision:
    param_dtype: Optional[torch.dtype] = None
    reduce_dtype: Optional[torch.dtype] = None
    buffer_dtype: Optional[torch.dtype] = None


def _select_units(root: nn.Module, policy: Optional[Callable]) -> List[nn.Module]:
    """Post-order traversal: children first, so nested units claim their parameters first."""
    units: List[nn.Module] = []

    def visit(m: nn.Module) -> int:
        numel = sum(p.numel() for p in m.parameters(recurse=False))
        for c in m.children():
            numel += visit(c)
        if m is not root and policy is not None and numel > 0 and policy(m, numel):
            units.append(m)
            return 0
        return numel

    visit(root)
    return units


# ------------------------------------------------------------------------------------ unit
class _SlotWork:
    """A collective issued through ``segments.eager``: under a segmented capture the issue is an
    eager action that refills ``slot`` on every replay, and ``wait()`` is its own action reading
    the replay's current handle (so the collective overlaps the segments in between)."""

    __slots__ = ("slot",)

    def __init__(self, fn):
        slot = [None]

        def issue():
            slot[0] = fn()

        _seg.eager(issue)
        self.slot = slot

    def wait(self):
        slot = self.slot
        _seg.eager(lambda: slot[0].wait())


class _Ring:
    """K fixed-address buffers shared by the units' gathered parameters (or full gradients) in
    ring mode: unit i lives in slot i % K while it is gathered, so memory is K x the largest unit
    (FULL_SHARD's reshard-after-forward bound) and every address is fixed — the step stays
    capturable as graph segments.  ``owner[k]``: the group whose data slot k holds."""

    def __init__(self, k: int, numel: int, dtype: torch.dtype, device: torch.device):
        self.bufs = [torch.empty(numel, dtype=dtype, device=device) for _ in range(k)]
        self.owner: List[Optional["_FlatGroup"]] = [None] * k

    @property
    def nbytes(self) -> int:
        return sum(b.numel() * b.element_size() for b in self.bufs)


class _FlatGroup:
    """One flat parameter: the trainable (fp32 master shard) or frozen (param-dtype shard) params of a unit."""

    def __init__(self, fsdp: "FullyShardedDataParallel", params: List[nn.Parameter], trainable: bool, tag: str,
                 ring_member: bool = False):
        self.fsdp = fsdp
        self.tag = tag
        self.trainable = trainable
        self.params = params
        self.shapes = [p.shape for p in params]
        self.numels = [p.numel() for p in params]
        self.offsets = [0]
        for n in self.numels[:-1]:
            self.offsets.append(self.offsets[-1] + n)
        self.numel = sum(self.numels)
        # resident: a frozen group kept whole on every rank (FSDP(replicate_frozen=...)): never
        # gathered, never freed — the base weights of a LoRA fine-tune fit 288 GB of HBM many times
        # (at world 1 every frozen group is resident: its one shard IS the full tensor — no copy)
        self.resident = (not trainable) and (fsdp.replicate_frozen or fsdp.identity)
        W, r = (1, 0) if self.resident else (fsdp.world, fsdp.rank)
        # shards of a multiple of 64 elements: every rank's slice of the gathered buffer (and every
        # reduce-scatter output) starts 128-byte aligned for RCCL and the vector kernels
        self.padded = int(math.ceil(max(self.numel, 1) / (W * 64)) * W * 64)
        self.shard_numel = self.padded // W
        dev = fsdp.device
        self.cdtype = fsdp.mp.param_dtype or torch.float32
        self.rdtype = fsdp.mp.reduce_dtype or self.cdtype
        # frozen weights are never updated: keep their shard in the compute dtype (half the memory)
        sdtype = torch.float32 if trainable else self.cdtype
        with torch.no_grad():
            flat = torch.zeros(self.padded, dtype=sdtype, device=dev)
            for p, o, n in zip(params, self.offsets, self.numels):
                flat[o : o + n].copy_(p.detach().reshape(-1))
            shard = flat[r * self.shard_numel : (r + 1) * self.shard_numel].clone()
        self.flat_param = nn.Parameter(shard, requires_grad=trainable)
        # ring mode: the gathered parameters / full gradient are views of a shared ring slot,
        # attached after every unit exists (attach_ring); nothing of their own is allocated
        self.ring: Optional[_Ring] = None
        self.grad_ring: Optional[_Ring] = None
        self.slot = -1
        self.ring_member = ring_member and not self.resident
        # pinned: buffers never released (persistent mode; in ring mode also the root unit's —
        # a capturable step allocates nothing)
        self.pinned = fsdp.persistent or bool(fsdp.ring)
        if self.ring_member:
            self.full = torch.empty(0, dtype=self.cdtype, device=dev)
            self.full_grad = torch.empty(0, dtype=self.rdtype, device=dev) if trainable else None
        else:
            self.full = self.flat_param.data if self.resident else torch.empty(self.padded, dtype=self.cdtype, device=dev)
            self.full_grad = torch.empty(self.padded, dtype=self.rdtype, device=dev) if trainable else None
        self._full_bytes = self.full.untyped_storage().nbytes()
        self._grad_bytes = self.full_grad.untyped_storage().nbytes() if trainable else 0
        self.gathered = True
        self.gather_work = None
        # persistent all-gather source in the compute dtype: cast ONCE per optimizer step (the
        # forward gather), reused by the backward re-gather; None when the shard already has it or
        # at world 1 without collectives (the gather is then one cast-copy straight into the buffer)
        self._send_buf = (torch.empty(self.shard_numel, dtype=self.cdtype, device=dev)
                          if self.flat_param.dtype != self.cdtype and not fsdp.identity else None)
        self.send_valid = False
        self.rs_work = None
        self.rs_out: Optional[torch.Tensor] = None
        # persistent reduce-scatter output / fp32 shard gradient (no per-step allocation or .to())
        self._rs_buf = (torch.empty(self.shard_numel, dtype=self.rdtype, device=dev)
                        if trainable and self.rdtype != torch.float32 and not fsdp.identity else None)
        self._grad_shard = torch.empty(self.shard_numel, dtype=torch.float32, device=dev) if trainable else None
        self.grad_ready: Set[int] = set()
        self._pending: List[Tuple[int, torch.Tensor]] = []  # (param index, grad) not yet in full_grad
        self.reduced = False
        if self.ring_member:
            self.gathered = False
            return
        # module parameters become views of the full buffer (the same Parameter objects)
        for p, o, n, shp in zip(params, self.offsets, self.numels, self.shapes):
            p.data = self.full[o : o + n].view(shp)
        if not (self.resident or self.pinned):
            self.free_full()
        elif not self.resident:
            self.gathered = False  # persistent: the full buffer is allocated but not filled yet
        if trainable:
            if self.pinned:
                self.full_grad.zero_()
            else:
                self.full_grad.untyped_storage().resize_(0)

    # -- storage ------------------------------------------------------------------------
    def attach_ring(self, ring: _Ring, grad_ring: Optional[_Ring], slot: int) -> None:
        """Ring mode: this group's full parameters (and full gradient) are views of slot ``slot``."""
        self.ring, self.grad_ring, self.slot = ring, grad_ring, slot
        self.full = ring.bufs[slot][: self.padded]
        self._full_bytes = self.full.untyped_storage().nbytes()
        for p, o, n, shp in zip(self.params, self.offsets, self.numels, self.shapes):
            p.data = self.full[o : o + n].view(shp)
        if self.trainable:
            self.full_grad = grad_ring.bufs[slot][: self.padded]
            self._grad_bytes = self.full_grad.untyped_storage().nbytes()
        self.gathered = False

    def holds_slot(self) -> bool:
        return self.ring is not None and self.ring.owner[self.slot] is self

    def free_full(self) -> None:
        if self.resident or self.pinned:
            # persistent: the storage stays, the content stays valid; ring: the slot is overwritten
            # by the unit that takes it next (no release, no re-allocation: fixed addresses)
            return
        if self.gather_work is not None:
            self.wait_gather()
        if self.gathered:
            self.full.untyped_storage().resize_(0)
            self.gathered = False

    def gather(self, async_op: bool = False) -> None:
        if self.ring is not None:
            prev = self.ring.owner[self.slot]
            if prev is not self:
                if prev is not None:  # evict: its later use re-gathers (same comm stream: ours lands last)
                    if getattr(prev, "unit", None) in self.fsdp._live_fwd:
                        raise RuntimeError(f"FSDP ring: gathering {self.tag} into slot {self.slot} would evict "
                                           f"{prev.tag}, whose forward is still running")
                    prev.gathered = False
                    prev.gather_work = None
                self.ring.owner[self.slot] = self
                self.gathered = False
        if self.resident or self.gathered or self.gather_work is not None:
            return
        st = self.full.untyped_storage()
        if st.nbytes() != self._full_bytes:
            st.resize_(self._full_bytes)
        if self.fsdp.identity:  # world 1: one cast-copy of the shard, no staging buffer
            with torch.no_grad():
                self.full.data.copy_(self.flat_param.detach())
            self.gathered = True
            return
        if self._send_buf is None:
            send = self.flat_param.detach()
        else:
            if not self.send_valid:  # params changed since the last cast (an optimizer step)
                with torch.no_grad():
                    self._send_buf.copy_(self.flat_param.detach())
                self.send_valid = True
            send = self._send_buf
        out = self.full.data  # fresh version counter: autograd's saved views stay valid
        comm = self.fsdp.comm
        self.gather_work = _SlotWork(lambda: comm.all_gather(out, send))
        if not async_op:
            self.wait_gather()

    def wait_gather(self) -> None:
        if self.gather_work is not None:
            self.gather_work.wait()
            self.gather_work = None
            self.gathered = True

    # -- gradients ------------------------------------------------------------------------
    def _grad_buf(self) -> torch.Tensor:
        if self.grad_ring is not None:
            occ = self.grad_ring.owner[self.slot]
            if occ is not self:
                if occ is not None and occ.rs_work is not None:
                    occ.rs_work.wait()  # its reduce-scatter still reads the slot (stream-ordered wait)
                    occ.rs_work = None
                self.grad_ring.owner[self.slot] = self
                if self.padded > self.numel:  # the previous occupant's bytes would enter the clip norm
                    with torch.no_grad():
                        self.full_grad.data[self.numel :].zero_()
            return self.full_grad.data
        st = self.full_grad.untyped_storage()
        if st.nbytes() != self._grad_bytes:
            st.resize_(self._grad_bytes)
            self.full_grad.data.zero_()
        return self.full_grad.data

    def start_backward(self) -> None:
        self.grad_ready = set()
        self._pending = []
        self.reduced = False

    def on_grad(self, i: int, p: nn.Parameter) -> bool:
        """Take one param's grad for the flat buffer; True once the group is complete.  The grads
        land together (one multi-tensor copy per group when it completes or reduces) instead of one
        small device copy per parameter."""
        if self.reduced or i in self.grad_ready:
            return False
        _flush_wgrad()  # a deferred weight-gradient reduce may still owe this gradient its values
        if p.grad.is_cuda:
            _streams.join(p.grad.device)  # produced on the weight-gradient side stream
        self._pending.append((i, p.grad))
        p.grad = None
        self.grad_ready.add(i)
        done = len(self.grad_ready) == len(self.params)
        if done:
            self._land_pending()
        return done

    def _land_pending(self) -> None:
        if not self._pending:
            return
        buf = self._grad_buf()
        pend = sorted(self._pending, key=lambda ig: ig[0])
        self._pending = []
        with torch.no_grad():
            if (len(pend) == len(self.params) and all(g.is_contiguous() and g.dtype == buf.dtype for _, g in pend)):
                # the whole group, in flat order: one concatenation kernel straight into the buffer
                torch.cat([g.reshape(-1) for _, g in pend], out=buf.narrow(0, 0, self.numel))
            else:
                dst = [buf[self.offsets[i] : self.offsets[i] + self.numels[i]].view(self.shapes[i]) for i, _ in pend]
                torch._foreach_copy_(dst, [g for _, g in pend])

    def reduce(self) -> None:
        if self.reduced:
            return
        self.reduced = True
        self._land_pending()
        buf = self._grad_buf()
        for i, (o, n) in enumerate(zip(self.offsets, self.numels)):
            if i not in self.grad_ready:  # unused this step: contributes zeros
                buf[o : o + n].zero_()
        if self.fsdp.identity:
            if self.grad_ring is not None:  # the slot is reused by a later unit: take the shard now
                with torch.no_grad():
                    if self.flat_param.grad is None:
                        self._grad_shard.copy_(buf[: self.shard_numel])
                        self.rs_out = self._grad_shard
                    else:
                        # .grad exists (accumulation, zero_grad(set_to_none=False), warm-up replays):
                        # it may BE _grad_shard, so add the slot's gradient into it right here —
                        # a copy into _grad_shard first would overwrite what is being accumulated
                        self.flat_param.grad.add_(buf[: self.shard_numel])
                        self.rs_out = None  # finish_reduce: nothing left to add
                self.rs_work = None
                return
            self.rs_out, self.rs_work = buf, None
            return
        # AVG in RCCL; the output lands in a persistent buffer — straight in the fp32 shard
        # gradient when the reduction runs in fp32 and nothing is being accumulated
        if self._rs_buf is None and self.flat_param.grad is None:
            self.rs_out = self._grad_shard
        else:
            self.rs_out = self._rs_buf if self._rs_buf is not None else torch.empty_like(self._grad_shard)
        comm, rs_out = self.fsdp.comm, self.rs_out
        self.rs_work = _SlotWork(lambda: comm.reduce_scatter(rs_out, buf, "avg"))

    def finish_reduce(self) -> None:
        if not self.reduced:
            self.reduce()
        if self.rs_work is not None:
            self.rs_work.wait()
            self.rs_work = None
        g = self.rs_out
        if g is None:  # identity ring: already accumulated into .grad by reduce()
            if not self.pinned:
                self.full_grad.untyped_storage().resize_(0)
            return
        if self.fsdp.identity:  # rs_out is the full flat gradient buffer (released below)
            g = g[: self.shard_numel]
        with torch.no_grad():
            if self.flat_param.grad is None:
                if g.data_ptr() != self._grad_shard.data_ptr():
                    self._grad_shard.copy_(g)  # (+ bf16 -> fp32)
                self.flat_param.grad = self._grad_shard
            else:
                self.flat_param.grad.add_(g)
        self.rs_out = None
        if not self.pinned:
            self.full_grad.untyped_storage().resize_(0)


class _Unit:
    """A wrapped module: its frozen and trainable parameter groups are gathered/released together."""

    def __init__(self, fsdp: "FullyShardedDataParallel", module: nn.Module, params: List[nn.Parameter], index: int,
                 ring_member: bool = False):
        self.fsdp = fsdp
        self.module = module
        self.index = index
        self.params = params
        train = [p for p in params if p.requires_grad]
        frozen = [p for p in params if not p.requires_grad]
        self.train = _FlatGroup(fsdp, train, True, f"u{index}t", ring_member) if train else None
        self.frozen = _FlatGroup(fsdp, frozen, False, f"u{index}f", ring_member) if frozen else None
        self.groups = [g for g in (self.frozen, self.train) if g is not None]
        for g in self.groups:
            g.unit_index = index
            g.unit = self
        self._pidx = {id(p): i for i, p in enumerate(train)}

    @property
    def numel(self) -> int:
        return sum(g.numel for g in self.groups)

    def gather(self, async_op: bool = False) -> None:
        for g in self.groups:
            g.gather(async_op=True)
        if not async_op:
            self.wait_gather()

    def wait_gather(self) -> None:
        for g in self.groups:
            g.wait_gather()

    def ring_slot_busy(self, active: Optional["_Unit"]) -> bool:
        """A prefetch of this unit would overwrite a ring slot that a running unit computes from:
        the ACTIVE one, or (nested units) an enclosing unit whose forward or backward is still in
        progress — with nesting, several units are live at once."""
        live = self.fsdp._live_fwd | self.fsdp._live_bwd
        for g in self.groups:
            if g.ring is None:
                continue
            occ = g.ring.owner[g.slot]
            if occ is None or occ in self.groups:
                continue
            if (active is not None and occ in active.groups) or getattr(occ, "unit", None) in live:
                return True
        return False

    def reshard(self) -> None:
        for g in self.groups:
            g.free_full()

    @property
    def reduced(self) -> bool:
        return self.train is None or self.train.reduced

    def start_backward(self) -> None:
        if self.train is not None:
            self.train.start_backward()

    def on_grad(self, p: nn.Parameter) -> None:
        if self.train is not None and self.train.on_grad(self._pidx[id(p)], p):
            self.train.reduce()
            if self.frozen is None:
                # the last weight-grad node of the unit also produced its input grad: nothing in this
                # unit's backward needs the full params any more.  (With frozen params — LoRA — the
                # unit's input-grad hook releases them instead: frozen weights are still read after
                # the last trainable grad lands.)
                self.fsdp._live_bwd.discard(self)
                self.reshard()

    def on_input_grads(self) -> None:
        """All grads w.r.t. the unit's inputs exist: its backward is over."""
        if self.train is not None and not self.train.reduced:
            self.train.reduce()
        self.fsdp._live_bwd.discard(self)
        self.reshard()

    def finish(self) -> None:
        if self.train is not None:
            self.train.finish_reduce()
        self.reshard()


# ------------------------------------------------------------------------------------ FSDP
class FullyShardedDataParallel(nn.Module):
    def __init__(
        self,
        module: nn.Module,
        process_group=None,
        auto_wrap_policy: Optional[Callable[[nn.Module, int], bool]] = None,
        mixed_precision: Optional[MixedPrecision] = None,
        device_id: Optional[torch.device] = None,
        sharding_strategy: str = "FULL_SHARD",
        forward_prefetch: bool = True,
        backward_prefetch: bool = True,
        sync_module_states: bool = True,
        comm=None,
        replicate_frozen=False,
        persistent=None,
        collectives_at_world_1: bool = False,
        ring: int = 0,
    ):
        """collectives_at_world_1: on a single rank, still run every gather / reduce-scatter as a
        collective (the native RCCL communicator on GPU) instead of the identity copies — the
        multi-GPU transport path, exercised and timed on one device.

        ring (FULL_SHARD, >= 2): the wrapped units' gathered parameters and full gradients live in
        a ring of ``ring`` fixed-address slots (unit i in slot i % ring) instead of being freed and
        re-allocated: reshard-after-forward memory (ring x the largest unit, not every unit) with
        the fixed addresses a captured step needs.  A unit keeps its slot until another unit takes
        it, so the last units of the forward are still gathered when the backward starts."""
        super().__init__()
        if sharding_strategy not in ("FULL_SHARD", "SHARD_GRAD_OP"):
            raise ValueError("sharding_strategy must be FULL_SHARD or SHARD_GRAD_OP (NO_SHARD = use DDP)")
        self.module = module
        self.group = process_group
        self._comm = comm
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0
        if device_id is None:
            device_id = next((p.device for p in module.parameters()), torch.device("cpu"))
        self.device = torch.device(device_id)
        # identity: world 1 with the collectives elided (a gather is one cast-copy, a reduce-scatter
        # nothing); collectives_at_world_1 keeps them, over RCCL when a process group exists on GPU
        self.identity = self.world == 1 and not collectives_at_world_1
        if (collectives_at_world_1 and self.world == 1 and comm is None and self.device.type == "cuda"
                and dist.is_available() and dist.is_initialized()):
            from ..ops import _native

            if _native.available():
                self._comm = NativeComm(self.device, process_group)
        module.to(self.device)
        self.mp = mixed_precision or MixedPrecision()
        # replicate_frozen: frozen (requires_grad=False) parameters stay whole on every rank in the
        # compute dtype — no all-gathers for them, ever; trainable ones are sharded as usual.
        # "auto": when the frozen bytes take at most a quarter of the device's memory (MI355X:
        # Llama-2-7B's 13.5 GB bf16 base vs 288 GB HBM — the LoRA step then moves only adapter
        # traffic over xGMI instead of re-gathering 13.5 GB per forward and per backward).
        if replicate_frozen == "auto":
            frozen_bytes = sum(p.numel() for p in module.parameters() if not p.requires_grad) * \
                torch.finfo(self.mp.param_dtype or torch.float32).bits // 8
            cap = torch.cuda.get_device_properties(self.device).total_memory if self.device.type == "cuda" else 0
            replicate_frozen = self.world > 1 and cap > 0 and frozen_bytes <= cap // 4
        self.replicate_frozen = bool(replicate_frozen)
        # persistent: every unit's gathered parameters and gradient buffer stay allocated (no
        # storage release / re-allocation per step) and the parameters gathered for the forward are
        # reused by the backward (one all-gather per unit per step instead of two).  That is the
        # memory-for-traffic trade 288 GB of HBM affords for the models here, and it makes the step
        # capturable (train/segments.py).  "auto"/None: on GPU when every unit's full parameters +
        # gradients take at most a quarter of the device memory.
        self.persistent_reason = "requested" if persistent is True else "off"
        if (not ring and persistent in (None, "auto") and sharding_strategy == "FULL_SHARD" and self.world > 1
                and self.device.type == "cuda"):
            # FULL_SHARD across ranks: the ring keeps the real reshard-after-forward memory bound
            # (3 units' worth, not the whole model on every rank) and a capturable step
            ring = 3
        if ring:
            persistent = False
        if persistent is None or persistent == "auto":
            if self.device.type == "cuda":
                need = sum(p.numel() for p in module.parameters()) * (
                    torch.finfo(self.mp.param_dtype or torch.float32).bits // 8 + 4)
                cap = torch.cuda.get_device_properties(self.device).total_memory
                persistent = need <= cap // 4
                self.persistent_reason = (f"auto: full params + grads {need / 2**30:.2f} GiB "
                                          f"{'<=' if persistent else '>'} a quarter of {cap / 2**30:.0f} GiB")
                if persistent and sharding_strategy == "FULL_SHARD":
                    # FULL_SHARD semantics change (no reshard after forward): say so, once per wrapper
                    log.warning("FSDP persistent=%s: FULL_SHARD keeps gathered parameters resident between "
                                "forward and backward (%s); pass persistent=False for reshard-after-forward",
                                persistent, self.persistent_reason)
            else:
                persistent = False
                self.persistent_reason = "auto: not a GPU device"
        self.ring = int(ring) if ring and sharding_strategy == "FULL_SHARD" else 0
        if self.ring == 1:
            raise ValueError("FSDP ring needs >= 2 slots (a unit and the one being prefetched)")
        if self.ring:
            persistent = False
            self.persistent_reason = f"ring of {self.ring} gathered-unit slots"
        self.persistent = bool(persistent)
        self.sharding = sharding_strategy
        self.reshard_after_forward = sharding_strategy == "FULL_SHARD" and not self.persistent
        self.forward_prefetch = forward_prefetch
        self.backward_prefetch = backward_prefetch
        if sync_module_states and self.world > 1:
            with torch.no_grad():
                src = _group_rank0(process_group)
                for t in list(module.parameters()) + list(module.buffers()):
                    dist.broadcast(t.data, src=src, group=process_group)
        if self.mp.buffer_dtype is not None:
            for m in module.modules():
                for name, b in list(m.named_buffers(recurse=False)):
                    if b is not None and b.is_floating_point():
                        setattr(m, name, b.to(self.mp.buffer_dtype))
        # units: policy-selected submodules (post-order, so nested units claim first), then the root
        unit_modules = _select_units(module, auto_wrap_policy)
        if self.ring and self._ring_slots(module, unit_modules, self.ring) is None:
            log.warning("FSDP ring=%d: wrapped units nest %d+ deep, no slot assignment keeps a unit "
                        "out of its ancestors' slots; using reshard-after-forward without the ring",
                        self.ring, self.ring)
            self.ring = 0
            self.persistent_reason = "ring disabled: nested units"
        claimed: Set[int] = set()
        self.units: List[_Unit] = []
        for um in unit_modules + [module]:
            params = []
            for p in um.parameters():
                if id(p) not in claimed:
                    claimed.add(id(p))
                    params.append(p)
            # the root unit (embeddings, head) stays gathered for the whole step: never in the ring
            self.units.append(_Unit(self, um, params, len(self.units), ring_member=bool(self.ring) and um is not module))
        self.root_unit = self.units[-1]
        self._rings: Dict[str, _Ring] = {}
        if self.ring:
            self._build_rings()
        self._active: Optional[_Unit] = None
        self._live_fwd: Set[_Unit] = set()  # units between their forward pre- and post-hooks
        self._live_bwd: Set[_Unit] = set()  # units whose backward started and has not finished
        self._unit_of_param = {id(p): u for u in self.units for p in u.params}
        self._fwd_order: List[_Unit] = []
        self._recording = True
        self._in_backward = False
        self._handles = []
        for u in self.units[:-1]:
            self._handles.append(u.module.register_forward_pre_hook(self._make_pre_fwd(u)))
            self._handles.append(u.module.register_forward_hook(self._make_post_fwd(u)))
        for u in self.units:
            for p in u.params:
                if p.requires_grad:
                    self._handles.append(p.register_post_accumulate_grad_hook(self._make_grad_hook(u)))

    @staticmethod
    def _ring_slots(root: nn.Module, unit_modules: List[nn.Module], k: int) -> Optional[List[int]]:
        """Ring slot of each wrapped unit (``unit_modules`` in unit-index order), or None when no
        assignment is safe.

        A unit nested inside another wrapped unit (size-based policies wrap ``linear1`` /
        ``linear2`` AND the rest of their encoder layer) is gathered while its
        ancestor still computes from its own slot, so a unit never shares a slot with any of its
        ancestors.  Units are visited ancestors-first and cycle through the slots they may use
        (unit i -> slot i % K for a flat stack of layers); a nesting K deep has no safe slot."""
        index = {id(m): i for i, m in enumerate(unit_modules)}
        ancestors: Dict[int, List[int]] = {}

        def visit(m: nn.Module, chain: List[int]) -> None:
            i = index.get(id(m))
            if i is not None:
                ancestors[i] = chain
                chain = chain + [i]
            for c in m.children():
                visit(c, chain)

        visit(root, [])
        slots: List[int] = [-1] * len(unit_modules)
        nxt = 0
        for i in sorted(range(len(unit_modules)), key=lambda i: (len(ancestors.get(i, [])), i)):
            banned = {slots[a] for a in ancestors.get(i, [])}
            free = [s for s in ((nxt + j) % k for j in range(k)) if s not in banned]
            if not free:
                return None
            slots[i] = free[0]
            nxt = free[0] + 1
        return slots

    def _build_rings(self) -> None:
        """One parameter ring per (kind, dtype) and one gradient ring, each slot sized to the
        largest member; slots come from ``_ring_slots`` (unit i -> slot i % K for a flat stack)."""
        members = [u for u in self.units if u is not self.root_unit]
        slot_of = self._ring_slots(self.module, [u.module for u in members], self.ring)
        assert slot_of is not None  # checked before the units were built (__init__)
        for kind in ("train", "frozen"):
            groups = [getattr(u, kind) for u in members if getattr(u, kind) is not None]
            groups = [g for g in groups if g.ring_member]
            if not groups:
                continue
            pr = _Ring(self.ring, max(g.padded for g in groups), groups[0].cdtype, self.device)
            gr = (_Ring(self.ring, max(g.padded for g in groups), groups[0].rdtype, self.device)
                  if kind == "train" else None)
            self._rings[kind] = pr
            if gr is not None:
                self._rings["grad"] = gr
            for g in groups:
                g.attach_ring(pr, gr, slot_of[g.unit_index])

    def memory_plan(self) -> Dict[str, float]:
        """GiB of gathered-parameter / full-gradient buffers this configuration keeps allocated."""
        gib = 2.0 ** 30
        if self.ring:
            ring = sum(r.nbytes for r in self._rings.values())
            root = sum(g._full_bytes + g._grad_bytes for g in self.root_unit.groups if not g.resident)
            return {"mode": f"ring{self.ring}", "gathered_gib": (ring + root) / gib}
        tot = sum(g.padded * (g.full.element_size() + (g.full_grad.element_size() if g.trainable else 0))
                  for g in self.flat_groups() if not g.resident)
        return {"mode": "persistent" if self.persistent else "reshard (peak: the units in flight)", "gathered_gib": tot / gib}

    @property
    def comm(self):
        """AG / RS transport: native RCCL communicator on GPU, torch.distributed elsewhere."""
        if self._comm is None:
            self._comm = get_comm(self.device, self.group)
        return self._comm

    # -- parameters the optimizer sees ------------------------------------------------------
    def parameters(self, recurse: bool = True) -> Iterator[nn.Parameter]:  # type: ignore[override]
        for u in self.units:
            if u.train is not None:
                yield u.train.flat_param

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True):  # type: ignore[override]
        for u in self.units:
            if u.train is not None:
                yield f"{prefix}flat_param_{u.index}", u.train.flat_param

    def flat_groups(self) -> List[_FlatGroup]:
        return [g for u in self.units for g in u.groups]

    # -- hooks ------------------------------------------------------------------------------
    def _make_pre_fwd(self, u: _Unit):
        def hook(module, args):
            if torch.is_grad_enabled():
                ins = [t for t in _flatten(args) if isinstance(t, torch.Tensor) and t.requires_grad]
                if ins:
                    torch.autograd.graph.register_multi_grad_hook(ins, lambda grads: self._input_grads(u), mode="all")
            if self._recording and u not in self._fwd_order:
                self._fwd_order.append(u)
            self._live_fwd.add(u)
            self._active = u
            u.gather()
            if self.forward_prefetch and not self._recording:
                nxt = self._neighbour(u, +1)
                if nxt is not None and not nxt.ring_slot_busy(u):
                    nxt.gather(async_op=True)
            return None

        return hook

    def _make_post_fwd(self, u: _Unit):
        def hook(module, args, output):
            self._live_fwd.discard(u)
            grad = torch.is_grad_enabled()
            if self.reshard_after_forward or not grad:
                u.reshard()
            if grad:
                tensors = [t for t in _flatten(output) if isinstance(t, torch.Tensor) and t.requires_grad]
                if tensors:
                    torch.autograd.graph.register_multi_grad_hook(tensors, self._make_pre_bwd(u), mode="any")
            return None

        return hook

    def _on_compute_stream(self):
        """Run a backward hook's work on the forward's stream (ops.streams.on_stream): a
        gradient copy or an RCCL issue ordered against another stream would race the backward
        kernels still writing the gradients (graph warm-up and capture run on side streams)."""
        return _streams.on_stream(getattr(self, "_compute_stream", None))

    def _make_pre_bwd(self, u: _Unit):
        def hook(grad):
            with self._on_compute_stream():
                self._ensure_backward_started()
                self._active = u
                self._live_bwd.add(u)
                u.gather()
                if self.backward_prefetch:
                    prv = self._neighbour(u, -1)
                    if prv is not None and not prv.reduced and not prv.ring_slot_busy(u):
                        prv.gather(async_op=True)

        return hook

    def _make_grad_hook(self, u: _Unit):
        def hook(p):
            with self._on_compute_stream():
                self._ensure_backward_started()
                u.on_grad(p)

        return hook

    def _neighbour(self, u: _Unit, step: int) -> Optional[_Unit]:
        try:
            k = self._fwd_order.index(u) + step
        except ValueError:
            return None
        return self._fwd_order[k] if 0 <= k < len(self._fwd_order) else None

    def _ensure_backward_started(self) -> None:
        if not self._in_backward:
            self._in_backward = True
            for u in self.units:
                u.start_backward()
            torch.autograd.Variable._execution_engine.queue_callback(self._post_backward)

    def _input_grads(self, u: _Unit) -> None:
        with self._on_compute_stream():
            u.on_input_grads()

    def _post_backward(self) -> None:
        with self._on_compute_stream():
            self._post_backward_body()

    def _post_backward_body(self) -> None:
        for u in self.units:
            u.finish()
            for g in u.groups:
                if not g.trainable:
                    continue  # frozen weights never change: a persistent gathered copy stays valid
                g.send_valid = False  # the optimizer steps next: recast on the next forward gather
                if g.pinned and not g.resident:
                    g.gathered = False  # ... and re-gather (the persistent buffer keeps its storage)
        self._in_backward = False
        self._active = None
        self._live_bwd.clear()

    def invalidate_gather_cache(self) -> None:
        """Call after changing the flat shards outside an optimizer step that follows backward."""
        for g in self.flat_groups():
            g.send_valid = False
            if g.pinned and not g.resident:
                g.gathered = False

    # -- forward ----------------------------------------------------------------------------
    def _root_pre(self) -> None:
        # the stream the step's compute runs on: backward hooks issue their copies and collectives
        # on it (see _on_compute_stream)
        self._compute_stream = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        self._live_fwd.clear()
        self.root_unit.gather()
        if self.forward_prefetch and not self._recording and self._fwd_order:
            self._fwd_order[0].gather(async_op=True)

    def _root_post(self) -> None:
        if self._fwd_order:
            self._recording = False
        if not torch.is_grad_enabled():
            self.root_unit.reshard()

    def forward(self, *args, **kwargs):
        self._root_pre()
        out = self.module(*args, **kwargs)
        self._root_post()
        return out

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            pass
        attr = getattr(self.module, name)
        if callable(attr) and not isinstance(attr, nn.Module) and getattr(attr, "__self__", None) is self.module:
            # methods such as ``forward_loss`` run the wrapped model: gather the root unit first
            def call(*args, **kwargs):
                self._root_pre()
                out = attr(*args, **kwargs)
                self._root_post()
                return out

            return call
        return attr

    # -- gradient clipping ---------------------------------------------------------------------
    def clip_grad_norm_(self, max_norm: float, defer_to=None) -> torch.Tensor:
        """Global L2 norm over every rank's shard (fixes the reference's local-shard clip, C25).
        ``defer_to``: a FusedAdam that applies the coefficient inside its step (ops.optim)."""
        return clip_grad_norm_(list(self.parameters()), max_norm, group=self.group, sharded=self.world > 1,
                               defer_to=defer_to)

    # -- state dicts (collective: call on EVERY rank) ---------------------------------------------
    @torch.no_grad()
    def full_state_dict(self, rank0_only: bool = True, offload_to_cpu: bool = True) -> Dict[str, torch.Tensor]:
        """All-gather every flat shard on all ranks; keys are the original module's.

        The reference entered this collective on rank 0 only (K13: a mismatched RCCL collective);
        here every rank participates and ``rank0_only`` just drops the result elsewhere.
        """
        full_params: Dict[int, torch.Tensor] = {}
        for g in self.flat_groups():
            full = torch.empty(g.padded, dtype=g.flat_param.dtype, device=self.device)
            if self.world > 1 and not g.resident:
                dist.all_gather_into_tensor(full, g.flat_param.detach(), group=self.group)
            else:
                full.copy_(g.flat_param.detach())
            for p, o, n, shp in zip(g.params, g.offsets, g.numels, g.shapes):
                full_params[id(p)] = full[o : o + n].view(shp)
        if rank0_only and self.rank != 0:
            return {}
        out: Dict[str, torch.Tensor] = {}
        for name, t in self.module.state_dict(keep_vars=True).items():
            v = full_params[id(t)] if id(t) in full_params else t.detach()
            v = v.clone()
            out[name] = v.cpu() if offload_to_cpu else v
        return out

    def state_dict(self, *args, **kwargs):  # full dict on every rank (collective)
        return self.full_state_dict(rank0_only=False, offload_to_cpu=False)

    @torch.no_grad()
    def load_full_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        """Every rank passes the full dict (e.g. from ``torch.load(weights_only=True)``); shards are sliced locally."""
        names = {id(t): n for n, t in self.module.state_dict(keep_vars=True).items()}
        for g in self.flat_groups():
            flat = torch.zeros(g.padded, dtype=g.flat_param.dtype, device=self.device)
            for p, o, n in zip(g.params, g.offsets, g.numels):
                flat[o : o + n].copy_(sd[names[id(p)]].reshape(-1).to(self.device, flat.dtype))
            r = 0 if g.resident else self.rank
            g.flat_param.data.copy_(flat[r * g.shard_numel : (r + 1) * g.shard_numel])
        self.invalidate_gather_cache()
        for n, t in self.module.state_dict(keep_vars=True).items():
            if id(t) not in self._unit_of_param and n in sd:
                t.data.copy_(sd[n].to(t.device, t.dtype))

    def load_state_dict(self, state_dict, strict: bool = True):
        self.load_full_state_dict(state_dict)

    def sharded_state_dict(self) -> Dict[str, object]:
        """This rank's flat shards + layout metadata (no communication)."""
        names = {id(t): n for n, t in self.module.state_dict(keep_vars=True).items()}
        groups = self.flat_groups()
        return {
            "world_size": self.world,
            "rank": self.rank,
            # resident (replicated frozen) groups: rank 0 holds the copy (no N-fold checkpoint)
            "flat_params": [None if (g.resident and self.rank != 0) else g.flat_param.detach().cpu().clone()
                            for g in groups],
            "meta": [{"tag": g.tag, "names": [names.get(id(p), "?") for p in g.params],
                      "shapes": [tuple(s) for s in g.shapes], "numel": g.numel, "padded": g.padded} for g in groups],
            "buffers": {n: b.detach().cpu().clone() for n, b in self.module.named_buffers()},
        }

    @torch.no_grad()
    def load_sharded_state_dict(self, sd: Dict[str, object]) -> None:
        if sd["world_size"] != self.world:
            raise ValueError(f"sharded checkpoint has world_size {sd['world_size']}, running with {self.world}")
        for g, t in zip(self.flat_groups(), sd["flat_params"]):
            if t is not None:
                g.flat_param.data.copy_(t.to(self.device))
            if g.resident and self.world > 1:  # group-rank 0's copy of a replicated frozen group
                dist.broadcast(g.flat_param.data, src=_group_rank0(self.group), group=self.group)
        self.invalidate_gather_cache()
        bufs = dict(self.module.named_buffers())
        for n, t in sd.get("buffers", {}).items():
            if n in bufs:
                bufs[n].copy_(t.to(bufs[n].device, bufs[n].dtype))

    def unit_sizes(self) -> List[int]:
        """Unsharded numel per unit (the all-gather / reduce-scatter message sizes)."""
        return [u.numel for u in self.units]


def _flatten(obj) -> Sequence:
    if isinstance(obj, torch.Tensor):
        return [obj]
    if isinstance(obj, (list, tuple)):
        return [t for o in obj for t in _flatten(o)]
    if isinstance(obj, dict):
        return [t for o in obj.values() for t in _flatten(o)]
    return []


FSDP = FullyShardedDataParallel
