"""Distributed trainers with the reference's names, signatures, CSV schemas and checkpoint layout.

Reference (``02_development/distributed_utils.py``):

* ``train_language_model_ddp(rank, world, epochs, base_dir)`` — SimpleTransformerLM-256, per-rank
  batch 32, AdamW 2e-4, CE(ignore pad), fp16 autocast + GradScaler, DDP (:132-200);
* ``train_cifar_model_ddp(rank, world, epochs, base_dir)`` — ResNet-18 (10 classes), batch 64,
  AdamW 1e-3, fp16 AMP, DDP, accuracy (:208-278);
* ``train_language_model_fsdp(rank, world, epochs, base_dir)`` — the LM under FSDP FULL_SHARD,
  size-based wrap (100k), bf16 mixed precision, clip 1.0, AdamW 1e-4 (:290-406);
* ``train_llama_fsdp(rank, world, *, epochs, base_dir, hf_token, model_id, lora, batch_size,
  progress_every)`` — Llama-2-7B, LoRA r16 (DDP) or full FSDP, AdamW 1e-5 wd .01, clip 1.0
  (:415-554).

Hyperion differences (each documented where it happens): synthetic data of the real shapes by
default (no network); seeded; device-side loss/accuracy accumulation (the reference synced with
``loss.item()`` every step, K15); global-norm clipping under FSDP; collective-safe checkpoints on
every rank; resume support; LoRA can also run under FSDP (the BASELINE config) with layer-class
wrapping (the reference's policy never recursed, K8); fault injection (``HYPERION_FAULT``).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader

from ..data import DistributedSampler, SyntheticCIFAR10, SyntheticWikiText2, WikiText2TorchDataset, load_wikitext2
from ..data.loader import DevicePrefetcher, DeviceTensorLoader, dataset_tensors
from ..models.simple_lm import GPT2_PAD, GPT2_VOCAB, simple_lm_256
from ..ops.optim import FusedAdam, clip_grad_norm_
from ..parallel.launch import cleanup, setup
from ..utils.fault import maybe_inject
from ..utils.seed import seed_everything
from .amp import LossScaler
from .checkpoint import load_checkpoint, restore_rng, rng_state, save_checkpoint
from .metrics import SCHEMAS, MetricsCSV, make_run_id, write_manifest

DEFAULT_BASE_DIR = os.environ.get("HYPERION_BASE_DIR", os.getcwd())


@dataclass
class RunOptions:
    """Knobs the reference hard-coded; defaults reproduce its settings."""

    synthetic: bool = True
    dataset_size: Optional[int] = None      # None = the real dataset's size
    max_steps_per_epoch: Optional[int] = None
    precision: Optional[str] = None         # override: fp32 | fp16 | bf16
    seed: int = 0
    save: bool = True
    ckpt_mode: str = "full"                 # full | sharded (FSDP)
    resume: Optional[str] = None            # checkpoint path, or "auto" = this run kind's latest checkpoint
    ckpt_every: Optional[int] = None        # also write the latest checkpoint every N steps (restartable)
    num_workers: int = 2
    causal: bool = False                    # reference LM had no causal mask
    timeout_s: float = 600.0
    # hipGraph-captured steps on GPU (the fwd + bwd + optimizer of one step replayed as one or two
    # graph launches; DDP: all-reduces eager between the two graphs).  None = on for CUDA.
    graph: Optional[bool] = None
    # GPU: tensor datasets resident in HBM and batched on the device (data/loader.py
    # DeviceTensorLoader) instead of DataLoader workers + per-step H2D copies
    device_data: bool = True
    # after training, all-gather per-parameter checksums and raise if the data-parallel replicas
    # differ (parallel/debug.py); the count of compared tensors is returned as "replicas"
    check_replicas: bool = False
    # FSDP FULL_SHARD ring slots (>= 2): gathered units share fixed-address buffers (reshard-after-
    # forward memory, capturable step); 0 = the wrapper's default (ring 3 at world > 1 on GPU,
    # persistent buffers at world 1)
    fsdp_ring: int = 0
    log: Callable[[str], None] = field(default=print)


def _out_dir(base_dir: str) -> str:
    d = os.path.join(base_dir, "data", "distributed")
    os.makedirs(d, exist_ok=True)
    return d


def _loader(ds, world, rank, batch, opts: RunOptions, device, drop_last=False):
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=opts.seed)
    if device.type == "cuda" and opts.device_data:
        tensors = dataset_tensors(ds)
        if tensors is not None:  # the whole dataset resident in HBM, batched on the device
            return sampler, DeviceTensorLoader(tensors, sampler, batch, device, drop_last=drop_last)
    dl = DataLoader(ds, batch_size=batch, sampler=sampler, num_workers=opts.num_workers if device.type == "cuda" else 0,
                    pin_memory=device.type == "cuda", drop_last=drop_last, persistent_workers=False)
    return sampler, DevicePrefetcher(dl, device)


def _wikitext(opts: RunOptions, base_dir: str):
    if not opts.synthetic:
        path = os.path.join(base_dir, "data", "processed", "wikitext2_tokenized")
        return WikiText2TorchDataset(load_wikitext2(path, "train"), split="train")
    kw = {} if opts.dataset_size is None else {"n": opts.dataset_size}
    return SyntheticWikiText2(seed=opts.seed, **kw)


def _reduce_mean(t: torch.Tensor, world: int) -> torch.Tensor:
    if world > 1:
        dist.all_reduce(t)
        t = t / world
    return t


def _shared_run_id(name: str, world: int) -> str:
    """Rank 0's clock names the run on every rank (per-rank clocks can straddle a second boundary
    and name the checkpoint / optimizer-shard files differently)."""
    when = [time.time()]
    if world > 1 and dist.is_available() and dist.is_initialized():
        dist.broadcast_object_list(when, src=0)
    return make_run_id(name, world, when[0])


def _amp(precision: str):
    return {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[precision]


class _EpochRunner:
    """Shared hot loop: device-side loss accumulation, fault hook, timing, and (on GPU) a
    hipGraph-captured step — the reference trainers' loops then replay one or two graphs per step
    instead of dispatching ~10^3 kernels from Python (trainers on the fast path)."""

    def __init__(self, rank, world, device, model, opt, scaler, amp_dtype, clip, sharded_clip, opts: RunOptions):
        self.rank, self.world, self.device = rank, world, device
        self.model, self.opt, self.scaler = model, opt, scaler
        self.amp_dtype = amp_dtype
        self.clip, self.sharded_clip = clip, sharded_clip
        self.opts = opts
        self.global_step = 0
        self.save_latest: Optional[Callable[[int, int], None]] = None  # (epoch, batches done in it)
        want = opts.graph if opts.graph is not None else device.type == "cuda"
        self.graph = bool(want) and device.type == "cuda" and torch.cuda.is_available()
        self._captured: Optional[_CapturedStep] = None
        self.graph_reason = ""  # why a requested graph fell back to eager (logged once)

    def after_step(self, epoch: int, done_in_epoch: int) -> None:
        """Periodic latest checkpoint (``RunOptions.ckpt_every``): collective for FSDP, every rank calls."""
        if self.save_latest is not None and self.opts.ckpt_every and self.global_step % self.opts.ckpt_every == 0:
            self.save_latest(epoch, done_in_epoch)

    def _autocast(self):
        return torch.autocast(self.device.type, dtype=self.amp_dtype or torch.float32,
                              enabled=self.amp_dtype is not None
                              and not (self.device.type == "cpu" and self.amp_dtype == torch.float16))

    def _graphable(self) -> bool:
        from ..parallel.ddp import DistributedDataParallel
        from ..parallel.fsdp import FullyShardedDataParallel

        why = ""
        if isinstance(self.model, FullyShardedDataParallel) and not (self.model.persistent or self.model.ring):
            why = "FSDP step without persistent or ring buffers (storage released / re-allocated per unit)"
        elif isinstance(self.model, DistributedDataParallel) and self.world > 1 and not self.model.bucketed:
            why = "DDP without gradient buckets"
        elif (isinstance(self.model, DistributedDataParallel) and self.world > 1 and self.model.broadcast_buffers
              and os.environ.get("HYPERION_DDP_CAPTURE", "segments") == "split"):
            # the split capture records fwd+bwd as ONE plain graph: the per-forward buffer broadcast
            # would be recorded into it (an RCCL call inside a graph) — only the segmented capture
            # turns it into an eager hole
            why = "split DDP capture with broadcast_buffers=True (per-forward buffer broadcast)"
        elif self.world > 1 and not isinstance(self.model, DistributedDataParallel):
            why = "non-Hyperion data parallel wrapper"
        elif os.environ.get("HYPERION_FAULT"):
            why = "fault injection needs host-side per-step control"
        if why and not self.graph_reason:
            self.graph_reason = why
            if self.rank == 0:
                self.opts.log(f"[graph] eager steps: {why}")
        return not why

    def step(self, loss_fn, inputs: Optional[tuple] = None):
        """``loss_fn(*inputs) -> (loss, extra)``; returns ``(loss fp32 detached, extra)``.  With
        ``inputs`` and a capturable model the step is replayed from a hipGraph."""
        if self.graph and inputs is not None and self._graphable():
            if self._captured is None:
                self._captured = _CapturedStep(self, loss_fn, inputs)
            if self._captured.fits(inputs):  # (a short last batch runs eagerly)
                self.global_step += 1
                return self._captured(inputs)
        inputs = inputs or ()
        cap = self._captured
        if cap is not None:
            # an eager step beside a captured one (a short last batch): the graphs and the fused
            # optimizer's pinned table hold the current .grad tensors, so they are zeroed in place and
            # accumulated into — dropping them (set_to_none) would leave later replays writing freed
            # blocks
            self.opt.zero_grad(set_to_none=False)
        else:
            self.opt.zero_grad(set_to_none=True)
        with self._autocast():
            loss, extra = loss_fn(*inputs)
        if maybe_inject(self.rank, self.global_step):
            loss = loss * float("nan")
        # a captured DDP step left the hooks in deferred mode (they only pack buckets): reduce here
        self._backward_update(loss, allreduce=cap.eager_allreduce() if cap is not None else None)
        self.global_step += 1
        return loss.detach().float(), extra

    def _backward_update(self, loss, allreduce: Optional[Callable[[], None]] = None) -> None:
        if self.scaler is not None and self.scaler.enabled:
            self.scaler.scale(loss).backward()
            if allreduce is not None:
                allreduce()
            if self.clip is not None:
                self.scaler.unscale_(self.opt)
                self._clip()
            self.scaler.step(self.opt)
            self.scaler.update()
        else:
            loss.backward()
            if allreduce is not None:
                allreduce()
            if self.clip is not None:
                self._clip(defer=True)
            self.opt.step()

    def _clip(self, defer: bool = False) -> None:
        """``defer``: FusedAdam applies the clip coefficient inside its step (one gradient pass fewer)."""
        from ..ops.optim import FusedAdam

        d = self.opt if defer and isinstance(self.opt, FusedAdam) else None
        if hasattr(self.model, "clip_grad_norm_"):
            self.model.clip_grad_norm_(self.clip, defer_to=d)
        else:
            clip_grad_norm_(self.model.parameters(), self.clip, sharded=self.sharded_clip, defer_to=d)


class _CapturedStep:
    """One trainer step as hipGraph(s): warm-up on a side stream, then capture.

    Single process: ONE graph (zero, forward, backward, unscale/clip, optimizer, scaler update).
    Hyperion DDP (default, ``HYPERION_DDP_CAPTURE=segments``): the whole step as graph segments;
    each bucket's all-reduce is an eager hole issued where the bucket completed inside the backward
    (and its wait where the backward ends), and a per-forward buffer broadcast (BN models,
    ``broadcast_buffers=True``) is a hole before the forward — RCCL overlaps the captured backward
    for every model.  ``HYPERION_DDP_CAPTURE=split``: graph 1 = forward + backward (hooks only
    pack, ``defer_allreduce``), eager bucket all-reduces, graph 2 = clip + optimizer.
    Hyperion FSDP (persistent buffers): the whole step as graph segments with every all-gather /
    reduce-scatter / clip all-reduce an eager hole between them (``train/segments.py``).
    No RCCL call is ever recorded into a graph.
    Inputs are copied into persistent buffers each step; outputs are the captured step's tensors.
    """

    def __init__(self, runner: "_EpochRunner", loss_fn, inputs: tuple, warmup: int = 3):
        from ..ops.multi_tensor import flush_pending
        from ..parallel.ddp import DistributedDataParallel
        from ..parallel.fsdp import FullyShardedDataParallel
        from .segments import SegmentedGraph

        self.r = runner
        self.seg: Optional[SegmentedGraph] = None
        self.fn = loss_fn
        self.static = [t.clone() if isinstance(t, torch.Tensor) else t for t in inputs]
        m = runner.model
        self.ddp = m if isinstance(m, DistributedDataParallel) and runner.world > 1 else None
        self.ddp_segments = self.ddp is not None and os.environ.get("HYPERION_DDP_CAPTURE", "segments") != "split"
        if self.ddp is not None and not self.ddp_segments:
            self.ddp.defer_allreduce = True
        scaled = runner.scaler is not None and runner.scaler.enabled
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            runner.opt.zero_grad(set_to_none=True)
            for _ in range(warmup):
                self._full(zero_in_place=True)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not scaled:  # let autograd steal fresh gradients inside the capture (no per-param add)
            runner.opt.zero_grad(set_to_none=True)
        zero_flag = getattr(runner.opt, "zero_grad_in_step", None)
        if zero_flag and not scaled:
            runner.opt.zero_grad_in_step = False
        self.g1 = torch.cuda.CUDAGraph()
        self.g2: Optional[torch.cuda.CUDAGraph] = None
        from ..ops.batchnorm import HostCounterReplay

        counters = HostCounterReplay(m)  # BN num_batches_tracked mirrors: undo the recording pass
        try:
            if isinstance(m, FullyShardedDataParallel) or self.ddp_segments:
                self.seg = SegmentedGraph()
                self.out = self.seg.capture(lambda: self._full(zero_in_place=scaled))
            elif self.ddp is None:
                with torch.cuda.graph(self.g1):
                    self.out = self._full(zero_in_place=scaled)
            else:
                with torch.cuda.graph(self.g1):
                    self.out = self._fwd_bwd(zero_in_place=scaled)
                self.g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g2, pool=self.g1.pool()):
                    self._update()
        finally:
            flush_pending()
            if zero_flag is not None:
                runner.opt.zero_grad_in_step = zero_flag
        self.counters = counters.captured()
        torch.cuda.synchronize()

    def _fwd_bwd(self, zero_in_place: bool):
        r = self.r
        if zero_in_place:
            r.opt.zero_grad(set_to_none=False)
        with r._autocast():
            loss, extra = self.fn(*self.static)
        if r.scaler is not None and r.scaler.enabled:
            r.scaler.scale(loss).backward()
        else:
            loss.backward()
        return loss.detach().float(), extra

    def _update(self) -> None:
        r = self.r
        if r.scaler is not None and r.scaler.enabled:
            if r.clip is not None:
                r.scaler.unscale_(r.opt)
                r._clip()
            r.scaler.step(r.opt)
            r.scaler.update()
        else:
            if r.clip is not None:
                r._clip()
            r.opt.step()

    def _full(self, zero_in_place: bool):
        out = self._fwd_bwd(zero_in_place)
        if self.ddp is not None and self.ddp.defer_allreduce:
            self.ddp.allreduce_buckets()
        self._update()
        return out

    def eager_allreduce(self) -> Optional[Callable[[], None]]:
        """What an eager step beside this capture must run after its backward: the deferred
        bucket all-reduce of the split-graph DDP mode (its hooks only pack), else nothing."""
        if self.ddp is not None and self.ddp.defer_allreduce:
            return self.ddp.allreduce_buckets
        return None

    def fits(self, inputs: tuple) -> bool:
        return all(not isinstance(st, torch.Tensor) or (isinstance(t, torch.Tensor) and t.shape == st.shape)
                   for st, t in zip(self.static, inputs))

    def __call__(self, inputs: tuple):
        for st, t in zip(self.static, inputs):
            if isinstance(st, torch.Tensor) and st.data_ptr() != t.data_ptr():
                st.copy_(t, non_blocking=True)
        self.counters.replayed()
        if self.seg is not None:
            self.seg.replay()
            return self.out
        self.g1.replay()
        if self.g2 is not None:
            self.ddp.allreduce_buckets()
            self.g2.replay()
        return self.out


def _replicas(opts: RunOptions, model, world: int) -> Optional[int]:
    from ..parallel.ddp import DistributedDataParallel

    if not (opts.check_replicas and world > 1 and isinstance(model, DistributedDataParallel)):
        return None
    from ..parallel.debug import assert_replicas_in_sync

    return assert_replicas_in_sync(model)


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


# ---------------------------------------------------------------------------------------- LM DDP
def train_language_model_ddp(rank: int, world: int, epochs: int = 3, base_dir: str = DEFAULT_BASE_DIR,
                             opts: Optional[RunOptions] = None, batch_size: int = 32) -> Dict:
    """C23: SimpleTransformerLM-256 + DDP + fp16 AMP; CSV ``epoch,loss,duration,gpus``."""
    from ..parallel.ddp import DDP

    opts = opts or RunOptions()
    device = setup(rank, world, timeout_s=opts.timeout_s) if world > 1 else _single_device()
    seed_everything(opts.seed, 0)  # identical init on every rank (DDP also broadcasts)
    out = _out_dir(base_dir)
    ds = _wikitext(opts, base_dir)
    sampler, loader = _loader(ds, world, rank, batch_size, opts, device)
    model = simple_lm_256(GPT2_VOCAB, causal=opts.causal).to(device)
    model = DDP(model) if world > 1 else model
    precision = opts.precision or ("fp16" if device.type == "cuda" else "fp32")
    opt = FusedAdam(model.parameters(), lr=2e-4, weight_decay=0.01, adamw=True)
    scaler = LossScaler(enabled=precision == "fp16", device=device)
    runner = _EpochRunner(rank, world, device, model, opt, scaler, _amp(precision), None, False, opts)
    inner = model.module if hasattr(model, "module") else model
    res = _maybe_resume(opts, model, opt, scaler, out, "language_ddp")
    run_id = res.run_id or _shared_run_id("language_ddp", world)
    csv = MetricsCSV(os.path.join(out, f"{run_id}_metrics.csv"), SCHEMAS["language_ddp"], enabled=rank == 0,
                     append=res.run_id is not None)
    runner.global_step = res.global_step
    _latest_saver(opts, out, "language_ddp", run_id, model, opt, scaler, runner)
    history = []
    for ep in range(res.start_epoch, epochs):
        sampler.set_epoch(ep)
        _sync(device)
        t0 = time.time()
        loss_sum = torch.zeros((), device=device)
        n = 0
        for i, (ids, _mask) in enumerate(loader):
            if opts.max_steps_per_epoch is not None and i >= opts.max_steps_per_epoch:
                break
            if res.skip_batch(ep, i):
                continue  # done before the checkpoint this run resumed from
            ddp_fwd = model if world > 1 else None

            def lm_loss(ids):
                x, y = ids[:, :-1], ids[:, 1:]
                if ddp_fwd is not None:  # DDP hooks need the wrapper's forward: run through it
                    return ddp_fwd(x, targets=y, ignore_index=GPT2_PAD), None
                return inner.forward_loss(x, y, ignore_index=GPT2_PAD), None

            loss, _ = runner.step(lm_loss, (ids,))
            loss_sum += loss
            n += 1
            runner.after_step(ep, i + 1)
        avg = _reduce_mean(loss_sum / max(n, 1), world).item()
        _sync(device)
        dur = time.time() - t0
        csv.append(epoch=ep + 1, loss=round(avg, 6), duration=round(dur, 4), gpus=world)
        history.append({"epoch": ep + 1, "loss": avg, "duration": dur, "steps": n})
        if runner.save_latest is not None:
            runner.save_latest(ep + 1, 0)
        if rank == 0:
            opts.log(f"[language_ddp] epoch {ep + 1}/{epochs} loss {avg:.4f} {dur:.2f}s ({n} steps)")
    ck = _finish(opts, out, run_id, model, opt, scaler, epochs, runner.global_step)
    _manifest(rank, out, run_id, history, batch_size, world, precision)
    replicas = _replicas(opts, model, world)
    if world > 1:
        cleanup()
    return {"replicas": replicas, "run_id": run_id, "history": history, "checkpoint": ck, "graphed": runner._captured is not None,
            "graph_reason": runner.graph_reason}


# ---------------------------------------------------------------------------------------- CIFAR DDP
def train_cifar_model_ddp(rank: int, world: int, epochs: int = 3, base_dir: str = DEFAULT_BASE_DIR,
                          opts: Optional[RunOptions] = None, batch_size: int = 64) -> Dict:
    """C24: ResNet-18 (10 classes, ImageNet stem on 32x32) + DDP + fp16 AMP; CSV with accuracy."""
    from ..data.datasets import CIFAR10TorchDataset, load_cifar10_pt
    from ..models.resnet import resnet18
    from ..parallel.ddp import DDP

    opts = opts or RunOptions()
    device = setup(rank, world, timeout_s=opts.timeout_s) if world > 1 else _single_device()
    seed_everything(opts.seed, 0)
    out = _out_dir(base_dir)
    if opts.synthetic:
        ds = SyntheticCIFAR10(seed=opts.seed, **({} if opts.dataset_size is None else {"n": opts.dataset_size}))
    else:
        ds = CIFAR10TorchDataset(load_cifar10_pt(os.path.join(base_dir, "data", "processed", "cifar10_train.pt")))
    sampler, loader = _loader(ds, world, rank, batch_size, opts, device)
    model = resnet18(num_classes=10).to(device)
    if device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    model = DDP(model, broadcast_buffers=True) if world > 1 else model
    precision = opts.precision or ("fp16" if device.type == "cuda" else "fp32")
    opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=0.01, adamw=True)
    scaler = LossScaler(enabled=precision == "fp16", device=device)
    runner = _EpochRunner(rank, world, device, model, opt, scaler, _amp(precision), None, False, opts)
    res = _maybe_resume(opts, model, opt, scaler, out, "cifar_ddp")
    run_id = res.run_id or _shared_run_id("cifar_ddp", world)
    csv = MetricsCSV(os.path.join(out, f"{run_id}_metrics.csv"), SCHEMAS["cifar"], enabled=rank == 0,
                     append=res.run_id is not None)
    runner.global_step = res.global_step
    _latest_saver(opts, out, "cifar_ddp", run_id, model, opt, scaler, runner)
    history = []
    for ep in range(res.start_epoch, epochs):
        sampler.set_epoch(ep)
        _sync(device)
        t0 = time.time()
        stats = torch.zeros(3, device=device, dtype=torch.float64)  # loss_sum, correct, total
        n = 0
        model.train()
        for i, (img, lbl) in enumerate(loader):
            if opts.max_steps_per_epoch is not None and i >= opts.max_steps_per_epoch:
                break
            if res.skip_batch(ep, i):
                continue
            if device.type == "cuda":
                img = img.contiguous(memory_format=torch.channels_last)

            def cifar_loss(img, lbl):
                logits = model(img)
                return F.cross_entropy(logits.float(), lbl), logits.detach()

            loss, logits = runner.step(cifar_loss, (img, lbl))
            stats[0] += loss
            stats[1] += (logits.argmax(1) == lbl).sum()
            stats[2] += lbl.numel()
            n += 1
            runner.after_step(ep, i + 1)
        if world > 1:
            dist.all_reduce(stats)
        loss_avg = (stats[0] / max(n, 1) / world).item()
        acc = (stats[1] / stats[2].clamp_min(1)).item() * 100.0
        _sync(device)
        dur = time.time() - t0
        csv.append(epoch=ep + 1, loss=round(loss_avg, 6), accuracy=round(acc, 4), duration=round(dur, 4), gpus=world)
        history.append({"epoch": ep + 1, "loss": loss_avg, "accuracy": acc, "duration": dur, "steps": n})
        if runner.save_latest is not None:
            runner.save_latest(ep + 1, 0)
        if rank == 0:
            opts.log(f"[cifar] epoch {ep + 1}/{epochs} loss {loss_avg:.4f} acc {acc:.2f}% {dur:.2f}s")
    ck = _finish(opts, out, run_id, model, opt, scaler, epochs, runner.global_step)
    _manifest(rank, out, run_id, history, batch_size, world, precision)
    replicas = _replicas(opts, model, world)
    if world > 1:
        cleanup()
    return {"replicas": replicas, "run_id": run_id, "history": history, "checkpoint": ck, "graphed": runner._captured is not None,
            "graph_reason": runner.graph_reason}


# ---------------------------------------------------------------------------------------- LM FSDP
def train_language_model_fsdp(rank: int, world: int, epochs: int = 3, base_dir: str = DEFAULT_BASE_DIR,
                              opts: Optional[RunOptions] = None, batch_size: int = 32,
                              model_fn: Optional[Callable[[], nn.Module]] = None, min_num_params: int = 100_000,
                              wrap: str = "size", run_name: str = "language_fsdp") -> Dict:
    """C25: the LM under FSDP FULL_SHARD, size-based wrap, bf16 mixed precision, global clip 1.0.

    ``model_fn`` / ``wrap='layer'`` / ``run_name``: the same trainer for other LMs — e.g.
    :func:`train_gpt2_fsdp` (BASELINE.json config 4) wraps one FSDP unit per transformer layer."""
    from ..models.transformer import TransformerEncoderLayer
    from ..parallel.fsdp import FSDP, MixedPrecision, size_based_auto_wrap_policy, transformer_auto_wrap_policy

    opts = opts or RunOptions()
    device = setup(rank, world, timeout_s=opts.timeout_s) if world > 1 else _single_device()
    seed_everything(opts.seed, 0)
    out = _out_dir(base_dir)
    ds = _wikitext(opts, base_dir)
    sampler, loader = _loader(ds, world, rank, batch_size, opts, device)
    base = (model_fn or (lambda: simple_lm_256(GPT2_VOCAB, causal=opts.causal)))()
    precision = opts.precision or ("bf16" if device.type == "cuda" else "fp32")
    pdt = _amp(precision)
    policy = (transformer_auto_wrap_policy({TransformerEncoderLayer}) if wrap == "layer"
              else size_based_auto_wrap_policy(min_num_params))
    model = FSDP(base, auto_wrap_policy=policy, device_id=device, mixed_precision=MixedPrecision(pdt, pdt, pdt),
                 ring=opts.fsdp_ring)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01, adamw=True)
    runner = _EpochRunner(rank, world, device, model, opt, None, None, 1.0, True, opts)
    res = _maybe_resume(opts, model, opt, None, out, run_name)
    run_id = res.run_id or _shared_run_id(run_name, world)
    csv = MetricsCSV(os.path.join(out, f"{run_id}_metrics.csv"), SCHEMAS.get(run_name, SCHEMAS["language_fsdp"]),
                     enabled=rank == 0, append=res.run_id is not None)
    runner.global_step = res.global_step
    _latest_saver(opts, out, run_name, run_id, model, opt, None, runner)
    history = []
    for ep in range(res.start_epoch, epochs):
        sampler.set_epoch(ep)
        _sync(device)
        t0 = time.time()
        loss_sum = torch.zeros((), device=device)
        n = 0
        for i, (ids, _mask) in enumerate(loader):
            if opts.max_steps_per_epoch is not None and i >= opts.max_steps_per_epoch:
                break
            if res.skip_batch(ep, i):
                continue
            loss, _ = runner.step(lambda ids: (model.forward_loss(ids[:, :-1], ids[:, 1:], ignore_index=GPT2_PAD), None),
                                  (ids,))
            loss_sum += loss
            n += 1
            runner.after_step(ep, i + 1)
        avg = _reduce_mean(loss_sum / max(n, 1), world).item()
        _sync(device)
        dur = time.time() - t0
        csv.append(epoch=ep + 1, loss=round(avg, 6), duration=round(dur, 4), gpus=world)
        history.append({"epoch": ep + 1, "loss": avg, "duration": dur, "steps": n})
        if runner.save_latest is not None:
            runner.save_latest(ep + 1, 0)
        if rank == 0:
            opts.log(f"[{run_name}] epoch {ep + 1}/{epochs} loss {avg:.4f} {dur:.2f}s")
    if world > 1:
        dist.barrier()
    ck = _finish(opts, out, run_id, model, opt, None, epochs, runner.global_step)
    _manifest(rank, out, run_id, history, batch_size, world, precision)
    replicas = _replicas(opts, model, world)
    if world > 1:
        cleanup()
    return {"replicas": replicas, "run_id": run_id, "history": history, "checkpoint": ck, "graphed": runner._captured is not None,
            "graph_reason": runner.graph_reason}


def train_gpt2_fsdp(rank: int, world: int, epochs: int = 3, base_dir: str = DEFAULT_BASE_DIR,
                    opts: Optional[RunOptions] = None, batch_size: int = 32) -> Dict:
    """BASELINE.json config 4: GPT-2-small-shaped causal LM (12 x 768, 12 heads, ff 3072, GELU,
    162.3M parameters: GPT-2-small's 124M plus an UNTIED 50257 x 768 output head, as the FSDP
    records report) under FSDP FULL_SHARD with one unit per transformer
    layer, bf16 mixed precision, global clip 1.0, on WikiText-2-shaped data (128 tokens).  The
    reference's FSDP run used the 2-layer 256-d LM (``distributed_utils.py:290-406``); this is the
    same trainer (:func:`train_language_model_fsdp`) on the larger model."""
    from ..models.simple_lm import gpt2_small_lm

    return train_language_model_fsdp(rank, world, epochs, base_dir, opts, batch_size,
                                     model_fn=lambda: gpt2_small_lm(GPT2_VOCAB), wrap="layer", run_name="gpt2_fsdp")


# ---------------------------------------------------------------------------------------- Llama
def train_llama_fsdp(rank: int, world: int, *, epochs: int = 1, base_dir: str = DEFAULT_BASE_DIR,
                     hf_token: Optional[str] = None, model_id: str = "NousResearch/Llama-2-7b-hf", lora: bool = False,
                     batch_size: int = 1, progress_every: int = 50, opts: Optional[RunOptions] = None,
                     config=None, lora_parallel: str = "fsdp", mask_pad_labels: bool = False,
                     replicate_frozen="auto") -> Dict:
    """C26: Llama fine-tune.  ``lora=True``: frozen bf16 base + r16 adapters on q/k/v/o.

    ``lora_parallel='fsdp'`` (default; the BASELINE.json config) wraps the model in FSDP with one
    unit per decoder layer and reduce-scatters only the adapters.  Whether the frozen base is
    sharded too is ``replicate_frozen``'s call (below): with the default ``"auto"`` it is
    REPLICATED whenever it fits (Llama-2-7B on MI355X: 13.5 GB of 288 GB), which makes the run
    FSDP over the adapters only — DDP-like traffic; ``replicate_frozen=False`` shards the base
    like the reference's torch FSDP.  ``'ddp'`` reproduces the reference (DDP over a replicated
    model).  ``lora=False``: full bf16 FSDP with ``LlamaDecoderLayer`` units.  ``model_id``: a LOCAL
    HF checkpoint directory (config.json + safetensors shards, models/hf_checkpoint.py) is loaded
    weights-only before LoRA / FSDP wrapping, as the reference's ``from_pretrained`` (:465-468,
    484-487); a hub id (no network here) falls back to random init of ``config`` (Llama-2-7B by
    default).  ``hf_token`` is accepted for CLI compatibility.
    ``mask_pad_labels`` fixes the reference's unmasked pad labels (:517) when set.
    ``replicate_frozen`` ("auto" | True | False): under FSDP keep the frozen base whole on every rank
    when it fits (auto: <= 1/4 of HBM — 13.5 GB of 288 GB on MI355X), so only the adapters are
    sharded and communicated; False shards the base like the reference's torch FSDP.
    """
    from ..models.llama import LlamaConfig, LlamaDecoderLayer, LlamaForCausalLM
    from ..models.lora import apply_lora, save_adapter
    from ..parallel.ddp import DDP
    from ..parallel.fsdp import FSDP, MixedPrecision, transformer_auto_wrap_policy

    del hf_token
    opts = opts or RunOptions()
    device = setup(rank, world, timeout_s=opts.timeout_s) if world > 1 else _single_device()
    seed_everything(opts.seed, 0)
    out = _out_dir(base_dir)
    from ..models.hf_checkpoint import is_hf_dir, load_hf_weights, load_llama_config

    pretrained = is_hf_dir(model_id)
    cfg = config or (load_llama_config(model_id) if pretrained else LlamaConfig.llama2_7b())
    ds = _wikitext(opts, base_dir)
    sampler, loader = _loader(ds, world, rank, batch_size, opts, device)
    precision = opts.precision or ("bf16" if device.type == "cuda" else "fp32")
    pdt = _amp(precision) or torch.float32
    with torch.device(device):
        base = LlamaForCausalLM(cfg)
    if pretrained:  # every rank reads the checkpoint; FSDP then keeps its own shard
        load_hf_weights(base, model_id)
        if rank == 0:
            opts.log(f"[llama] weights from {model_id}")
    elif rank == 0 and model_id and not os.path.isdir(str(model_id)):
        opts.log(f"[llama] {model_id}: not a local HF checkpoint directory -> random-init weights")
    if lora:
        base = apply_lora(base, r=16, alpha=32, dropout=0.05)
        mode = f"lora_{precision}"
    else:
        mode = f"fsdp_{precision}"
    policy = transformer_auto_wrap_policy({LlamaDecoderLayer})
    if lora and (lora_parallel == "ddp" or world == 1):
        model = base.to(pdt)
        model = DDP(model) if world > 1 else model
    else:
        model = FSDP(base, auto_wrap_policy=policy, device_id=device, mixed_precision=MixedPrecision(pdt, pdt, pdt),
                     replicate_frozen=replicate_frozen if lora else False, ring=opts.fsdp_ring)
    opt = FusedAdam([p for p in model.parameters() if p.requires_grad], lr=1e-5, weight_decay=0.01, adamw=True)
    runner = _EpochRunner(rank, world, device, model, opt, None, None, 1.0, isinstance(model, FSDP), opts)
    res = _maybe_resume(opts, model, opt, None, out, "llama")
    run_id = res.run_id or _shared_run_id("llama", world)
    csv = MetricsCSV(os.path.join(out, f"{run_id}_metrics.csv"), SCHEMAS["llama"], enabled=rank == 0,
                     append=res.run_id is not None)
    runner.global_step = res.global_step
    _latest_saver(opts, out, "llama", run_id, model, opt, None, runner)
    history = []
    for ep in range(res.start_epoch, epochs):
        sampler.set_epoch(ep)
        _sync(device)
        t0 = time.time()
        loss_sum = torch.zeros((), device=device)
        n = 0
        for i, (ids, msk) in enumerate(loader):
            if opts.max_steps_per_epoch is not None and i >= opts.max_steps_per_epoch:
                break
            if res.skip_batch(ep, i):
                continue
            ids = ids % cfg.vocab_size  # GPT-2-tokenized synthetic ids folded into the Llama vocab
            labels = ids.masked_fill(msk == 0, -100) if mask_pad_labels else ids.clone()

            def llama_loss(ids, msk, labels):
                return model(ids, attention_mask=msk, labels=labels).loss, None

            loss, _ = runner.step(llama_loss, (ids, msk, labels))
            loss_sum += loss
            n += 1
            runner.after_step(ep, i + 1)
            if rank == 0 and progress_every and n % progress_every == 0:
                opts.log(f"[llama] epoch {ep + 1} step {n} loss {loss.item():.4f}")
        avg = _reduce_mean(loss_sum / max(n, 1), world).item()
        _sync(device)
        dur = time.time() - t0
        csv.append(epoch=ep + 1, loss=round(avg, 6), duration_s=round(dur, 4), gpus=world, mode=mode)
        history.append({"epoch": ep + 1, "loss": avg, "duration_s": dur, "steps": n, "mode": mode})
        if runner.save_latest is not None:
            runner.save_latest(ep + 1, 0)
        if rank == 0:
            opts.log(f"[llama] epoch {ep + 1}/{epochs} loss {avg:.4f} {dur:.2f}s mode {mode}")
    ck = None
    if opts.save:
        if lora:
            # adapters only (PEFT save_pretrained layout); FSDP gathers them collectively first
            if isinstance(model, FSDP):
                sd = model.full_state_dict(rank0_only=True)
                if rank == 0:
                    ck = _save_adapter_from_sd(sd, os.path.join(out, f"{run_id}_{mode}"))
            elif rank == 0:
                inner = model.module if hasattr(model, "module") else model
                ck = save_adapter(inner, os.path.join(out, f"{run_id}_{mode}"))
        else:
            ck = save_checkpoint(os.path.join(out, f"{run_id}_{mode}.pt"), model, None, None, epochs,
                                 runner.global_step, mode=opts.ckpt_mode)
    _manifest(rank, out, run_id, history, batch_size, world, precision)
    replicas = _replicas(opts, model, world)
    if world > 1:
        cleanup()
    return {"replicas": replicas, "run_id": run_id, "history": history, "checkpoint": ck, "mode": mode,
            "graphed": runner._captured is not None, "graph_reason": runner.graph_reason,
            "weights": f"pretrained:{model_id}" if pretrained else "random-init"}


def _save_adapter_from_sd(sd: Dict[str, torch.Tensor], out_dir: str) -> str:
    import json

    from safetensors.torch import save_file

    from ..models.lora import lora_config_dict

    os.makedirs(out_dir, exist_ok=True)
    ad = {"base_model.model." + k.replace(".default.", "."): v.contiguous() for k, v in sd.items()
          if ".lora_A." in k or ".lora_B." in k}
    save_file(ad, os.path.join(out_dir, "adapter_model.safetensors"))
    with open(os.path.join(out_dir, "adapter_config.json"), "w") as f:
        json.dump(lora_config_dict(16, 32, 0.05, ["k_proj", "o_proj", "q_proj", "v_proj"]), f, indent=2)
    return out_dir


# ---------------------------------------------------------------------------------------- helpers
def _single_device() -> torch.device:
    from ..utils.device import get_device

    d = get_device()
    if d.type == "cuda":
        torch.cuda.set_device(d)
    return d


@dataclass
class _Resume:
    """Where a resumed run picks up: epoch (completed epochs), batches already done in it."""

    start_epoch: int = 0
    skip: int = 0
    run_id: Optional[str] = None
    global_step: int = 0
    rng: Optional[Dict] = None

    def skip_batch(self, epoch: int, i: int) -> bool:
        """True for batches done before the checkpoint.  The generator states are restored at the
        first batch that runs: creating the epoch's DataLoader iterator draws from the global
        generator, so restoring earlier would shift every later dropout mask."""
        if epoch != self.start_epoch:
            return False
        if i < self.skip:
            return True
        if self.rng is not None:
            restore_rng(self.rng)
            self.rng = None
        return False


def _latest_path(out: str, run_name: str) -> str:
    return os.path.join(out, f"{run_name}_latest.pt")


def _maybe_resume(opts: RunOptions, model, opt, scaler, out: Optional[str] = None,
                  run_name: Optional[str] = None) -> _Resume:
    """Restore from ``opts.resume`` (a path, or ``"auto"`` = the latest checkpoint of this run kind
    in ``out`` if one exists): model / optimizer / scaler / RNG state and the position in the data
    stream, so an interrupted run continues bit-for-bit where its last checkpoint was taken."""
    path = opts.resume
    if path == "auto":
        path = _latest_path(out, run_name) if out and run_name else None
        if path is None or not os.path.exists(path):
            return _Resume()
    if not path:
        return _Resume()
    meta = load_checkpoint(path, model, opt, scaler)
    rng = {k: v for k, v in meta.items() if k.startswith("rng_")} or None
    return _Resume(int(meta.get("epoch", 0)), int(meta.get("step_in_epoch", 0)), meta.get("run_id"),
                   int(meta.get("step", 0)), rng)


def _latest_saver(opts: RunOptions, out: str, run_name: str, run_id: str, model, opt, scaler, runner) -> None:
    if not opts.ckpt_every:
        return

    def save(epoch: int, done: int) -> None:
        save_checkpoint(_latest_path(out, run_name), model, opt, scaler, epoch, runner.global_step,
                        mode=opts.ckpt_mode, extra={"step_in_epoch": done, "run_id": run_id, **rng_state()})

    runner.save_latest = save


def _finish(opts: RunOptions, out: str, run_id: str, model, opt, scaler, epoch: int, step: int):
    if not opts.save:
        return None
    return save_checkpoint(os.path.join(out, f"{run_id}_model.pt"), model, opt, scaler, epoch, step, mode=opts.ckpt_mode)


def _manifest(rank: int, out: str, run_id: str, history, batch: int, world: int, precision: str) -> None:
    if rank != 0 or not history:
        return
    steady = history[len(history) // 3:] or history
    dur_key = "duration" if "duration" in steady[0] else "duration_s"
    steps = sum(h["steps"] for h in steady)
    secs = sum(h[dur_key] for h in steady)
    write_manifest(os.path.join(out, f"{run_id}_run.json"), {
        "run_id": run_id, "world": world, "per_rank_batch": batch, "precision": precision, "history": history,
        "samples_per_s": (steps * batch * world / secs) if secs > 0 else None,
        "ms_per_step": (secs / steps * 1e3) if steps else None,
        "peak_mem_mb": torch.cuda.max_memory_allocated() / 2**20 if torch.cuda.is_available() else None,
    })
