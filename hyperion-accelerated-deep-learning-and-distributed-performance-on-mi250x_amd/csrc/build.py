"""In-tree build of the ``hyperion._C`` extension for gfx950.

No setuptools/BuildExtension (that path hipifies sources); this drives ``hipcc`` directly:

* every ``kernels/*.hip`` is pure HIP device code with ``extern "C"``-style launchers (no torch
  headers, so each compiles in seconds);
* ``bindings/*.cpp`` and ``comm/*.cpp`` include the torch C++ API and wrap the launchers;
* objects are cached under ``csrc/build/`` and rebuilt when the source or any header in
  ``csrc/`` changes; the shared object lands next to the package ``__init__`` as ``_C.so`` so it
  travels with the repo snapshot to the GPU box.

Usage: ``python -m hyperion.csrc.build [--force] [-j N] [--debug]``.

``--debug`` builds ``_C_debug.so`` (objects under ``csrc/build_debug/``): ``-O1``, ``HYP_DEBUG``
device checks (``HYP_DASSERT``: staging addresses inside their operands, shape invariants) — the
kernel bounds-check build of SURVEY §5.2, loaded instead of ``_C`` when ``HYPERION_DEBUG_BUILD=1``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import re
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List

CSRC = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(CSRC)
BUILD = os.path.join(CSRC, "build")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("HYPERION_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm at /opt/rocm)")


def _torch_paths():
    import torch  # noqa: F401
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    return inc, lib, bool(torch._C._GLIBCXX_USE_CXX11_ABI)


_INCLUDE = re.compile(rb'^\s*#\s*include\s+"([^"]+)"', re.M)


def _headers_digest(src: str) -> str:
    """Digest of the in-tree headers ``src`` includes, transitively (quoted includes resolved
    against the including file's directory, then csrc/): a header edit rebuilds only its users."""
    h = hashlib.sha1()
    seen, stack = set(), [src]
    while stack:
        cur = stack.pop()
        with open(cur, "rb") as f:
            text = f.read()
        if cur != src:
            h.update(cur.encode() + text)
        for inc in _INCLUDE.findall(text):
            inc = inc.decode()
            for base in (os.path.dirname(cur), CSRC):
                cand = os.path.normpath(os.path.join(base, inc))
                if os.path.isfile(cand):
                    if cand not in seen:
                        seen.add(cand)
                        stack.append(cand)
                    break
    return h.hexdigest()[:12]


def _sources() -> List[str]:
    srcs = []
    for sub, pat in (("kernels", "*.hip"), ("comm", "*.cpp"), ("bindings", "*.cpp")):
        srcs += sorted(glob.glob(os.path.join(CSRC, sub, pat)))
    return srcs


def _common_flags(inc, abi, debug: bool = False) -> List[str]:
    flags = [
        "-O1" if debug else "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-munsafe-fp-atomics",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-D_GLIBCXX_USE_CXX11_ABI={int(abi)}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        "-I" + CSRC,
    ]
    if debug:
        flags += ["-DHYP_DEBUG=1", "-DHYP_MODULE_NAME=_C_debug"]
    return flags


def _compile(src: str, obj: str, flags: List[str], torch_flags: List[str], verbose: bool) -> str:
    cmd = [_hipcc(), "-c", src, "-o", obj] + flags
    if src.endswith(".cpp"):
        cmd = [_hipcc(), "-x", "hip", "-c", src, "-o", obj] + flags + torch_flags
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = False, debug: bool = False) -> str:
    inc, torch_lib, abi = _torch_paths()
    BUILD = os.path.join(CSRC, "build_debug" if debug else "build")
    OUT = os.path.join(PKG, "_C_debug.so" if debug else "_C.so")
    os.makedirs(BUILD, exist_ok=True)
    flags = _common_flags(inc, abi, debug)
    py_inc = sysconfig.get_paths()["include"]
    torch_flags = [f"-I{p}" for p in inc] + [
        f"-I{py_inc}",
        "-DTORCH_EXTENSION_NAME=" + ("_C_debug" if debug else "_C"),
        "-DTORCH_API_INCLUDE_EXTENSION_H",
    ]
    todo, objs = [], []
    for src in _sources():
        hdr = _headers_digest(src)
        with open(src, "rb") as f:
            digest = hashlib.sha1(f.read() + hdr.encode() + " ".join(flags).encode()).hexdigest()[:12]
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(BUILD, f"{rel}.{digest}.o")
        objs.append(obj)
        if force or not os.path.exists(obj):
            todo.append((src, obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(_compile, s, o, flags, torch_flags, verbose) for s, o in todo]
            for fu in cf.as_completed(futs):
                fu.result()
    need_link = force or bool(todo) or not os.path.exists(OUT)
    if not need_link:
        out_m = os.path.getmtime(OUT)
        need_link = any(os.path.getmtime(o) > out_m for o in objs)
    if need_link:
        tmp = OUT + ".tmp"
        # Link with plain clang++ (hipcc would append /opt/rocm's libamdhip64.so.7) and do NOT name
        # the HIP runtime or RCCL at all: their symbols resolve at load time through libtorch_hip's
        # own dependencies (torch/lib/libamdhip64.so, torch/lib/librccl.so).  The process then holds
        # ONE HIP runtime and ONE RCCL — our kernels launch on torch's streams and our communicator
        # shares torch's RCCL.  (Naming them here would add NEEDED libamdhip64.so.7 / librccl.so.1,
        # which resolve to /opt/rocm's copies: a second runtime in the process.)
        cmd = (
            [os.path.join(os.path.dirname(os.path.realpath(_hipcc())), "..", "lib", "llvm", "bin", "clang++"),
             "-shared", "-o", tmp]
            + objs
            + ["-fPIC", f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}"]
            + ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
        )
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT)
    # drop stale objects from older source versions
    keep = set(objs)
    for o in glob.glob(os.path.join(BUILD, "*.o")):
        if o not in keep:
            try:
                os.remove(o)
            except OSError:
                pass
    return OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true", help="bounds-checked -O1 -g build -> _C_debug.so")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose, debug=a.debug)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
