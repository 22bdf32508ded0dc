"""Build libibldpc.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libibldpc.so")
SOURCES = ["ib_kernels.hip", "float_kernels.hip", "channel_kernels.hip", "encoder_kernels.hip", "capi.hip", "comm.hip"]
ARCH = os.environ.get("IBLDPC_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
         "-Wno-unused-result", "-Wno-pass-failed"]
# per-source flags (variants may override them). float_kernels: messages are never NaN (ibldpc.h's
# precondition), so min / max / median need no NaN quieting (-fno-honor-nans), and the kernels run with
# the IEEE mode bit off (C3 +2 % on one box against -fno-honor-nans alone, identical instruction mix).
# The IEEE-mode attribute differs from the device libraries', which then do not inline: the source
# takes its work-item geometry from builtins (fl_tid ...), so only the fp64 box-plus's exp / log (the
# strict-precision build) remain calls.
SRC_FLAGS = {"float_kernels.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee"]}


def _stale(out: str, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, defines=(), lib: str = LIB, tag: str = "",
          src_flags=None) -> str:
    """Compile the HIP sources and link `lib`. `defines` (e.g. ["IBL_W=2"]) select kernel variants,
    `src_flags` replaces SRC_FLAGS; variant objects go to build/<tag>/."""
    src_flags = SRC_FLAGS if src_flags is None else src_flags
    objdir = os.path.join(PKG, "build", tag) if tag else os.path.join(PKG, "build")
    os.makedirs(objdir, exist_ok=True)
    headers = [os.path.join(INCLUDE, "ibldpc.h")] + \
        [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".inc", ".h"))]
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src.replace(".hip", ".o"))
        if force or _stale(o, [s] + headers):
            jobs.append([HIPCC, *FLAGS, *src_flags.get(src, []), *[f"-D{d}" for d in defines], "-c", s, "-o", o])
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            for cmd, r in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
                if r.returncode != 0:
                    sys.stderr.write(r.stdout + r.stderr)
                    raise RuntimeError(f"hipcc failed: {' '.join(cmd)}")
                if verbose:
                    sys.stderr.write(r.stderr)
    objs = [os.path.join(objdir, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or _stale(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o", lib]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("link failed")
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
