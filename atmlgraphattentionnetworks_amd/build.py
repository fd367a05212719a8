"""In-tree build of libgat_amd.so for gfx950 (no JIT cache: the .so travels
with the repo snapshot to the GPU box).

The library is five HIP translation units (csrc/*.hip, sharing
csrc/gat_common.h); each compiles to an object under build/obj in its own
hipcc process, in parallel, and one link makes the shared library.  Objects
are rebuilt when their source, the shared header or include/gat_amd.h is
newer.

    python -m atmlgraphattentionnetworks_amd.build [--force]
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SRCS = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
COMMON = os.path.join(CSRC, "gat_common.h")
HDR = os.path.join(ROOT, "include", "gat_amd.h")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(PKG, "libgat_amd.so")
ARCH = os.environ.get("GAT_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-munsafe-fp-atomics"]
# GAT_AB_KERNELS=1: a tools-only build that also carries the measured-slower
# kernels kept for A/B (the fp32-MFMA k_project_pipe2 behind GAT_PROJ_X3=0);
# the product library never defines it.  Use --force when switching.
if os.environ.get("GAT_AB_KERNELS"):
    FLAGS.append("-DGAT_AB_KERNELS")


def hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return os.path.join(rocm, "bin", "hipcc")


def _stale(target: str, deps: list[str]) -> bool:
    return (not os.path.exists(target)
            or os.path.getmtime(target) < max(os.path.getmtime(d) for d in deps))


def build(force: bool = False, verbose: bool = True) -> str:
    if not SRCS:
        raise RuntimeError(f"no HIP sources under {CSRC}")
    os.makedirs(OBJ, exist_ok=True)
    objs, jobs = [], []
    for src in SRCS:
        obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, COMMON, HDR]):
            cmd = [hipcc(), f"--offload-arch={ARCH}", *FLAGS, "-c", "-o", obj + ".tmp", src]
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            jobs.append((obj, subprocess.Popen(cmd)))
    failed = [obj for obj, p in jobs if p.wait() != 0]
    if failed:
        raise RuntimeError("hipcc failed for " + ", ".join(os.path.basename(o) for o in failed))
    for obj, _ in jobs:
        os.replace(obj + ".tmp", obj)
    if force or jobs or _stale(LIB, objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp", *objs]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
