"""In-tree build of libgat_amd.so for gfx950 (no JIT cache: the .so travels
with the repo snapshot to the GPU box).

    python -m atmlgraphattentionnetworks_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "gat_amd.hip")
HDR = os.path.join(ROOT, "include", "gat_amd.h")
LIB = os.path.join(PKG, "libgat_amd.so")
ARCH = os.environ.get("GAT_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    return os.path.join(rocm, "bin", "hipcc")


def build(force: bool = False, verbose: bool = True) -> str:
    deps = [SRC, HDR]
    if (not force and os.path.exists(LIB)
            and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps)):
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
           "-o", LIB + ".tmp", SRC]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
