#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch usage of the built library (reads the
gfx950 code object's AMDGPU metadata note; no GPU needed).

    python3 tools/kernel_resources.py [substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "atmlgraphattentionnetworks_amd", "libgat_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    pats = sys.argv[1:]
    with tempfile.TemporaryDirectory() as d:
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", LIB], cwd=d, check=True,
                       capture_output=True)
        # the bundles are written next to the input: move it into the temp dir
        for f in os.listdir(os.path.dirname(LIB)):
            if re.match(r"libgat_amd\.so\.\d+\.", f):
                os.replace(os.path.join(os.path.dirname(LIB), f), os.path.join(d, f))
        # one code object per translation unit (csrc/*.hip)
        notes = "".join(
            subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(d, co)],
                           capture_output=True, text=True, check=True).stdout
            for co in sorted(os.listdir(d)) if "gfx950" in co)
    rows = []
    for blk in notes.split("  - .agpr_count:")[1:]:
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "-"])[1]
        name = get("name")
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if pats and not any(p in dem for p in pats):
            continue
        rows.append((dem, blk.split()[0], get("vgpr_count"), get("sgpr_count"),
                     get("group_segment_fixed_size"), get("private_segment_fixed_size"),
                     get("vgpr_spill_count")))
    print(f"{'agpr':>4} {'vgpr':>4} {'sgpr':>4} {'lds':>6} {'scr':>4} {'spill':>5}  kernel")
    for dem, a, v, s, l, p, sp in sorted(rows):
        print(f"{a:>4} {v:>4} {s:>4} {l:>6} {p:>4} {sp:>5}  {dem[:150]}")


if __name__ == "__main__":
    main()
