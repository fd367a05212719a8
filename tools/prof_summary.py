#!/usr/bin/env python3
"""Condense a rocprofv3 ``*_kernel_stats.csv`` into a short, readable CSV
(kernel names shortened; durations unchanged) for ``profiles/``.

    python tools/prof_summary.py gpurun_out/prof_x/run_kernel_stats.csv > profiles/rNN/foo.csv
"""
import csv
import re
import sys


def short_name(name: str) -> str:
    n = name
    if n.startswith("void "):
        n = n[5:]
    n = n.replace("(anonymous namespace)::", "")
    if "rocprim" in n:
        kind = re.search(r"radix_sort_onesweep_(\w+?)<", n)
        return "rocprim::radix_sort_onesweep_" + (kind.group(1) if kind else "?")
    if n.startswith("at::native::"):
        m = re.match(r"at::native::(?:\w+::)*?(\w+)<", n)
        return "torch:" + (m.group(1) if m else n[:60])
    depth, out = 0, []
    for ch in n:  # cut at the argument list, keep template args
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out)[:100]


def main(path):
    rows = list(csv.DictReader(open(path)))
    w = csv.writer(sys.stdout)
    w.writerow(["Kernel", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in rows:
        w.writerow([short_name(r["Name"]), r["Calls"], r["TotalDurationNs"],
                    f"{float(r['AverageNs']):.1f}", f"{float(r['Percentage']):.2f}", r["MinNs"],
                    r["MaxNs"]])


if __name__ == "__main__":
    main(sys.argv[1])
