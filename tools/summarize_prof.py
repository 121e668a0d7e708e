#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per (kernel, grid) dispatch group, the call
count and mean/min/max duration, so templated GEMM launches of different shapes are
distinguishable (rocprofv3 demangles without template arguments, so instantiations are told
apart by Kernel_Id). Usage: summarize_prof.py <run_kernel_trace.csv> [--top N] [--filter SUBSTR]
(--filter: only kernels whose name contains SUBSTR, e.g. "mvae::" for the library's own kernels
without the bench harness's torch kernels)"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    rows = [r for r in csv.DictReader(open(path)) if flt in r["Kernel_Name"]]
    g = collections.defaultdict(list)
    for r in rows:
        name = f'{r["Kernel_Name"]} #{r.get("Kernel_Id", "")}'
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        g[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in g.values())
    print(f"| kernel | workgroups | calls | mean us | min us | max us | % of GPU time |")
    print("|---|---|---|---|---|---|---|")
    for (name, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        short = name if len(name) < 90 else name[:87] + "..."
        print(f"| `{short}` | {grid} | {len(v)} | {sum(v) / len(v) / 1e3:.1f} | {min(v) / 1e3:.1f} | "
              f"{max(v) / 1e3:.1f} | {100 * sum(v) / tot:.1f} |")


if __name__ == "__main__":
    main()
