#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 counter passes: mean value per dispatch of every counter,
grouped by kernel (template arguments stripped unless --full), plus the derived HBM bytes
(FETCH_SIZE x 2 on gfx950 + WRITE_SIZE, MI355X_MICROARCH.md §HBM) and the kernel-trace mean
duration. Each pass directory is one `rocprofv3 --pmc ... --kernel-trace --output-format csv -d DIR`.

  python tools/pmc_kernels.py DIR1 DIR2 ... [--match gemm_bf16] [--full]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def short(name, full, grid=None):
    if full:
        return name
    n = re.sub(r"^void ", "", name).replace("mvae::(anonymous namespace)::", "")
    n = n[:n.index("(")] if "(" in n else n
    return n + (f" grid={grid}" if grid else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--full", action="store_true")
    args = ap.parse_args()
    val = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> values per dispatch
    dur = defaultdict(list)
    for d in args.dirs:
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in rows(d, "counter_collection.csv"):
            k = r["Kernel_Name"]
            if args.match and args.match not in k:
                continue
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            names[did] = short(k, args.full, r.get("Grid_Size"))
        for did, cs in per.items():
            for c, v in cs.items():
                val[names[did]][c].append(v)
        for r in rows(d, "kernel_trace.csv"):
            k = r["Kernel_Name"]
            if args.match and args.match not in k:
                continue
            dur[short(k, args.full, r.get("Grid_Size"))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k in sorted(set(val) | set(dur)):
        print(k)
        if dur.get(k):
            print(f"  duration_us            {sum(dur[k]) / len(dur[k]) / 1e3:14.2f}  (n={len(dur[k])})")
        cs = val.get(k, {})
        for c in sorted(cs):
            v = cs[c]
            print(f"  {c:22s} {sum(v) / len(v):14.1f}  (n={len(v)})")
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 2048
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
            print(f"  hbm_MB (2xFETCH+WRITE) {(f + w) / 1e6:14.2f}  fetch {f / 1e6:.2f} write {w / 1e6:.2f}")


if __name__ == "__main__":
    main()
