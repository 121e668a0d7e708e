#!/usr/bin/env python3
"""HBM bytes per launch of the bench's dominant GEMM from two rocprofv3 counter passes
(MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE cannot share a pass; on gfx950
FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B stores; both are in KB).

  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/fetch -o run -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT/write -o run -- python3 bench.py ...
  python3 tools/pmc_traffic.py --fetch OUT/fetch --write OUT/write --region enc_bwd_w_0 \
      --config C2 --precision f32x > profiles/pmc_traffic.json

The dominant GEMM is identified as the (kernel, grid) dispatch group with the largest total
duration among GEMM kernels — the same launch bench.py's roofline names (its region mean and
this group's mean duration are both written out so the match can be checked).
"""
import argparse
import collections
import csv
import glob
import json
import os


def _rows(d, suffix):
    paths = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not paths:
        raise SystemExit(f"no *{suffix} under {d}")
    out = []
    for p in paths:
        out.extend(csv.DictReader(open(p)))
    return out


def _grid(r):
    g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    w = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
    return g // max(w, 1)


def _per_dispatch(d, counter):
    vals = {}
    for r in _rows(d, "counter_collection.csv"):
        if r.get("Counter_Name") == counter:
            key = int(r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    trace = {int(r["Dispatch_Id"]): r for r in _rows(d, "kernel_trace.csv")}
    return vals, trace


def _dominant(trace):
    g = collections.defaultdict(list)
    for did, r in trace.items():
        if "gemm" not in r["Kernel_Name"]:
            continue
        g[(r["Kernel_Name"], _grid(r))].append(did)
    dur = {k: sum(int(trace[i]["End_Timestamp"]) - int(trace[i]["Start_Timestamp"]) for i in v)
           for k, v in g.items()}
    key = max(dur, key=dur.get)
    return key, g[key], dur[key] / len(g[key]) / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--region", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--precision", required=True)
    args = ap.parse_args()
    fv, ft = _per_dispatch(args.fetch, "FETCH_SIZE")
    wv, wt = _per_dispatch(args.write, "WRITE_SIZE")
    (kname, grid), fids, fus = _dominant(ft)
    wids = [i for i, r in wt.items() if r["Kernel_Name"] == kname and _grid(r) == grid]
    fetch = [fv[i] * 1024 * 2 for i in fids if i in fv]   # KB -> B, x2 gfx950 correction
    write = [wv[i] * 1024 for i in wids if i in wv]
    if not fetch or not write:
        raise SystemExit("counter values missing for the dominant kernel")
    fb = sum(fetch) / len(fetch)
    wb = sum(write) / len(write)
    print(json.dumps({
        "config": args.config, "precision": args.precision,
        "regions": {args.region: {
            "hbm_bytes_per_launch": round(fb + wb),
            "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
            "kernel": kname, "workgroups": grid, "launches": len(fetch),
            "mean_us_under_counters": round(fus, 2)}},
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with "
                  "--kernel-trace; FETCH_SIZE x2 (gfx950), KB x1024",
    }, indent=1))


if __name__ == "__main__":
    main()
