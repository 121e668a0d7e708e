#!/usr/bin/env python3
"""One training step's kernel sequence from a rocprofv3 kernel trace of bench.py: the library's
kernels (mvae::) from one de-interleave launch (the start of a step) to the next, for the step
whose kernels overlap least (the bench's region pass serialises them on one stream), with start
offsets, durations and the gap before each launch.  usage: python tools/step_trace.py <csv>"""
import csv
import re
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mvae::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step starts at the de-interleave (the bits form, or the plane form; not the gated grey pass)
    ad = [i for i, r in enumerate(rows) if re.search(r"::(deint_bits|deinterleave_vec)", r["Kernel_Name"])]
    best = None
    for k in range(1, len(ad)):
        seg = rows[ad[k - 1]:ad[k]]
        ov, last = 0, 0
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            ov += s < last
            last = max(last, e)
        if best is None or ov < best[0]:
            best = (ov, seg)
    seg = best[1]
    t0 = int(seg[0]["Start_Timestamp"])
    prev_end = t0
    busy = 0.0
    print(f"{'kernel':62s} {'wgs':>6s} {'start':>8s} {'us':>8s} {'gap':>6s}")
    for r in seg:
        m = re.search(r"::(\w+)(<[^(]*>)?\(", r["Kernel_Name"])
        nm = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += (e - s) / 1e3
        print(f"{nm[:62]:62s} {wg:6d} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:6.1f}")
        prev_end = max(prev_end, e)
    print(f"span {(prev_end - t0) / 1e3:.1f} us, kernel time {busy:.1f} us, overlapping launches {best[0]}")


if __name__ == "__main__":
    main()
