#!/usr/bin/env python3
"""Per-step span and idle time of the library's kernels in a rocprofv3 kernel trace of bench.py
(steps split at the de-interleave launch; both streams; idle = the part of the span no kernel
covers), with the five largest gaps and where the next step starts. The timed loop's steps are
the ones with idle time of a few tens of us (the region pass serialises its launches behind
event records). usage: python tools/step_gaps.py <kernel_trace.csv>"""
import csv
import re
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mvae::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step starts at the de-interleave (the bits form, or the plane form; not the gated grey pass)
    ad = [i for i, r in enumerate(rows) if re.search(r"::(deint_bits|deinterleave_vec)", r["Kernel_Name"])]
    for k in range(1, len(ad)):
        seg = rows[ad[k - 1]:ad[k]]
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
        t0 = iv[0][0]
        end, idle, gaps = t0, 0, []
        for s, e in iv:
            if s > end:
                idle += s - end
                gaps.append(s - end)
            end = max(end, e)
        gaps.sort(reverse=True)
        nxt = (int(rows[ad[k]]["Start_Timestamp"]) - t0) / 1e3
        print(f"step {k}: {len(seg)} kernels, span {(end - t0) / 1e3:.1f} us, idle {idle / 1e3:.1f} us, "
              f"largest gaps {[round(g / 1e3, 1) for g in gaps[:5]]}, next step at {nxt:.1f} us")


if __name__ == "__main__":
    main()
