#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV: the last complete training
step (from one deinterleave dispatch to the next), every kernel with its start offset,
duration, queue and workgroups, plus busy/idle totals (union of kernel intervals).

  python tools/timeline.py <run_kernel_trace.csv> [--step -2]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else -2
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "deinterleave" in r["Kernel_Name"]]
    a, b = starts[k - 1], starts[k]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    iv = []
    for r in step:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        iv.append((s, e))
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        name = r["Kernel_Name"].split("(")[0][:60]
        print(f"{s / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  q{r.get('Queue_Id', '?'):>3} wg {wg:6d}  {name} #{r.get('Kernel_Id', '')}")
    iv.sort()
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = int(rows[b]["Start_Timestamp"]) - t0
    print(f"step span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us, "
          f"sum of kernel durations {sum(e - s for s, e in iv) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
