#!/usr/bin/env python3
"""The timed loop's steps in a rocprofv3 kernel trace of one bench.py configuration
(``bench.py --config X --no-configs ...``): per launch of a step -- keyed by (kernel, workgroups,
occurrence within the step), so the side stream's interleaving does not matter -- the mean start
offset and duration over the timed steps, in launch order; and, with ``--mark-dominant`` runs,
the kernels between each pair of region markers summed per step (the dominant region's launches
-- e.g. the layer-0 weight gradient's row chunks and their split-K reductions -- against the
bench line's roofline.avg_ms). Timed steps: those after the region pass (whose steps idle
> 100 us behind their event records) with idle below that.
usage: python tools/timed_steps.py <kernel_trace.csv> [--idle-us 100]"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"::(\w+)(<[^(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    path = sys.argv[1]
    lim = float(sys.argv[sys.argv.index("--idle-us") + 1]) if "--idle-us" in sys.argv else 100.0
    rows = [r for r in csv.DictReader(open(path)) if "mvae::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["wg"] = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        r["nm"] = short(r["Kernel_Name"])
    # a step starts at the de-interleave (the bits form, or the plane form; not the gated grey pass)
    ad = [i for i, r in enumerate(rows) if re.match(r"(deint_bits|deinterleave_vec)", r["nm"])]
    steps = []
    for k in range(1, len(ad)):
        seg = rows[ad[k - 1]:ad[k]]
        end, idle = seg[0]["s"], 0
        for r in sorted(seg, key=lambda r: r["s"]):
            if r["s"] > end:
                idle += r["s"] - end
            end = max(end, r["e"])
        steps.append((seg, idle / 1e3, (end - seg[0]["s"]) / 1e3))
    # the longest run of consecutive low-idle steps with one kernel count that follows a high-idle
    # step (the warm-up steps before the region pass are low-idle too, but shorter)
    best, run = (0, 0), []
    for i, st in enumerate(steps):
        if st[1] <= lim and (not run or len(st[0]) == len(steps[run[0]][0])):
            run.append(i)
        else:
            run = [i] if st[1] <= lim else []
        if run and len(run) >= best[1] - best[0] and run[0] > 0 and steps[run[0] - 1][1] > lim:
            best = (run[0], run[-1] + 1)
    timed = steps[best[0]:best[1]]
    if not timed:
        sys.exit("no timed steps found")
    n = len(timed)
    print(f"# {n} timed steps (steps {best[0]}..{best[1] - 1} of the trace); span per step mean "
          f"{sum(t[2] for t in timed) / n:.1f} us, idle mean {sum(t[1] for t in timed) / n:.1f} us")
    acc = collections.OrderedDict()
    for seg, _, _ in timed:
        t0 = seg[0]["s"]
        seen = collections.Counter()
        for r in seg:
            key = (r["nm"], r["wg"], seen[(r["nm"], r["wg"])])
            seen[(r["nm"], r["wg"])] += 1
            a = acc.setdefault(key, [0.0, 0.0, 0])
            a[0] += (r["s"] - t0) / 1e3
            a[1] += (r["e"] - r["s"]) / 1e3
            a[2] += 1
    print(f"| # | kernel | workgroups | start us | mean us |")
    print("|---|---|---|---|---|")
    tot = 0.0
    for i, ((nm, wg, occ), (s, d, c)) in enumerate(sorted(acc.items(), key=lambda kv: kv[1][0] / kv[1][2])):
        tot += d / c
        print(f"| {i} | `{nm[:70]}`{' #' + str(occ) if occ else ''} | {wg} | {s / c:.1f} | {d / c:.1f} |")
    print(f"kernel time per step {tot:.1f} us")
    # marker-bracketed launches (grid >= 4096 workgroups of 64 threads: mvae_region_marker), on the
    # markers' own queue (the side stream's kernels in between are not the region's)
    qk = next((k for k in ("Stream_Id", "Queue_Id") if k in rows[0]), None)
    per = []
    for seg, _, _ in timed:
        mk = [i for i, r in enumerate(seg) if "region_marker" in r["nm"]]
        tot_m = 0.0
        for a, b in zip(mk[0::2], mk[1::2]):
            q = seg[a][qk] if qk else None
            tot_m += sum((r["e"] - r["s"]) / 1e3 for r in seg[a + 1:b] if not qk or r[qk] == q)
        if mk:
            per.append((tot_m, len(mk) // 2))
    if per:
        print(f"marked region: {sum(p[0] for p in per) / len(per):.1f} us per step over {per[0][1]} "
              f"marker pair(s) per step (the kernels between each pair, summed)")


if __name__ == "__main__":
    main()
