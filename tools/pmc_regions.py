#!/usr/bin/env python3
"""Per-region PMC counters of the training step: one rocprofv3 --pmc pass per counter group over
a short bench.py child run whose named regions are bracketed by marker kernels (the same
attribution bench.py uses for roofline.traffic). Prints one JSON object: region -> counter ->
mean value per launch (summed over the region's dispatches, i.e. GEMM + its reduction).

  python tools/pmc_regions.py --regions enc_bwd_w_0,dec_fwd_out_bce --config C2 \
      --groups "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES" "FETCH_SIZE" > out.json

Each group must fit one pass (MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC (FETCH_SIZE uses 3,
WRITE_SIZE 2), <= 4 TCP counters); every pass runs under its own 120 s limit."""
import argparse
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def region_ids(args):
    """Region name -> id from a libmvae context of the same configuration (no GPU work)."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from magic_amd.config import baseline_config\nfrom magic_amd.engine import Engine\n"
            "cfg = baseline_config(%r)\n" % (ROOT, args.config) +
            ("cfg = cfg.replace(precision=%r)\n" % args.precision if args.precision else "") +
            "e = Engine(cfg, 0)\nprint(','.join(e.timing_names()))\ne.close()\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        raise SystemExit(out.stderr[-2000:])
    return out.stdout.strip().splitlines()[-1].split(",")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regions", required=True)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--precision", default="")
    ap.add_argument("--groups", nargs="+", required=True)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc_regions"))
    args = ap.parse_args()
    names = region_ids(args)
    want = args.regions.split(",")
    ids = {n: names.index(n) for n in want}
    exe = shutil.which("rocprofv3")
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child",
             ",".join(str(i) for i in ids.values()), "--config", args.config, "--steps", "2",
             "--warmup", "1"]
    if args.precision:
        child += ["--precision", args.precision]
    os.makedirs(args.out, exist_ok=True)
    res = {n: {} for n in want}
    for gi, group in enumerate(args.groups):
        d = tempfile.mkdtemp(prefix=f"g{gi}_", dir=args.out)
        cmd = [exe, "--pmc", *group.split(","), "--kernel-trace", "--output-format", "csv", "-d", d,
               "-o", "run", "--", *child]
        with open(d + ".log", "w") as log:
            p = subprocess.Popen(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=log,
                                 stderr=subprocess.STDOUT, start_new_session=True)
            try:
                rc = p.wait(timeout=120)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                raise SystemExit(f"pass {group} timed out")
        if rc != 0:
            raise SystemExit(f"pass {group} rc={rc} (log {d}.log)")
        for c in group.split(","):
            vals = bench._region_counter(d, c, list(ids.values()))
            for n, rid in ids.items():
                if rid in vals:
                    res[n][c] = vals[rid]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
