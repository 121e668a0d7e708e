#!/usr/bin/env python3
"""Tabulate bench.py A/B runs: pairs/s, ms/step and chosen region times of each
gpurun_out/<name>.json / .err pair.  usage: python tools/ab_table.py NAME... [--keys a,b,c]"""
import json
import re
import sys

DEFAULT_KEYS = "enc_bwd_w_0,enc_fwd_0,dec_fwd_out_bce,dec_bwd_d_out,dec_bwd_w_out,deinterleave"


def main():
    argv = sys.argv[1:]
    keys = DEFAULT_KEYS
    if "--keys" in argv:
        i = argv.index("--keys")
        keys = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    keys = keys.split(",")
    for name in argv:
        base = name if name.startswith("gpurun_out/") else "gpurun_out/" + name
        d = json.load(open(base + ".json"))
        reg = {}
        for line in open(base + ".err"):
            m = re.match(r"\[bench\] (\S+)\s+([\d.]+) ms/step", line)
            if m and m.group(1) not in reg:
                reg[m.group(1)] = float(m.group(2))
        cells = " ".join(f"{k}={reg.get(k, float('nan')):.4f}" for k in keys)
        print(f"{name.split('/')[-1]:14s} {d['value']:10.0f} {d['ms_per_step']:.3f} ms  {cells}")


if __name__ == "__main__":
    main()
