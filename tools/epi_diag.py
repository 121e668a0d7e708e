#!/usr/bin/env python3
"""Timing diagnostics of one GEMM shape with its step epilogue (kernel diag bits: 1 = no operand
copies after the prologue, 2 = no epilogue global stores, 4 = no LDS transpose, 8 = no
transcendental math; results meaningless). Interleaved rounds in one process.

  python tools/epi_diag.py --shape dec_fwd_out --prec 32 --diags 0,2,4,8,14,1,15
"""
import argparse
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from magic_amd import _lib  # noqa: E402
from magic_amd.config import baseline_config  # noqa: E402
from tools.gemm_bench import shapes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="dec_fwd_out")
    ap.add_argument("--prec", type=int, default=32, help="16 bf16, 32 f32x (variant bits 4-7)")
    ap.add_argument("--diags", default="0,2,4,8,14,1,15")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    lib = _lib.load()
    torch.cuda.init()
    st = torch.cuda.current_stream().cuda_stream
    sh = {s[0]: s for s in shapes(baseline_config(args.config))}[args.shape]
    name, M, N, K, at, bt, batch, epi = sh
    diags = [int(x) for x in args.diags.split(",")]
    res = {d: [] for d in diags}
    for _ in range(args.rounds):
        for d in diags:
            ms = C.c_float()
            v = args.prec | (epi << 8) | (d << 12)
            rc = lib.mvae_bench_gemm(M, N, K, at, bt, batch, v, args.iters, st, C.byref(ms))
            if rc != 0:
                raise RuntimeError(lib.mvae_last_error(None))
            res[d].append(ms.value)
    print(f"{name} {M}x{N}x{K} batch {batch} epi {epi} prec {args.prec}")
    for d in diags:
        print(f"  diag {d:2d}: {statistics.median(res[d]) * 1e3:8.1f} us")


if __name__ == "__main__":
    main()
