#!/usr/bin/env python3
"""Library baseline for the step's GEMM shapes: torch.matmul on ROCm (hipBLASLt) in bf16 with
fp32 accumulation, timed with HIP events in one process, beside the library's own kernel
(mvae_bench_gemm, default plan, store epilogue) on the same shapes. Not part of the step: a
yardstick for the hand-written kernels.  usage: python tools/blas_probe.py [--config C3]"""
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


def t_torch(M, N, K, at, bt, batch, iters=10, rounds=3):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = (torch.rand((batch, K, M) if at else (batch, M, K), device="cuda", generator=g) * 2 - 1).bfloat16()
    B = (torch.rand((batch, N, K) if bt else (batch, K, N), device="cuda", generator=g) * 2 - 1).bfloat16()
    a = A.transpose(1, 2) if at else A
    b = B.transpose(1, 2) if bt else B
    out = []
    for _ in range(rounds):
        torch.matmul(a, b)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            torch.matmul(a, b)
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--shapes", default="enc_bwd_w_0,enc_fwd_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,"
                    "enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,dec_fwd_2,square4096")
    args = ap.parse_args()
    lib = _lib.load()
    torch.cuda.init()
    st = torch.cuda.current_stream().cuda_stream
    cfg = baseline_config(args.config)
    want = set(args.shapes.split(","))
    print(f"{'shape':16s} {'MxNxK':>22s} batch {'hipBLASLt bf16':>15s} {'mvae bf16':>10s}   (TF/s; us)")
    for name, M, N, K, at, bt, batch, _ in shapes(cfg):
        if name not in want:
            continue
        tt = t_torch(M, N, K, at, bt, batch)
        res = []
        for _ in range(3):
            ms = C.c_float()
            rc = lib.mvae_bench_gemm(M, N, K, at, bt, batch, 16, 10, st, C.byref(ms))
            if rc != 0:
                raise RuntimeError(lib.mvae_last_error(None))
            res.append(ms.value)
        tm = statistics.median(res)
        fl = 2.0 * M * N * K * batch
        print(f"{name:16s} {f'{M}x{N}x{K}':>22s} {batch:5d} {fl / tt / 1e9:15.1f} {fl / tm / 1e9:10.1f}"
              f"   {tt * 1e3:.1f} {tm * 1e3:.1f}")


if __name__ == "__main__":
    main()
