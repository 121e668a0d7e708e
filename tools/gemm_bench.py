#!/usr/bin/env python3
"""A/B the GEMM kernel variants on the training step's shapes, interleaved rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24). Prints TFLOP/s per (shape, variant).

  python tools/gemm_bench.py [--variants 0,1,2] [--rounds 3] [--config C2]
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


def shapes(cfg):
    B, D, e, L = cfg.batch, cfg.D, cfg.enc[0], cfg.latent
    d1 = cfg.dec[1]
    # (name, M, N, K, at, bt, batch, epilogue: 0 store, 1 act, 2 dact, 3 bce)
    return [
        ("enc_fwd_0", 3 * B, e, D + 1, 0, 0, 1, 1),
        ("enc_bwd_w_0", D + 1, e, 2 * B, 1, 0, 2, 0),
        ("dec_fwd_out", B, D, d1 + 1, 0, 0, 1, 3),
        ("dec_bwd_d_out", B, d1, D, 0, 1, 1, 2),
        ("dec_bwd_w_out", d1 + 1, D, B, 1, 0, 1, 0),
        ("enc_fwd_h", 3 * B, e, e + 1, 0, 0, 1, 1),
        ("enc_bwd_d_h", 4 * B, e, e, 0, 1, 1, 2),
        ("enc_bwd_w_h", e + 1, e, 2 * B, 1, 0, 2, 0),
        ("head_fwd", 3 * B, 2 * L, e + 1, 0, 0, 1, 0),
        ("head_bwd_d", 4 * B, e, 2 * L, 0, 1, 1, 2),
        ("head_bwd_w", e + 1, 2 * L, 2 * B, 1, 0, 2, 0),
        ("dec_fwd_1", B, cfg.dec[0], L + 1, 0, 0, 1, 1),
        ("dec_bwd_w_1", L + 1, cfg.dec[0], B, 1, 0, 1, 0),
        ("dec_bwd_d_z", B, L, cfg.dec[0], 0, 1, 1, 0),
        ("dec_fwd_2", B, d1, cfg.dec[0] + 1, 0, 0, 1, 1),
        ("dec_bwd_d_2", B, cfg.dec[0], d1, 0, 1, 1, 2),
        ("dec_bwd_w_2", cfg.dec[0] + 1, d1, B, 1, 0, 1, 0),
        ("square4096", 4096, 4096, 4096, 0, 0, 1, 0),
        # L2-resident probes of the k-loop's operand path: one tile re-run from a warm L2, and
        # 64 tiles over 16 MB of operands
        ("l2_one", 256, 256, 2048, 0, 0, 1, 0),
        ("l2_64", 2048, 2048, 2048, 0, 0, 1, 0),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,16,17,18,32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--epilogues", action="store_true", help="run each shape with its step epilogue")
    ap.add_argument("--diag", default="0", help="kernel diagnostics bits (PParams::diag), comma list")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default: all)")
    ap.add_argument("--extra", action="append", default=[],
                    help="extra shape NAME:M:N:K:AT:BT:BATCH (repeatable)")
    args = ap.parse_args()
    lib = _lib.load()
    torch.cuda.init()
    st = torch.cuda.current_stream().cuda_stream
    cfg = baseline_config(args.config)
    # a variant may end in "b" (A of 0/1 values: the layer-0 pixels) or "B" (... and read as a
    # BitMat by the eight-phase kernel's bits path): mvae_bench_gemm variant bits 20 / 21
    def vparse(v):
        f = 0
        if v.endswith("b"):
            v, f = v[:-1], 1 << 20
        elif v.endswith("B"):
            v, f = v[:-1], 3 << 20
        return int(v) | f
    variants = [(vparse(v), int(d)) for v in args.variants.split(",") for d in args.diag.split(",")]
    want = set(args.shapes.split(",")) if args.shapes else None
    extra = []
    for e in args.extra:
        f = e.split(":")
        extra.append((f[0], *[int(v) for v in f[1:7]], 0))
    sh = [s for s in shapes(cfg) if want is None or s[0] in want] + extra
    res = {}
    for _ in range(args.rounds):
        for name, M, N, K, at, bt, batch, epi in sh:
            for v in variants:
                ms = C.c_float()
                vv = v[0] | (epi << 8 if args.epilogues else 0) | (v[1] << 12)
                rc = lib.mvae_bench_gemm(M, N, K, at, bt, batch, vv, args.iters, st, C.byref(ms))
                if rc != 0:
                    raise RuntimeError(lib.mvae_last_error(None))
                res.setdefault((name, v), []).append(ms.value)
    lab = [f"v{v & 0xfffff}" + {0: "", 1: "b", 3: "B"}[v >> 20] + (f"d{d}" if d else "") for v, d in variants]
    print(f"{'shape':16s} {'MxNxK':>22s} batch " + " ".join(f"{x + ' TF/s':>12s}" for x in lab))
    for name, M, N, K, at, bt, batch, epi in sh:
        fl = 2.0 * M * N * K * batch
        cells = []
        for v in variants:
            med = statistics.median(res[(name, v)])
            cells.append(f"{fl / med / 1e9:12.1f}")
        cells.append("  us: " + " ".join(f"{statistics.median(res[(name, v)]) * 1e3:.1f}" for v in variants))
        print(f"{name:16s} {f'{M}x{N}x{K}':>22s} {batch:5d} " + " ".join(cells))


if __name__ == "__main__":
    main()
