#!/usr/bin/env python3
"""A/B the de-interleave forms (mvae_bench_deint) at a config's batch shape, interleaved rounds in
one process: ms per launch and GB/s of the bytes each form must move (variant + 1000: four X
images read in turn, so the last-level cache holds none of the next launch's input).

  python tools/deint_bench.py [--config C3] [--variants 100,0,1,2,3,4] [--rounds 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--variants", default="100,0,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    torch.cuda.init()
    st = torch.cuda.current_stream().cuda_stream
    cfg = baseline_config(a.config)
    B, D = cfg.batch, cfg.D
    vs = [int(v) for v in a.variants.split(",")]
    res = {v: [] for v in vs}
    for _ in range(a.rounds):
        for v in vs:
            ms = C.c_float()
            rc = lib.mvae_bench_deint(B, D, v, a.iters, st, C.byref(ms))
            if rc:
                raise RuntimeError(lib.mvae_last_error(None))
            res[v].append(ms.value)
    read = B * 3 * D * 4
    for v in vs:
        m = statistics.median(res[v])
        vv = v % 1000  # (v + 1000: four X images in turn, none cached; + 2000 / 4000: a GEMM / 1 GB memset before each)
        wr = 3 * B * D * 2 + B * D / 8 if vv == 100 else 2 * 3 * B * (D + 64) / 8 + B * D / 8
        print(f"{a.config} variant {v:3d}: {m * 1e3:8.1f} us  {(read + wr) / m / 1e6:7.0f} GB/s "
              f"(read {read / 1e6:.0f} MB, write {wr / 1e6:.0f} MB)")


if __name__ == "__main__":
    main()
