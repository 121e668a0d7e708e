#!/usr/bin/env python3
"""Repeat one wide-kernel GEMM case (debug GEMM entry) N times in one process and report the
worst error against float64 -- a check for nondeterministic (race) results."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from magic_amd import _lib  # noqa: E402


def run(M, N, K, ldc, epi, act, prec, variant, planes, reps):
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + 31 * epi + act)
    A = torch.randn(M, K, device="cuda", generator=g) * 0.3
    ldb = (N + 7) // 8 * 8
    Bm = torch.zeros(K, ldb, device="cuda")
    Bm[:, :N] = torch.randn(K, N, device="cuda", generator=g) * 0.3
    pre = torch.randn(M, ldb, device="cuda", generator=g)
    aux = torch.tanh(pre)
    acc = A.double() @ Bm[:, :N].double()
    a = aux[:, :N].double()
    ref = acc * (1 - a * a) if epi == 2 else torch.tanh(acc)
    errs = []
    for _ in range(reps):
        C = torch.full((M, ldc), float("nan"), device="cuda")
        rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), K, 0, Bm.data_ptr(), ldb, 0, C.data_ptr(), ldc,
                                 epi | (prec << 4) | (variant << 8) | (planes << 12), act,
                                 aux.data_ptr(), ldb, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        errs.append((C[:, :N].double() - ref).abs().max().item())
    bad = sum(e > 1e-3 for e in errs)
    print(f"M{M} N{N} K{K} ldc{ldc} epi{epi} prec{prec} v{variant} planes{planes}: "
          f"max err {max(errs):.3e}, {bad}/{reps} bad", flush=True)


if __name__ == "__main__":
    for v in (12, 0, 11):
        for planes in (1, 0):
            for epi in (2, 1):
                run(600, 520, 304, 520, epi, 0, 2, v, planes, 40)
