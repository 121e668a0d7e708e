"""Round 6: the layer-0 pixel operand as bits (BitMat, mvae_internal.h) -- the eight-phase kernel's
bits path against its plane path on the same 0/1 operand (bitwise: the same products, summed in
the same order) and against float64."""
import pytest
import torch

from magic_amd import _lib

pytestmark = pytest.mark.gpu


def _bin(rows, cols, g, ld=None):
    ld = ld or (cols + 7) // 8 * 8
    x = (torch.rand(rows, ld, device="cuda", generator=g) < 0.37).float()
    x[:, cols:] = 0
    return x


def _gemm(lib, M, N, K, A, at, Bm, ldc, flags, act=0):
    C = torch.full((M, ldc), float("nan"), device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), A.shape[1], at, Bm.data_ptr(), Bm.shape[1], 0,
                             C.data_ptr(), ldc, flags, act, None, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    torch.cuda.synchronize()
    return C


@pytest.mark.parametrize("prec", [2, 1], ids=["f32x", "bf16"])
@pytest.mark.parametrize("at", [0, 1], ids=["fwd", "wgrad"])
@pytest.mark.parametrize("epi", [0, 1], ids=["store", "act"])
@pytest.mark.parametrize("M,N,K", [(600, 520, 300), (256, 256, 64), (130, 257, 1001), (300, 500, 4099),
                                   (700, 260, 10001)])
def test_gemm_bits_path_bitwise_equal_planes(prec, at, epi, M, N, K):
    """variant 13 forces the eight-phase kernel; epi bit 14 hands it A as a BitMat too: the bits
    path must reproduce the plane path bit for bit in bf16, to fp32 rounding in f32x (ragged M / N /
    K, partial k-tiles, split-K at K 4099 / 10001, one-block shapes), and float64 at the bars."""
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M * 3 + N * 7 + K + 11 * at + epi)
    A = _bin(K, M, g) if at else _bin(M, K, g)
    Bm = torch.randn(K, (N + 7) // 8 * 8, device="cuda", generator=g) * 0.1
    ldc = (N + 7) // 8 * 8
    flags = epi | (prec << 4) | (13 << 8)
    Cp = _gemm(lib, M, N, K, A, at, Bm, ldc, flags)
    Cb = _gemm(lib, M, N, K, A, at, Bm, ldc, flags | (1 << 14))
    Ad = A[:, :M].double().T if at else A[:, :K].double()
    acc = Ad @ Bm[:, :N].double()
    ref = torch.tanh(acc) if epi == 1 else acc
    mag = (Ad @ Bm[:, :N].double().abs()).max().item()
    bound = (2e-6 if prec == 2 else 1e-2) * mag + 1e-6
    assert (Cb[:, :N].double() - ref).abs().max().item() <= bound
    if prec == 1:
        assert torch.equal(Cb[:, :N], Cp[:, :N])
    else:  # f32x: the bits path walks the plane pairs of a k-tile innermost (its fragments reused),
        # the plane path k-tiles in pairs: the same products summed in another order
        assert (Cb[:, :N].double() - Cp[:, :N].double()).abs().max().item() <= 1e-6 * mag + 1e-7


def test_gemm_bits_grey_operand_takes_plane_path():
    """A BitMat whose source plane held a value other than 0 / 1 raises the not-binary word, and the
    kernel then reads the planes: the result is the plane path's."""
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = 300, 260, 700
    A = _bin(M, K, g)
    A[7, 13] = 0.5
    Bm = torch.randn(K, 264, device="cuda", generator=g) * 0.1
    flags = (1 << 4) | (13 << 8)
    Cp = _gemm(lib, M, N, K, A, 0, Bm, 264, flags)
    Cb = _gemm(lib, M, N, K, A, 0, Bm, 264, flags | (1 << 14))
    assert torch.equal(Cb[:, :N], Cp[:, :N])
