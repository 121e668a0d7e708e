"""The plane-stacked f32x ring kernel (create option x3, gemm_bf16.hip gemm_bf16x_kernel): every
layout, both ring tile heights, the store / activation / dgrad epilogues, ragged shapes, partial
k-tiles and split-K -- against float64 at the f32x bar and against the (k-tile, pair) ring kernel
to fp32 rounding (the same plane products summed in another order); whole C2 steps against the
float64 oracle and against the ring kernel's steps."""
import pytest
import torch

from magic_amd import _lib

pytestmark = pytest.mark.gpu


def _gemm(lib, M, N, K, A, at, Bm, bt, ldc, flags, act=0, aux=None):
    C = torch.full((M, ldc), float("nan"), device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), A.shape[1], at, Bm.data_ptr(), Bm.shape[1], bt,
                             C.data_ptr(), ldc, flags, act, aux.data_ptr() if aux is not None else None,
                             aux.shape[1] if aux is not None else 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    torch.cuda.synchronize()
    return C


@pytest.mark.parametrize("tm", [256, 192, "w256"])
@pytest.mark.parametrize("at,bt", [(0, 0), (1, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("epi", [0, 1, 2], ids=["store", "act", "dact"])
@pytest.mark.parametrize("M,N,K", [(12288, 500, 501), (600, 260, 300), (700, 130, 4099), (501, 500, 8192),
                                   (256, 128, 32), (300, 200, 10001)])
def test_x3_gemm_matches_float64_and_ring(tm, at, bt, epi, M, N, K):
    """tm 256 / 192: the tile-N-128 form (ring variant 11, x3 = 1); w256: the 256x256 form (ring
    variant 12, x3 = 2; 192-row plans stay on the ring kernel)."""
    if tm == 192 and at:
        pytest.skip("192-row tiles need a k-contiguous A")
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K + 11 * at + 13 * bt + epi)
    r8 = lambda n: (n + 7) // 8 * 8
    A = torch.randn((K, r8(M)) if at else (M, r8(K)), device="cuda", generator=g)
    Bm = torch.randn((N, r8(K)) if bt else (K, r8(N)), device="cuda", generator=g) * 0.05
    if not at:
        A[:, K:] = 0
    if bt:
        Bm[:, K:] = 0
    ldc = r8(N)
    aux = torch.tanh(torch.randn(M, ldc, device="cuda", generator=g)) if epi == 2 else None
    flags = epi | (2 << 4) | ((12 if tm == "w256" else 11) << 8) | ((1 << 13) if tm == 192 else 0)
    Cr = _gemm(lib, M, N, K, A, at, Bm, bt, ldc, flags, 0, aux)
    Cx = _gemm(lib, M, N, K, A, at, Bm, bt, ldc, flags | ((2 if tm == "w256" else 1) << 16), 0, aux)
    Ad = (A[:, :M].T if at else A[:, :K]).double()
    Bd = (Bm[:, :K].T if bt else Bm[:, :N]).double()
    acc = Ad @ Bd
    if epi == 1:
        ref = torch.tanh(acc)
    elif epi == 2:
        ref = acc * (1 - aux[:, :N].double() ** 2)
    else:
        ref = acc
    mag = (Ad.abs() @ Bd.abs()).max().item()
    assert torch.isfinite(Cx[:, :N]).all()
    assert (Cx[:, :N].double() - ref).abs().max().item() <= 2e-6 * mag + 1e-6
    assert (Cx[:, :N].double() - Cr[:, :N].double()).abs().max().item() <= 1e-6 * mag + 1e-7


@pytest.mark.parametrize("x3", [1, 2])
def test_x3_c2_step_vs_oracle(x3):
    """C2 (f32x) with x3: losses, gradients and the post-Adam parameters against the float64 oracle
    at the f32x bars of the other C2 step tests."""
    from magic_amd.config import baseline_config
    from tests.test_gpu_parity import check_step
    check_step(baseline_config("C2").replace(options=f"x3={x3}"), adam=True)


@pytest.mark.parametrize("x3", [1, 2])
def test_x3_c2_steps_match_ring_kernel(x3):
    """C2 with and without x3 on the same inputs: both gradients of one backward to fp32 rounding
    (the same plane products summed in another order), and the losses of three training steps (the
    second batch grey). Parameters are not compared bitwise-close: TF-Adam's m / sqrt(v) turns a
    rounding-level difference of a near-zero gradient into up to a learning-rate-sized step."""
    from magic_amd import _lib as L_
    from magic_amd.config import baseline_config
    from magic_amd.engine import Engine
    from tests.gpu_helpers import make_params
    from tests.test_gpu_r6 import _batches
    cfg = baseline_config("C2")
    P = make_params(cfg)
    batches = _batches(cfg, 3, 1, 17)
    res = []
    for opt in ("x3=0", f"x3={x3}"):
        eng = Engine(cfg.replace(options=opt), 0)
        try:
            eng.load_params(P)
            x, a = batches[0]
            eng.forward(x)
            eng.metric(a)
            eng.backward()
            torch.cuda.synchronize()
            grads = {(kind, k): v.cpu().double() for kind in (L_.KIND_GRAD1, L_.KIND_GRAD2)
                     for k, v in eng.tensors(kind).items()}
            eng.load_params(P)
            L = []
            for x, a in batches:
                eng.train_step(x, a)
                L.append(eng.losses.clone())
            torch.cuda.synchronize()
            res.append((grads, torch.stack(L).cpu().double()))
        finally:
            eng.close()
    (g0, l0), (g1, l1) = res
    assert ((l0 - l1).abs() <= 1e-5 * l0.abs() + 1e-6).all(), (l0, l1)
    for k in g0:
        d = (g0[k] - g1[k]).abs().max().item()
        assert d <= 2e-5 * g0[k].abs().max().item() + 1e-12, (k, d)
