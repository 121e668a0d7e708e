"""GPU parity for the eight-phase 256x256 GEMM kernel (gemm_bf16e.hip, round 4) on every
operand layout, ragged edge and fused epilogue, and whole training steps with it forced onto
every 256-row bf16 DMA GEMM (create option e8=2) or excluded (e8=0), against the float64 oracle at
the fp32 bar (f32x) and the documented bf16 bar; plus the round-3 items (chunked layer-0
gradient, 192-row ring tiles, latent sampling grid)."""
import pytest
import torch

from magic_amd import _lib
from magic_amd.config import baseline_config, preset
from tests.test_gpu_parity import _padded, check_step

pytestmark = pytest.mark.gpu

BF16 = dict(tol=5e-2, loss_tol=2e-3, dist_tol=2e-2)  # documented bf16 tolerance


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# ------------------------------------------------------------------ eight-phase kernel
@pytest.mark.parametrize("prec", [2, 1], ids=["f32x", "bf16"])
@pytest.mark.parametrize("at,bt", [(0, 0), (1, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("M,N,K,variant", [(128, 128, 64, 13), (300, 517, 1001, 13), (1000, 600, 4099, 13),
                                           (513, 260, 130, 14), (40, 70, 200, 13), (2100, 500, 700, 14),
                                           (129, 40, 8193, 13), (1, 8, 1, 13), (256, 256, 192, 13),
                                           (520, 770, 320, 13), (256, 256, 192, 6)])
def test_gemm_e8_kernel(at, bt, M, N, K, variant, prec):
    """Variant 13 / 14 force the eight-phase kernel (14 also routes fp32-only outputs through its
    LDS row-major epilogue, as every eight-phase output does; 6 = 13); ragged M / N / K edges,
    tiles smaller than 256 x 256, odd k-tile counts (the pipeline's tail waits) and the planner's
    split-K (K 4099, 8193)."""
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M * 5 + N * 11 + K + variant)
    A = _padded(K, M, g) if at else _padded(M, K, g)
    Bm = _padded(N, K, g) if bt else _padded(K, N, g)
    C = torch.full((M, N), float("nan"), device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), A.shape[1], at, Bm.data_ptr(), Bm.shape[1], bt,
                             C.data_ptr(), N, (prec << 4) | (variant << 8), 0, None, 0,
                             torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    Ad = (A[:, :M].double().T if at else A[:, :K].double())
    Bd = (Bm[:, :K].double().T if bt else Bm[:, :N].double())
    ref = Ad @ Bd
    err = (C.double() - ref).abs().max().item()
    mag = (Ad.abs() @ Bd.abs()).max().item()
    bound = (2e-6 if prec != 1 else 1e-2) * mag + 1e-6
    assert err <= bound, (err, bound)


@pytest.mark.parametrize("prec", [2, 1], ids=["f32x", "bf16"])
@pytest.mark.parametrize("epi,act", [(1, 0), (1, 1), (2, 0), (2, 1), (4, 0)])
@pytest.mark.parametrize("M,N,ldc", [(600, 520, 520), (300, 500, 500), (130, 257, 264), (280, 300, 301)])
@pytest.mark.parametrize("variant,planes", [(13, 0), (13, 1), (14, 0)])
def test_gemm_e8_epilogues(prec, epi, act, M, N, ldc, variant, planes):
    """Fused ACT / DACT / SIGMOID epilogues of the eight-phase kernel against float64, in both its
    epilogue forms (C/D layout; LDS row-major with 16-B stores and element tails, ld 301 falls
    back to the C/D layout); nothing written past column N."""
    lib = _lib.load()
    K = 304
    g = torch.Generator(device="cuda").manual_seed(M + 7 * N + 31 * epi + act + variant)
    A = torch.randn(M, K, device="cuda", generator=g) * 0.3
    Bm = _padded(K, N, g) * 0.3
    ld_aux = (N + 7) // 8 * 8
    pre = torch.randn(M, ld_aux, device="cuda", generator=g)
    aux = torch.tanh(pre) if act == 0 else torch.nn.functional.elu(pre)
    C = torch.full((M, ldc), float("nan"), device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), K, 0, Bm.data_ptr(), Bm.shape[1], 0, C.data_ptr(),
                             ldc, epi | (prec << 4) | (variant << 8) | (planes << 12), act,
                             aux.data_ptr(), ld_aux, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    acc = A.double() @ Bm[:, :N].double()
    a = aux[:, :N].double()
    if epi == 1:
        ref = torch.tanh(acc) if act == 0 else torch.where(acc < 0, torch.exp(acc) - 1, acc)
    elif epi == 2:
        ref = acc * (1 - a * a) if act == 0 else torch.where(a < 0, acc * (a + 1), acc)
    else:
        ref = torch.sigmoid(acc)
    mag = (A.double().abs() @ Bm[:, :N].double().abs()).max().item()
    bound = (2e-6 if prec == 2 else 1e-2) * mag + 1e-6
    if planes and prec == 1:  # one RN bf16 plane of the output
        bound += 2.0 ** -8 * ref.abs().max().item()
    err = (C[:, :N].double() - ref).abs().max().item()
    assert err <= bound, (err, bound)
    if ldc > N and not planes:
        assert torch.isnan(C[:, N:]).all()


@pytest.mark.parametrize("mode", ["0", "2"], ids=["ring_only", "e8_everywhere"])
@pytest.mark.parametrize("prec", ["f32x", "bf16"])
@pytest.mark.parametrize("grey", [False, True], ids=["binary", "grey"])
def test_step_e8_modes(mode, prec, grey):
    """A whole step with every 256-row bf16 DMA GEMM on the eight-phase kernel (BCE head with fp32
    or bf16-plane target, DACT row remap, batch-2 weight gradients, split-K) or on the ring
    kernels only."""
    cfg = preset("8c", image_size=20, batch=288, precision=prec).replace(enc=(300, 260, 280),
                                                                        options=f"e8={mode}")
    if prec == "f32x":
        check_step(cfg, grey=grey, recon=True)
    else:
        check_step(cfg, grey=grey, recon=True, **BF16)


@pytest.mark.parametrize("mode", ["1", "2"], ids=["planner", "e8_everywhere"])
def test_step_c3_shape_e8(mode):
    """BASELINE C3's shapes (8d, bf16, 100x100, enc [500]*4, L = 200) at B = 2048 with the default
    plan and with the eight-phase kernel everywhere, documented bf16 bar."""
    check_step(baseline_config("C3").replace(batch=2048, options=f"e8={mode}"), adam=False, **BF16)


def test_step_c2_f32x_e8_everywhere():
    """The benched C2 configuration (f32x, B = 4096) with the eight-phase kernel on every 256-row
    bf16 GEMM, at the fp32 bar."""
    check_step(preset("8c", image_size=100, batch=4096, precision="f32x", options="e8=2"), adam=False)


# ------------------------------------------------------------------ chunked layer-0 gradient
@pytest.mark.parametrize("chunks", [1, 2, 4, 8])
@pytest.mark.parametrize("prec,conv", [("f32x", False), ("bf16", False), ("f32", True)])
def test_wgrad0_chunks_tile_grads_and_match_backward(chunks, prec, conv):
    """Option "wgrad0_chunks" = R: the backward in R + 2 parts; the ranges the parts report cover
    MVAE_BUF_GRADS exactly once, and the chunked gradients equal the one-GEMM backward (the
    chunk GEMMs plan their own split-K, so agreement is to the GEMM's rounding, not bitwise)."""
    from magic_amd.engine import Engine
    from tests.gpu_helpers import make_inputs, make_params, max_rel, to_dev
    if conv:
        cfg = preset("8c", image_size=20, batch=24, conv=True, precision=prec).replace(enc=(64, 40))
    else:
        cfg = preset("8c", image_size=40, batch=96, precision=prec).replace(enc=(300, 260))
    eng = Engine(cfg, 0)
    try:
        P = make_params(cfg)
        X, areas, eps = make_inputs(cfg, cfg.batch)
        eng.load_params(P)
        eng.forward(to_dev(X), to_dev(eps))
        eng.metric(to_dev(areas))
        eng.backward()
        torch.cuda.synchronize()
        ref = eng.grads.cpu().numpy().copy()
        eng.set_option("wgrad0_chunks", chunks)
        assert 3 <= eng.N_BACKWARD_PARTS <= chunks + 2  # fewer chunks than 256-row tiles allow
        eng.load_params(P)
        eng.forward(to_dev(X), to_dev(eps))
        eng.metric(to_dev(areas))
        cover = torch.zeros(eng.grads.numel(), dtype=torch.int32)
        base = eng.grads.data_ptr()
        for part in range(eng.N_BACKWARD_PARTS):
            eng.backward_part(part)
            for v in eng.grad_ranges(part):
                off = (v.data_ptr() - base) // 4
                cover[off:off + v.numel()] += 1
        torch.cuda.synchronize()
        assert int(cover.min()) == 1 and int(cover.max()) == 1, "ranges must tile grads exactly once"
        got = eng.grads.cpu().numpy()
        assert max_rel(got, ref) <= (1e-5 if prec != "bf16" else 1e-2), max_rel(got, ref)
        with pytest.raises(Exception):
            eng.set_option("wgrad0_chunks", 3)
    finally:
        eng.close()


# ------------------------------------------------------------------ 192-row ring tiles
@pytest.mark.parametrize("prec", [2, 1], ids=["f32x", "bf16"])
@pytest.mark.parametrize("bt", [0, 1])
@pytest.mark.parametrize("M,N,K,mode", [(192, 256, 64, 0), (193, 500, 501, 1), (1000, 600, 4099, 0),
                                        (600, 130, 300, 1), (385, 517, 1001, 2), (24576 // 8, 500, 501, 1)])
def test_gemm_tile192(bt, M, N, K, mode, prec):
    """epi bit 13 forces the ring kernel's 192-row tiles (MI = 3, k-contiguous A): ragged M / N /
    K edges, the planner's split-K (K 4099), and the ACT / DACT epilogues (mode 1 / 2)."""
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M * 13 + N * 7 + K + mode)
    A = _padded(M, K, g)
    Bm = _padded(N, K, g) if bt else _padded(K, N, g)
    aux = torch.rand(M, (N + 7) // 8 * 8, device="cuda", generator=g) * 1.6 - 0.8
    C = torch.full((M, N), float("nan"), device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), A.shape[1], 0, Bm.data_ptr(), Bm.shape[1], bt,
                             C.data_ptr(), N, mode | (prec << 4) | (1 << 13), 0,
                             aux.data_ptr() if mode == 2 else None, aux.shape[1],
                             torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    Ad = A[:, :K].double()
    Bd = Bm[:, :K].double().T if bt else Bm[:, :N].double()
    ref = Ad @ Bd
    mag = (Ad.abs() @ Bd.abs()).max().item()
    if mode == 1:
        ref = torch.tanh(ref)
    elif mode == 2:
        y = aux[:, :N].double()
        ref = ref * (1 - y * y)
    err = (C.double() - ref).abs().max().item()
    bound = (2e-6 if prec != 1 else 1e-2) * mag + 1e-6
    assert err <= bound, (err, bound)


def test_sample_latent_space_gpu():
    """11a/utils.py:401-422 on the GPU decoder: every tile of the batched canvas equals a
    single-row generate of its grid point (L = 2, preset 11a at 20 x 20, batch 8)."""
    import numpy as np
    from magic_amd.vae import TangoEncoder, sample_latent_space
    cfg = preset("11a", image_size=20, batch=8)
    cfg.latent = 2
    vae = TangoEncoder(None, config=cfg)
    try:
        c = sample_latent_space(vae, nx=4, ny=4)
        assert c.shape == (80, 80) and np.isfinite(c).all()
        v = np.linspace(-3, 3, 4)
        for i, j in [(0, 0), (1, 3), (3, 2)]:
            one = vae.generate(np.array([[v[j], v[i]]], dtype=np.float32))[0].reshape(20, 20)
            tile = c[(4 - i - 1) * 20:(4 - i) * 20, j * 20:(j + 1) * 20]
            np.testing.assert_allclose(tile, one, rtol=0, atol=1e-6)
    finally:
        vae.close()
