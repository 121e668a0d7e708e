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


@pytest.mark.parametrize("reg", [0, 1], ids=["lds", "reg"])
@pytest.mark.parametrize("prec", [2, 1], ids=["f32x", "bf16"])
@pytest.mark.parametrize("at", [0, 1], ids=["fwd", "wgrad"])
@pytest.mark.parametrize("epi", [0, 1], ids=["store", "act"])
@pytest.mark.parametrize("M,N,K", [(600, 520, 300), (256, 256, 64), (130, 257, 1001), (300, 500, 4099),
                                   (700, 260, 10001)])
def test_gemm_bits_path_bitwise_equal_planes(reg, prec, at, epi, M, N, K):
    """variant 13 forces the eight-phase kernel; epi bit 14 hands it A as a BitMat too: the bits
    path must reproduce the plane path bit for bit in bf16, to fp32 rounding in f32x (ragged M / N /
    K, partial k-tiles, split-K at K 4099 / 10001, one-block shapes), and float64 at the bars.
    reg (epi bit 15): the words loaded to registers by each wave (the fused de-interleave's form)
    instead of through an LDS copy of the block."""
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M * 3 + N * 7 + K + 11 * at + epi)
    A = _bin(K, M, g) if at else _bin(M, K, g)
    Bm = torch.randn(K, (N + 7) // 8 * 8, device="cuda", generator=g) * 0.1
    ldc = (N + 7) // 8 * 8
    flags = epi | (prec << 4) | (13 << 8)
    Cp = _gemm(lib, M, N, K, A, at, Bm, ldc, flags)
    Cb = _gemm(lib, M, N, K, A, at, Bm, ldc, flags | (1 << 14) | (reg << 15))
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


# ------------------------------------------------------------------ the fused de-interleave

def _batches(cfg, n, grey_at, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = []
    for i in range(n):
        x = (torch.rand(cfg.batch, 3 * cfg.D, device="cuda", generator=g) < 0.1).float()
        if i == grey_at:  # a batch with pixels other than 0 / 1: the grey pass + plane-path fallback
            x = x * torch.randint(1, 256, x.shape, device="cuda", generator=g).float() / 255.0
        a = torch.randint(296, 6427, (cfg.batch,), device="cuda", generator=g).float()
        out.append((x, a))
    return out


def test_deint_fuse_c3_steps_bitwise():
    """C3 (bf16, B = 8192, 100x100, L = 200): the de-interleave's workers inside the layer-0
    forward's launch (create option deint_fuse; 192 tiles + 64 workers, the tiles polling the
    workers' chunk counters) against the separate de-interleave launch -- the same forward split
    (1), so three training steps (the second batch grey: the plane-path fallback) leave bitwise
    identical parameters and losses."""
    from magic_amd.config import baseline_config
    from magic_amd.engine import Engine
    from tests.gpu_helpers import make_params
    cfg = baseline_config("C3")
    assert cfg.precision == "bf16" and cfg.batch == 8192
    P = make_params(cfg)
    batches = _batches(cfg, 3, 1, 7)
    res = []
    for fuse in (0, 1):
        eng = Engine(cfg.replace(options=f"deint_fuse={fuse}"), 0)
        try:
            eng.load_params(P)
            L = []
            for x, a in batches:
                eng.train_step(x, a)
                L.append(eng.losses.clone())
            torch.cuda.synchronize()
            res.append(({k: v.cpu() for k, v in eng.params().items()}, torch.stack(L).cpu()))
        finally:
            eng.close()
    (p0, l0), (p1, l1) = res
    assert torch.equal(l0, l1), (l0, l1)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k


def test_deint_fuse_c2_gradients_match():
    """C2 (f32x, B = 4096): the fused launch runs the forward at split 2 (96 tiles x 2 + 64
    workers), the separate path at the planner's split: the same products summed in another order,
    so one binary and one grey batch's losses and gradients agree to fp32 rounding."""
    from magic_amd.config import baseline_config
    from magic_amd.engine import Engine
    from tests.gpu_helpers import make_params
    cfg = baseline_config("C2")
    assert cfg.precision == "f32x"
    P = make_params(cfg)
    batches = _batches(cfg, 2, 1, 9)
    res = []
    for fuse in (0, 1):
        eng = Engine(cfg.replace(options=f"deint_fuse={fuse}"), 0)
        try:
            eng.load_params(P)
            r = []
            for x, a in batches:
                eng.forward(x)
                eng.metric(a)
                eng.backward()
                torch.cuda.synchronize()
                r.append((eng.losses.cpu().double(),
                          {k: v.cpu().double() for k, v in eng.tensors(_lib.KIND_GRAD1).items()},
                          {k: v.cpu().double() for k, v in eng.tensors(_lib.KIND_GRAD2).items()}))
            res.append(r)
        finally:
            eng.close()
    for (l0, g10, g20), (l1, g11, g21) in zip(*res):
        assert ((l0 - l1).abs() <= 1e-5 * l0.abs().clamp_min(1e-3)).all(), (l0, l1)
        for g0, g1 in ((g10, g11), (g20, g21)):
            for k in g0:
                scale = g0[k].abs().max().clamp_min(1e-30)
                assert (g0[k] - g1[k]).abs().max() / scale <= 1e-4, k


@pytest.mark.parametrize("prec", ["f32x", "bf16"])
@pytest.mark.parametrize("grey", [False, True], ids=["binary", "grey"])
def test_deint_fuse_small_step_vs_oracle(prec, grey):
    """The fused launch at a small ragged shape (20x20 images, B = 320, 300/260/280-wide encoder:
    8 tiles + 248 workers, more workers than tasks, a partial last chunk) against the float64
    oracle at the bars of test_step_wide_kernels."""
    from magic_amd.config import preset
    from tests.test_gpu_parity import check_step
    cfg = preset("8c", image_size=20, batch=320, precision=prec).replace(enc=(300, 260, 280),
                                                                       options="deint_fuse=1")
    if prec == "f32x":
        check_step(cfg, grey=grey, recon=True)
    else:
        check_step(cfg, grey=grey, tol=5e-2, loss_tol=2e-3, dist_tol=2e-2, recon=True)


# ------------------------------------------------------------------ xbw transposed from xbf

@pytest.mark.parametrize("case", ["C3", "C2", "small"])
def test_xbw_split_steps_bitwise(case):
    """Option xbw_split: the de-interleave writes the forward BitMat only and the layer-0 weight
    gradient's BitMat is transposed from it on the side stream (bits_transpose_kernel), joined
    before the weight gradient. The same bits, so three training steps (the second batch grey:
    the planes path) leave bitwise identical parameters and losses -- at C3 (bf16), C2 (f32x) and a
    ragged small shape (D = 400: a partial last pixel tile; B = 320)."""
    from magic_amd.config import baseline_config, preset
    from magic_amd.engine import Engine
    from tests.gpu_helpers import make_params
    if case == "small":
        cfg = preset("8c", image_size=20, batch=320, precision="bf16").replace(enc=(300, 260, 280))
    else:
        cfg = baseline_config(case)
    _steps_bitwise(cfg, "xbw_split=0", "xbw_split=1")


def _steps_bitwise(cfg, opt_a, opt_b):
    """Three training steps (the second batch grey) under two create options: bitwise identical
    parameters and losses."""
    from magic_amd.engine import Engine
    from tests.gpu_helpers import make_params
    P = make_params(cfg)
    batches = _batches(cfg, 3, 1, 11)
    res = []
    for opt in (opt_a, opt_b):
        eng = Engine(cfg.replace(options=opt), 0)
        try:
            eng.load_params(P)
            L = []
            for x, a in batches:
                eng.train_step(x, a)
                L.append(eng.losses.clone())
            torch.cuda.synchronize()
            res.append(({k: v.cpu() for k, v in eng.params().items()}, torch.stack(L).cpu()))
        finally:
            eng.close()
    (p0, l0), (p1, l1) = res
    assert torch.equal(l0, l1), (l0, l1)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k


# ------------------------------------------------------------------ one-launch column statistics

@pytest.mark.parametrize("case", ["C2", "C3", "wide"])
def test_cs_one_steps_bitwise(case):
    """Option cs_one: the cosine metric's column statistics (colsq, coldot; 8c/vae.py:449-450) in
    one launch whose last chunk's workgroup sums the partials in the two-launch form's order -- the
    same bits over three steps, at C2 (64 row chunks, one column block) and at a ragged shape with
    several column blocks (L = 100: 200 colsq columns; B = 1000: a partial last chunk)."""
    from magic_amd.config import baseline_config, preset
    if case == "wide":
        cfg = preset("8c", image_size=20, batch=1000, precision="bf16").replace(latent=100)
    else:
        cfg = baseline_config(case)
    assert cfg.metric == "cosine"
    _steps_bitwise(cfg, "cs_one=0", "cs_one=1")  # (forced on: the default is on only where L <= 32)


# ------------------------------------------------------------------ coalesced de-interleave loads

@pytest.mark.parametrize("case", ["C3", "C2", "small"])
def test_deint_coalesced_steps_bitwise(case):
    """deint_variant 8: the de-interleave's X loads coalesced through an LDS stage (deint_load_co)
    -- the same BitMats, target bits and not-binary word, so three steps (the second batch grey)
    are bitwise the default's; C3 takes its weight-gradient-words-free form (xbw_split), C2 the
    whole form, and the small shape (D = 400) a partial last pixel task."""
    from magic_amd.config import baseline_config, preset
    if case == "small":
        cfg = preset("8c", image_size=20, batch=320, precision="bf16").replace(enc=(300, 260, 280))
    else:
        cfg = baseline_config(case)
    _steps_bitwise(cfg, "", "deint_variant=8")
