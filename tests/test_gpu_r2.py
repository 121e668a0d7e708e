"""GPU parity for the round-2 items: the L = 2000 configurations (BASELINE C5 and preset 8e),
the benched C3 / C2 shapes themselves, BCE saturation semantics, the inference-surface RNG
streams, the sharded eps sampler, generate() through the plane-image GEMMs, and the driver
on the reference's own images. Tolerances are written per test (the fp32 bar of
test_gpu_parity.py: max|gpu - oracle| <= 1e-4 * max|oracle| per tensor, cancellation-aware)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from magic_amd import _lib
from magic_amd.config import baseline_config, preset
from oracle import mvae_oracle as O
from tests.gpu_helpers import (gpu_phases, make_inputs, make_params, max_rel, oracle_cfg,
                               oracle_phases, to_dev)
from tests.test_gpu_parity import check_step

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BF16 = dict(tol=5e-2, loss_tol=2e-3, dist_tol=2e-2)  # documented bf16 tolerance


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _engine(cfg):
    from magic_amd.engine import Engine
    return Engine(cfg, 0)


# ------------------------------------------------------------------ L = 2000
@pytest.mark.parametrize("prec", ["f32", "f32x", "bf16"])
def test_c5_reciprocal_sqdiff_L2000(prec):
    """BASELINE C5's flavour (``11a/vae.py:306-313``: reciprocal squared difference) at
    L = 2000 (``8e/vae.py:49``), 100x100, B = 256: the head GEMMs are 4000 wide and the latent
    kernels move 160 KB per pair."""
    cfg = baseline_config("C5").replace(batch=256, precision=prec)
    assert cfg.latent == 2000 and cfg.metric == "sqdiff" and cfg.reciprocal
    check_step(cfg, recon=True, **(BF16 if prec == "bf16" else {}))


@pytest.mark.parametrize("prec", ["f32", "f32x", "bf16"])
def test_8e_cosine_L2000(prec):
    """Preset 8e as the reference ran it: axis-0 cosine distance over L = 2000 columns."""
    cfg = preset("8e", image_size=100, batch=256, precision=prec)
    check_step(cfg, **(BF16 if prec == "bf16" else {}))


# ------------------------------------------------------------------ benched shapes
def test_c3_benched_shape_bf16():
    """BASELINE C3 exactly as bench.py --config C3 runs it (8d, bf16, B = 8192): split-K
    plans, 24576-row stacks and tile counts of the benched shape, documented bf16 bar."""
    cfg = baseline_config("C3")
    assert cfg.batch == 8192 and cfg.precision == "bf16"
    check_step(cfg, adam=False, **BF16)


def test_c2_benched_shape_with_adam():
    """BASELINE C2 (f32x, B = 4096) including both TF-Adam updates, at the fp32 bar."""
    check_step(baseline_config("C2"), adam=True)


# ------------------------------------------------------------------ BCE saturation
def _saturated_case(cfg):
    P = make_params(cfg)
    P["dec_out_mean_b"][:7] = 60.0      # u >= 60 - |d2 Vo| on pixels 0..6 -> y == 1.0
    X, areas, eps = make_inputs(cfg, cfg.batch)
    X[:, 0:21:3] = 0.0                   # lock pixels 0..6 are 0: log(1 - y) = log(0)
    return P, X, areas, eps


@pytest.mark.parametrize("prec", ["f32", "f32x", "bf16"])
def test_bce_saturation_forward_inf_gradients_finite(prec):
    """``11a/vae.py:266-267`` has no epsilon: saturated pixels make r_l and cost +inf (as in
    TF). The build's gradient dU = (y - x)/B stays finite and equals the oracle's (TF's would
    be NaN; TangoEncoder reproduces that downstream, next test)."""
    cfg = preset("8c", image_size=20, batch=64, precision=prec)
    eng = _engine(cfg)
    try:
        P, X, areas, eps = _saturated_case(cfg)
        eng.load_params(P)
        lg, dg, g1g, g2g = gpu_phases(eng, X, areas, eps)
        lo, do, g1o, g2o, c = oracle_phases(cfg, P, X, areas, eps)
        assert np.all(c["y"][:, :7] == 1.0) and np.isposinf(lo[0]) and np.isposinf(lo[2])
        assert np.isposinf(lg[0]) and np.isposinf(lg[2]), lg
        tol = 5e-2 if prec == "bf16" else 1e-4
        for i in (1, 3, 4):
            assert abs(lg[i] - lo[i]) <= (2e-3 if prec == "bf16" else 1e-4) * max(abs(lo[i]), 1e-3)
        m1, m2 = c["mag"]
        for k in g1o:
            assert np.all(np.isfinite(g1g[k])), k
            assert max_rel(g1g[k], g1o[k], m1[k]) <= tol, k
        for k in g2o:
            assert max_rel(g2g[k], g2o[k], m2[k]) <= tol, k
    finally:
        eng.close()


def test_bce_saturation_reference_guard_fires_next_step():
    """TangoEncoder after a +inf cost: the next partial_fit reports NaN (the reference's
    parameters are NaN after TF's inf*0 gradient), and the driver's guard raises
    TrainingException on that step (``11a/main.py:77-78``)."""
    from magic_amd.main import TrainingException, train
    from magic_amd.vae import TangoEncoder
    cfg = preset("11a", image_size=20, batch=16)
    vae = TangoEncoder(None, config=cfg)
    try:
        P, X, areas, eps = _saturated_case(cfg)
        vae.engine.load_params(P)
        feed = iter([(X, areas)] * 8)
        fits = []
        orig = vae.partial_fit

        def spy(Xb, a):
            out = orig(Xb, a)
            fits.append(out[0])
            return out
        vae.partial_fit = spy
        with pytest.raises(TrainingException):
            train(vae, feed, 8 * cfg.batch, training_epochs=1, log=lambda s: None)
        assert np.isposinf(fits[0]) and np.isnan(fits[1]) and len(fits) == 2
    finally:
        vae.close()


# ------------------------------------------------------------------ RNG streams
def test_inference_draws_do_not_shift_training_noise():
    """transform draws nothing; predict/reconstruct draw from the inference stream; the
    counters round-trip through TangoEncoder.state_dict."""
    from magic_amd.vae import TangoEncoder
    cfg = preset("8c", image_size=12, batch=8).replace(enc=(24, 16), latent=5)
    X, areas, _ = make_inputs(cfg, cfg.batch)
    a = TangoEncoder(None, config=cfg)
    b = TangoEncoder(None, config=cfg)
    try:
        a.transform(X)
        a.get_predictions(X)
        a.reconstruct(X)
        assert a.engine.get_rng() == (0, 2)
        ra = a.partial_fit(X, areas)
        rb = b.partial_fit(X, areas)
        np.testing.assert_array_equal(np.array(ra[:5]), np.array(rb[:5]))
        assert a.engine.get_rng() == (1, 2) and b.engine.get_rng() == (1, 0)
        sd = a.state_dict()
        c = TangoEncoder(None, config=cfg, init_seed=7)
        c.load_state_dict(sd)
        assert c.engine.get_rng() == (1, 2)
        np.testing.assert_array_equal(np.array(a.partial_fit(X, areas)[:5]),
                                      np.array(c.partial_fit(X, areas)[:5]))
        c.close()
    finally:
        a.close()
        b.close()


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist
    from magic_amd.engine import Engine
    from magic_amd.parallel import DataParallelStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = preset("8c", image_size=16, batch=24, metric="cosine")
    half = cfg.batch // world
    eng = Engine(cfg.replace(batch=half, global_batch=cfg.batch), 0)
    eng.load_params(make_params(cfg))
    X, areas, _ = make_inputs(cfg, cfg.batch)
    sl = slice(rank * half, (rank + 1) * half)
    DataParallelStep(eng).step(to_dev(X[sl]), to_dev(areas[sl]), None)  # internal eps
    torch.cuda.synchronize()
    q.put((rank, eng.buffer(_lib.BUF_EPS).cpu().numpy(), eng.grads.cpu().numpy()))
    eng.close()
    dist.destroy_process_group()


def test_sharded_sampler_equals_single_process_draw():
    """With eps drawn internally, rank r of a 2-way data-parallel step draws exactly rows
    [r B/2, (r+1) B/2) of the single process's eps, so the all-reduced gradients match the
    full-batch step (fp32 bar)."""
    cfg = preset("8c", image_size=16, batch=24, metric="cosine")
    eng = _engine(cfg)
    eng.load_params(make_params(cfg))
    X, areas, _ = make_inputs(cfg, cfg.batch)
    eng.forward(to_dev(X), None)
    eng.metric(to_dev(areas))
    eng.backward()
    torch.cuda.synchronize()
    eps_ref = eng.buffer(_lib.BUF_EPS).cpu().numpy().reshape(3, cfg.batch, cfg.latent)
    g_ref = eng.grads.cpu().numpy()
    eng.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (e, g) for r, e, g in (q.get(timeout=300) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    half = cfg.batch // 2
    for r in range(2):
        e, g = res[r]
        np.testing.assert_array_equal(e.reshape(3, half, cfg.latent),
                                      eps_ref[:, r * half:(r + 1) * half])
        assert max_rel(g, g_ref) <= 1e-4


# ------------------------------------------------------------------ generate via plane GEMMs
@pytest.mark.parametrize("prec", ["f32x", "bf16"])
def test_generate_plane_modes_wide_decoder(prec):
    """generate() re-points the decoder's first GEMM at the z buffer it feeds; with L + 1 > 64
    and B >= 256 that GEMM runs on the 256x256 plane kernel, which must read zgen's own plane
    images (stride B*ldz)."""
    cfg = preset("10a", image_size=20, batch=256, precision=prec)
    assert cfg.latent + 1 > 64
    eng = _engine(cfg)
    try:
        P = make_params(cfg)
        eng.load_params(P)
        z = np.random.default_rng(3).standard_normal((cfg.batch, cfg.latent)).astype(np.float32)
        yg = eng.generate(to_dev(z)).cpu().numpy()
        _, _, _, yo = O.decode({k: v.astype(np.float64) for k, v in P.items()}, z.astype(np.float64),
                               oracle_cfg(cfg))
        assert max_rel(yg, yo) <= (2e-2 if prec == "bf16" else 1e-4)
        y5 = eng.generate(to_dev(z[:5])).cpu().numpy()
        assert max_rel(y5, yo[:5]) <= (2e-2 if prec == "bf16" else 1e-4)
    finally:
        eng.close()


# ------------------------------------------------------------------ driver on real images
def test_driver_on_reference_images():
    """Two short epochs of magic_amd.main.train (11a driver) on the reference's
    overlap_micro images (tests/golden/overlap_micro.npz) through the HIP batch producer."""
    from magic_amd import overlap_input
    from magic_amd.main import train
    from magic_amd.vae import TangoEncoder
    npz = os.path.join(ROOT, "tests", "golden", "overlap_micro.npz")
    cfg = preset("11a", image_size=200, batch=8)
    vae = TangoEncoder(None, config=cfg)
    try:
        stream = overlap_input.inputs(normalize=True, reshape=True, rotation=True, batch_size=8,
                                      image_size=200, data_dir=npz)
        logs = []
        _, hist = train(vae, stream, 48, training_epochs=2, log=logs.append)
        eps_ = [h for h in hist if h[0] == "epoch"]
        assert len(eps_) == 2 and all(np.isfinite(h[2]) for h in eps_)
        assert [h[:3] for h in hist if h[0] == "mse"] == [("mse", 0, 3)]
        x, a = next(stream)
        assert x.shape == (8, 200 * 200 * 3) and float(x.max()) == 1.0
        raw = overlap_input.inputs(normalize=False, reshape=False, rotation=True, batch_size=8,
                                   image_size=200, data_dir=npz)
        xr, _ = next(raw)
        assert xr.shape == (8, 200, 200, 3) and float(xr.max()) == 255.0
    finally:
        vae.close()


# ------------------------------------------------------------------ schedule switches
@pytest.mark.parametrize("prec", ["f32x", "bf16"])
def test_side_stream_schedule_is_bitwise_identical(prec):
    """Weight gradients on the side stream (default) vs all on the caller's stream: the same
    GEMMs with their own split-K workspaces -> bitwise identical gradients and losses, through
    mvae_backward and through the three-part (data-parallel) entry."""
    cfg = preset("8c", image_size=40, batch=768, precision=prec).replace(enc=(400, 300, 260))
    eng = _engine(cfg)
    try:
        P = make_params(cfg)
        X, areas, eps = make_inputs(cfg, cfg.batch)
        outs = []
        for side in (1, 0):
            eng.set_option("side_stream", side)
            eng.load_params(P)
            outs.append(gpu_phases(eng, X, areas, eps))
        eng.set_option("side_stream", 1)
        x, a, e = to_dev(X), to_dev(areas), to_dev(eps)
        eng.forward(x, e)
        eng.metric(a)
        for part in range(eng.N_BACKWARD_PARTS):
            eng.backward_part(part)
        torch.cuda.synchronize()
        parts = eng.grads.cpu().numpy()
        for o in outs[1:]:
            for u, v in zip(outs[0][:2], o[:2]):
                np.testing.assert_array_equal(u, v)
            for d in (2, 3):
                for k in outs[0][d]:
                    np.testing.assert_array_equal(outs[0][d][k], o[d][k])
        eng.forward(x, e)
        eng.metric(a)
        eng.backward()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(parts, eng.grads.cpu().numpy())
    finally:
        eng.close()


# ------------------------------------------------------------------ fp32 VALU kernel (skinny GEMMs)

@pytest.mark.parametrize("prec", ["f32x", "bf16"])
def test_early_adam_is_bitwise_identical(prec):
    """Option early_adam (Adam of the blocks after layer 0 on the side stream, beside the layer-0
    weight gradient) vs one Adam launch after the backward, and mvae_train_step (which uses it
    in the plane modes), with the layer-0 weight gradient as one GEMM or in two row chunks (chunk
    0's rows updated beside chunk 1's GEMM: option early_chunks):
    all bitwise identical parameters after three steps."""
    cfg = preset("8c", image_size=40, batch=768, precision=prec).replace(enc=(400, 300, 260))
    P = make_params(cfg)
    X, areas, eps = make_inputs(cfg, cfg.batch)
    x, a, e = to_dev(X), to_dev(areas), to_dev(eps)
    outs, outs2 = [], []
    for mode in ("early", "late", "train_step", "early2", "late2", "train_step2"):
        eng = _engine(cfg)  # fresh Adam state per mode
        try:
            eng.set_option("early_adam", 1 if mode.startswith("early") else 0)
            if mode == "train_step2":  # two chunks under the early Adam
                eng.set_option("early_chunks", 2)
            elif mode.endswith("2"):  # layer-0 weight gradient in two chunks: chunk 0's Adam early
                eng.set_option("wgrad0_chunks", 2)
            else:  # one layer-0 GEMM, also with the early Adam (the default: early_chunks = 1)
                eng.set_option("early_chunks", 1)
            eng.load_params(P)
            for _ in range(3):
                if mode.startswith("train_step"):
                    eng.train_step(x, a, e)
                else:
                    eng.forward(x, e)
                    eng.metric(a)
                    eng.backward()
                    eng.adam()
            torch.cuda.synchronize()
            (outs2 if mode.endswith("2") else outs).append({k: v.cpu().numpy() for k, v in eng.params().items()})
        finally:
            eng.close()
    # the chunk GEMMs keep the one-GEMM plan (split-K, kernel): all six bitwise equal, the default
    # train_step (two chunks under the early Adam) and the plain sequence included
    group = outs + outs2
    for o in group[1:]:
        for k in group[0]:
            np.testing.assert_array_equal(group[0][k], o[k])



@pytest.mark.parametrize("prec", ["f32x", "bf16"])
def test_bce_split_matches_one_launch(prec):
    """The BCE head in whole rounds plus 256x128 ring tiles for the remaining columns (option
    bce_split; 66 x 66 images, B = 4096: 16 x 18 = 288 tiles of 256x256 -> 16 n-tiles + 272
    columns) vs one launch: bitwise identical in bf16; in f32x the eight-phase kernel's
    image-reusing walk sums the plane pairs in another order than the ring kernel, so the
    remainder columns agree to fp32 rounding (losses, distance and gradients within 1e-6)."""
    cfg = preset("8c", image_size=66, batch=4096, precision=prec).replace(enc=(300, 260))
    P = make_params(cfg)
    X, areas, eps = make_inputs(cfg, cfg.batch)
    eng = _engine(cfg)
    try:
        outs = []
        for split in (1, 0):
            eng.set_option("bce_split", split)
            eng.load_params(P)
            outs.append(gpu_phases(eng, X, areas, eps))
        def same(u, v):
            if prec == "bf16":
                np.testing.assert_array_equal(u, v)
            else:
                u, v = np.asarray(u, np.float64), np.asarray(v, np.float64)
                assert np.abs(u - v).max() <= 1e-6 * max(np.abs(v).max(), 1e-30)
        for u, v in zip(outs[0][:2], outs[1][:2]):
            same(u, v)
        for d in (2, 3):
            for k in outs[0][d]:
                same(outs[0][d][k], outs[1][d][k])
    finally:
        eng.close()

@pytest.mark.parametrize("at,bt", [(0, 0), (1, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 53, 29), (12288, 40, 501), (21, 500, 4096),
                                   (4096, 20, 500), (16384, 500, 40), (501, 40, 8192), (70, 130, 65)])
def test_gemm_valu_layouts(at, bt, M, N, K):
    """The skinny-shape fp32 VALU kernel (variant 9) on every layout and the step's skinny
    shapes at L = 20 (head forward / weight gradient, decoder layer 1 and its gradients, the
    latent-head dgrad), incl. its split-K, against float64 at the fp32 bound."""
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(M * 3 + N * 7 + K)
    A = torch.randn((K, M) if at else (M, K), device="cuda", generator=g)
    Bm = torch.randn((N, K) if bt else (K, N), device="cuda", generator=g)
    C = torch.full((M, N), float("nan"), device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), A.shape[1], at, Bm.data_ptr(), Bm.shape[1], bt,
                             C.data_ptr(), N, 9 << 8, 0, None, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    Ad = A.double().T if at else A.double()
    Bd = Bm.double().T if bt else Bm.double()
    err = (C.double() - Ad @ Bd).abs().max().item()
    mag = (Ad.abs() @ Bd.abs()).max().item()
    assert err <= 2e-6 * mag + 1e-6, (err, mag)


@pytest.mark.parametrize("epi,act", [(1, 0), (1, 1), (2, 0), (2, 1), (4, 0)])
def test_gemm_valu_epilogues(epi, act):
    lib = _lib.load()
    M, N, K = 300, 500, 21
    g = torch.Generator(device="cuda").manual_seed(11 + epi + act)
    A = torch.randn(M, K, device="cuda", generator=g) * 0.3
    Bm = torch.randn(K, N, device="cuda", generator=g) * 0.3
    aux = torch.tanh(torch.randn(M, N, device="cuda", generator=g)) if act == 0 else \
        torch.nn.functional.elu(torch.randn(M, N, device="cuda", generator=g))
    C = torch.empty(M, N, device="cuda")
    rc = lib.mvae_debug_gemm(M, N, K, A.data_ptr(), K, 0, Bm.data_ptr(), N, 0, C.data_ptr(), N,
                             epi | (9 << 8), act, aux.data_ptr(), N, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.mvae_last_error(None)
    acc = A.double() @ Bm.double()
    if epi == 1:
        ref = torch.tanh(acc) if act == 0 else torch.where(acc < 0, torch.exp(acc) - 1, acc)
    elif epi == 2:
        a = aux.double()
        ref = acc * (1 - a * a) if act == 0 else torch.where(a < 0, acc * (a + 1), acc)
    else:
        ref = torch.sigmoid(acc)
    assert (C.double() - ref).abs().max().item() < 1e-5
