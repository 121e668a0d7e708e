"""Data-parallel step on the real HIP kernels: 2 ranks sharing the box's one GPU (gloo
all-reduce of device tensors), each with half the batch, vs one process on the full
batch. The all-reduced gradient bucket and the global losses must match the single-
process step within the fp32 parity tolerance (1e-4 relative)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from magic_amd.config import preset
from tests.gpu_helpers import make_inputs, make_params, max_rel

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, metric, q, conv=False, size=24, chunks=4, cfg=None, early=False, comm=False):
    import torch.distributed as dist
    from magic_amd.engine import Engine
    from magic_amd.parallel import DataParallelStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = cfg or preset("8c", image_size=size, batch=32, metric=metric, conv=conv)
    B = cfg.batch
    half = B // world
    eng = Engine(cfg.replace(batch=half, global_batch=B), 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, B)
    sl = slice(rank * half, (rank + 1) * half)
    if early:  # an engine left with Adam-on-the-side-stream on (e.g. by a collective-free step)
        eng.set_option("early_adam", 1)
    st = DataParallelStep(eng, wgrad0_chunks=chunks)
    st.comm_timing = comm  # HIP-event timing of the collective waits (bench.py's comm block)
    if chunks > 1:
        assert eng.N_BACKWARD_PARTS > 3  # the layer-0 weight gradient really runs in row chunks
    st.step(torch.from_numpy(X[sl]).cuda(), torch.from_numpy(areas[sl]).cuda(),
            torch.from_numpy(np.ascontiguousarray(eps[:, sl])).cuda())
    torch.cuda.synchronize()
    q.put((rank, eng.grads.cpu().numpy(), eng.losses.cpu().numpy(),
           {k: v.cpu().numpy() for k, v in eng.params().items()}, st.comm_stats() if comm else None))
    eng.close()
    dist.destroy_process_group()


def _dp2(cfg, metric="cosine", chunks=4, early=False, comm=False):
    """2 spawned gloo ranks on this GPU, each half of cfg.batch: {rank: (grads, losses, params,
    comm_stats)}"""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, metric, q),
                         kwargs=dict(chunks=chunks, cfg=cfg, early=early, comm=comm)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, l, P, c)) for r, g, l, P, c in (q.get(timeout=600) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _single(cfg):
    """one process on the whole batch: grads, losses, and the parameters after Adam"""
    from magic_amd.engine import Engine
    eng = Engine(cfg, 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, cfg.batch)
    eng.forward(torch.from_numpy(X).cuda(), torch.from_numpy(eps).cuda())
    eng.metric(torch.from_numpy(areas).cuda())
    eng.backward()
    torch.cuda.synchronize()
    g, l = eng.grads.cpu().numpy(), eng.losses.cpu().numpy()
    eng.adam()
    P = {k: v.cpu().numpy() for k, v in eng.params().items()}
    eng.close()
    return g, l, P


@pytest.mark.parametrize("prec", ["f32x", "f32"])
def test_dp2_early_adam_left_on_waits_for_the_all_reduce(prec):
    """An engine whose early_adam option was left on: a collective step must not run
    Adam on the side stream before the gradient all-reduce -- both replicas end bitwise equal,
    and equal to the single-process step on the whole batch (1e-4)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = preset("8c", image_size=24, batch=32, precision=prec)
    g_ref, l_ref, P_ref = _single(cfg)
    res = _dp2(cfg, early=True)
    for k in P_ref:
        np.testing.assert_array_equal(res[0][2][k], res[1][2][k])
        assert max_rel(res[0][2][k], P_ref[k]) <= 1e-4, k
    assert max_rel(res[0][0], g_ref) <= 1e-4


def test_dp2_c4_per_rank_shape_matches_full_batch():
    """BASELINE C4's per-rank workload through DataParallelStep on this GPU: 2 gloo ranks at C3's
    shape each (8d, L = 200, bf16, B = 8192 per rank, wgrad0_chunks = 4, cosine colsq / coldot
    all-reduces, async loss reduce) against one process on the concatenated 16 384-pair batch:
    losses and the whole all-reduced gradient bucket at the documented bf16 bar."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.config import baseline_config
    cfg = baseline_config("C3").replace(batch=16384)
    g_ref, l_ref, _ = _single(cfg)
    res = _dp2(cfg, chunks=4)
    for r in range(2):
        g, l, _, _ = res[r]
        np.testing.assert_allclose(l, l_ref, rtol=2e-3)
        err = max_rel(g, g_ref)
        print(f"C4 per-rank shape, rank {r}: losses {l.tolist()} vs {l_ref.tolist()}; bucket max-rel {err:.3e}")
        assert err <= 5e-2, err
    np.testing.assert_array_equal(res[0][0], res[1][0])


def test_dp2_c5_per_rank_shape_matches_full_batch():
    """BASELINE C5's per-rank workload (8e: L = 2000, reciprocal squared-difference metric -- no
    mid-step statistics collective -- bf16, B = 8192 per rank) through DataParallelStep: 2 gloo
    ranks on this GPU against one process on the concatenated 16 384-pair batch, losses and the
    whole all-reduced bucket at the bf16 bar; the collectives timed with HIP events as bench.py's
    comm block does (the exposed all-reduce wait, the bucket: the whole [g1 | g2] buffer)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.config import baseline_config
    cfg = baseline_config("C5").replace(batch=16384)
    assert cfg.latent == 2000 and cfg.reciprocal and cfg.metric == "sqdiff"
    g_ref, l_ref, _ = _single(cfg)
    res = _dp2(cfg, chunks=4, comm=True)
    for r in range(2):
        g, l, _, c = res[r]
        np.testing.assert_allclose(l, l_ref, rtol=2e-3)
        err = max_rel(g, g_ref)
        print(f"C5 per-rank shape, rank {r}: losses {l.tolist()} vs {l_ref.tolist()}; bucket max-rel "
              f"{err:.3e}; comm {c}")
        assert err <= 5e-2, err
        assert c["steps"] == 1 and c["bucket_bytes"] == g.nbytes and c["exposed_allreduce_wait_ms"] >= 0
        assert c["blocking_stats_allreduce_ms"] == 0  # squared difference: no statistics collective
    np.testing.assert_array_equal(res[0][0], res[1][0])


@pytest.mark.parametrize("metric,conv,size,chunks", [("cosine", False, 24, 4), ("sqdiff", False, 24, 4),
                                                     ("sqdiff", True, 24, 4), ("cosine", False, 48, 4),
                                                     ("cosine", False, 48, 1)])
def test_dp2_on_gpu_matches_full_batch(metric, conv, size, chunks):
    """2 ranks (async loss all-reduce beside the backward; layer-0 weight gradient in
    ``wgrad0_chunks`` row chunks, each all-reduced as it completes) vs one process."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.engine import Engine
    cfg = preset("8c", image_size=size, batch=32, metric=metric, conv=conv)
    eng = Engine(cfg, 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, cfg.batch)
    eng.forward(torch.from_numpy(X).cuda(), torch.from_numpy(eps).cuda())
    eng.metric(torch.from_numpy(areas).cuda())
    eng.backward()
    torch.cuda.synchronize()
    g_ref, l_ref = eng.grads.cpu().numpy(), eng.losses.cpu().numpy()
    eng.close()

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, metric, q, conv, size, chunks)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, l)) for r, g, l, _, _ in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        g, l = res[r]
        np.testing.assert_allclose(l, l_ref, rtol=1e-4)
        assert max_rel(g, g_ref) <= 1e-4
    np.testing.assert_array_equal(res[0][0], res[1][0])


def _rccl_worker(port, metric, conv, q):
    import torch.distributed as dist
    from magic_amd.engine import Engine
    from magic_amd.parallel import DataParallelStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cfg = preset("8c", image_size=24, batch=32, metric=metric, conv=conv)
    eng = Engine(cfg, 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, cfg.batch)
    st = DataParallelStep(eng, force_collectives=True)
    assert st.coll
    for _ in range(2):
        st.step(torch.from_numpy(X).cuda(), torch.from_numpy(areas).cuda(), torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    q.put((eng.params()["enc_h0_W"].cpu().numpy(), eng.grads.cpu().numpy(), eng.losses.cpu().numpy()))
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("metric,conv", [("cosine", False), ("sqdiff", True)])
def test_rccl_collective_path_one_rank(metric, conv):
    """The RCCL code path of DataParallelStep (backend "nccl": async all-reduces of the
    library-owned gradient ranges while the later backward parts run, colsq/coldot and loss
    all-reduces) in a one-rank group on this box's GPU: two steps must equal two plain steps
    bitwise (a one-rank SUM is the identity)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.engine import Engine
    cfg = preset("8c", image_size=24, batch=32, metric=metric, conv=conv)
    eng = Engine(cfg, 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, cfg.batch)
    for _ in range(2):
        eng.train_step(torch.from_numpy(X).cuda(), torch.from_numpy(areas).cuda(), torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    w_ref, g_ref = eng.params()["enc_h0_W"].cpu().numpy(), eng.grads.cpu().numpy()
    eng.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, metric, conv, q))
    p.start()
    w, g, _ = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    np.testing.assert_array_equal(g, g_ref)
    np.testing.assert_array_equal(w, w_ref)


def _predict_worker(rank, world, port, q):
    import torch.distributed as dist
    from magic_amd.engine import Engine
    from magic_amd.parallel import DataParallelStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = preset("8c", image_size=24, batch=32, metric="cosine")
    half = cfg.batch // world
    eng = Engine(cfg.replace(batch=half, global_batch=cfg.batch), 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, cfg.batch)
    sl = slice(rank * half, (rank + 1) * half)
    st = DataParallelStep(eng)
    pred = st.predict(torch.from_numpy(X[sl]).cuda(), torch.from_numpy(np.ascontiguousarray(eps[:, sl])).cuda())
    q.put((rank, pred.cpu().numpy()))
    eng.close()
    dist.destroy_process_group()


def test_dp2_predictions_use_global_cosine_norms():
    """get_predictions under data parallelism: the cosine distance normalises each latent
    column over the GLOBAL batch (8c/vae.py:449-450); 2 ranks x half the rows must give the
    single-process predictions on the whole batch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.engine import Engine
    cfg = preset("8c", image_size=24, batch=32, metric="cosine")
    eng = Engine(cfg, 0)
    eng.load_params(make_params(cfg))
    X, areas, eps = make_inputs(cfg, cfg.batch)
    ref = eng.predict(torch.from_numpy(X).cuda(), torch.from_numpy(eps).cuda()).cpu().numpy()
    eng.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_predict_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.concatenate([res[0], res[1]])
    assert max_rel(got, ref) <= 1e-4, max_rel(got, ref)
