"""Data-parallel host logic (magic_amd.parallel) on CPU with gloo, world_size 2.

Each rank holds half the batch; after one DataParallelStep every rank's parameters must
equal (to float64 rounding) the single-process step on the concatenated batch — for the
squared-difference metric (no mid-step collective) and for the batch-coupled cosine
metric (axis-0 l2_normalize: colsq/coldot all-reduces)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from magic_amd.config import MVAEConfig
from magic_amd.parallel import DataParallelStep, shard_rows
from oracle import mvae_oracle as O
from tests.cpu_engine import OracleEngine


def _cfg(metric, recip, conv=False):
    return MVAEConfig(image_size=8, batch=6, enc=(20, 16), dec=(12, 10), latent=5, act="tanh",
                      metric=metric, reciprocal=recip, deform_weight=10.0, lr=(1e-3, 1e-4), conv=conv)


def _inputs(cfg, B):
    rng = np.random.default_rng(3)
    X = (rng.random((B, 3 * cfg.D)) < 0.3).astype(np.float64)
    areas = rng.integers(296, 6427, B).astype(np.float64)
    eps = rng.standard_normal((3, B, cfg.latent))
    return torch.from_numpy(X), torch.from_numpy(areas), torch.from_numpy(eps)


def _worker(rank, world, port, metric, recip, q, overlap=True, conv=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg(metric, recip, conv)
    full_B = cfg.batch * world
    cfg = cfg.replace(global_batch=full_B)
    oc = O.OracleConfig(image_size=cfg.image_size, enc=cfg.enc, dec=cfg.dec, latent=cfg.latent, conv=conv)
    P = O.init_params(oc, seed=0, dtype=np.float64)
    X, A, E = _inputs(cfg, full_B)
    eng = OracleEngine(cfg, P)
    step = DataParallelStep(eng, overlap=overlap)
    for _ in range(2):
        losses = step.step(shard_rows(X, rank, world), shard_rows(A, rank, world),
                           E[:, rank * cfg.batch:(rank + 1) * cfg.batch].contiguous())
    pred = step.predict(shard_rows(X, rank, world), E[:, rank * cfg.batch:(rank + 1) * cfg.batch].contiguous())
    q.put((rank, {k: v.copy() for k, v in eng.P.items()}, losses.numpy().copy(), pred.numpy().copy()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("metric,recip,overlap,conv", [("sqdiff", True, True, False), ("cosine", False, True, False),
                                                       ("cosine", True, True, False), ("cosine", True, False, False),
                                                       ("sqdiff", True, True, True), ("cosine", False, True, True)])
def test_dp2_equals_single_process(metric, recip, overlap, conv):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, metric, recip, q, overlap, conv))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (P, l, pr)) for r, P, l, pr in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process on the full batch
    cfg = _cfg(metric, recip, conv)
    B = cfg.batch * world
    cfg = cfg.replace(batch=B)
    oc = O.OracleConfig(image_size=cfg.image_size, enc=cfg.enc, dec=cfg.dec, latent=cfg.latent,
                        metric=metric, reciprocal=recip, lr=cfg.lr, conv=conv)
    P = O.init_params(oc, seed=0, dtype=np.float64)
    st = O.adam_init(oc, P)
    X, A, E = _inputs(cfg, B)
    for _ in range(2):
        losses, _, P, st, _ = O.train_step(P, st, X.numpy(), A.numpy(), E.numpy(), oc)
    # get_predictions after the two steps: global-batch cosine norms on every rank
    pred_full = O.predictions(P, X.numpy(), E.numpy(), oc)
    np.testing.assert_allclose(np.concatenate([res[r][2] for r in range(world)]), pred_full, rtol=1e-9)
    for r in range(world):
        Pr, lr_, _ = res[r]
        np.testing.assert_allclose(lr_, losses, rtol=1e-10)
        for k in O.trained_names(oc):
            np.testing.assert_allclose(Pr[k], P[k], rtol=1e-9, atol=1e-12, err_msg=k)
    # replicas stay identical across ranks
    for k in res[0][0]:
        np.testing.assert_array_equal(res[0][0][k], res[1][0][k])


def test_dp_rejects_wrong_global_batch():
    cfg = _cfg("sqdiff", False).replace(global_batch=99)
    oc = O.OracleConfig(image_size=cfg.image_size, enc=cfg.enc, dec=cfg.dec, latent=cfg.latent)
    with pytest.raises(ValueError):
        DataParallelStep(OracleEngine(cfg, O.init_params(oc, 0, np.float64)))
