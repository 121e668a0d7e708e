"""The HIP path against the COMMITTED golden vectors (tests/golden/step_*.npz, written by
tests/golden/make_golden.py from the oracle): same inputs, eps and parameters as stored in the
fixture, the fp32 bar of the north star (1e-4 max-norm relative per tensor, cancellation-aware
with the oracle's sum-of-|terms| scale as in test_gpu_parity.py) for the five losses, the
distance vector and every gradient of both optimizers."""
import glob
import os

import numpy as np
import pytest
import torch

from magic_amd import _lib
from magic_amd.config import MVAEConfig
from oracle import mvae_oracle as O
from tests.gpu_helpers import max_rel, to_dev
from tests.test_golden import GOLD, load_step

pytestmark = pytest.mark.gpu
STEPS = sorted(glob.glob(os.path.join(GOLD, "step_*.npz")))


@pytest.mark.parametrize("prec", ["f32", "f32x"])
@pytest.mark.parametrize("path", STEPS, ids=[os.path.basename(p)[5:-4] for p in STEPS])
def test_gpu_step_matches_golden_vectors(path, prec):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.engine import Engine
    oc, z, P, g1, g2, _ = load_step(path)
    B = z["X"].shape[0]
    cfg = MVAEConfig(image_size=oc.image_size, batch=B, enc=tuple(oc.enc), dec=tuple(oc.dec),
                     latent=oc.latent, act=oc.act, metric=oc.metric, reciprocal=oc.reciprocal,
                     deform_weight=oc.deform_weight, lr=tuple(oc.lr), precision=prec, conv=oc.conv)
    eng = Engine(cfg, 0)
    try:
        eng.load_params({k: v.astype(np.float32) for k, v in P.items()})
        eng.forward(to_dev(z["X"].astype(np.float32)), to_dev(z["eps"].astype(np.float32)))
        eng.metric(to_dev(z["areas"].astype(np.float32)))
        eng.backward()
        torch.cuda.synchronize()
        losses = eng.losses.cpu().numpy().astype(np.float64)[:5]
        dist = eng.dist.cpu().numpy().astype(np.float64)
        h1 = {k: v.cpu().numpy().astype(np.float64) for k, v in eng.tensors(_lib.KIND_GRAD1).items()}
        h2 = {k: v.cpu().numpy().astype(np.float64) for k, v in eng.tensors(_lib.KIND_GRAD2).items()}
    finally:
        eng.close()
    # the cancellation scale (sum of |terms|) of the same step, from the oracle
    c = O.forward(P, z["X"], z["eps"], oc)
    O.metric(c, z["areas"], oc, B)
    m1, m2 = O.backward(c, oc, B, magnitude=True)
    rel = np.abs(losses - z["losses"]) / np.maximum(np.abs(z["losses"]), 1e-3)
    assert np.all(rel <= 1e-4), rel
    assert max_rel(dist, z["dist"]) <= 1e-4
    assert set(h1) >= set(g1) and set(h2) == set(g2)
    for k in g1:
        assert max_rel(h1[k], g1[k], m1[k]) <= 1e-4, ("g1", k, max_rel(h1[k], g1[k], m1[k]))
    for k in g2:
        assert max_rel(h2[k], g2[k], m2[k]) <= 1e-4, ("g2", k, max_rel(h2[k], g2[k], m2[k]))
