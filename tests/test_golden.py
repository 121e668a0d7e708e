"""Committed fixtures (tests/golden/, made by make_golden.py): the reference's own data
files (labels, micro image set) and oracle golden vectors for one step per flavour."""
import glob
import os

import numpy as np
import pytest

from oracle import mvae_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STEPS = sorted(glob.glob(os.path.join(GOLD, "step_*.npz")))


def load_step(path):
    z = np.load(path)
    name = os.path.basename(path)[5:-4]
    from tests.golden.make_golden import FLAVOURS, golden_cfg
    cfg = golden_cfg(FLAVOURS[name])
    get = lambda pre: {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}  # noqa: E731
    return cfg, z, get("P/"), get("g1/"), get("g2/"), get("Pn/")


def test_overlap_areas_fixture_matches_reference_statistics():
    """2000 int64 labels, range 296-6426, mean 1972.8, sd 1179.6."""
    a = np.load(os.path.join(os.path.dirname(GOLD), "..", "magic_amd", "data", "overlap_areas.npy"))
    assert a.shape == (2000,) and a.dtype == np.int64
    assert a.min() == 296 and a.max() == 6426
    assert abs(a.mean() - 1972.8) < 0.1 and abs(a.std() - 1179.6) < 1.0


def test_micro_images_fixture():
    z = np.load(os.path.join(GOLD, "overlap_micro.npz"))
    n, h, w = z["shape"]
    assert (n, h, w) == (100, 200, 200)
    lock = np.unpackbits(z["lock_bits"], axis=-1)[..., :w]
    fg = lock.reshape(n, -1).mean(1)
    assert 0.02 < fg.mean() < 0.2  # SURVEY: 5-13% foreground on sampled pairs


@pytest.mark.parametrize("path", STEPS, ids=[os.path.basename(p) for p in STEPS])
def test_oracle_reproduces_golden_step(path):
    cfg, z, P, g1, g2, Pn = load_step(path)
    st = O.adam_init(cfg, P)
    losses, dist, Pn2, _, (h1, h2) = O.train_step(P, st, z["X"], z["areas"], z["eps"], cfg)
    np.testing.assert_allclose(losses, z["losses"], rtol=1e-12)
    np.testing.assert_allclose(dist, z["dist"], rtol=1e-12)
    for k in g1:
        np.testing.assert_allclose(h1[k], g1[k], rtol=1e-10, atol=1e-14)
    for k in g2:
        np.testing.assert_allclose(h2[k], g2[k], rtol=1e-10, atol=1e-14)
    for k in Pn:
        np.testing.assert_allclose(Pn2[k], Pn[k], rtol=1e-12)
    assert len(STEPS) == 5
