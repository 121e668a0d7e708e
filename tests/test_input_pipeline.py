"""Batch producer (``11a/overlap_input.py:127-261``): the HIP kernel
``mvae_make_batch`` against the oracle restatement (bit-exact: given the per-example fp32
rotation coefficients the gather is integer work), on the reference's own images
(tests/golden/overlap_micro.npz = ``overlap_micro.zip``)."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import input_oracle as IO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def micro(n=20):
    z = np.load(os.path.join(GOLD, "overlap_micro.npz"))
    _, h, w = z["shape"]
    L = (np.unpackbits(z["lock_bits"][:n], axis=-1)[..., :w] * 255).astype(np.uint8)
    K = (np.unpackbits(z["key_bits"][:n], axis=-1)[..., :w] * 255).astype(np.uint8)
    return L, K


def test_oracle_rotation_kats():
    """angle 0 = identity; pi = both axes flipped; pi/2 maps a pixel as TF's projective
    transform does (output (x, y) samples input (-y + (W-1+H-1)/2 ... ))."""
    L, _ = micro(2)
    img = L[0]
    h, w = img.shape
    c0 = IO.rotation_coefficients([0.0], h, w)[0]
    np.testing.assert_array_equal(IO.rotate_nearest(img, c0), img)
    cpi = IO.rotation_coefficients([math.pi], h, w)[0]
    np.testing.assert_array_equal(IO.rotate_nearest(img, cpi), img[::-1, ::-1])
    c90 = IO.rotation_coefficients([math.pi / 2], h, w)[0]
    r = IO.rotate_nearest(img, c90)
    # square image: x' = (W-1) - y, y' = x  ->  out[y, x] = in[x, W-1-y]
    np.testing.assert_array_equal(r, img[:, ::-1].T)


def test_oracle_batch_layout():
    L, K = micro(3)
    coef = IO.rotation_coefficients([0.0, 0.0], 200, 200)
    X = IO.make_batch(L, K, [2, 0], coef)
    assert X.shape == (2, 200 * 200 * 3)
    np.testing.assert_array_equal(X[0, 0::3], L[2].reshape(-1) / 255.0)
    np.testing.assert_array_equal(X[0, 1::3], L[2].reshape(-1) / 255.0)
    np.testing.assert_array_equal(X[1, 2::3], K[0].reshape(-1) / 255.0)
    assert set(np.unique(X)) <= {0.0, 1.0}


@pytest.mark.gpu
def test_hip_batch_producer_bit_exact():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.overlap_input import make_batch, rotation_coefficients
    L, K = micro(20)
    rng = np.random.default_rng(5)
    B = 64
    idx = rng.integers(0, 20, B).astype(np.int32)
    ang = rng.uniform(0, 2 * math.pi, B).astype(np.float32)
    ang[:6] = [0.0, math.pi / 2, math.pi, 3 * math.pi / 2, 2 * math.pi - 1e-6, 1e-6]
    coef = rotation_coefficients(ang, 200, 200)
    np.testing.assert_array_equal(coef, IO.rotation_coefficients(ang, 200, 200))
    X = make_batch(torch.from_numpy(L).cuda(), torch.from_numpy(K).cuda(),
                   torch.from_numpy(idx).cuda(), torch.from_numpy(coef).cuda()).cpu().numpy()
    ref = IO.make_batch(L, K, idx, coef)
    np.testing.assert_array_equal(X, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(200, 200), (100, 100), (199, 197), (64, 36)],
                         ids=["vec_200", "vec_100_partial_segment", "scalar_odd", "vec_small"])
@pytest.mark.parametrize("normalize", [True, False], ids=["div255", "raw"])
def test_hip_batch_producer_paths(h, w, normalize):
    """Both kernel paths (4 pixels per thread through LDS when H*W % 4 == 0, else one pixel per
    thread) bit-exact against the oracle, on grey uint8 tables (every byte value, so every
    quotient v/255 occurs) and raw 0..255 output."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.overlap_input import make_batch, rotation_coefficients
    rng = np.random.default_rng(h * 7 + w)
    n, B = 7, 33
    L = rng.integers(0, 256, (n, h, w), dtype=np.uint8)
    K = rng.integers(0, 256, (n, h, w), dtype=np.uint8)
    idx = rng.integers(0, n, B).astype(np.int32)
    ang = rng.uniform(0, 2 * math.pi, B).astype(np.float32)
    ang[:3] = [0.0, math.pi / 2, math.pi]
    coef = rotation_coefficients(ang, h, w)
    X = make_batch(torch.from_numpy(L).cuda(), torch.from_numpy(K).cuda(), torch.from_numpy(idx).cuda(),
                   torch.from_numpy(coef).cuda(), normalize=normalize).cpu().numpy()
    ref = IO.make_batch(L, K, idx, coef, scale_div=255.0 if normalize else 1.0)
    np.testing.assert_array_equal(X, ref)


@pytest.mark.gpu
def test_batch_stream_on_reference_images():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from magic_amd.overlap_input import inputs
    bs = inputs(normalize=True, reshape=True, rotation=True, batch_size=24, image_size=200,
                data_dir=os.path.join(GOLD, "overlap_micro.npz"))
    x, a = next(bs)
    assert x.shape == (24, 200 * 200 * 3) and a.shape == (24,)
    xs = x.cpu().numpy()
    assert set(np.unique(xs)) <= {0.0, 1.0}
    # rotation preserves the foreground mass up to nearest-neighbour edge effects
    lock, rot = xs[:, 0::3].sum(1), xs[:, 1::3].sum(1)
    assert np.all(np.abs(rot - lock) <= 0.15 * lock + 50)
