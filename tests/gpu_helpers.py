"""Shared helpers for the GPU parity tests: build a case, run the HIP step phase by phase
through the C ABI, run the oracle on the same seeded inputs, compare."""
from __future__ import annotations

import numpy as np
import torch

from magic_amd import _lib
from magic_amd.config import MVAEConfig
from oracle import mvae_oracle as O


def oracle_cfg(cfg: MVAEConfig) -> O.OracleConfig:
    return O.OracleConfig(image_size=cfg.image_size, enc=tuple(cfg.enc), dec=tuple(cfg.dec),
                          latent=cfg.latent, act=cfg.act, deform_weight=cfg.deform_weight,
                          metric=cfg.metric, reciprocal=cfg.reciprocal, lr=tuple(cfg.lr),
                          beta1=cfg.beta1, beta2=cfg.beta2, epsilon=cfg.epsilon,
                          conv=getattr(cfg, "conv", False))


def make_inputs(cfg: MVAEConfig, B: int, seed: int = 1, density: float = 0.1, grey: bool = False):
    """Binary pixels (HWC-interleaved), areas in the reference's range, eps [3,B,L].
    grey: foreground pixels take k/255 values (not exact in bf16: the fp32-target paths)."""
    rng = np.random.default_rng(seed)
    X = (rng.random((B, 3 * cfg.D)) < density).astype(np.float32)
    if grey:
        X *= (rng.integers(1, 256, size=X.shape) / 255.0).astype(np.float32)
    areas = rng.integers(296, 6427, size=B).astype(np.float32)
    eps = np.random.default_rng(seed + 1).standard_normal((3, B, cfg.latent)).astype(np.float32)
    return X, areas, eps


def make_params(cfg: MVAEConfig, seed: int = 0, bias_scale: float = 0.05):
    P = O.init_params(oracle_cfg(cfg), seed=seed, dtype=np.float32)
    rng = np.random.default_rng(seed + 100)
    for k in P:  # non-zero biases exercise the folded-bias (ones column) path
        if k.endswith("_b"):
            P[k] = (rng.standard_normal(P[k].shape) * bias_scale).astype(np.float32)
    return P


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def gpu_phases(eng, X, areas, eps):
    """forward -> metric -> backward; returns losses, dist, g1, g2 (host numpy)."""
    x, a, e = to_dev(X), to_dev(areas), to_dev(eps)
    eng.forward(x, e)
    eng.metric(a)
    eng.backward()
    torch.cuda.synchronize()
    losses = eng.losses.cpu().numpy().astype(np.float64)
    dist = eng.dist.cpu().numpy().astype(np.float64)
    g1 = {k: v.cpu().numpy().astype(np.float64) for k, v in eng.tensors(_lib.KIND_GRAD1).items()}
    g2 = {k: v.cpu().numpy().astype(np.float64) for k, v in eng.tensors(_lib.KIND_GRAD2).items()}
    return losses, dist, g1, g2


def oracle_phases(cfg, P, X, areas, eps):
    oc = oracle_cfg(cfg)
    B = X.shape[0]
    c = O.forward(P, X.astype(np.float64), eps.astype(np.float64), oc)
    O.metric(c, areas.astype(np.float64), oc, B)
    losses = O.loss_sums(c, B)
    g1, g2 = O.backward(c, oc, B)
    c["mag"] = O.backward(c, oc, B, magnitude=True)
    return losses, c["dist"], g1, g2, c


def max_rel(a, b, mag=None):
    """max|a - b| / max|b|. With ``mag`` (the oracle's sum-of-|terms| for the same tensor)
    the denominator is max(max|b|, 1e-2 * max|mag|): a tensor whose exact value cancels
    (true value ~0) is judged against 1% of the magnitude of its summed terms."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.abs(b).max()
    if mag is not None:
        scale = max(scale, 1e-2 * np.abs(np.asarray(mag, np.float64)).max())
    return float(np.abs(a - b).max() / max(scale, 1e-30))
