"""ORACLE — TEST INFRASTRUCTURE ONLY. Never imported by the product (``magic_amd``).

CPU restatement (numpy, float64 or float32) of ONE training step of the "magic"
asymmetric metric-VAE, ``TangoEncoder`` from the reference:

  * graph / hyper-parameters : ``11a/vae.py:22-332`` and the 8c-family presets
    ``8c/vae.py:22-326`` (encoder widths :30, latent :49, tanh :56, lrs :63,
    deformation x10 :287, cosine distance :301, ``cosine_distance`` :438-452);
  * 11a differences: elu (``11a/vae.py:58``), deformation x100 (``:293``),
    reciprocal distance (``:307,309``);
  * init: ``xavier_init`` ``11a/utils.py:484-491``; zero biases ``11a/vae.py:116-135``;
  * step: ``partial_fit`` ``11a/vae.py:385-411`` = forward + gradients of ``cost``
    and of ``training_loss`` + two ``AdamOptimizer.minimize`` (``11a/vae.py:320-327``).

The reference's arithmetic lives in TensorFlow 1.x (unpinned, ~1.2/1.3 by the log
headers ``8c/nohup.out:1-14``), which is absent here and Python-2-only in the
reference. This module restates the TF1 op semantics used on the path:
  - ``tf.nn.l2_normalize(a, 0)`` = a * rsqrt(max(sum_over_batch(a^2), 1e-12))
    (axis 0 = the BATCH axis, as the reference calls it, ``8c/vae.py:449-450``);
  - reconstruction ``-sum log(y^x (1-y)^(1-x))`` with TF ``pow(0,0)=1`` semantics
    and no epsilon (``11a/vae.py:266-269``);
  - ``EluGrad`` g*(y+1) where y<0; ``TanhGrad`` g*(1-y^2);
  - ``ApplyAdam``: lr_t = lr*sqrt(1-b2^t)/(1-b1^t) in fp32, m += (g-m)(1-b1),
    v += (g^2-v)(1-b2), var -= lr_t*m/(sqrt(v)+eps); beta powers are fp32
    variables multiplied after each step.
Semantics the reference leaves undefined and this oracle fixes:
  - ``eps`` (``tf.random_normal``, TF Philox) cannot be reproduced: it is an INPUT,
    shape [3, B, L] in the reference's call order (lock, rotated lock, key);
  - both optimizers' gradients come from the pre-step parameters and
    theta_new = (theta - delta1) - delta2 (the reference runs both ApplyAdam ops in
    one ``sess.run`` with no ordering, ``11a/vae.py:399-400``).

PARITY UNPINNED at the TensorFlow boundary: the reference has no tests, fixtures or
golden vectors for this path. This oracle is pinned instead by
(1) known-answer tests derived from the reference semantics (tests/test_oracle_kat.py),
(2) an independent differentiator (torch.autograd in float64, tests/test_oracle_autograd.py),
(3) the step-0 loss magnitudes logged in ``{8c,8d,8e}/nohup.out:27`` (statistical check).

The step is split into the same phases the product exposes, so the data-parallel host
logic can be tested against it: ``forward`` -> [all-reduce colsq] -> ``metric`` ->
[all-reduce coldot] -> ``backward`` -> [all-reduce grads] -> ``adam``.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import conv_oracle as CV

L2_EPS = 1e-12  # tf.nn.l2_normalize default epsilon


@dataclasses.dataclass
class OracleConfig:
    image_size: int = 100
    enc: Tuple[int, ...] = (500, 500, 500, 500)
    dec: Tuple[int, int] = (500, 500)
    latent: int = 20
    act: str = "tanh"            # "tanh" (8c family) | "elu" (10b/11a)
    deform_weight: float = 10.0  # 10 (8c) | 100 (11a)
    metric: str = "cosine"       # "cosine" | "sqdiff"
    reciprocal: bool = False     # 9a/10a/11a: distance = 1/raw
    lr: Tuple[float, float] = (1e-4, 1e-6)
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8
    conv: bool = False           # conv-encoder variant (conv_oracle.py)

    @property
    def D(self) -> int:
        return self.image_size * self.image_size


# --------------------------------------------------------------------------- params
def param_shapes(cfg) -> List[Tuple[str, Tuple[int, ...]]]:
    """Variables in creation order, ``11a/vae.py:85-153`` (dead log-sigma decoder last)."""
    D, L = cfg.D, cfg.latent
    out = []
    fan_in = D
    if getattr(cfg, "conv", False):  # the CifarNet tower comes first (encoder variables)
        out += CV.param_shapes()
        fan_in = CV.feat_dim(cfg.image_size)
    for i, e in enumerate(cfg.enc):
        out.append((f"enc_h{i}_W", (fan_in, e)))
        out.append((f"enc_h{i}_b", (e,)))
        fan_in = e
    out += [("enc_out_mean_W", (fan_in, L)), ("enc_out_mean_b", (L,)),
            ("enc_out_log_sigma_W", (fan_in, L)), ("enc_out_log_sigma_b", (L,)),
            ("dec_h1_W", (L, cfg.dec[0])), ("dec_h1_b", (cfg.dec[0],)),
            ("dec_h2_W", (cfg.dec[0], cfg.dec[1])), ("dec_h2_b", (cfg.dec[1],)),
            ("dec_out_mean_W", (cfg.dec[1], D)), ("dec_out_mean_b", (D,)),
            ("dec_out_log_sigma_W", (cfg.dec[1], D)), ("dec_out_log_sigma_b", (D,))]
    return out


DEAD = ("dec_out_log_sigma_W", "dec_out_log_sigma_b")


def trained_names(cfg) -> List[str]:
    return [n for n, _ in param_shapes(cfg) if n not in DEAD]


def encoder_names(cfg) -> List[str]:
    return [n for n in trained_names(cfg) if n.startswith("enc_")]


def xavier_init(rng: np.random.Generator, fan_in: int, fan_out: int, dtype=np.float32):
    """``11a/utils.py:484-491``: U(+-sqrt(6/(fan_in+fan_out)))."""
    hi = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-hi, hi, size=(fan_in, fan_out)).astype(dtype)


def init_params(cfg, seed: int = 0, dtype=np.float32) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    P = {}
    for name, shp in param_shapes(cfg):
        if len(shp) == 2:
            fi, fo = CV.xavier_fans(name, shp)
            hi = np.sqrt(6.0 / (fi + fo))
            P[name] = rng.uniform(-hi, hi, size=shp).astype(dtype)
        else:
            P[name] = np.zeros(shp, dtype)
    return P


# --------------------------------------------------------------------------- ops
def act_fwd(a, kind):
    if kind == "tanh":
        return np.tanh(a)
    if kind == "elu":  # TF: features < 0 ? exp(features) - 1 : features
        return np.where(a < 0, np.exp(np.minimum(a, 0)) - 1, a)
    raise ValueError(kind)


def act_grad(y, g, kind):
    """TF TanhGrad / EluGrad, both written in terms of the activation OUTPUT y."""
    if kind == "tanh":
        return g * (1 - y * y)
    if kind == "elu":
        return np.where(y < 0, g * (y + 1), g)
    raise ValueError(kind)


def split_input(X, cfg):
    """``11a/vae.py:172-185``: reshape [B,H,W,3] + split(axis=3): channel c at (h*W+w)*3+c.
    Contiguous copies, so the matmuls run in BLAS (strided operands fall off the BLAS path)."""
    return tuple(np.ascontiguousarray(X[:, c::3]) for c in range(3))


def encode(P, x, cfg):
    """``get_latent_representation`` ``11a/vae.py:335-367`` without the sampling. With
    ``cfg.conv`` the FC layers read the conv tower's features (hs[0]); the tower's cache is
    returned as the 4th value (None otherwise)."""
    tc = None
    if getattr(cfg, "conv", False):
        x, tc = CV.tower_forward(P, x, cfg.image_size)
    hs = [x]
    h = x
    for i in range(len(cfg.enc)):
        h = act_fwd(h @ P[f"enc_h{i}_W"] + P[f"enc_h{i}_b"], cfg.act)
        hs.append(h)
    mu = h @ P["enc_out_mean_W"] + P["enc_out_mean_b"]
    s = h @ P["enc_out_log_sigma_W"] + P["enc_out_log_sigma_b"]
    return hs, mu, s, tc


def decode(P, z, cfg):
    """``11a/vae.py:227-232``."""
    d1 = act_fwd(z @ P["dec_h1_W"] + P["dec_h1_b"], cfg.act)
    d2 = act_fwd(d1 @ P["dec_h2_W"] + P["dec_h2_b"], cfg.act)
    u = d2 @ P["dec_out_mean_W"] + P["dec_out_mean_b"]
    y = 1.0 / (1.0 + np.exp(-u))
    return d1, d2, u, y


def bce_rows(y, x):
    """R_b = -sum log(y^x (1-y)^(1-x)), TF pow(0,0)=1 semantics, no epsilon (``11a/vae.py:266-269``)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = np.where(x != 0, x * np.log(y), 0.0)
        t2 = np.where(x != 1, (1 - x) * np.log(1 - y), 0.0)
    return -(t1 + t2).sum(axis=1)


# --------------------------------------------------------------------------- phases
def forward(P, X, eps, cfg, dtype=np.float64):
    """Forward pass over the LOCAL rows. Returns a cache; cache['colsq'] holds the
    per-column sums over local rows of z_lock^2 and z_key^2 ([2, L]) which the
    cosine metric needs summed over the GLOBAL batch."""
    X = np.asarray(X, dtype)
    eps = np.asarray(eps, dtype)
    P = {k: np.asarray(v, dtype) for k, v in P.items()}
    xl, xr, xk = split_input(X, cfg)
    c = {"P": P, "xl": xl, "eps": eps}
    for tag, x, e in (("l", xl, eps[0]), ("r", xr, eps[1]), ("k", xk, eps[2])):
        hs, mu, s, tc = encode(P, x, cfg)
        sig = np.sqrt(np.exp(s))                       # tf.sqrt(tf.exp(s)), 11a/vae.py:376
        z = mu + sig * e
        c.update({f"tc_{tag}": tc, f"hs_{tag}": hs, f"mu_{tag}": mu, f"s_{tag}": s, f"sig_{tag}": sig, f"z_{tag}": z})
    d1, d2, u, y = decode(P, c["z_l"], cfg)
    c.update(d1=d1, d2=d2, u=u, y=y)
    c["R"] = bce_rows(y, xl)                                                   # 11a/vae.py:266-269
    c["K"] = -0.5 * (1 + c["s_l"] - c["mu_l"] ** 2 - np.exp(c["s_l"])).sum(1)  # :281-284
    c["F"] = cfg.deform_weight * ((c["z_l"] - c["z_r"]) ** 2).sum(1)          # :293-294
    c["colsq"] = np.stack([(c["z_l"] ** 2).sum(0), (c["z_k"] ** 2).sum(0)])
    return c


def metric(c, areas, cfg, B_global: int, colsq_global=None):
    """Distance (``11a/vae.py:306-311``, ``cosine_distance`` ``:444-458``) and the metric
    loss ``training_loss`` (``:313``) over the local rows; fills the per-row gradient
    scale ``draw`` and (cosine) the local column sums ``coldot`` = sum_b draw_b nl nk."""
    areas = np.asarray(areas, c["z_l"].dtype)
    zl, zk = c["z_l"], c["z_k"]
    if cfg.metric == "cosine":
        cs = c["colsq"] if colsq_global is None else np.asarray(colsq_global, zl.dtype)
        rl = 1.0 / np.sqrt(np.maximum(cs[0], L2_EPS))
        rk = 1.0 / np.sqrt(np.maximum(cs[1], L2_EPS))
        nl, nk = zl * rl, zk * rk
        raw = (nl * nk).sum(1)
        c.update(rl=rl, rk=rk, nl=nl, nk=nk, cs=cs)
    elif cfg.metric == "sqdiff":
        raw = ((zl - zk) ** 2).sum(1)
    else:
        raw = None
        raise ValueError(cfg.metric)
    dist = 1.0 / raw if cfg.reciprocal else raw
    T = (dist - areas) ** 2
    g = 2.0 * (dist - areas) / B_global
    draw = -g * dist * dist if cfg.reciprocal else g      # tf.reciprocal grad: -dy * y^2
    c.update(raw=raw, dist=dist, T=T, draw=draw)
    if cfg.metric == "cosine":
        c["coldot"] = (draw[:, None] * c["nl"] * c["nk"]).sum(0)
    return c


def loss_sums(c, B_global: int):
    """Local contributions to (cost, training_loss, r_l, l_l, d_l) — global means after a sum."""
    inv = 1.0 / B_global
    R, K, F, T = c["R"].sum() * inv, c["K"].sum() * inv, c["F"].sum() * inv, c["T"].sum() * inv
    return np.array([R + K + F, T, R, K, F])


def _enc_backward(P, hs, dmu, ds, cfg, acc: Dict[str, np.ndarray], mag: bool = False, tc=None):
    A = np.abs if mag else (lambda v: v)
    h = A(hs[-1])
    for nm, d in (("enc_out_mean", dmu), ("enc_out_log_sigma", ds)):
        acc[nm + "_W"] = acc.get(nm + "_W", 0) + h.T @ d
        acc[nm + "_b"] = acc.get(nm + "_b", 0) + d.sum(0)
    dh = dmu @ A(P["enc_out_mean_W"]).T + ds @ A(P["enc_out_log_sigma_W"]).T
    for i in reversed(range(len(cfg.enc))):
        dz = A(act_grad(hs[i + 1], dh, cfg.act))
        acc[f"enc_h{i}_W"] = acc.get(f"enc_h{i}_W", 0) + A(hs[i]).T @ dz
        acc[f"enc_h{i}_b"] = acc.get(f"enc_h{i}_b", 0) + dz.sum(0)
        if i > 0 or tc is not None:
            dh = dz @ A(P[f"enc_h{i}_W"]).T
    if tc is not None:  # through the conv tower (dh = dL/d features)
        CV.tower_backward(P, tc, dh, acc, mag)
    return acc


def backward(c, cfg, B_global: int, coldot_global=None, magnitude: bool = False):
    """Hand-derived gradients of ``cost`` (g1: every trained variable) and of
    ``training_loss`` (g2: encoder variables only), SURVEY.md Appendix A.2/A.3.

    ``magnitude=True`` returns instead the same sums taken over ABSOLUTE values of every
    term (the scale sum|terms| of the standard floating-point error bound). Tests use it as
    the yardstick for gradients whose exact value cancels (e.g. the squared-difference
    g2 bias: lock and key contributions are equal and opposite)."""
    A = np.abs if magnitude else (lambda v: v)
    P = {k: A(v) for k, v in c["P"].items()}
    inv = 1.0 / B_global
    w = cfg.deform_weight
    g1: Dict[str, np.ndarray] = {}
    # decoder + reconstruction: dcost/du = (y - x)/B  (sigmoid-BCE, exact for x in [0,1])
    dU = A(c["y"] - c["xl"]) * inv
    d1, d2, zl_ = A(c["d1"]), A(c["d2"]), A(c["z_l"])
    g1["dec_out_mean_W"] = d2.T @ dU
    g1["dec_out_mean_b"] = dU.sum(0)
    dz2 = A(act_grad(c["d2"], dU @ P["dec_out_mean_W"].T, cfg.act))
    g1["dec_h2_W"] = d1.T @ dz2
    g1["dec_h2_b"] = dz2.sum(0)
    dz1 = A(act_grad(c["d1"], dz2 @ P["dec_h2_W"].T, cfg.act))
    g1["dec_h1_W"] = zl_.T @ dz1
    g1["dec_h1_b"] = dz1.sum(0)
    dzl_dec = dz1 @ P["dec_h1_W"].T
    # deformation + KL + reparameterisation (g1)
    diff = A(c["z_l"] - c["z_r"])
    el, er, ek = A(c["eps"][0]), A(c["eps"][1]), A(c["eps"][2])
    if magnitude:
        dzl1 = dzl_dec + 2 * w * diff * inv
        dzr1 = 2 * w * diff * inv
        dmu_l1 = dzl1 + np.abs(c["mu_l"]) * inv
        ds_l1 = 0.5 * dzl1 * el * c["sig_l"] + 0.5 * (np.exp(c["s_l"]) + 1) * inv
    else:
        dzl1 = dzl_dec + 2 * w * diff * inv
        dzr1 = -2 * w * diff * inv
        dmu_l1 = dzl1 + c["mu_l"] * inv
        ds_l1 = 0.5 * dzl1 * el * c["sig_l"] + 0.5 * (np.exp(c["s_l"]) - 1) * inv
    dmu_r1, ds_r1 = A(dzr1), A(0.5 * dzr1 * er * c["sig_r"])
    _enc_backward(P, c["hs_l"], A(dmu_l1), A(ds_l1), cfg, g1, magnitude, c.get("tc_l"))
    _enc_backward(P, c["hs_r"], dmu_r1, ds_r1, cfg, g1, magnitude, c.get("tc_r"))
    # metric (g2)
    draw = A(c["draw"][:, None])
    if cfg.metric == "sqdiff":
        dzl2 = 2 * draw * A(c["z_l"] - c["z_k"])
        dzk2 = dzl2 if magnitude else -dzl2
    else:
        cd = c["coldot"] if coldot_global is None else np.asarray(coldot_global, dzl_dec.dtype)
        ml = (c["cs"][0] >= L2_EPS).astype(dzl_dec.dtype)   # tf.maximum grad routes to ss only when ss >= eps
        mk = (c["cs"][1] >= L2_EPS).astype(dzl_dec.dtype)
        if magnitude:
            cdm = (draw * np.abs(c["nl"] * c["nk"])).sum(0)
            dzl2 = c["rl"] * (draw * np.abs(c["nk"]) + np.abs(c["nl"]) * cdm * ml)
            dzk2 = c["rk"] * (draw * np.abs(c["nl"]) + np.abs(c["nk"]) * cdm * mk)
        else:
            dzl2 = c["rl"] * (draw * c["nk"] - c["nl"] * cd * ml)
            dzk2 = c["rk"] * (draw * c["nl"] - c["nk"] * cd * mk)
    g2: Dict[str, np.ndarray] = {}
    _enc_backward(P, c["hs_l"], dzl2, A(0.5 * dzl2 * el * c["sig_l"]), cfg, g2, magnitude, c.get("tc_l"))
    _enc_backward(P, c["hs_k"], dzk2, A(0.5 * dzk2 * ek * c["sig_k"]), cfg, g2, magnitude, c.get("tc_k"))
    return g1, g2


# --------------------------------------------------------------------------- Adam
def adam_init(cfg, P, dtype=None) -> dict:
    """Slots in ``dtype`` (default: float64 for float64 parameters, else float32)."""
    f32 = np.float32
    st = {"t": 0}
    for o, names in ((1, trained_names(cfg)), (2, encoder_names(cfg))):
        dt = dtype or (np.float64 if P[names[0]].dtype == np.float64 else np.float32)
        st[f"m{o}"] = {n: np.zeros_like(P[n], dtype=dt) for n in names}
        st[f"v{o}"] = {n: np.zeros_like(P[n], dtype=dt) for n in names}
        st[f"b1p{o}"] = f32(cfg.beta1)
        st[f"b2p{o}"] = f32(cfg.beta2)
    return st


def adam_lr_t(lr, b1p, b2p):
    """TF ApplyAdam's lr_t, evaluated in fp32 exactly as the TF fp32 kernel does."""
    f32 = np.float32
    return f32(f32(f32(lr) * np.sqrt(f32(1) - f32(b2p), dtype=f32)) / f32(f32(1) - f32(b1p)))


def adam(P, g1, g2, st, cfg, dtype=np.float64):
    """Both ``AdamOptimizer.minimize`` ops of one ``partial_fit`` (``11a/vae.py:320-327``)."""
    P = {k: np.asarray(v, dtype).copy() for k, v in P.items()}
    b1, b2, e = cfg.beta1, cfg.beta2, cfg.epsilon
    for o, g in ((1, g1), (2, g2)):
        lr_t = float(adam_lr_t(cfg.lr[o - 1], st[f"b1p{o}"], st[f"b2p{o}"]))
        for n, gn in g.items():
            sd = st[f"m{o}"][n].dtype
            m = st[f"m{o}"][n] = (st[f"m{o}"][n] + (gn - st[f"m{o}"][n]) * (1 - b1)).astype(sd, copy=False)
            v = st[f"v{o}"][n] = (st[f"v{o}"][n] + (gn * gn - st[f"v{o}"][n]) * (1 - b2)).astype(sd, copy=False)
            P[n] = (P[n] - (lr_t * m) / (np.sqrt(v) + e)).astype(dtype, copy=False)
        st[f"b1p{o}"] = np.float32(st[f"b1p{o}"] * np.float32(b1))
        st[f"b2p{o}"] = np.float32(st[f"b2p{o}"] * np.float32(b2))
    st["t"] += 1
    return P, st


# --------------------------------------------------------------------------- step
def train_step(P, st, X, areas, eps, cfg, dtype=np.float64):
    """``partial_fit`` ``11a/vae.py:385-411``: returns pre-update
    (cost, training_loss, r_l, l_l, d_l), distance[B], new params, new Adam state, grads."""
    B = X.shape[0]
    c = forward(P, X, eps, cfg, dtype)
    metric(c, areas, cfg, B)
    losses = loss_sums(c, B)
    g1, g2 = backward(c, cfg, B)
    P_new, st = adam(P, g1, g2, st, cfg, dtype)
    return losses, c["dist"], P_new, st, (g1, g2)


def predictions(P, X, eps, cfg, dtype=np.float64):
    """``get_predictions`` ``11a/vae.py:413-414``: the (sampled) distance."""
    c = forward(P, X, eps, cfg, dtype)
    metric(c, np.zeros(X.shape[0]), cfg, X.shape[0])
    return c["dist"]


def overlap_mse(pred_dist, areas, invert: bool):
    """Eval "overlap-MSE" ``11a/main.py:99-111`` (11a inverts the reciprocal distance)."""
    p = 1.0 / np.asarray(pred_dist, np.float64) if invert else np.asarray(pred_dist, np.float64)
    return float(((p - np.asarray(areas, np.float64)) ** 2).mean())
