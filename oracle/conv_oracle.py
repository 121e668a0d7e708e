"""ORACLE — TEST INFRASTRUCTURE ONLY. Never imported by the product (``magic_amd``).

CPU restatement (numpy, float64) of the conv-encoder variant of the metric-VAE encoder
(BASELINE config 5). PARITY UNPINNED BY NATURE: the reference has no
conv VAE. The tower is the reference's only conv net, the CifarNet tower of the siamese
overlap regressor, ``6b/net.py:50-60``:

    conv1 5x5x64 (SAME, ReLU)  ->  max_pool 2x2/2 (VALID)  ->  lrn(4, 1.0, 0.001/9, 0.75)
    conv2 5x5x64 (SAME, ReLU)  ->  lrn(4, 1.0, 0.001/9, 0.75)  ->  max_pool 2x2/2  ->  flatten

``slim.conv2d`` defaults (``6b/net.py:50,55`` are called without the arg scope): ReLU,
xavier-uniform weights over fans (k*k*c_in, k*k*c_out), zero biases. ``slim.flatten`` of the
NHWC [N, S/4, S/4, 64] map gives feature index (h*W4 + w)*64 + c. The flat features feed the
VAE's fully connected encoder (``11a/vae.py:335-367``) in place of the raw pixels; the three
encoder passes (lock, rotated lock, key) share the tower's weights as they share the FC
weights.

TF1 op semantics restated:
  - ``tf.nn.lrn``: s_c = bias + alpha * sum_{|j-c|<=r} a_j^2 (window clipped at the channel
    ends), out_c = a_c * s_c^-beta; LRNGrad: da_j = g_j s_j^-beta
    - 2 alpha beta a_j sum_{|c-j|<=r} g_c a_c s_c^(-beta-1);
  - ``max_pool`` gradient: to the FIRST maximum of the window in row-major order (TF's
    MaxPoolGrad keeps the first position on ties: binary images make exact ties common);
  - ``ReluGrad``: g * (y > 0).
Weight layout: W[(ky*5 + kx)*c_in + ci, co] (TF HWIO flattened), as the product stores it.
"""
from __future__ import annotations

from typing import Callable, Dict

import numpy as np

K = 5            # conv kernel size
C = 64           # channels of both conv layers (6b/net.py:50,55)
LRN_R, LRN_BIAS, LRN_ALPHA, LRN_BETA = 4, 1.0, 0.001 / 9.0, 0.75   # 6b/net.py:54,57


def feat_dim(image_size: int) -> int:
    return (image_size // 2 // 2) ** 2 * C


def param_shapes():
    return [("enc_conv1_W", (K * K, C)), ("enc_conv1_b", (C,)),
            ("enc_conv2_W", (K * K * C, C)), ("enc_conv2_b", (C,))]


def xavier_fans(name: str, shape):
    """(fan_in, fan_out) of slim's xavier initializer: a conv kernel counts its receptive
    field on both sides (k*k*c_in, k*k*c_out)."""
    if name.startswith("enc_conv"):
        return shape[0], K * K * shape[1]
    return shape


def im2col(x):
    """x [N,H,W,Ci] -> [N,H,W,25*Ci] with column (ky*5+kx)*Ci + ci, SAME zero padding."""
    N, H, W, Ci = x.shape
    p = K // 2
    xp = np.pad(x, ((0, 0), (p, p), (p, p), (0, 0)))
    cols = np.stack([xp[:, ky:ky + H, kx:kx + W, :] for ky in range(K) for kx in range(K)], axis=3)
    return cols.reshape(N, H, W, K * K * Ci)


def conv(x, W, b):
    return im2col(x) @ W + b


def rot_weights(W, ci: int):
    """SAME-conv data gradient as a conv: Wr[(t', co), ci] = W[(24 - t', ci), co]."""
    co = W.shape[1]
    return W.reshape(K * K, ci, co)[::-1].transpose(0, 2, 1).reshape(K * K * co, ci)


def maxpool(a):
    """2x2 stride 2 VALID; returns (p, arg) with arg = dy*2 + dx of the first maximum."""
    N, H, W, Ch = a.shape
    H2, W2 = H // 2, W // 2
    v = a[:, :2 * H2, :2 * W2].reshape(N, H2, 2, W2, 2, Ch).transpose(0, 1, 3, 2, 4, 5)
    v = v.reshape(N, H2, W2, 4, Ch)
    arg = v.argmax(axis=3)                           # first occurrence on ties
    p = np.take_along_axis(v, arg[:, :, :, None, :], 3)[:, :, :, 0]
    return p, arg


def unpool(g, arg, shape):
    """MaxPoolGrad: g [N,H2,W2,C] to the argmax position of each window; zeros elsewhere."""
    N, H, W, Ch = shape
    H2, W2 = g.shape[1], g.shape[2]
    v = np.zeros((N, H2, W2, 4, Ch), g.dtype)
    np.put_along_axis(v, arg[:, :, :, None, :], g[:, :, :, None, :], 3)
    v = v.reshape(N, H2, W2, 2, 2, Ch).transpose(0, 1, 3, 2, 4, 5).reshape(N, 2 * H2, 2 * W2, Ch)
    out = np.zeros(shape, g.dtype)
    out[:, :2 * H2, :2 * W2] = v
    return out


def _window_sum(v):
    """sum over channels j with |j - c| <= r (clipped), last axis."""
    cs = np.concatenate([np.zeros(v.shape[:-1] + (1,), v.dtype), np.cumsum(v, axis=-1)], axis=-1)
    Ch = v.shape[-1]
    hi = np.minimum(np.arange(Ch) + LRN_R + 1, Ch)
    lo = np.maximum(np.arange(Ch) - LRN_R, 0)
    return cs[..., hi] - cs[..., lo]


def lrn_scale(a):
    return LRN_BIAS + LRN_ALPHA * _window_sum(a * a)


def lrn(a):
    return a * lrn_scale(a) ** -LRN_BETA


def lrn_bwd(a, g, A: Callable = lambda v: v):
    """LRNGrad of out = lrn(a) w.r.t. a, given dout = g. A = abs: the sum-of-|terms| bound."""
    s = lrn_scale(a)
    inner = _window_sum(A(g * a * s ** (-LRN_BETA - 1)))
    t2 = 2 * LRN_ALPHA * LRN_BETA * A(a) * inner
    return A(g) * s ** -LRN_BETA + (t2 if A is np.abs else -t2)


def tower_forward(P, x, S: int):
    """x [N, S*S] (one image channel per row) -> (features [N, F], cache)."""
    N = x.shape[0]
    x4 = x.reshape(N, S, S, 1)
    a1 = np.maximum(conv(x4, P["enc_conv1_W"], P["enc_conv1_b"]), 0)
    p1, arg1 = maxpool(a1)
    n1 = lrn(p1)
    a2 = np.maximum(conv(n1, P["enc_conv2_W"], P["enc_conv2_b"]), 0)
    n2 = lrn(a2)
    p2, arg2 = maxpool(n2)
    cache = dict(x4=x4, a1=a1, p1=p1, arg1=arg1, n1=n1, a2=a2, arg2=arg2)
    return p2.reshape(N, -1), cache


def tower_backward(P, cache, df, acc: Dict[str, np.ndarray], magnitude: bool = False):
    """Accumulate the tower's weight gradients into ``acc`` given dL/d(features)."""
    A = np.abs if magnitude else (lambda v: v)
    a2, n1, a1 = cache["a2"], cache["n1"], cache["a1"]
    dn2 = unpool(df.reshape(a2.shape[0], a2.shape[1] // 2, a2.shape[2] // 2, C), cache["arg2"], a2.shape)
    da2 = lrn_bwd(a2, dn2, A) * (a2 > 0)
    N, H1, W1, _ = a2.shape
    acc["enc_conv2_W"] = acc.get("enc_conv2_W", 0) + A(im2col(n1)).reshape(-1, K * K * C).T @ da2.reshape(-1, C)
    acc["enc_conv2_b"] = acc.get("enc_conv2_b", 0) + da2.sum((0, 1, 2))
    dn1 = im2col(da2) @ rot_weights(A(P["enc_conv2_W"]), C)
    dp1 = lrn_bwd(cache["p1"], dn1, A)
    da1 = unpool(dp1, cache["arg1"], a1.shape) * (a1 > 0)
    acc["enc_conv1_W"] = acc.get("enc_conv1_W", 0) + A(im2col(cache["x4"])).reshape(-1, K * K).T @ da1.reshape(-1, C)
    acc["enc_conv1_b"] = acc.get("enc_conv1_b", 0) + da1.sum((0, 1, 2))
    return acc
