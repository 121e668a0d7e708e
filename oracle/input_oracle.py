"""ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement (numpy) of the reference's batch
producer for the hot path (``11a/overlap_input.py:127-261``, ``11a/utils.py:453-464``):

  lock, key   decode_png -> float32 [H, W, 1]                       (``:41-73``)
  rotated     tf.contrib.image.rotate(lock, angle), NEAREST, zero fill (``11a/utils.py:462``)
  example     concat([lock, rotated, key], axis=2)                   (``:201``)
  batch       / 255.0                                                (``:113-115``)
              reshape [B, H*W*3]                                     (``:117-119``)

``tf.contrib.image.rotate`` (TF 1.x) = ``angles_to_projective_transforms`` +
``ImageProjectiveTransform``: output pixel (x, y) samples the input at
  x' = cos*x - sin*y + x_off,  y' = sin*x + cos*y + y_off,
  x_off = ((W-1) - (cos*(W-1) - sin*(H-1))) / 2,  y_off = ((H-1) - (sin*(W-1) + cos*(H-1))) / 2
in float32, NEAREST = round half away from zero, outside [0, W-1] x [0, H-1] -> 0.
The per-example coefficients (cos, sin, x_off, y_off) are computed on the host in float32
(``rotation_coefficients``); given them, the gather is exact integer work, so the HIP kernel
must match this restatement bit for bit. The uniform angle draw (``tf.random_uniform``,
TF Philox) is not reproducible and is an input here.
"""
from __future__ import annotations

import numpy as np


def rotation_coefficients(angles, height: int, width: int) -> np.ndarray:
    """[B] radians -> [B, 4] float32 (cos, sin, x_off, y_off), TF's float32 arithmetic."""
    a = np.asarray(angles, np.float32)
    c = np.cos(a).astype(np.float32)
    s = np.sin(a).astype(np.float32)
    w1 = np.float32(width - 1)
    h1 = np.float32(height - 1)
    xo = ((w1 - (c * w1 - s * h1)) / np.float32(2.0)).astype(np.float32)
    yo = ((h1 - (s * w1 + c * h1)) / np.float32(2.0)).astype(np.float32)
    return np.stack([c, s, xo, yo], axis=1).astype(np.float32)


def _round_half_away(v):
    """C ``roundf`` (half away from zero), exactly: v - trunc(v) is exact in float."""
    t = np.trunc(v)
    return np.where(np.abs(v - t) >= np.float32(0.5), t + np.sign(v), t).astype(np.float32)


def rotate_nearest(img: np.ndarray, coef: np.ndarray) -> np.ndarray:
    """One image [H, W] with coefficients [4] -> rotated [H, W] (same dtype)."""
    h, w = img.shape
    c, s, xo, yo = (np.float32(v) for v in coef)
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing="ij")
    # float32, no fused multiply-add: ((c*x) - (s*y)) + x_off
    xin = ((c * xs).astype(np.float32) - (s * ys).astype(np.float32)).astype(np.float32) + xo
    yin = ((s * xs).astype(np.float32) + (c * ys).astype(np.float32)).astype(np.float32) + yo
    xr = _round_half_away(xin)
    yr = _round_half_away(yin)
    inside = (xr >= 0) & (xr <= w - 1) & (yr >= 0) & (yr <= h - 1)
    out = np.zeros_like(img)
    out[inside] = img[yr[inside].astype(np.int64), xr[inside].astype(np.int64)]
    return out


def make_batch(locks: np.ndarray, keys: np.ndarray, idx, coef: np.ndarray,
               scale_div: float = 255.0) -> np.ndarray:
    """locks/keys uint8 [n, H, W]; idx [B]; coef [B, 4] -> X float32 [B, H*W*3]."""
    idx = np.asarray(idx, np.int64)
    B = len(idx)
    n, h, w = locks.shape
    X = np.empty((B, h * w * 3), np.float32)
    d = np.float32(scale_div)
    for b in range(B):
        lk = locks[idx[b]].astype(np.float32)
        ky = keys[idx[b]].astype(np.float32)
        rt = rotate_nearest(lk, coef[b])
        X[b] = (np.stack([lk, rt, ky], axis=2) / d).reshape(-1)
    return X
