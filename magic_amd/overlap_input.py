"""Batch producer with the reference's layout (``11a/overlap_input.py:76-261``), assembled on
the GPU by the HIP kernel ``mvae_make_batch``.

``inputs(normalize=True, reshape=True, rotation=True)`` returns a ``BatchStream``; each
``next(stream)`` (the reference's ``sess.run([images_batch, labels_batch])``) yields

  images: float32 [B, H*W*3] — per pixel (h*W+w) three channels (lock, rotated lock, key),
          ``tf.concat([lock, rotated_lock, key], axis=2)`` (``:201``) reshaped (``:117-119``),
          divided by 255 (``:113-115``);
  labels: float32 [B] overlap areas.

Sources: a directory or .zip of ``{N}_L.png`` / ``{N}_K.png`` pairs with an areas array
(``.npy``), or the synthetic shape generator (``synthetic=True``; BASELINE.json asks for
100x100 synthetic pairs). The rotated lock is the lock rotated by U[0, 2pi) about the image
centre with nearest-neighbour sampling and zero fill, the ``tf.contrib.image.rotate``
semantics (``11a/utils.py:453-464``); decoded images live in HBM as uint8 tables and each
batch is gathered, rotated, interleaved and normalised by one HIP kernel.
"""
from __future__ import annotations

import io
import math
import os
import zipfile
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .constants import FLAGS


def rotation_coefficients(angles, height: int, width: int) -> np.ndarray:
    """Per-example ``tf.contrib.image.rotate`` coefficients (cos, sin, x_off, y_off), float32
    as TF's ``angles_to_projective_transforms`` computes them; [B] radians -> [B, 4]."""
    a = np.asarray(angles, np.float32)
    c = np.cos(a).astype(np.float32)
    s = np.sin(a).astype(np.float32)
    w1, h1 = np.float32(width - 1), np.float32(height - 1)
    xo = ((w1 - (c * w1 - s * h1)) / np.float32(2.0)).astype(np.float32)
    yo = ((h1 - (s * w1 + c * h1)) / np.float32(2.0)).astype(np.float32)
    return np.ascontiguousarray(np.stack([c, s, xo, yo], axis=1), dtype=np.float32)


def make_batch(locks: torch.Tensor, keys: torch.Tensor, idx: torch.Tensor, coef: torch.Tensor,
               out: Optional[torch.Tensor] = None, normalize: bool = True) -> torch.Tensor:
    """HIP batch producer (``mvae_make_batch``): uint8 device tables [n, H, W], idx int32 [B],
    coef float32 [B, 4] -> X float32 [B, H*W*3] = per pixel (lock, rotated lock, key) / 255
    (``normalize=False``: the raw 0..255 values, ``11a/overlap_input.py:113-115``)."""
    from . import _lib
    lib = _lib.load()
    n, h, w = locks.shape
    B = idx.shape[0]
    for t, dt in ((locks, torch.uint8), (keys, torch.uint8), (idx, torch.int32), (coef, torch.float32)):
        if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
            raise ValueError("make_batch: device tensors (uint8 tables, int32 idx, float32 coef) expected")
    out = out if out is not None else torch.empty(B, 3 * h * w, device=locks.device)
    rc = lib.mvae_make_batch(locks.data_ptr(), keys.data_ptr(), h, w, idx.data_ptr(), coef.data_ptr(),
                             B, 255.0 if normalize else 1.0, out.data_ptr(),
                             torch.cuda.current_stream(locks.device).cuda_stream)
    _lib.check(lib, None, rc)
    return out


def random_shapes(n: int, size: int, gen: torch.Generator, device) -> torch.Tensor:
    """Binary images {0,1} of 1-3 random filled ellipses/rectangles (foreground ~3-15%, like
    the reference's overlap_micro PNGs), [n, size, size] float32."""
    dev = torch.device(device)
    ys, xs = torch.meshgrid(torch.arange(size, dtype=torch.float32),
                            torch.arange(size, dtype=torch.float32), indexing="ij")
    ys, xs = ys.to(dev), xs.to(dev)
    img = torch.zeros(n, size, size, device=dev)
    for _ in range(3):
        u = torch.rand(n, 7, generator=gen).to(dev)
        cx, cy = (0.25 + 0.5 * u[:, 0]) * size, (0.25 + 0.5 * u[:, 1]) * size
        ra, rb = (0.05 + 0.12 * u[:, 2]) * size, (0.05 + 0.12 * u[:, 3]) * size
        th = u[:, 4] * math.pi
        keep = (u[:, 5] < 0.7).float().reshape(n, 1, 1)
        kind = (u[:, 6] < 0.5).reshape(n, 1, 1)
        dx = xs[None] - cx.reshape(n, 1, 1)
        dy = ys[None] - cy.reshape(n, 1, 1)
        ct, st = torch.cos(th).reshape(n, 1, 1), torch.sin(th).reshape(n, 1, 1)
        px, py = ct * dx + st * dy, -st * dx + ct * dy
        ell = (px / ra.reshape(n, 1, 1)) ** 2 + (py / rb.reshape(n, 1, 1)) ** 2 <= 1.0
        rect = (px.abs() <= ra.reshape(n, 1, 1)) & (py.abs() <= rb.reshape(n, 1, 1))
        m = torch.where(kind, ell, rect).float() * keep
        img = torch.maximum(img, m)
    return img


# areas resampled from the reference's 2a/OVERLAP_AREAS empirical
# distribution (range 296-6426). magic_amd/data/overlap_areas.npy holds the 2000 values (package
# data, extracted as text without unpickling by tests/golden/make_golden.py); a log-normal fit is
# the fallback when the table is absent.
_AREAS_FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "overlap_areas.npy")


def area_distribution() -> np.ndarray:
    if os.path.exists(_AREAS_FIXTURE):
        return np.load(_AREAS_FIXTURE).astype(np.float32)
    rng = np.random.default_rng(1)
    return np.clip(np.exp(rng.normal(7.4, 0.62, 2000)), 296, 6426).round().astype(np.float32)


def synthetic_batch(batch: int, image_size: int, seed: int = 1, device="cuda",
                    dtype=torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
    """One seeded synthetic batch (X [B, 3D] in {0,1}, areas [B]) through the HIP producer."""
    gen = torch.Generator().manual_seed(seed)
    dev = torch.device(device)
    lock = (random_shapes(batch, image_size, gen, device) * 255).to(torch.uint8).contiguous()
    key = (random_shapes(batch, image_size, gen, device) * 255).to(torch.uint8).contiguous()
    ang = torch.rand(batch, generator=gen).numpy() * (2 * math.pi)
    coef = torch.from_numpy(rotation_coefficients(ang, image_size, image_size)).to(dev)
    idx = torch.arange(batch, dtype=torch.int32, device=dev)
    x = make_batch(lock, key, idx, coef).to(dtype)
    dist = area_distribution()
    sel = torch.randint(0, len(dist), (batch,), generator=gen).numpy()
    areas = torch.from_numpy(dist[sel]).to(dev)
    return x, areas


class PairSource:
    """Lock/key PNG pairs from a directory or a zip (``{N}_L.png``/``{N}_K.png``)."""

    def __init__(self, path: str, areas: Optional[np.ndarray] = None, limit: Optional[int] = None):
        from PIL import Image
        self.locks, self.keys = [], []
        if path.endswith(".zip"):
            z = zipfile.ZipFile(path)
            names = set(z.namelist())
            prefix = os.path.commonprefix([n for n in names if n.endswith("_L.png")]).rsplit("/", 1)
            prefix = prefix[0] + "/" if len(prefix) == 2 else ""
            read = lambda n: z.read(prefix + n)  # noqa: E731
            exists = lambda n: (prefix + n) in names  # noqa: E731
        else:
            read = lambda n: open(os.path.join(path, n), "rb").read()  # noqa: E731
            exists = lambda n: os.path.exists(os.path.join(path, n))  # noqa: E731
        i = 0
        while exists(f"{i}_L.png") and exists(f"{i}_K.png") and (limit is None or i < limit):
            for lst, nm in ((self.locks, f"{i}_L.png"), (self.keys, f"{i}_K.png")):
                a = np.array(Image.open(io.BytesIO(read(nm))).convert("L"), dtype=np.float32)
                lst.append(a)
            i += 1
        if i == 0:
            raise ValueError(f"no {{N}}_L.png/{{N}}_K.png pairs under {path}")
        self.locks = np.stack(self.locks)
        self.keys = np.stack(self.keys)
        if areas is None:
            areas = area_distribution()
        self.areas = np.asarray(areas, np.float32)[:i]

    @classmethod
    def from_packed(cls, npz_path: str, areas: Optional[np.ndarray] = None, limit: Optional[int] = None):
        """Pairs from a packed-bit archive (``lock_bits``, ``key_bits``, ``shape``) such as
        tests/golden/overlap_micro.npz, the reference's overlap_micro.zip images."""
        z = np.load(npz_path)
        n, h, w = (int(v) for v in z["shape"])
        n = n if limit is None else min(n, limit)
        self = cls.__new__(cls)
        self.locks = np.unpackbits(z["lock_bits"][:n], axis=-1)[..., :w].astype(np.float32) * 255.0
        self.keys = np.unpackbits(z["key_bits"][:n], axis=-1)[..., :w].astype(np.float32) * 255.0
        self.areas = np.asarray(areas if areas is not None else area_distribution(), np.float32)[:n]
        return self

    def __len__(self):
        return len(self.locks)


class BatchStream:
    """Shuffled epochs over a source (``slice_input_producer(shuffle=True)`` +
    ``shuffle_batch``), a uniform [0, 2pi) rotation per example, /255 normalisation — the
    per-batch assembly runs in the HIP batch producer (``mvae_make_batch``)."""

    def __init__(self, batch: int, image_size: int, source: Optional[PairSource] = None,
                 normalize: bool = True, seed: int = 1, device="cuda", synthetic_pool: int = 960,
                 reshape: bool = True, fp16: bool = False):
        self.batch, self.size = batch, image_size
        self.normalize, self.reshape, self.fp16 = normalize, reshape, fp16
        self.device = torch.device(device)
        self.rng = np.random.default_rng(seed)
        if source is None:  # synthetic pool of pairs, re-rotated every draw
            g = torch.Generator().manual_seed(seed + 1000)
            lock = random_shapes(synthetic_pool, image_size, g, "cpu") * 255.0
            key = random_shapes(synthetic_pool, image_size, g, "cpu") * 255.0
            dist = area_distribution()
            idx = torch.randint(0, len(dist), (synthetic_pool,), generator=g).numpy()
            locks, keys, self.areas = lock, key, torch.from_numpy(dist[idx])
        else:
            if source.locks.shape[1] != image_size:
                raise ValueError(f"images are {source.locks.shape[1]}px, expected {image_size}")
            locks, keys = torch.from_numpy(source.locks), torch.from_numpy(source.keys)
            self.areas = torch.from_numpy(source.areas)
        self.locks = locks.round().clamp(0, 255).to(torch.uint8).contiguous().to(self.device)
        self.keys = keys.round().clamp(0, 255).to(torch.uint8).contiguous().to(self.device)
        self.areas = self.areas.float().to(self.device)
        self._perm = np.empty(0, dtype=np.int64)
        self._pos = 0

    def _take(self, n):
        out = []
        while n > 0:
            if self._pos >= len(self._perm):
                self._perm = self.rng.permutation(len(self.locks))
                self._pos = 0
            k = min(n, len(self._perm) - self._pos)
            out.append(self._perm[self._pos:self._pos + k])
            self._pos += k
            n -= k
        return np.concatenate(out)

    def __iter__(self) -> Iterator:
        return self

    def __next__(self):
        idx = self._take(self.batch)
        ang = self.rng.uniform(0.0, 2 * math.pi, self.batch)
        coef = torch.from_numpy(rotation_coefficients(ang, self.size, self.size)).to(self.device)
        idx_t = torch.from_numpy(idx.astype(np.int32)).to(self.device)
        x = make_batch(self.locks, self.keys, idx_t, coef, normalize=self.normalize)
        a = self.areas[idx_t.long()]
        if not self.reshape:  # [B, H, W, 3] (11a/overlap_input.py:117-119 not applied)
            x = x.view(self.batch, self.size, self.size, 3)
        if self.fp16:  # FLAGS.USE_FP16 casts images and labels (11a/overlap_input.py:109-111)
            x, a = x.half(), a.half()
        return x, a


def inputs(normalize: bool = False, reshape: bool = False, rotation: bool = False,
           batch_size: Optional[int] = None, image_size: Optional[int] = None,
           data_dir: Optional[str] = None, device="cuda", seed: int = 1) -> BatchStream:
    """``11a/overlap_input.py:76-122``: images [B, H*W*3] (``reshape=True``) or [B, H, W, 3],
    divided by 255 when ``normalize``, cast to float16 with labels when ``FLAGS.USE_FP16``;
    ``rotation=False`` raises as in the reference (``:95-96``)."""
    if not rotation:
        raise ValueError("Rotation has to be True.")
    size = image_size or FLAGS.IMAGE_SIZE
    bs = batch_size or FLAGS.BATCH_SIZE
    d = data_dir if data_dir is not None else FLAGS.DATA_DIR
    src = None
    if d:
        lim = FLAGS.NUM_EXAMPLES_TO_LOAD_INTO_QUEUE
        src = PairSource.from_packed(d, limit=lim) if d.endswith(".npz") else PairSource(d, limit=lim)
    return BatchStream(bs, size, src, normalize=normalize, seed=seed, device=device, reshape=reshape,
                       fp16=bool(getattr(FLAGS, "USE_FP16", False)))
