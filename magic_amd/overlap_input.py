"""Batch producer with the reference's layout (``11a/overlap_input.py:76-261``).

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
semantics (``11a/utils.py:453-464``). Rotation and assembly run as torch ops on the
stream's device (input plumbing, outside the timed training step).
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


def rotate_nearest(img: torch.Tensor, angle: torch.Tensor) -> torch.Tensor:
    """``tf.contrib.image.rotate(images, angles)`` (NEAREST, zero fill) for img [N, H, W].

    Output pixel (x, y) samples input (x', y') = R(angle)·(x, y) + offset with
    R = [[cos, -sin], [sin, cos]], offset so the centre ((W-1)/2, (H-1)/2) is fixed;
    nearest = round half away from zero."""
    n, h, w = img.shape
    dev = img.device
    a = angle.to(dev, torch.float32).reshape(n, 1, 1)
    c, s = torch.cos(a), torch.sin(a)
    xo = ((w - 1) - (c * (w - 1) - s * (h - 1))) / 2.0
    yo = ((h - 1) - (s * (w - 1) + c * (h - 1))) / 2.0
    ys, xs = torch.meshgrid(torch.arange(h, device=dev, dtype=torch.float32),
                            torch.arange(w, device=dev, dtype=torch.float32), indexing="ij")
    xin = c * xs - s * ys + xo
    yin = s * xs + c * ys + yo
    xr = torch.sign(xin) * torch.floor(torch.abs(xin) + 0.5)
    yr = torch.sign(yin) * torch.floor(torch.abs(yin) + 0.5)
    inside = (xr >= 0) & (xr <= w - 1) & (yr >= 0) & (yr <= h - 1)
    idx = (yr.clamp(0, h - 1) * w + xr.clamp(0, w - 1)).long()
    out = torch.gather(img.reshape(n, h * w), 1, idx.reshape(n, h * w)).reshape(n, h, w)
    return torch.where(inside, out, torch.zeros((), device=dev, dtype=img.dtype))


def assemble(lock: torch.Tensor, rot: torch.Tensor, key: torch.Tensor) -> torch.Tensor:
    """[N,H,W] x3 -> [N, H*W*3] channel-interleaved (lock, rotated lock, key)."""
    n = lock.shape[0]
    return torch.stack([lock, rot, key], dim=3).reshape(n, -1).contiguous()


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
# distribution (range 296-6426). tests/golden/overlap_areas.npy holds the 2000 values
# (extracted without unpickling, tests/golden/make_golden.py); a log-normal fit is the
# fallback when the fixture is absent.
_AREAS_FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "tests", "golden", "overlap_areas.npy")


def area_distribution() -> np.ndarray:
    if os.path.exists(_AREAS_FIXTURE):
        return np.load(_AREAS_FIXTURE).astype(np.float32)
    rng = np.random.default_rng(1)
    return np.clip(np.exp(rng.normal(7.4, 0.62, 2000)), 296, 6426).round().astype(np.float32)


def synthetic_batch(batch: int, image_size: int, seed: int = 1, device="cuda",
                    dtype=torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
    """One seeded synthetic batch (X [B, 3D] in {0,1}, areas [B])."""
    gen = torch.Generator().manual_seed(seed)
    lock = random_shapes(batch, image_size, gen, device)
    key = random_shapes(batch, image_size, gen, device)
    ang = torch.rand(batch, generator=gen) * (2 * math.pi)
    rot = rotate_nearest(lock, ang)
    x = assemble(lock, rot, key).to(dtype)
    dist = area_distribution()
    idx = torch.randint(0, len(dist), (batch,), generator=gen).numpy()
    areas = torch.from_numpy(dist[idx]).to(device)
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

    def __len__(self):
        return len(self.locks)


class BatchStream:
    """Shuffled epochs over a source (``slice_input_producer(shuffle=True)`` +
    ``shuffle_batch``), random rotation per example, /255 normalisation."""

    def __init__(self, batch: int, image_size: int, source: Optional[PairSource] = None,
                 normalize: bool = True, seed: int = 1, device="cuda", synthetic_pool: int = 960):
        self.batch, self.size, self.normalize = batch, image_size, normalize
        self.device = torch.device(device)
        self.gen = torch.Generator().manual_seed(seed)
        if source is None:  # synthetic pool of pairs, re-rotated every draw
            g = torch.Generator().manual_seed(seed + 1000)
            lock = random_shapes(synthetic_pool, image_size, g, "cpu") * 255.0
            key = random_shapes(synthetic_pool, image_size, g, "cpu") * 255.0
            dist = area_distribution()
            idx = torch.randint(0, len(dist), (synthetic_pool,), generator=g).numpy()
            self.locks, self.keys, self.areas = lock, key, torch.from_numpy(dist[idx])
        else:
            if source.locks.shape[1] != image_size:
                raise ValueError(f"images are {source.locks.shape[1]}px, expected {image_size}")
            self.locks = torch.from_numpy(source.locks)
            self.keys = torch.from_numpy(source.keys)
            self.areas = torch.from_numpy(source.areas)
        self.locks = self.locks.to(self.device)
        self.keys = self.keys.to(self.device)
        self._perm = torch.empty(0, dtype=torch.long)
        self._pos = 0

    def _take(self, n):
        out = []
        while n > 0:
            if self._pos >= len(self._perm):
                self._perm = torch.randperm(len(self.locks), generator=self.gen)
                self._pos = 0
            k = min(n, len(self._perm) - self._pos)
            out.append(self._perm[self._pos:self._pos + k])
            self._pos += k
            n -= k
        return torch.cat(out)

    def __iter__(self) -> Iterator:
        return self

    def __next__(self):
        idx = self._take(self.batch)
        lock = self.locks[idx.to(self.device)]
        key = self.keys[idx.to(self.device)]
        ang = torch.rand(self.batch, generator=self.gen) * (2 * math.pi)
        rot = rotate_nearest(lock, ang)
        x = assemble(lock, rot, key)
        if self.normalize:
            x = x / 255.0
        return x.contiguous(), self.areas[idx].to(self.device).float()


def inputs(normalize: bool = False, reshape: bool = False, rotation: bool = False,
           batch_size: Optional[int] = None, image_size: Optional[int] = None,
           data_dir: Optional[str] = None, device="cuda", seed: int = 1) -> BatchStream:
    """``11a/overlap_input.py:76``. ``reshape`` is implied (the stream yields [B, 3D])."""
    if not rotation:
        raise ValueError("Rotation has to be True.")
    size = image_size or FLAGS.IMAGE_SIZE
    bs = batch_size or FLAGS.BATCH_SIZE
    d = data_dir if data_dir is not None else FLAGS.DATA_DIR
    src = PairSource(d, limit=FLAGS.NUM_EXAMPLES_TO_LOAD_INTO_QUEUE) if d else None
    return BatchStream(bs, size, src, normalize=normalize, seed=seed, device=device)
