"""Engine: one libmvae context on one GPU, with torch views of its device memory.

PyTorch is plumbing here (device memory, streams, RNG for inputs, torch.distributed);
every arithmetic step of the training path runs in the HIP kernels of ``libmvae.so``.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .config import MVAEConfig

PARAM_ORDER_DEAD = ("dec_out_log_sigma_W", "dec_out_log_sigma_b")


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError("expected a contiguous float32 device tensor")
    return t.data_ptr()


class Engine:
    """Owns an ``mvae_ctx``. Tensors passed in must be contiguous float32 on ``device``."""

    def __init__(self, cfg: MVAEConfig, device: int = 0):
        if not torch.cuda.is_available():
            raise _lib.MVAELibraryError("no GPU visible: libmvae runs on MI355X (gfx950) only")
        self.lib = _lib.load()
        self.cfg = cfg
        self.device = device
        self.dev = torch.device("cuda", device)
        c = _lib.mvae_cfg()
        c.image_size = cfg.image_size
        c.batch = cfg.batch
        c.global_batch = cfg.gbatch
        c.n_enc = len(cfg.enc)
        if not 1 <= c.n_enc <= _lib.MVAE_MAX_ENC:
            raise ValueError("encoder depth out of range")
        for i, e in enumerate(cfg.enc):
            c.enc[i] = e
        c.dec[0], c.dec[1] = cfg.dec
        c.latent = cfg.latent
        c.act = _lib.ACT[cfg.act]
        c.metric = _lib.METRIC[cfg.metric]
        c.reciprocal = int(cfg.reciprocal)
        c.deform_weight = cfg.deform_weight
        c.lr[0], c.lr[1] = cfg.lr
        c.beta1, c.beta2, c.epsilon = cfg.beta1, cfg.beta2, cfg.epsilon
        c.precision = _lib.PREC[cfg.precision]
        c.seed = cfg.seed
        c.conv = int(getattr(cfg, "conv", False))
        torch.cuda.set_device(device)
        torch.cuda.init()
        h = C.c_void_p()
        opts = getattr(cfg, "options", "") or None
        rc = self.lib.mvae_create_ex(C.byref(c), device, opts.encode() if opts else None, C.byref(h))
        if rc != 0:
            raise _lib.MVAEError(rc, (self.lib.mvae_last_error(None) or b"").decode())
        self.ctx = h.value
        self._keep = []
        self._views: Dict[tuple, Dict[str, torch.Tensor]] = {}
        self.losses = self.buffer(_lib.BUF_LOSSES)
        self.grads = self.buffer(_lib.BUF_GRADS)
        self.colsq = self.buffer(_lib.BUF_COLSQ)
        self.coldot = self.buffer(_lib.BUF_COLDOT)
        self.dist = self.buffer(_lib.BUF_DIST)

    # ------------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "ctx", None):
            torch.cuda.synchronize(self.dev)
            self._views.clear()
            self.losses = self.grads = self.colsq = self.coldot = self.dist = None
            self.lib.mvae_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        return _lib.check(self.lib, self.ctx, rc)

    @property
    def stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    # ------------------------------------------------------------------ memory views
    def buffer(self, which: int) -> torch.Tensor:
        p = C.c_void_p()
        n = C.c_size_t()
        self._check(self.lib.mvae_buffer(self.ctx, which, C.byref(p), C.byref(n)))
        return _lib.device_view(p.value, (n.value,), (1,), self.device, self._keep)

    def tensors(self, kind: int = _lib.KIND_PARAM) -> Dict[str, torch.Tensor]:
        """Name -> view, in the reference's variable creation order (``11a/vae.py:85-153``).
        Weights are [fan_in, fan_out] (y = x W), biases [fan_out]."""
        key = (kind,)
        if key in self._views:
            return self._views[key]
        out = {}
        n = self.lib.mvae_param_count(self.ctx)
        t = _lib.mvae_tensor()
        for i in range(n):
            rc = self.lib.mvae_param_info(self.ctx, kind, i, C.byref(t))
            if rc != 0:
                continue  # e.g. decoder variables have no metric-optimizer state
            name = t.name.decode()
            if t.rows == 1 and not name.endswith("_W"):
                v = _lib.device_view(t.data, (t.cols,), (1,), self.device, self._keep)
            else:
                v = _lib.device_view(t.data, (t.rows, t.cols), (t.ld, 1), self.device, self._keep)
            out[name] = v
        self._views[key] = out
        return out

    def params(self) -> Dict[str, torch.Tensor]:
        return self.tensors(_lib.KIND_PARAM)

    def sync_params(self):
        """Refresh the bf16 plane images of the parameters after writing the fp32 masters
        through the views (bf16 / f32x modes; a no-op in fp32 mode)."""
        self._check(self.lib.mvae_sync_params(self.ctx, self.stream))

    def load_params(self, P: Dict[str, np.ndarray]):
        views = self.params()
        for k, v in P.items():
            views[k].copy_(torch.as_tensor(np.asarray(v, np.float32)).to(self.dev))
        self.sync_params()
        torch.cuda.synchronize(self.dev)

    def init_params(self, seed: int = 0):
        """Xavier-uniform weights (``11a/utils.py:484-491``), zero biases (``11a/vae.py:116-153``),
        drawn on the host from a seeded generator in the reference's creation order."""
        rng = np.random.default_rng(seed)
        views = self.params()
        for name, v in views.items():
            if v.dim() == 2:
                fan_in, fan_out = v.shape
                if name.startswith("enc_conv"):  # slim xavier: receptive field on both fans
                    fan_out *= 25
                hi = np.sqrt(6.0 / (fan_in + fan_out))
                v.copy_(torch.from_numpy(rng.uniform(-hi, hi, size=tuple(v.shape)).astype(np.float32)).to(self.dev))
            else:
                v.zero_()
        self.sync_params()
        torch.cuda.synchronize(self.dev)

    def get_step(self):
        a, b = C.c_int64(), C.c_int64()
        self._check(self.lib.mvae_get_step(self.ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_step(self, t1: int, t2: int):
        self._check(self.lib.mvae_set_step(self.ctx, t1, t2))

    def set_shard(self, row_offset: int):
        """This rank's first row in the global batch (the internal eps sampler draws the
        rank's slice of the global stream)."""
        self._check(self.lib.mvae_set_shard(self.ctx, row_offset))

    def get_rng(self):
        a, b = C.c_uint64(), C.c_uint64()
        self._check(self.lib.mvae_get_rng(self.ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_rng(self, train: int, eval_: int):
        self._check(self.lib.mvae_set_rng(self.ctx, train, eval_))

    # ------------------------------------------------------------------ step phases
    def _xin(self, x):
        if x.shape != (self.cfg.batch, 3 * self.cfg.D):
            raise ValueError(f"X must be [{self.cfg.batch}, {3 * self.cfg.D}] (got {tuple(x.shape)})")
        return _ptr(x)

    def forward(self, x: torch.Tensor, eps: Optional[torch.Tensor] = None):
        if eps is not None and eps.shape != (3, self.cfg.batch, self.cfg.latent):
            raise ValueError("eps must be [3, B, L] (lock, rotated lock, key)")
        self._check(self.lib.mvae_forward(self.ctx, self._xin(x), _ptr(eps), self.stream))

    def metric(self, areas: torch.Tensor):
        if areas.shape != (self.cfg.batch,):
            raise ValueError("overlap_areas must be [B]")
        self._check(self.lib.mvae_metric(self.ctx, _ptr(areas), self.stream))

    def backward(self):
        self._check(self.lib.mvae_backward(self.ctx, self.stream))

    @property
    def N_BACKWARD_PARTS(self) -> int:
        """Backward parts of the current schedule (2 + the layer-0 weight-gradient chunks)."""
        return self.lib.mvae_backward_nparts(self.ctx)

    def backward_part(self, part: int):
        """Part ``part`` (0, 1, 2 in order) of ``backward``; see ``grad_ranges``."""
        self._check(self.lib.mvae_backward_part(self.ctx, part, self.stream))

    def grad_ranges(self, part: int):
        """Views of ``grads`` that are final once ``backward_part(part)`` has run."""
        base = self.grads.data_ptr()
        out = []
        for i in range(8):
            p = C.c_void_p()
            n = C.c_size_t()
            if self.lib.mvae_grad_range(self.ctx, part, i, C.byref(p), C.byref(n)) != 0:
                break
            off = (p.value - base) // 4
            if n.value:
                out.append(self.grads[off:off + n.value])
        return out

    def set_option(self, name: str, value: int):
        self._check(self.lib.mvae_set_option(self.ctx, name.encode(), int(value)))

    def adam(self):
        self._check(self.lib.mvae_adam(self.ctx, self.stream))

    def train_step(self, x, areas, eps=None, losses_out=None, dist_out=None):
        if areas.shape != (self.cfg.batch,):
            raise ValueError("overlap_areas must be [B]")
        self._check(self.lib.mvae_train_step(self.ctx, self._xin(x), _ptr(areas), _ptr(eps),
                                             _ptr(losses_out), _ptr(dist_out), self.stream))

    def predict(self, x, eps=None, out=None):
        out = out if out is not None else torch.empty(self.cfg.batch, device=self.dev)
        self._check(self.lib.mvae_predict(self.ctx, self._xin(x), _ptr(eps), _ptr(out), self.stream))
        return out

    def predict_encode(self, x, eps=None):
        """First phase of ``predict``: encoder + (cosine) the local column sums ``colsq``."""
        self._check(self.lib.mvae_predict_encode(self.ctx, self._xin(x), _ptr(eps), self.stream))

    def predict_finish(self, out=None):
        """Second phase: distances with the current ``colsq`` (all-reduced under DP)."""
        out = out if out is not None else torch.empty(self.cfg.batch, device=self.dev)
        self._check(self.lib.mvae_predict_finish(self.ctx, _ptr(out), self.stream))
        return out

    def transform(self, x, out=None):
        out = out if out is not None else torch.empty(self.cfg.batch, self.cfg.latent, device=self.dev)
        self._check(self.lib.mvae_transform(self.ctx, self._xin(x), _ptr(out), self.stream))
        return out

    def reconstruct(self, x, eps=None, out=None):
        out = out if out is not None else torch.empty(self.cfg.batch, self.cfg.D, device=self.dev)
        self._check(self.lib.mvae_reconstruct(self.ctx, self._xin(x), _ptr(eps), _ptr(out), self.stream))
        return out

    def generate(self, z: torch.Tensor, out=None):
        z = z.reshape(-1, self.cfg.latent).contiguous()
        n = z.shape[0]
        out = out if out is not None else torch.empty(n, self.cfg.D, device=self.dev)
        self._check(self.lib.mvae_generate(self.ctx, _ptr(z), n, _ptr(out), self.stream))
        return out

    # ------------------------------------------------------------------ timing regions
    def timing_enable(self, on: bool = True):
        self._check(self.lib.mvae_timing_enable(self.ctx, int(on)))

    def timing_select(self, name: Optional[str] = None):
        """Record only region ``name`` (None: all regions)."""
        r = -1
        if name is not None:
            names = [self.lib.mvae_timing_name(self.ctx, i).decode()
                     for i in range(self.lib.mvae_timing_regions(self.ctx))]
            r = names.index(name)
        self._check(self.lib.mvae_timing_select(self.ctx, r))

    def timing_names(self):
        return [self.lib.mvae_timing_name(self.ctx, i).decode()
                for i in range(self.lib.mvae_timing_regions(self.ctx))]

    def timing_marker(self, name: str, on: bool = True):
        """Bracket region ``name`` with marker kernels (rocprofv3 counter attribution)."""
        self._check(self.lib.mvae_timing_marker(self.ctx, self.timing_names().index(name), int(on)))

    def timing_reset(self):
        self._check(self.lib.mvae_timing_reset(self.ctx))

    def timing_read(self) -> Dict[str, tuple]:
        """Region name -> (total ms, launches) over the HIP events recorded while enabled."""
        out = {}
        tot, cnt = C.c_double(), C.c_int64()
        for r in range(self.lib.mvae_timing_regions(self.ctx)):
            self._check(self.lib.mvae_timing_read(self.ctx, r, C.byref(tot), C.byref(cnt)))
            if cnt.value:
                out[self.lib.mvae_timing_name(self.ctx, r).decode()] = (tot.value, cnt.value)
        return out
