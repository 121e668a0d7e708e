"""Hyper-parameter presets of the reference's metric-VAE lineage and the
BASELINE.json run configurations.

The reference hard-codes these in ``TangoEncoder.__init__`` (``11a/vae.py:30-65``,
``8c/vae.py:30-63``) and in ``FLAGS`` (``11a/constants.py:32,52,60``); here they are one
dataclass so every preset is reachable by name.
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Tuple


@dataclasses.dataclass
class MVAEConfig:
    image_size: int = 100
    batch: int = 64
    global_batch: Optional[int] = None       # None -> batch (single rank)
    enc: Tuple[int, ...] = (500, 500, 500, 500)
    dec: Tuple[int, int] = (500, 500)
    latent: int = 20
    act: str = "tanh"
    metric: str = "cosine"
    reciprocal: bool = False
    deform_weight: float = 10.0
    lr: Tuple[float, float] = (1e-4, 1e-6)
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8
    precision: str = "f32"
    seed: int = 2
    conv: bool = False   # conv-encoder variant: CifarNet tower (6b/net.py:50-60) before the FC encoder
    # plan-time kernel switches of libmvae (mvae_create_ex options, "name=value,..."; A/B and
    # tests: e8, thin_ring, valu, dact_planes, bce_split, plan_log, conv2_*); "" = measured defaults
    options: str = ""

    @property
    def D(self) -> int:
        return self.image_size * self.image_size

    @property
    def gbatch(self) -> int:
        return self.global_batch or self.batch

    def replace(self, **kw) -> "MVAEConfig":
        return dataclasses.replace(self, **kw)

    def flops_per_pair(self) -> float:
        """Algorithmic FLOPs of one training pair: 3 encoder forwards,
        1 decoder forward, decoder backward, 4 encoder backward passes (lock x2, rot, key)."""
        D, L = self.D, self.latent
        S1 = self.image_size // 2
        F0 = (S1 // 2) ** 2 * 64 if self.conv else D      # layer-0 fan-in
        widths = [F0] + list(self.enc)
        enc_fwd = sum(2 * a * b for a, b in zip(widths[:-1], widths[1:])) + 2 * self.enc[-1] * 2 * L
        dec_layers = [(L, self.dec[0]), (self.dec[0], self.dec[1]), (self.dec[1], D)]
        dec_fwd = sum(2 * a * b for a, b in dec_layers)
        dec_bwd = 2 * dec_fwd  # wgrad + dgrad (the dgrad into z is counted, cheap)
        # encoder backward per pass: wgrad of every layer + dgrad of every layer but the first
        # (the first is conv1 in the conv variant: 25 MACs x 64 per pixel; conv2: 1600 x 64
        # per pooled pixel)
        first = 2 * F0 * self.enc[0]
        if self.conv:
            first = 2 * D * 25 * 64
            enc_fwd += first + 2 * S1 * S1 * 1600 * 64
        enc_w = enc_fwd
        enc_d = enc_fwd - first
        enc_bwd = 4 * (enc_w + enc_d)
        return float(3 * enc_fwd + dec_fwd + dec_bwd + enc_bwd)


# SURVEY.md §2.3 (reference IMAGE_SIZE is 200; BASELINE runs use 100 — pass image_size=)
PRESETS = {
    "8c": dict(enc=(500, 500, 500, 500), latent=20, act="tanh", deform_weight=10.0,
               lr=(1e-4, 1e-6), metric="cosine", reciprocal=False),
    "8d": dict(enc=(500, 500, 500, 500), latent=200, act="tanh", deform_weight=10.0,
               lr=(1e-4, 1e-6), metric="cosine", reciprocal=False),
    "8e": dict(enc=(500, 500, 500, 500), latent=2000, act="tanh", deform_weight=10.0,
               lr=(1e-4, 1e-6), metric="cosine", reciprocal=False),
    "8f": dict(enc=(10000, 5000, 1000, 500), latent=2000, act="tanh", deform_weight=10.0,
               lr=(1e-4, 1e-6), metric="cosine", reciprocal=False),
    "9a": dict(enc=(500, 500, 500, 500), latent=2, act="tanh", deform_weight=10.0,
               lr=(1e-4, 1e-6), metric="cosine", reciprocal=True),
    "10a": dict(enc=(500, 500, 500, 500), latent=80, act="tanh", deform_weight=10.0,
                lr=(1e-4, 1e-8), metric="cosine", reciprocal=True),
    "11a": dict(enc=(500, 500), latent=80, act="elu", deform_weight=100.0,
                lr=(1e-6, 1e-8), metric="sqdiff", reciprocal=True),
    "shapes": dict(enc=(500, 500), latent=200, act="tanh", deform_weight=100.0,
                   lr=(1e-6, 1e-8), metric="sqdiff", reciprocal=True),
}
PRESET_BATCH = {"8c": 100, "8d": 100, "8e": 100, "8f": 100, "9a": 24, "10a": 24, "11a": 24,
                "shapes": 24}


def preset(name: str, image_size: int = 100, batch: Optional[int] = None, **kw) -> MVAEConfig:
    p = dict(PRESETS[name])
    p.update(kw)
    return MVAEConfig(image_size=image_size, batch=batch or PRESET_BATCH[name], **p)


# BASELINE.json "configs" 
def baseline_config(cid: str) -> MVAEConfig:
    cid = cid.upper()
    if cid == "C1":
        return preset("8c", batch=64)
    if cid == "C2":
        # "fp32": the exact 3-term bf16 split (f32x) is fp32-accurate (products exact, fp32
        # accumulation; tests hold it to the native fp32 kernel's error bound) and faster
        # than native fp32 MFMA on gfx950; precision="f32" selects the native path
        return preset("8c", batch=4096, precision="f32x")
    if cid in ("C3", "C4"):
        return preset("8d", batch=8192, precision="bf16")
    if cid == "C5":
        return preset("8e", batch=8192, metric="sqdiff", reciprocal=True, precision="bf16")
    if cid == "C5CONV":
        # BASELINE config 5's conv-encoder variant: the CifarNet tower in front of the 8e
        # encoder (latent 2000, reciprocal squared difference), bf16 MFMA
        return preset("8e", batch=512, metric="sqdiff", reciprocal=True, precision="bf16", conv=True)
    raise KeyError(cid)
