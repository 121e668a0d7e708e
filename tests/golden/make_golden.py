#!/usr/bin/env python3
"""Regenerate the committed fixtures under tests/golden/ (run here, where the read-only
reference is mounted; the GPU box only reads the committed files).

  magic_amd/data/overlap_areas.npy  the 2000 int64 labels of the reference's ``2a/OVERLAP_AREAS``
                         (package data: the synthetic batches resample it)
                         (a Python-2 protocol-0 pickle of numpy int64 scalars). The file is
                         NOT unpickled: its ``S'...'`` string literals (8 raw little-endian
                         bytes each) are parsed as text and decoded with escape rules only.
  overlap_micro.npz      the reference's ``overlap_micro.zip`` (100 lock/key pairs, 200x200
                         binary PNGs) as packed bits: data, not code.
  step_<flavour>.npz     oracle (float64) golden vectors for one training step of a tiny
                         config per preset flavour (and the conv-encoder variant): inputs,
                         5 losses, distance, g1, g2, post-Adam parameters.

Usage: python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import codecs
import io
import os
import re
import sys
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import mvae_oracle as O  # noqa: E402

FLAVOURS = {
    "8c_cosine_tanh": dict(act="tanh", metric="cosine", reciprocal=False, deform_weight=10.0),
    "9a_recip_cosine": dict(act="tanh", metric="cosine", reciprocal=True, deform_weight=10.0),
    "11a_recip_sqdiff_elu": dict(act="elu", metric="sqdiff", reciprocal=True, deform_weight=100.0),
    "sqdiff_tanh": dict(act="tanh", metric="sqdiff", reciprocal=False, deform_weight=10.0),
    # conv-encoder variant (tower of 6b/net.py:50-60): image side a multiple of 4
    "conv_recip_sqdiff": dict(act="tanh", metric="sqdiff", reciprocal=True, deform_weight=10.0,
                              conv=True, image_size=12),
}
TINY = dict(image_size=10, enc=(24, 16), dec=(12, 14), latent=4, lr=(1e-3, 1e-4))
TINY_B = 8


def parse_overlap_areas(path: str) -> np.ndarray:
    raw = open(path, "rb").read().decode("latin-1")
    vals = []
    # Python 2's repr quotes with ' unless the bytes contain ' (then with ")
    for lit in re.findall(r"S(?:'((?:[^'\\]|\\.)*)'|\"((?:[^\"\\]|\\.)*)\")\n", raw):
        b = codecs.escape_decode((lit[0] or lit[1]).encode("latin-1"))[0]
        if len(b) == 8:
            vals.append(np.frombuffer(b, "<i8")[0])
    return np.array(vals, np.int64)


def pack_micro(path: str) -> dict:
    from PIL import Image
    z = zipfile.ZipFile(path)
    locks, keys = [], []
    i = 0
    while f"overlap_micro/{i}_L.png" in z.namelist():
        for lst, nm in ((locks, f"{i}_L"), (keys, f"{i}_K")):
            a = np.array(Image.open(io.BytesIO(z.read(f"overlap_micro/{nm}.png"))).convert("L"))
            assert set(np.unique(a)) <= {0, 255}
            lst.append(a > 0)
        i += 1
    L, K = np.stack(locks), np.stack(keys)
    return {"lock_bits": np.packbits(L, axis=-1), "key_bits": np.packbits(K, axis=-1),
            "shape": np.array(L.shape)}


def golden_cfg(flav: dict) -> O.OracleConfig:
    return O.OracleConfig(**dict(TINY, **flav))


def step_golden(name: str, flav: dict) -> dict:
    cfg = golden_cfg(flav)
    P = O.init_params(cfg, seed=0, dtype=np.float64)
    rng = np.random.default_rng(7)
    for k in P:
        if k.endswith("_b"):
            P[k] = rng.normal(0, 0.05, P[k].shape)
    X = (np.random.default_rng(1).random((TINY_B, 3 * cfg.D)) < 0.2).astype(np.float64)
    areas = np.random.default_rng(1).integers(296, 6427, TINY_B).astype(np.float64)
    eps = np.random.default_rng(2).standard_normal((3, TINY_B, cfg.latent))
    st = O.adam_init(cfg, P)
    losses, dist, Pn, st, (g1, g2) = O.train_step(P, st, X, areas, eps, cfg)
    out = {"X": X, "areas": areas, "eps": eps, "losses": losses, "dist": dist}
    for k, v in P.items():
        out["P/" + k] = v
    for k, v in g1.items():
        out["g1/" + k] = v
    for k, v in g2.items():
        out["g2/" + k] = v
    for k, v in Pn.items():
        out["Pn/" + k] = v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    areas = parse_overlap_areas(os.path.join(args.reference, "2a", "OVERLAP_AREAS"))
    np.save(os.path.join(os.path.dirname(os.path.dirname(HERE)), "magic_amd", "data", "overlap_areas.npy"), areas)
    print("overlap_areas", areas.shape, areas.min(), areas.max(), areas.mean())
    np.savez_compressed(os.path.join(HERE, "overlap_micro.npz"),
                        **pack_micro(os.path.join(args.reference, "overlap_micro.zip")))
    for name, flav in FLAVOURS.items():
        np.savez_compressed(os.path.join(HERE, f"step_{name}.npz"), **step_golden(name, flav))
        print("wrote", name)


if __name__ == "__main__":
    main()
