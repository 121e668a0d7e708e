"""(diagnostics) One step of a config with create option bits=0 vs bits=1: per-tensor max-norm
relative difference of g1 / g2, losses, and the plan log."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from magic_amd import _lib
from magic_amd.config import preset
from magic_amd.engine import Engine
from tests.gpu_helpers import gpu_phases, make_inputs, make_params

for name, cfg in [("8d100b64", preset("8d", image_size=100, batch=64, precision="bf16")),
                  ("8c20b64", preset("8c", image_size=20, batch=64, precision="bf16")),
                  ("8d24b64", preset("8d", image_size=24, batch=64, precision="bf16").replace(enc=(500,) * 4, latent=255)),
                  ("8d24b128", preset("8d", image_size=24, batch=128, precision="bf16"))]:
    res = {}
    for opt in ("bits=0", "bits=1"):
        eng = Engine(cfg.replace(options=opt), 0)
        P = make_params(cfg)
        eng.load_params(P)
        X, areas, eps = make_inputs(cfg, cfg.batch)
        res[opt] = gpu_phases(eng, X, areas, eps)
        eng.close()
    a, b = res["bits=0"], res["bits=1"]
    print(name, "losses", a[0][:5], b[0][:5])
    for i, lab in ((2, "g1"), (3, "g2")):
        for k in a[i]:
            d = np.abs(a[i][k] - b[i][k]).max() / max(np.abs(a[i][k]).max(), 1e-30)
            if d > 1e-3:
                print(f"  {name} {lab} {k}: rel diff {d:.3e}")
    sys.stdout.flush()
