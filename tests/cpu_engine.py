"""TEST-ONLY stand-in engine: the oracle's phases behind the same interface as
``magic_amd.engine.Engine`` (forward / metric / backward / adam + the ``colsq``,
``coldot``, ``grads``, ``losses`` tensors), so the data-parallel host logic
(``magic_amd.parallel``) can be exercised with gloo on CPU. Never used by the product."""
from __future__ import annotations

import numpy as np
import torch

from oracle import mvae_oracle as O


class OracleEngine:
    def __init__(self, cfg, P):
        self.cfg = cfg
        self.oc = O.OracleConfig(image_size=cfg.image_size, enc=tuple(cfg.enc), dec=tuple(cfg.dec),
                                 latent=cfg.latent, act=cfg.act, deform_weight=cfg.deform_weight,
                                 metric=cfg.metric, reciprocal=cfg.reciprocal, lr=tuple(cfg.lr),
                                 conv=getattr(cfg, "conv", False))
        self.P = {k: np.asarray(v, np.float64) for k, v in P.items()}
        self.st = O.adam_init(self.oc, self.P)
        self.names1 = O.trained_names(self.oc)
        self.names2 = O.encoder_names(self.oc)
        n1 = sum(self.P[n].size for n in self.names1)
        n2 = sum(self.P[n].size for n in self.names2)
        L = cfg.latent
        self.colsq = torch.zeros(2 * L, dtype=torch.float64)
        self.coldot = torch.zeros(L, dtype=torch.float64)
        self.grads = torch.zeros(n1 + n2, dtype=torch.float64)
        self.losses = torch.zeros(5, dtype=torch.float64)
        self.dist = None

    def forward(self, x, eps=None):
        self.c = O.forward(self.P, x.numpy(), eps.numpy(), self.oc)
        self.colsq.copy_(torch.from_numpy(self.c["colsq"].reshape(-1)))

    def metric(self, areas):
        cs = self.colsq.numpy().reshape(2, -1)
        O.metric(self.c, areas.numpy(), self.oc, self.cfg.gbatch, colsq_global=cs)
        self.losses.copy_(torch.from_numpy(O.loss_sums(self.c, self.cfg.gbatch)))
        self.dist = torch.from_numpy(self.c["dist"])
        if self.cfg.metric == "cosine":
            self.coldot.copy_(torch.from_numpy(self.c["coldot"]))

    def backward(self):
        cd = self.coldot.numpy() if self.cfg.metric == "cosine" else None
        g1, g2 = O.backward(self.c, self.oc, self.cfg.gbatch, coldot_global=cd)
        flat = [g1[n].reshape(-1) for n in self.names1] + [g2[n].reshape(-1) for n in self.names2]
        self.grads.copy_(torch.from_numpy(np.concatenate(flat)))

    # the HIP engine's three-part backward: here part 0 computes everything and the
    # ranges are a fixed partition of ``grads`` released part by part (host-logic test)
    N_BACKWARD_PARTS = 3

    def backward_part(self, part):
        if part == 0:
            self.backward()

    def grad_ranges(self, part):
        n = self.grads.numel()
        cuts = [0, n // 5, n // 2, n]
        return [self.grads[cuts[part]:cuts[part + 1]]]

    def adam(self):
        g = self.grads.numpy()
        g1, g2, o = {}, {}, 0
        for n in self.names1:
            g1[n] = g[o:o + self.P[n].size].reshape(self.P[n].shape)
            o += self.P[n].size
        for n in self.names2:
            g2[n] = g[o:o + self.P[n].size].reshape(self.P[n].shape)
            o += self.P[n].size
        self.P, self.st = O.adam(self.P, g1, g2, self.st, self.oc)

    # get_predictions in the engine's two phases (colsq all-reduced between them under DP)
    def predict_encode(self, x, eps=None):
        self.pc = O.forward(self.P, x.numpy(), eps.numpy(), self.oc)
        self.colsq.copy_(torch.from_numpy(self.pc["colsq"].reshape(-1)))

    def predict_finish(self):
        cs = self.colsq.numpy().reshape(2, -1)
        O.metric(self.pc, np.zeros(self.pc["z_l"].shape[0]), self.oc, self.cfg.gbatch, colsq_global=cs)
        return torch.from_numpy(self.pc["dist"].copy())
