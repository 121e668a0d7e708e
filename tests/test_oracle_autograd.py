"""Pin the oracle's hand-derived backward against an INDEPENDENT differentiator:
torch.autograd (float64) applied to a direct restatement of the reference's TF graph
(``11a/vae.py:172-313``, ``cosine_distance`` ``:444-458``), op for op — including the
``log(pow(y,x)*pow(1-y,1-x))`` reconstruction form and ``l2_normalize``'s ``maximum``."""
import numpy as np
import pytest
import torch

from oracle import mvae_oracle as O

FLAVOURS = [
    # act, metric, reciprocal, w
    ("tanh", "cosine", False, 10.0),   # 8c / 8d / 8e
    ("tanh", "cosine", True, 10.0),    # 9a / 10a
    ("elu", "sqdiff", True, 100.0),    # 10b / 11a
    ("tanh", "sqdiff", False, 10.0),
    ("elu", "cosine", False, 100.0),
    ("elu", "sqdiff", False, 10.0),
]


def tiny_cfg(act, metric, recip, w, enc=(16, 12), L=4):
    return O.OracleConfig(image_size=6, enc=enc, dec=(10, 14), latent=L, act=act,
                          deform_weight=w, metric=metric, reciprocal=recip)


def tiny_batch(cfg, B, seed=1):
    rng = np.random.default_rng(seed)
    X = (rng.random((B, 3 * cfg.D)) < 0.3).astype(np.float64)
    areas = rng.integers(296, 6427, size=B).astype(np.float64)
    eps = np.random.default_rng(seed + 1).standard_normal((3, B, cfg.latent))
    return X, areas, eps


def torch_graph(P, X, areas, eps, cfg):
    """Direct TF-graph restatement; returns (cost, training_loss, distance)."""
    act = torch.tanh if cfg.act == "tanh" else torch.nn.functional.elu
    xl, xr, xk = X[:, 0::3], X[:, 1::3], X[:, 2::3]

    def enc(x, e):
        h = x
        for i in range(len(cfg.enc)):
            h = act(h @ P[f"enc_h{i}_W"] + P[f"enc_h{i}_b"])
        mu = h @ P["enc_out_mean_W"] + P["enc_out_mean_b"]
        s = h @ P["enc_out_log_sigma_W"] + P["enc_out_log_sigma_b"]
        return mu, s, mu + torch.sqrt(torch.exp(s)) * e

    mu, s, zl = enc(xl, eps[0])
    _, _, zr = enc(xr, eps[1])
    _, _, zk = enc(xk, eps[2])
    d1 = act(zl @ P["dec_h1_W"] + P["dec_h1_b"])
    d2 = act(d1 @ P["dec_h2_W"] + P["dec_h2_b"])
    y = torch.sigmoid(d2 @ P["dec_out_mean_W"] + P["dec_out_mean_b"])
    rec = -torch.sum(torch.log(torch.pow(y, xl) * torch.pow(1.0 - y, 1.0 - xl)), 1)
    lat = -0.5 * torch.sum(1 + s - mu ** 2 - torch.exp(s), 1)
    dfm = cfg.deform_weight * torch.sum((zl - zr) ** 2, 1)
    cost = torch.mean(rec + lat + dfm)
    if cfg.metric == "cosine":
        na = zl * torch.rsqrt(torch.clamp(torch.sum(zl ** 2, 0, keepdim=True), min=O.L2_EPS))
        nb = zk * torch.rsqrt(torch.clamp(torch.sum(zk ** 2, 0, keepdim=True), min=O.L2_EPS))
        dist = torch.sum(na * nb, 1)
    else:
        dist = torch.sum((zl - zk) ** 2, 1)
    if cfg.reciprocal:
        dist = 1.0 / dist
    tl = torch.mean((dist - areas) ** 2)
    return cost, tl, dist, (rec.mean(), lat.mean(), dfm.mean())


@pytest.mark.parametrize("flav", FLAVOURS)
def test_backward_matches_autograd(flav):
    cfg = tiny_cfg(*flav)
    B = 7
    P = O.init_params(cfg, seed=3, dtype=np.float64)
    # non-zero biases so bias paths are exercised
    rng = np.random.default_rng(9)
    for k in P:
        if k.endswith("_b"):
            P[k] = rng.normal(0, 0.1, P[k].shape)
    X, areas, eps = tiny_batch(cfg, B)
    c = O.forward(P, X, eps, cfg)
    O.metric(c, areas, cfg, B)
    losses = O.loss_sums(c, B)
    g1, g2 = O.backward(c, cfg, B)

    TP = {k: torch.tensor(v, requires_grad=True) for k, v in P.items()}
    cost, tl, dist, (r, l, d) = torch_graph(TP, torch.tensor(X), torch.tensor(areas), torch.tensor(eps), cfg)
    np.testing.assert_allclose(losses, [cost.item(), tl.item(), r.item(), l.item(), d.item()], rtol=1e-12)
    np.testing.assert_allclose(c["dist"], dist.detach().numpy(), rtol=1e-12)

    names = O.trained_names(cfg)
    gc = torch.autograd.grad(cost, [TP[n] for n in names], allow_unused=True, retain_graph=True)
    gt = torch.autograd.grad(tl, [TP[n] for n in names], allow_unused=True)
    for n, a, b in zip(names, gc, gt):
        np.testing.assert_allclose(g1[n], a.numpy(), rtol=1e-9, atol=1e-12 * max(1, np.abs(a.numpy()).max()), err_msg=n)
        if n.startswith("enc_"):
            np.testing.assert_allclose(g2[n], b.numpy(), rtol=1e-9, atol=1e-12 * max(1, np.abs(b.numpy()).max()), err_msg=n)
        else:  # the decoder receives no gradient from training_loss
            assert b is None or not np.any(b.numpy()), n
            assert n not in g2


def test_adam_matches_torch_formula():
    """TF ApplyAdam vs an independent re-statement over several steps."""
    cfg = tiny_cfg("tanh", "cosine", False, 10.0)
    P = O.init_params(cfg, seed=0, dtype=np.float64)
    st = O.adam_init(cfg, P)
    rng = np.random.default_rng(0)
    names = O.trained_names(cfg)
    ref = {n: P[n].copy() for n in names}
    m = {o: {n: 0.0 for n in names} for o in (1, 2)}
    v = {o: {n: 0.0 for n in names} for o in (1, 2)}
    for t in range(1, 5):
        g1 = {n: rng.normal(size=P[n].shape) for n in names}
        g2 = {n: rng.normal(size=P[n].shape) for n in O.encoder_names(cfg)}
        P, st = O.adam(P, g1, g2, st, cfg)
        for o, g in ((1, g1), (2, g2)):
            lr = cfg.lr[o - 1] * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
            for n, gn in g.items():
                m[o][n] = 0.9 * m[o][n] + 0.1 * gn
                v[o][n] = 0.999 * v[o][n] + 0.001 * gn * gn
                ref[n] = ref[n] - lr * m[o][n] / (np.sqrt(v[o][n]) + 1e-8)
        for n in names:
            # TF keeps beta powers in fp32: 1 - 0.999f carries a 1.3e-5 relative error,
            # so the fp32 lr_t differs from the float64 formula by ~1e-5 of the update.
            np.testing.assert_allclose(P[n], ref[n], rtol=0, atol=1e-4 * sum(cfg.lr))
