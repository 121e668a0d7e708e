"""Pin the conv-encoder oracle (oracle/conv_oracle.py) against an
INDEPENDENT differentiator: torch.autograd (float64) on torch's own conv2d / max_pool2d /
local_response_norm, composed as the CifarNet tower of ``6b/net.py:50-60`` and fed into the
VAE graph of ``11a/vae.py:172-313``. Parity with TF itself is unpinned by nature (the
reference has no conv VAE); the op semantics restated are TF1's (module docstring)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import conv_oracle as CV
from oracle import mvae_oracle as O
from tests.test_oracle_autograd import tiny_batch


def torch_tower(P, x, S):
    """x [N, S*S] -> flat NHWC features, torch ops only."""
    N = x.shape[0]
    xi = x.reshape(N, 1, S, S)
    w1 = P["enc_conv1_W"].reshape(5, 5, 1, 64).permute(3, 2, 0, 1)   # HWIO -> OIHW
    w2 = P["enc_conv2_W"].reshape(5, 5, 64, 64).permute(3, 2, 0, 1)
    lrn = lambda a: F.local_response_norm(a, size=2 * CV.LRN_R + 1, alpha=CV.LRN_ALPHA * (2 * CV.LRN_R + 1),
                                          beta=CV.LRN_BETA, k=CV.LRN_BIAS)
    a1 = F.relu(F.conv2d(xi, w1, P["enc_conv1_b"], padding=2))
    n1 = lrn(F.max_pool2d(a1, 2, 2))
    a2 = F.relu(F.conv2d(n1, w2, P["enc_conv2_b"], padding=2))
    p2 = F.max_pool2d(lrn(a2), 2, 2)
    return p2.permute(0, 2, 3, 1).reshape(N, -1)


def test_lrn_and_pool_match_torch():
    rng = np.random.default_rng(0)
    a = np.maximum(rng.normal(size=(3, 6, 7, 64)), 0) * 3
    t = torch.tensor(a).permute(0, 3, 1, 2)
    ref = F.local_response_norm(t, 9, alpha=CV.LRN_ALPHA * 9, beta=CV.LRN_BETA, k=1.0).permute(0, 2, 3, 1)
    np.testing.assert_allclose(CV.lrn(a), ref.numpy(), rtol=1e-13)
    p, arg = CV.maxpool(a)
    np.testing.assert_array_equal(p, F.max_pool2d(t, 2, 2).permute(0, 2, 3, 1).numpy())
    # ties (relu zeros, equal values): gradient to the FIRST max in row-major window order
    b = np.zeros((1, 2, 2, 64))
    b[0, 1, 0, :] = 1.0
    b[0, 1, 1, :] = 1.0
    p, arg = CV.maxpool(b)
    assert (arg == 2).all()
    g = CV.unpool(np.ones((1, 1, 1, 64)), arg, b.shape)
    assert g[0, 1, 0].sum() == 64 and g.sum() == 64


def test_lrn_bwd_matches_autograd():
    rng = np.random.default_rng(1)
    a = np.abs(rng.normal(size=(2, 3, 3, 64))) * 2
    g = rng.normal(size=a.shape)
    t = torch.tensor(a, requires_grad=True)
    out = F.local_response_norm(t.permute(0, 3, 1, 2), 9, alpha=CV.LRN_ALPHA * 9, beta=CV.LRN_BETA, k=1.0)
    (gt,) = torch.autograd.grad(out, t, torch.tensor(g).permute(0, 3, 1, 2))
    np.testing.assert_allclose(CV.lrn_bwd(a, g), gt.numpy(), rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("flav", [("tanh", "sqdiff", True, 10.0), ("tanh", "cosine", False, 10.0),
                                  ("elu", "sqdiff", False, 100.0)])
def test_conv_backward_matches_autograd(flav):
    act, metric, recip, w = flav
    S = 8
    cfg = O.OracleConfig(image_size=S, enc=(16, 12), dec=(10, 14), latent=4, act=act,
                         deform_weight=w, metric=metric, reciprocal=recip, conv=True)
    B = 5
    P = O.init_params(cfg, seed=3, dtype=np.float64)
    assert P["enc_h0_W"].shape == (CV.feat_dim(S), 16)
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
    Xt = torch.tensor(X)
    feats = [torch_tower(TP, Xt[:, ch::3], S) for ch in range(3)]
    Fcat = torch.stack(feats, 2).reshape(B, -1)          # interleaved: column f*3 + channel
    cost, tl, dist, (r, l, d) = _graph_with_features(TP, Fcat, Xt, torch.tensor(areas),
                                                     torch.tensor(eps), cfg)
    np.testing.assert_allclose(losses, [cost.item(), tl.item(), r.item(), l.item(), d.item()], rtol=1e-11)
    np.testing.assert_allclose(c["dist"], dist.detach().numpy(), rtol=1e-11)
    names = O.trained_names(cfg)
    gc = torch.autograd.grad(cost, [TP[n] for n in names], allow_unused=True, retain_graph=True)
    gt = torch.autograd.grad(tl, [TP[n] for n in names], allow_unused=True)
    for n, a, b in zip(names, gc, gt):
        np.testing.assert_allclose(g1[n], a.numpy(), rtol=1e-9, atol=1e-11 * max(1, np.abs(a.numpy()).max()), err_msg=n)
        if n.startswith("enc_"):
            np.testing.assert_allclose(g2[n], b.numpy(), rtol=1e-9, atol=1e-11 * max(1, np.abs(b.numpy()).max()), err_msg=n)
    # the tower's gradients are non-trivial (relu/pool masks leave most of them alive)
    assert np.abs(g1["enc_conv1_W"]).max() > 0 and np.abs(g2["enc_conv2_W"]).max() > 0


def _graph_with_features(P, Fcat, X, areas, eps, cfg):
    """``torch_graph`` with the encoder reading ``Fcat`` (interleaved features) and the
    decoder reconstructing the lock PIXELS of ``X``."""
    act = torch.tanh if cfg.act == "tanh" else torch.nn.functional.elu
    fl, fr, fk = Fcat[:, 0::3], Fcat[:, 1::3], Fcat[:, 2::3]
    xl = X[:, 0::3]

    def enc(h, e):
        for i in range(len(cfg.enc)):
            h = act(h @ P[f"enc_h{i}_W"] + P[f"enc_h{i}_b"])
        mu = h @ P["enc_out_mean_W"] + P["enc_out_mean_b"]
        s = h @ P["enc_out_log_sigma_W"] + P["enc_out_log_sigma_b"]
        return mu, s, mu + torch.sqrt(torch.exp(s)) * e

    mu, s, zl = enc(fl, eps[0])
    _, _, zr = enc(fr, eps[1])
    _, _, zk = enc(fk, eps[2])
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
