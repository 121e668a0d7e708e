"""Known-answer tests for the oracle, derived from the reference semantics
(SURVEY.md §8c "KATs derivable from reference semantics")."""
import numpy as np
import pytest

from oracle import mvae_oracle as O


def cfg8c(image=10, enc=(32, 32, 32, 32), L=20, **kw):
    return O.OracleConfig(image_size=image, enc=enc, dec=(32, 32), latent=L, **kw)


def zero_params(cfg):
    return {k: np.zeros_like(v, dtype=np.float64) for k, v in O.init_params(cfg).items()}


def test_kat_zero_weights_recon_is_D_ln2():
    """(i) all weights/biases 0 -> y = 0.5 -> r_l = D ln 2 (binary x); (ii) mu=s=0 -> l_l = 0."""
    cfg = cfg8c()
    B = 5
    X = (np.random.default_rng(1).random((B, 3 * cfg.D)) < 0.1).astype(np.float64)
    c = O.forward(zero_params(cfg), X, np.random.default_rng(2).standard_normal((3, B, cfg.latent)), cfg)
    np.testing.assert_allclose(c["R"], cfg.D * np.log(2.0), rtol=1e-12)
    np.testing.assert_allclose(c["K"], 0.0, atol=1e-15)


def test_kat_identical_latents_zero_deformation():
    """(iii) z_lock == z_rot (same image, same eps) -> d_l = 0; sqdiff distance to itself is 0."""
    cfg = cfg8c(metric="sqdiff")
    B = 4
    lock = (np.random.default_rng(1).random((B, cfg.D)) < 0.2).astype(np.float64)
    X = np.stack([lock, lock, lock], axis=2).reshape(B, 3 * cfg.D)
    e = np.random.default_rng(2).standard_normal((1, B, cfg.latent))
    c = O.forward(O.init_params(cfg, dtype=np.float64), X, np.repeat(e, 3, 0), cfg)
    O.metric(c, np.zeros(B), cfg, B)
    np.testing.assert_allclose(c["F"], 0.0, atol=1e-20)
    np.testing.assert_allclose(c["dist"], 0.0, atol=1e-20)


def test_kat_cosine_batch_of_one_is_sign_agreement():
    """(v) cosine with B=1: each latent column normalises to +-1 over the batch axis ->
    dist = sum_i sign(a_i) sign(b_i)  (axis-0 l2_normalize, ``8c/vae.py:449-450``)."""
    cfg = cfg8c()
    P = O.init_params(cfg, seed=5, dtype=np.float64)
    X = (np.random.default_rng(3).random((1, 3 * cfg.D)) < 0.3).astype(np.float64)
    eps = np.random.default_rng(4).standard_normal((3, 1, cfg.latent))
    c = O.forward(P, X, eps, cfg)
    O.metric(c, np.zeros(1), cfg, 1)
    expect = np.sum(np.sign(c["z_l"][0]) * np.sign(c["z_k"][0]))
    np.testing.assert_allclose(c["dist"][0], expect, rtol=1e-12)


def test_kat_first_adam_step_is_lr_sign():
    """(vi) first TF Adam step: delta = lr_t*m/(sqrt(v)+eps) ~= lr*sign(g) for |g| >> 1e-8."""
    cfg = cfg8c()
    P = O.init_params(cfg, seed=0, dtype=np.float64)
    st = O.adam_init(cfg, P)
    g1 = {n: np.full(P[n].shape, 0.37) for n in O.trained_names(cfg)}
    g2 = {n: np.full(P[n].shape, -2.0) for n in O.encoder_names(cfg)}
    Pn, st = O.adam(P, g1, g2, st, cfg)
    for n in O.encoder_names(cfg):
        np.testing.assert_allclose(P[n] - Pn[n], cfg.lr[0] * 1 - cfg.lr[1] * 1, rtol=1e-5)
    for n in O.trained_names(cfg):
        if n.startswith("dec_"):
            np.testing.assert_allclose(P[n] - Pn[n], cfg.lr[0], rtol=1e-5)
    assert st["b1p1"] == np.float32(0.9) * np.float32(0.9)


def test_kat_sigmoid_bce_gradient():
    """(vii) dcost/du = (y - x)/B for the sigmoid-BCE head: check the decoder-output
    bias gradient equals the column sums of (y - x)/B."""
    cfg = cfg8c()
    B = 6
    P = O.init_params(cfg, seed=1, dtype=np.float64)
    X = (np.random.default_rng(7).random((B, 3 * cfg.D)) < 0.4).astype(np.float64)
    eps = np.random.default_rng(8).standard_normal((3, B, cfg.latent))
    c = O.forward(P, X, eps, cfg)
    O.metric(c, np.ones(B), cfg, B)
    g1, _ = O.backward(c, cfg, B)
    np.testing.assert_allclose(g1["dec_out_mean_b"], ((c["y"] - c["xl"]) / B).sum(0), rtol=1e-12)


@pytest.mark.parametrize("L,logged_deform", [(20, 470.783), (200, 4471.0)])
def test_statistical_step0_magnitudes(L, logged_deform):
    """(iv) at xavier init E[d_l] ~ w * 2L and r_l ~ D ln 2: compare with the step-0
    losses logged by the reference (``8c/nohup.out:27``, ``8d/nohup.out:27``:
    recon 27734.2 / 27749.8, KL 1.72 / 16.0, deform 470.8 / 4471) at the reference's
    own 200x200, B=100 shape, on synthetic binary images (foreground ~5-13%, as the
    reference's overlap_micro PNGs). Statistical, not bitwise: TF's init RNG cannot be
    reproduced."""
    cfg = O.OracleConfig(image_size=200, enc=(500, 500, 500, 500), latent=L)
    B = 100
    rng = np.random.default_rng(11)
    X = (rng.random((B, 3 * cfg.D)) < 0.08).astype(np.float32)
    P = O.init_params(cfg, seed=0, dtype=np.float32)
    eps = np.random.default_rng(12).standard_normal((3, B, L)).astype(np.float32)
    c = O.forward(P, X, eps, cfg, dtype=np.float32)
    r, k, d = c["R"].mean(), c["K"].mean(), c["F"].mean()
    assert abs(r - 27734.2) / 27734.2 < 0.01, r
    assert abs(d - logged_deform) / logged_deform < 0.25, d
    assert 0 < k < 20 * (L / 20), k


def test_kat_bce_saturation_forward_inf_gradient_finite():
    """BCE with no epsilon (``11a/vae.py:266-267``): once the sigmoid rounds to 1.0 on a 0
    pixel, log(pow(1-y, 1-x)) = log(0) and R = +inf (np.isnan(inf) is False, so the
    reference's guard ``11a/main.py:77`` lets the step through). The restatement keeps that
    forward value and the analytic gradient dU = (y - x)/B, which stays finite (TF's pow/log
    chain rule gives NaN there: DESIGN.md §2, "BCE saturation")."""
    cfg = cfg8c(image=4, enc=(8, 8), L=3)
    B = 3
    P = O.init_params(cfg, seed=0, dtype=np.float64)
    P["dec_out_mean_b"][0] = 60.0          # pixel 0: u >= 60 - |d2 Vo| -> y == 1.0 exactly
    X = np.zeros((B, 3 * cfg.D))           # all-zero target at pixel 0
    X[:, 3 * 5] = 1.0
    eps = np.random.default_rng(2).standard_normal((3, B, cfg.latent))
    c = O.forward(P, X, eps, cfg)
    assert np.all(c["y"][:, 0] == 1.0)
    assert np.all(np.isposinf(c["R"]))
    O.metric(c, np.full(B, 500.0), cfg, B)
    losses = O.loss_sums(c, B)
    assert np.isposinf(losses[0]) and np.isposinf(losses[2]) and np.isfinite(losses[1])
    g1, g2 = O.backward(c, cfg, B)
    assert all(np.all(np.isfinite(v)) for v in list(g1.values()) + list(g2.values()))
    np.testing.assert_allclose(g1["dec_out_mean_b"][0], 1.0, rtol=0)  # sum_b (1 - 0)/B
