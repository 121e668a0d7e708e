"""GPU parity for round 5's fused hidden-layer chains (enc_chain.hip): the bf16 encoder's and
decoder's hidden layers in one launch each, activation block resident in LDS, against the float64
oracle at the documented bf16 bar and against the per-layer GEMMs they replace (create options
enc_chain=0 / dec_chain=0)."""
import numpy as np
import pytest
import torch

from magic_amd.config import baseline_config, preset
from tests.gpu_helpers import make_inputs, make_params, to_dev
from tests.test_gpu_parity import check_step

pytestmark = pytest.mark.gpu

BF16 = dict(tol=5e-2, loss_tol=2e-3, dist_tol=2e-2)  # documented bf16 tolerance


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("opts", ["enc_chain=1", "enc_chain=0", "enc_chain_rows=32", "enc_chain_rows=64",
                                  "enc_chain_rows=96", "dec_chain=0", "enc_chain=0,dec_chain=0"])
def test_enc_chain_step_c3_shape(opts):
    """C3's encoder (4 x 500, tanh) at B = 2048: 6144 rows, 16 rows per workgroup (auto), and
    forced 32 / 64 / 96-row blocks (four, three and two weight steps in LDS)."""
    check_step(baseline_config("C3").replace(batch=2048, options=opts), adam=False, **BF16)


@pytest.mark.parametrize("enc,act,batch,latent", [((400, 300, 260), "elu", 100, 16),
                                                  ((500, 500, 500, 500, 300), "tanh", 50, 16),
                                                  ((300, 200, 511), "tanh", 37, 16), ((300, 200, 511), "tanh", 37, 250),
                                                  ((500, 500, 500, 500), "tanh", 64, 255),
                                                  ((500, 500, 500, 500, 300, 200), "elu", 40, 20)])
def test_enc_chain_step_widths(enc, act, batch, latent):
    """Ragged widths (a 511-wide hidden layer: its ones column is the block's last), four fused
    layers, five (no chain), 500 / 510-column latent heads after the chain, elu, and row counts
    that leave the last workgroup's block partly past M."""
    cfg = preset("8d", image_size=24, batch=batch, precision="bf16").replace(enc=enc, act=act, latent=latent)
    check_step(cfg, adam=False, **BF16)


@pytest.mark.parametrize("latent,dec,act,batch", [(200, (500, 500), "tanh", 4096), (16, (400, 300), "elu", 100),
                                                  (31, (511, 200), "tanh", 37), (8, (64, 500), "tanh", 1000)])
def test_dec_chain_step(latent, dec, act, batch):
    """The decoder's two hidden layers in one launch (option dec_chain, default on in bf16 mode):
    C3's decoder, ragged latent / hidden widths (511: the ones column is the block's last), elu,
    and row counts that leave the last workgroup's block partly past B."""
    cfg = preset("8d", image_size=24, batch=batch, precision="bf16").replace(latent=latent, dec=dec, act=act)
    check_step(cfg, adam=False, **BF16)


def _recon(cfg, X):
    from magic_amd.engine import Engine
    eng = Engine(cfg, 0)
    try:
        eng.load_params(make_params(cfg))
        out = eng.reconstruct(to_dev(X))
        torch.cuda.synchronize()
        return out.cpu().numpy().astype(np.float64)
    finally:
        eng.close()


def test_dec_chain_matches_per_layer_gemms():
    """Reconstructions at C3's full shape: the decoder chain against one GEMM per hidden layer
    (the same bf16 arithmetic, another accumulation order)."""
    cfg = baseline_config("C3")
    X, _, _ = make_inputs(cfg, cfg.batch, seed=5)
    a = _recon(cfg.replace(options="dec_chain=1"), X)
    b = _recon(cfg.replace(options="dec_chain=0"), X)
    assert np.all(np.isfinite(a))
    assert np.abs(a - b).max() <= 2e-2


def _means(cfg, X):
    from magic_amd.engine import Engine
    eng = Engine(cfg, 0)
    try:
        eng.load_params(make_params(cfg))
        out = eng.transform(to_dev(X))
        torch.cuda.synchronize()
        return out.cpu().numpy().astype(np.float64)
    finally:
        eng.close()


def test_enc_chain_matches_per_layer_gemms():
    """transform (the encoder's latent means) at C3's full shape (24576 stacked rows, 96 rows
    per workgroup): the chain against one GEMM per layer -- the same bf16 arithmetic in another
    accumulation order, so the means agree to bf16 rounding of the activations."""
    cfg = baseline_config("C3")
    X, _, _ = make_inputs(cfg, cfg.batch, seed=3)
    a = _means(cfg.replace(options="enc_chain=1"), X)
    b = _means(cfg.replace(options="enc_chain=0"), X)
    assert np.all(np.isfinite(a))
    err = np.abs(a - b).max() / max(np.abs(b).max(), 1e-6)
    assert err <= 2e-2, err
