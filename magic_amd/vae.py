"""``TangoEncoder`` — drop-in mirror of the reference class (``11a/vae.py:13-441``,
``8c/vae.py:13-435``) backed by the MI355X HIP step in ``libmvae.so``.

Same constructor entry (``TangoEncoder(sess)``; hyper-parameters via ``config=``), same
methods and return values:

  partial_fit(X, overlap_areas) -> (cost, training_loss, rec_loss, lat_loss, def_loss, distance)
                                   (11a, ``:385-411``; 5-tuple without distance when
                                   ``compat="8c"``, ``8c/vae.py:379-405``)
  get_predictions(X, overlap_areas) -> distance[B]       (``:413-414``)
  transform(X, overlap_areas)       -> z_mean[B, L]      (``:416-420``)
  generate(z_mu=None)               -> x_reconstructed_mean (``:422-434``)
  reconstruct(X, overlap_areas)     -> x_reconstructed_mean[B, D] (``:436-440``)
  cosine_distance (module function)  (``:444-458``) — host-side helper for tests/tools

X is ``[B, H*W*3]`` float32, HWC-interleaved (lock, rotated lock, key) exactly as
``overlap_input.inputs(normalize=True, reshape=True, rotation=True)`` yields it. Inputs may
be numpy arrays (copied host->device, as ``feed_dict`` did) or float32 device tensors
(no copy). Outputs are numpy arrays like ``sess.run`` results.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .config import MVAEConfig, preset
from .constants import FLAGS, metric_name
from .engine import Engine


def _default_config() -> MVAEConfig:
    # 11a/vae.py:30-65 with the FLAGS of 11a/constants.py
    return preset("11a", image_size=FLAGS.IMAGE_SIZE, batch=FLAGS.BATCH_SIZE,
                  metric=metric_name(FLAGS.DISTANCE_METRIC))


class TangoEncoder(object):
    def __init__(self, sess=None, config: Optional[MVAEConfig] = None, device: int = 0,
                 compat: str = "11a", init_seed: int = 0, data_parallel=None,
                 tf_nonfinite: bool = True):
        self.sess = sess  # kept for signature compatibility (11a/vae.py:22)
        cfg = config or _default_config()
        self.config = cfg
        self.encoder_neurons = list(cfg.enc)
        self.decoder_neurons = list(cfg.dec)
        assert len(self.encoder_neurons) > 0
        assert len(self.decoder_neurons) == 2
        self.num_input_neurons = cfg.D * 3
        self.latent_dimensions = cfg.latent
        self.learning_rates = list(cfg.lr)
        self.batch_size = cfg.batch
        self.compat = compat
        self.engine = Engine(cfg, device)
        self.engine.init_params(init_seed)
        self._dp = None
        if data_parallel is not None:
            from .parallel import DataParallelStep
            self._dp = DataParallelStep(self.engine, group=None if data_parallel is True else data_parallel)
        self._losses = torch.empty(5, device=self.engine.dev)
        self._dist = torch.empty(cfg.batch, device=self.engine.dev)
        # Non-finite cost (e.g. BCE saturation: the sigmoid rounds to 1.0 on a 0 pixel, so
        # log(pow(1-y, 1-x)) = log(0) and R = +inf with no epsilon, 11a/vae.py:266-267).
        # TF's gradient of that pow/log chain is NaN (inf * 0), so after such a step every
        # reference parameter is NaN and the NEXT partial_fit returns cost = nan, which the
        # driver's guard turns into TrainingException (11a/main.py:77-78). This build's
        # gradient dU = (y - x)/B stays finite; tf_nonfinite=True reproduces the reference's
        # observable behaviour by reporting NaN losses from the step after a non-finite cost.
        # Only partial_fit is emulated: get_predictions / transform / reconstruct / generate keep
        # running on the (finite) parameters, and load_state_dict clears the flag.
        self.tf_nonfinite = tf_nonfinite
        self._poisoned = False

    # ----------------------------------------------------------------- helpers
    def _dev(self, a, shape):
        dev = self.engine.dev
        if isinstance(a, torch.Tensor):
            t = a.to(device=dev, dtype=torch.float32)
        else:
            t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev, non_blocking=False)
        t = t.reshape(shape).contiguous()
        return t

    def _x(self, X):
        return self._dev(X, (self.batch_size, self.num_input_neurons))

    # ----------------------------------------------------------------- reference API
    def partial_fit(self, X, overlap_areas, eps=None):
        """One training step (both Adam updates). Returns the PRE-update losses."""
        x = self._x(X)
        a = self._dev(overlap_areas, (self.batch_size,))
        e = None if eps is None else self._dev(eps, (3, self.batch_size, self.latent_dimensions))
        if self._poisoned:
            nan = float("nan")
            if self.compat == "8c":
                return nan, nan, nan, nan, nan
            return nan, nan, nan, nan, nan, np.full(self.batch_size, np.nan, np.float32)
        if self._dp is None:
            self.engine.train_step(x, a, e, losses_out=self._losses, dist_out=self._dist)
            losses = self._losses
        else:
            losses = self._dp.step(x, a, e)
            self._dist.copy_(self.engine.dist)
        l = losses.cpu().numpy().astype(np.float64)
        cost, training_loss, rec_loss, lat_loss, def_loss = (float(v) for v in l[:5])
        if self.tf_nonfinite and not np.isfinite(cost):
            self._poisoned = True
        if self.compat == "8c":
            return cost, training_loss, rec_loss, lat_loss, def_loss
        return cost, training_loss, rec_loss, lat_loss, def_loss, self._dist.cpu().numpy()

    def get_predictions(self, X, overlap_areas=None, eps=None):
        e = None if eps is None else self._dev(eps, (3, self.batch_size, self.latent_dimensions))
        if self._dp is not None:  # cosine column norms over the global batch
            return self._dp.predict(self._x(X), e).cpu().numpy()
        return self.engine.predict(self._x(X), e).cpu().numpy()

    def transform(self, X, overlap_areas=None):
        return self.engine.transform(self._x(X)).cpu().numpy()

    def generate(self, z_mu=None):
        if z_mu is None:
            z_mu = np.random.normal(size=self.latent_dimensions)
        z = self._dev(z_mu, (-1, self.latent_dimensions))
        return self.engine.generate(z).cpu().numpy()

    def reconstruct(self, X, overlap_areas=None, eps=None):
        e = None if eps is None else self._dev(eps, (3, self.batch_size, self.latent_dimensions))
        return self.engine.reconstruct(self._x(X), e).cpu().numpy()

    # ----------------------------------------------------------------- extras
    def parameters(self):
        """Name -> torch view of the device parameters (reference variable meanings)."""
        return self.engine.params()

    def state_dict(self):
        out = {f"param/{k}": v.detach().cpu().clone() for k, v in self.engine.params().items()}
        for kind, tag in ((3, "m1"), (4, "v1"), (5, "m2"), (6, "v2")):
            for k, v in self.engine.tensors(kind).items():
                out[f"{tag}/{k}"] = v.detach().cpu().clone()
        t1, t2 = self.engine.get_step()
        out["step"] = torch.tensor([t1, t2])
        out["rng"] = torch.tensor(list(self.engine.get_rng()), dtype=torch.int64)
        return out

    def load_state_dict(self, sd):
        views = {3: "m1", 4: "v1", 5: "m2", 6: "v2"}
        for k, v in self.engine.params().items():
            v.copy_(sd[f"param/{k}"].to(v.device))
        for kind, tag in views.items():
            for k, v in self.engine.tensors(kind).items():
                v.copy_(sd[f"{tag}/{k}"].to(v.device))
        t1, t2 = (int(x) for x in sd["step"])
        self.engine.set_step(t1, t2)
        if "rng" in sd:
            self.engine.set_rng(*(int(x) for x in sd["rng"]))
        self.engine.sync_params()
        torch.cuda.synchronize(self.engine.dev)
        self._poisoned = False  # restored parameters are finite again

    def close(self):
        self.engine.close()


def sample_latent_space(vae, nx: int = 20, ny: int = 20, lo: float = -3.0, hi: float = 3.0):
    """The 2-D latent-space sampling grid of ``11a/utils.py:401-422`` as an array (the reference
    plots it to a PNG; plotting is out of scope): tile (nx - i - 1, j) = ``vae.generate`` of
    z = (w[j], v[i]) with v = linspace(lo, hi, nx), w = linspace(lo, hi, ny), as the reference's
    loop over ``yi in x_values`` / ``xi in y_values`` places it, so the canvas is nx tiles tall
    and ny tiles wide, (nx*S) x (ny*S) for image side S (the reference hard-codes nx = ny = 20,
    where its (ny*S) x (nx*S) canvas is the same shape). The reference runs one
    ``generate`` per grid point on a batch of identical rows and keeps row 0; here the grid points
    are the rows of ``ceil(nx*ny / batch_size)`` batched ``generate`` calls. Returns None unless
    the latent space is 2-D (the reference prints a message instead).
    """
    if vae.latent_dimensions != 2:
        return None
    x_values = np.linspace(lo, hi, nx)
    y_values = np.linspace(lo, hi, ny)
    z = np.array([[xi, yi] for yi in x_values for xi in y_values], dtype=np.float32)
    rows = []
    for s0 in range(0, len(z), vae.batch_size):
        rows.append(np.asarray(vae.generate(z[s0:s0 + vae.batch_size])))
    imgs = np.concatenate(rows, axis=0)
    side = int(round(np.sqrt(imgs.shape[1])))
    canvas = np.empty((side * nx, side * ny), dtype=imgs.dtype)
    for i in range(len(x_values)):
        for j in range(len(y_values)):
            canvas[(nx - i - 1) * side:(nx - i) * side, j * side:(j + 1) * side] = \
                imgs[i * len(y_values) + j].reshape(side, side)
    return canvas


def cosine_distance(a, b):
    """``11a/vae.py:444-458``: l2-normalise along axis 0 (the batch axis), then the row-wise
    dot product. Host helper (numpy) for tools and tests; the step computes this in HIP."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    na = a / np.sqrt(np.maximum((a * a).sum(0, keepdims=True), np.float32(1e-12)))
    nb = b / np.sqrt(np.maximum((b * b).sum(0, keepdims=True), np.float32(1e-12)))
    return (na * nb).sum(1)
