"""Training driver — mirror of ``11a/main.py:42-133`` (and the 8c variant ``8c/main.py:33-94``)
on the HIP step. No HTTP "poor man's tensorboard" (``11a/utils.py:256-266``) and no plots.

  python -m magic_amd.main --preset 8c --image-size 100 --batch 4096 --epochs 2
"""
from __future__ import annotations

import argparse
import sys
import time

import numpy as np

from . import overlap_input
from .config import preset
from .constants import FLAGS
from .vae import TangoEncoder


class TrainingException(Exception):
    """``11a/excps.py:3-4``."""


def train(vae: TangoEncoder, batches, n_samples: int, training_epochs: int = 60,
          eval_every_epochs: int = 10, eval_step: int = 3, paired_eval: bool = True,
          log=print):
    """``11a/main.py:42-133``: per-step ``partial_fit``, NaN guard, overlap-MSE eval at
    (epoch % 10 == 0, i == 3) on a fresh batch, epoch averages. With
    ``paired_eval=False`` the eval images and labels come from two different draws, as
    ``8c/main.py:44-45,67-68`` fetched them (reproduces the README's MSE setting)."""
    batch_size = vae.batch_size
    invert = vae.config.reciprocal
    history = []
    try:
        for epoch in range(training_epochs):
            avg_cost = 0.0
            avg_loss = 0.0
            total_batch = int(n_samples / batch_size)
            for i in range(total_batch):
                batch_xs, overlap_areas = next(batches)
                out = vae.partial_fit(batch_xs, overlap_areas)
                cost, training_loss = out[0], out[1]
                if np.isnan(cost):
                    raise TrainingException("Got cost=nan")
                if epoch % eval_every_epochs == 0 and i == eval_step:
                    test_x, test_a = next(batches)
                    if not paired_eval:
                        _, test_a = next(batches)
                    pred = vae.get_predictions(test_x, test_a)
                    if invert:
                        pred = 1.0 / pred  # 11a/main.py:100
                    a = test_a.cpu().numpy() if hasattr(test_a, "cpu") else np.asarray(test_a)
                    mse = float(((np.asarray(pred, np.float64) - a) ** 2).mean())
                    log(f"mse: {mse}")
                    history.append(("mse", epoch, mse))
                avg_cost += cost / n_samples * batch_size
                avg_loss += training_loss / n_samples * batch_size
            log(f"Epoch: {epoch}".ljust(20) + f"Average cost: {int(avg_cost)}".ljust(35)
                + f"Average loss: {int(avg_loss)}".ljust(35))
            history.append(("epoch", epoch, avg_cost, avg_loss))
    except KeyboardInterrupt:
        pass
    return vae, history


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="11a")
    ap.add_argument("--image-size", type=int, default=FLAGS.IMAGE_SIZE)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--data", default=None, help="dir/.zip of {N}_L.png/{N}_K.png (default synthetic)")
    ap.add_argument("--samples-per-epoch", type=int, default=FLAGS.NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN)
    ap.add_argument("--unpaired-eval", action="store_true", help="8c driver semantics")
    args = ap.parse_args(argv)
    cfg = preset(args.preset, image_size=args.image_size, batch=args.batch or None)
    vae = TangoEncoder(None, config=cfg, compat="8c" if args.preset in ("8c", "8d", "8e", "8f") else "11a")
    batches = overlap_input.inputs(normalize=True, reshape=True, rotation=True, batch_size=cfg.batch,
                                   image_size=cfg.image_size, data_dir=args.data)
    t0 = time.time()
    train(vae, batches, max(args.samples_per_epoch, cfg.batch), args.epochs,
          paired_eval=not args.unpaired_eval)
    print(f"done in {time.time() - t0:.1f}s", file=sys.stderr)
    vae.close()


if __name__ == "__main__":
    main()
