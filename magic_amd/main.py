"""Training driver — mirror of ``11a/main.py:42-133`` and of the 8c variant ``8c/main.py:33-94``
on the HIP step. No HTTP "poor man's tensorboard" (``11a/utils.py:256-266``) and no plots.

  python -m magic_amd.main --preset 8c --image-size 100 --batch 4096 --epochs 2

The two reference drivers differ in four ways, all reproduced (``driver=``):

  =============  ===========================================  ================================
                 11a (``11a/main.py``)                         8c (``8c/main.py``)
  =============  ===========================================  ================================
  eval cadence   ``epoch % 10 == 0 and i == 3`` (:93)          ``i % 24 == 0`` (:66)
  eval fetch     images + labels of ONE dequeue (:94)          two dequeues: images and labels
                                                               do not match (:67-68)
  predictions    ``1. / predictions`` (:100)                   as returned (:69)
  epoch log      average cost and average loss (:121-126)      average cost every 5th epoch
                                                               (:84,87-89)
  =============  ===========================================  ================================

Both raise ``TrainingException("Got cost=nan")`` when ``partial_fit`` returns a NaN cost
(11a :77-78, 8c :51-52) and swallow ``KeyboardInterrupt`` (11a :130-131, 8c :91-92).
"""
from __future__ import annotations

import argparse
import sys
import time

import numpy as np

from . import overlap_input
from .config import preset
from .constants import FLAGS


class TrainingException(Exception):
    """``11a/excps.py:3-4`` (``8c/main.py:29-30``)."""


DRIVERS = {
    # eval predicate (epoch, i), paired eval fetch, invert predictions, log both averages
    "11a": dict(eval_at=lambda epoch, i: epoch % 10 == 0 and i == 3, paired=True, invert=True),
    "8c": dict(eval_at=lambda epoch, i: i % 24 == 0, paired=False, invert=False),
}


def _host(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def train(vae, batches, n_samples: int, training_epochs: int = 60, driver: str = "11a",
          invert=None, paired_eval=None, eval_at=None, display_step: int = 5, log=print):
    """Run the reference training loop. ``batches`` yields (images, labels) like the
    reference's ``sess.run([images_batch, labels_batch])``.

    invert: ``1/pred`` before the MSE; default: the driver's choice for a reciprocal model
    (11a inverts because its distance is the reciprocal, ``11a/vae.py:307,309``; a model
    without the reciprocal is never inverted). Returns (vae, history): history holds
    ("mse", epoch, i, mse) and ("epoch", epoch, avg_cost, avg_loss) records."""
    d = DRIVERS[driver]
    eval_at = eval_at or d["eval_at"]
    paired = d["paired"] if paired_eval is None else paired_eval
    if invert is None:
        invert = d["invert"] and bool(getattr(vae.config, "reciprocal", True))
    batch_size = vae.batch_size
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
                if eval_at(epoch, i):
                    test_x, test_a = next(batches)
                    if not paired:
                        _, test_a = next(batches)  # 8c: a second dequeue for the labels
                    pred = np.asarray(vae.get_predictions(test_x, test_a), np.float64)
                    if invert:
                        pred = 1.0 / pred
                    mse = float(((pred - _host(test_a).astype(np.float64)) ** 2).mean())
                    log(f"mse: {mse}")
                    history.append(("mse", epoch, i, mse))
                avg_cost += cost / n_samples * batch_size
                avg_loss += training_loss / n_samples * batch_size
            if driver == "8c":
                if epoch % display_step == 0:
                    log(f"Epoch: {epoch + 1:04d} cost= {avg_cost:.9f}")
            else:
                log(f"Epoch: {epoch}".ljust(20) + f"Average cost: {int(avg_cost)}".ljust(35)
                    + f"Average loss: {int(avg_loss)}".ljust(35))
            history.append(("epoch", epoch, avg_cost, avg_loss))
    except KeyboardInterrupt:
        pass
    return vae, history


def main(argv=None):
    from .vae import TangoEncoder
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="11a")
    ap.add_argument("--image-size", type=int, default=FLAGS.IMAGE_SIZE)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--data", default=None, help="dir/.zip of {N}_L.png/{N}_K.png or a packed .npz "
                                                 "(default: synthetic shapes)")
    ap.add_argument("--samples-per-epoch", type=int, default=FLAGS.NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN)
    ap.add_argument("--driver", choices=sorted(DRIVERS), default=None,
                    help="reference driver semantics (default: 8c for the 8c-family presets)")
    args = ap.parse_args(argv)
    cfg = preset(args.preset, image_size=args.image_size, batch=args.batch or None)
    eight_c = args.preset in ("8c", "8d", "8e", "8f")
    driver = args.driver or ("8c" if eight_c else "11a")
    vae = TangoEncoder(None, config=cfg, compat="8c" if eight_c else "11a")
    batches = overlap_input.inputs(normalize=True, reshape=True, rotation=True, batch_size=cfg.batch,
                                   image_size=cfg.image_size, data_dir=args.data)
    t0 = time.time()
    train(vae, batches, max(args.samples_per_epoch, cfg.batch), args.epochs, driver=driver)
    print(f"done in {time.time() - t0:.1f}s", file=sys.stderr)
    vae.close()


if __name__ == "__main__":
    main()
