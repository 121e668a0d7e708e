"""magic_amd — MI355X (gfx950) native training step of the "magic" asymmetric metric-VAE
(reference: ag8/magic ``TangoEncoder``), hand-written HIP kernels behind a C ABI
(``include/mvae.h``), with the reference's Python call surface on top.

  magic_amd.vae.TangoEncoder      reference class mirror (partial_fit, get_predictions, ...)
  magic_amd.overlap_input.inputs  batch producer, reference layout [B, H*W*3]
  magic_amd.engine.Engine         low-level context (phases, device views)
  magic_amd.parallel              data-parallel step (torch.distributed / RCCL)
"""
from .config import MVAEConfig, PRESETS, baseline_config, preset  # noqa: F401

__version__ = "0.1.0"
