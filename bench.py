#!/usr/bin/env python3
"""Benchmark: training steps of the "magic" metric-VAE (``TangoEncoder.partial_fit``,
reference ``11a/vae.py:385-411``) on MI355X through libmvae's HIP kernels.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]
  N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step = one pass of the hot path over one batch of synthetic 100x100 shape pairs already
resident in HBM: de-interleave, eps sampling, 3 encoder passes, decoder, five-loss head,
both gradients, (N>1: RCCL all-reduces), both Adam updates. Weak scaling: the per-GPU batch
is fixed; ``value`` = pairs processed by ALL ranks / max-over-ranks wall time.

Rank 0 prints ONE JSON line. Extra diagnostics (per-region HIP-event timings) go to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from magic_amd import _lib  # noqa: E402
from magic_amd.config import baseline_config  # noqa: E402

METRIC = "shape-pairs/sec/GPU (train step) + overlap-MSE, 100×100 pairs, 1/2/4/8 GPUs"
F32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (exact fp32)
BF16_MFMA_PEAK_TFLOPS = 2500.0   # dense
HBM_PEAK_GBS = 8000.0


def region_flops(cfg, name: str) -> float:
    """Algorithmic FLOPs of one launch of a timed GEMM region (2*M*N*K, K = fan-in)."""
    B, D, L = cfg.batch, cfg.D, cfg.latent
    widths = [D] + list(cfg.enc)
    e, (d0, d1) = cfg.enc[-1], cfg.dec
    if name.startswith("enc_fwd_"):
        i = int(name.rsplit("_", 1)[1])
        return 2.0 * 3 * B * widths[i] * widths[i + 1]
    if name.startswith("enc_bwd_w_"):
        i = int(name.rsplit("_", 1)[1])
        return 2 * 2.0 * 2 * B * widths[i] * widths[i + 1]
    if name.startswith("enc_bwd_d_"):
        i = int(name.rsplit("_", 1)[1])
        return 2.0 * 4 * B * widths[i] * widths[i + 1]
    table = {
        "head_fwd": 2.0 * 3 * B * e * 2 * L,
        "dec_fwd_1": 2.0 * B * L * d0, "dec_fwd_2": 2.0 * B * d0 * d1,
        "dec_fwd_out_bce": 2.0 * B * d1 * D,
        "dec_bwd_w_out": 2.0 * B * d1 * D, "dec_bwd_d_out": 2.0 * B * D * d1,
        "dec_bwd_w_2": 2.0 * B * d0 * d1, "dec_bwd_d_2": 2.0 * B * d0 * d1,
        "dec_bwd_w_1": 2.0 * B * L * d0, "dec_bwd_d_z": 2.0 * B * d0 * L,
        "head_bwd_w": 2 * 2.0 * 2 * B * e * 2 * L, "head_bwd_d": 2.0 * 4 * B * 2 * L * e,
    }
    return table.get(name, 0.0)


def cpu_baseline(cfg, seconds: float):
    """The oracle (CPU restatement, numpy fp32 + BLAS) timed on this host on a bounded
    sample of the same workload: C2 widths, a 256-pair batch, >= 2 steps, ~`seconds`."""
    from oracle import mvae_oracle as O
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    oc = O.OracleConfig(image_size=cfg.image_size, enc=tuple(cfg.enc), dec=tuple(cfg.dec),
                        latent=cfg.latent, act=cfg.act, deform_weight=cfg.deform_weight,
                        metric=cfg.metric, reciprocal=cfg.reciprocal, lr=tuple(cfg.lr))
    Bc = 256
    rng = np.random.default_rng(1)
    X = (rng.random((Bc, 3 * cfg.D)) < 0.08).astype(np.float32)
    areas = rng.integers(296, 6427, Bc).astype(np.float32)
    P = O.init_params(oc, seed=0, dtype=np.float32)
    st = O.adam_init(oc, P)
    eps = rng.standard_normal((3, Bc, cfg.latent)).astype(np.float32)
    O.train_step(P, st, X, areas, eps, oc, dtype=np.float32)  # warm-up
    t0 = time.perf_counter()
    n = 0
    while n < 2 or time.perf_counter() - t0 < seconds:
        _, _, P, st, _ = O.train_step(P, st, X, areas, eps, oc, dtype=np.float32)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * Bc / dt, 2), "unit": "shape-pairs/s", "cores": int(cores),
            "kind": "port",
            "sample": f"oracle/mvae_oracle.py train_step, numpy float32 + OpenBLAS, {n} steps x "
                      f"{Bc} pairs of the {cfg.image_size}x{cfg.image_size} {len(cfg.enc)}x{cfg.enc[0]} "
                      f"L={cfg.latent} step, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2", help="BASELINE config id (C2 fp32 B=4096 default)")
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch")
    ap.add_argument("--precision", default="", help="override GEMM arithmetic: f32 | f32x | bf16")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="disable per-region HIP events")
    ap.add_argument("--region-steps", type=int, default=10,
                    help="extra steps with every region timed (per-kernel table, dominant GEMM)")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from magic_amd.engine import Engine
    from magic_amd.overlap_input import synthetic_batch
    from magic_amd.parallel import DataParallelStep

    cfg = baseline_config(args.config)
    if args.batch:
        cfg = cfg.replace(batch=args.batch)
    if args.precision:
        cfg = cfg.replace(precision=args.precision)
    cfg = cfg.replace(global_batch=cfg.batch * world, seed=1000 + rank)
    eng = Engine(cfg, local)
    eng.init_params(0)  # identical replicas on every rank
    stepper = DataParallelStep(eng, reduce_losses=True)

    # synthetic inputs resident in HBM: a pool of 2 batches cycled through the steps
    pool = [synthetic_batch(cfg.batch, cfg.image_size, seed=17 + 101 * rank + j, device=dev)
            for j in range(2)]
    torch.cuda.synchronize()

    for i in range(args.warmup):
        x, a = pool[i % 2]
        stepper.step(x, a)
    torch.cuda.synchronize()
    regions = {}
    dom = None
    if not args.no_timing:
        # region pass (outside the timed loop): HIP events around every region, for the
        # per-kernel table and to pick the dominant GEMM
        eng.timing_reset()
        eng.timing_enable(True)
        for i in range(args.region_steps):
            x, a = pool[i % 2]
            stepper.step(x, a)
        torch.cuda.synchronize()
        eng.timing_enable(False)
        regions = eng.timing_read()
        gemms = {k: v for k, v in regions.items() if region_flops(cfg, k) > 0}
        dom = max(gemms, key=lambda k: gemms[k][0])
        # timed loop: events around the dominant GEMM only (one pair per step)
        eng.timing_reset()
        eng.timing_select(dom)
        eng.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        x, a = pool[i % 2]
        stepper.step(x, a)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    eng.timing_enable(False)
    dom_timed = eng.timing_read().get(dom) if dom else None
    eng.timing_select(None)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    losses = eng.losses.cpu().numpy().tolist()
    if not np.all(np.isfinite(losses)):
        raise RuntimeError(f"non-finite losses after the timed steps: {losses}")

    # overlap-MSE on a held-out seeded batch (11a/main.py:94-111; 1/pred for reciprocal)
    xe, ae = synthetic_batch(cfg.batch, cfg.image_size, seed=999, device=dev)
    pred = eng.predict(xe).double()
    if cfg.reciprocal:
        pred = 1.0 / pred
    mse = float(((pred - ae.double()) ** 2).mean().item())

    if rank == 0:
        pairs = cfg.batch * world * args.steps
        value = pairs / elapsed
        roofline = None
        if regions and dom_timed:
            gemms = {k: v for k, v in regions.items() if region_flops(cfg, k) > 0}
            ms_avg = dom_timed[0] / dom_timed[1]  # HIP events over the timed loop
            flops = region_flops(cfg, dom)
            achieved = flops / (ms_avg * 1e-3) / 1e12
            peak = BF16_MFMA_PEAK_TFLOPS if cfg.precision == "bf16" else F32_MFMA_PEAK_TFLOPS
            extra = {}
            if cfg.precision == "f32x":
                # the exact 3-term split runs the plane pairs (i, j), i + j < 3, as bf16 MFMA
                # work: 6 pairs, or 3 when the A operand (the pixels) is exact in bf16. Its
                # algorithm's FLOPs are pairs x 2MNK at the bf16 peak; the fp32-equivalent
                # rate (2MNK / time) is reported beside it.
                dyn = int(eng.buffer(_lib.BUF_DYN).view(torch.int32).item())
                pairs = 3 if dom in ("enc_fwd_0", "enc_bwd_w_0") and dyn == 0 else 6
                extra = {"fp32_equivalent_tflops": round(achieved, 2), "bf16_plane_pairs": pairs}
                achieved *= pairs
                flops *= pairs
                peak = BF16_MFMA_PEAK_TFLOPS
            traffic = None
            try:
                with open(args.traffic_json) as f:
                    tj = json.load(f)
                if (tj.get("config") == args.config and tj.get("precision") == cfg.precision
                        and dom in tj.get("regions", {})):
                    traffic = tj["regions"][dom]["hbm_bytes_per_launch"]
            except (OSError, ValueError):
                pass
            roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                        "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                        "kernel": dom, "flops_per_launch": flops, "avg_ms": round(ms_avg, 4), **extra}
            rs = args.region_steps
            total_gemm_ms = sum(v[0] for v in gemms.values()) / rs
            gemm_flops = sum(region_flops(cfg, k) * v[1] for k, v in gemms.items()) / rs
            print(f"[bench] region pass ({rs} steps): GEMM time/step {total_gemm_ms:.3f} ms, "
                  f"{gemm_flops / total_gemm_ms / 1e9:.1f} TFLOP/s over all GEMMs; timed step "
                  f"{elapsed / args.steps * 1e3:.3f} ms; {dom} {ms_avg:.4f} ms in the timed loop",
                  file=sys.stderr)
            for k, (ms, n) in sorted(regions.items(), key=lambda kv: -kv[1][0]):
                fl = region_flops(cfg, k)
                extra = f"  {fl / (ms / n * 1e-3) / 1e12:7.1f} TF/s" if fl else ""
                print(f"[bench] {k:18s} {ms / n:9.4f} ms x{n}{extra}", file=sys.stderr)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(cfg, args.cpu_seconds)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "shape-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"f32": "f32", "f32x": "f32 (exact 3-term bf16 split MFMA, fp32 accumulate)",
                      "bf16": "bf16 GEMM operands, fp32 accumulate"}[cfg.precision],
            "data": "synthetic 100x100 binary shape pairs (random ellipses/rectangles, nearest-"
                    "neighbour rotated lock), areas resampled from the reference's OVERLAP_AREAS; "
                    "random xavier init",
            "config": {"workload": f"BASELINE {args.config}: preset "
                                   f"{'8c' if cfg.latent == 20 else '8d/8e'} enc {list(cfg.enc)} "
                                   f"L={cfg.latent} {cfg.act} {cfg.metric}",
                       "global_batch": cfg.batch * world, "per_gpu_batch": cfg.batch,
                       "image": f"{cfg.image_size}x{cfg.image_size}", "parallelism": f"dp{world}"},
            "per_gpu_value": round(value / world, 2),
            "overlap_mse": round(mse, 2),
            "losses": {"cost": losses[0], "training_loss": losses[1], "r_l": losses[2],
                       "l_l": losses[3], "d_l": losses[4]},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
