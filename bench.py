#!/usr/bin/env python3
"""Benchmark: training steps of the "magic" metric-VAE (``TangoEncoder.partial_fit``,
reference ``11a/vae.py:385-411``) on MI355X through libmvae's HIP kernels.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]

``--gpus N`` with N > 1 and no torchrun environment starts N local ranks itself
(``torch.distributed.run``, one process per GPU, RCCL); under torchrun it is one of them.

A step = one pass of the hot path over one batch of synthetic 100x100 shape pairs already
resident in HBM: de-interleave, eps sampling, 3 encoder passes, decoder, five-loss head,
both gradients, (N > 1: RCCL all-reduces), both Adam updates. Weak scaling: the per-GPU
batch is fixed; ``value`` = pairs processed by ALL ranks / max-over-ranks wall time.

Rank 0 prints ONE JSON line; per-region HIP-event timings go to stderr. Besides the
contract's fields the line carries:
  roofline       the dominant GEMM: algorithmic FLOPs (2*M*N*K once) / its
                 mean HIP-event duration in the timed loop, against the dense MFMA peak of
                 the arithmetic it runs on; f32x (fp32-accurate bf16 plane split) adds
                 mfma_pipe_frac = plane-pair bf16 work / time / bf16 peak. traffic = HBM
                 bytes per step of that region (its launches: the layer-0 weight gradient runs
                 as 2 row chunks under the early Adam) from rocprofv3 FETCH_SIZE / WRITE_SIZE
                 passes run by this process (child runs, marker-bracketed, MI355X_MICROARCH.md
                 §HBM); achieved and avg_ms are per step as well.
  loss_roofline  the HBM-bound kernels (de-interleave, sampler, latent head, metric, Adam)
                 and the BCE epilogue: algorithmic bytes per launch / time vs 8 TB/s.
  cpu_baseline   the CPU restatement (oracle, numpy fp32 + BLAS) on this host: the
                 GPU-batch workload with all threads, C1 (B=64) with all threads and with 1
                 thread, and the in-run parity of the GPU C1 step against it.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "shape-pairs/sec/GPU (train step) + overlap-MSE, 100×100 pairs, 1/2/4/8 GPUs"
F32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 (exact fp32)
BF16_MFMA_PEAK_TFLOPS = 2500.0   # dense
HBM_PEAK_GBS = 8000.0
PMC_REGIONS_BW = ("deinterleave", "deint_fwd0", "latent_bwd", "adam")
# the layer-0 pair and the decoder-output trio: HBM traffic and the MFMA-busy fraction per region
PMC_REGIONS_MFMA = ("enc_fwd_0", "enc_bwd_w_0", "dec_fwd_out_bce", "dec_bwd_d_out", "dec_bwd_w_out")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2", help="BASELINE config id (C2 fp32 B=4096 default)")
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch")
    ap.add_argument("--precision", default="", help="override GEMM arithmetic: f32 | f32x | bf16")
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="per CPU-baseline timing leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="disable per-region HIP events")
    ap.add_argument("--region-steps", type=int, default=10,
                    help="extra steps with every region timed (per-kernel table, dominant GEMM)")
    ap.add_argument("--pmc", default="auto", choices=["auto", "off"],
                    help="rocprofv3 FETCH_SIZE/WRITE_SIZE child passes for roofline.traffic")
    ap.add_argument("--pmc-child", default="", help=argparse.SUPPRESS)
    ap.add_argument("--opt", action="append", default=[],
                    help="libmvae schedule switch NAME=VALUE (mvae_set_option), repeatable")
    ap.add_argument("--create-opt", action="append", default=[],
                    help="libmvae plan-time kernel switch NAME=VALUE (mvae_create_ex), repeatable")
    ap.add_argument("--mark-dominant", action="store_true",
                    help="profiler runs: marker kernels around the dominant GEMM region's launches in "
                         "the timed loop, so a kernel trace attributes them (tools/timed_steps.py)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the configs block (C3 / C5 on one GPU; C4 / C5 with N ranks)")
    ap.add_argument("--no-h2d", action="store_true", help="skip the PCIe-inclusive h2d leg")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip the input-pipeline leg (inputs() -> HIP batch producer -> step)")
    ap.add_argument("--plan", action="store_true",
                    help="print the per-rank plan of a --gpus N run (configs, batches, collectives) "
                         "as one JSON line and exit: no ranks, no GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launcher / data-parallel / timing / JSON path "
                         "(gloo, a stand-in engine; no GPU, no kernels, not a measurement)")
    args = ap.parse_args(argv)
    if args.region_steps < 1:
        ap.error("--region-steps must be >= 1 (the roofline's dominant kernel comes from the region pass)")
    return args


# ------------------------------------------------------------------------ launcher
def self_launch(args, argv) -> int:
    """N > 1 without a torchrun environment: start N local ranks (one process per GPU) as a
    child torch.distributed.run before this process touches the GPU, and exit with its code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


# ------------------------------------------------------------------------ work models
def region_flops(cfg, name: str) -> float:
    """Algorithmic FLOPs of one launch of a timed GEMM region (2*M*N*K, K = fan-in)."""
    B, D, L = cfg.batch, cfg.D, cfg.latent
    S1 = cfg.image_size // 2
    F0 = (S1 // 2) ** 2 * 64 if cfg.conv else D   # layer-0 fan-in: pixels or tower features
    widths = [F0] + list(cfg.enc)
    e, (d0, d1) = cfg.enc[-1], cfg.dec
    if cfg.conv:  # the 5x5x64x64 conv as an implicit GEMM (K = 25 taps x 64 channels)
        conv2 = 2.0 * S1 * S1 * 1600 * 64
        if name == "conv2_fwd":
            return 3 * B * conv2
        if name in ("conv2_dgrad", "conv2_wgrad"):
            return 4 * B * conv2
    if name == "deint_fwd0":  # the de-interleave's workers inside the layer-0 forward's launch
        name = "enc_fwd_0"
    if name == "enc_fwd_chain":  # the hidden layers 1 .. n-1 in one launch
        return sum(2.0 * 3 * B * widths[i] * widths[i + 1] for i in range(1, len(cfg.enc)))
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
        "dec_fwd_chain": 2.0 * B * L * d0 + 2.0 * B * d0 * d1,  # both hidden layers, one launch
        "dec_fwd_out_bce": 2.0 * B * d1 * D,
        "dec_bwd_w_out": 2.0 * B * d1 * D, "dec_bwd_d_out": 2.0 * B * D * d1,
        "dec_bwd_w_2": 2.0 * B * d0 * d1, "dec_bwd_d_2": 2.0 * B * d0 * d1,
        "dec_bwd_w_1": 2.0 * B * L * d0, "dec_bwd_d_z": 2.0 * B * d0 * L,
        "head_bwd_w": 2 * 2.0 * 2 * B * e * 2 * L, "head_bwd_d": 2.0 * 4 * B * 2 * L * e,
    }
    return table.get(name, 0.0)


def plane_pairs(cfg, name: str, exact_pixels: bool) -> int:
    """bf16 MFMA products per fp32 product in the f32x split: 6 plane pairs (i + j < 3), 3 when
    the A operand is the exact binary pixel operand (layer 0)."""
    return 3 if name in ("enc_fwd_0", "enc_bwd_w_0") and exact_pixels else 6


def bits_on(cfg) -> bool:
    """The library's bits path for the layer-0 pixel operand (create option bits, default on):
    plane modes, FC encoder, 64-row batch blocks, whole 8-pixel groups."""
    return (cfg.precision in ("bf16", "f32x") and not cfg.conv and cfg.batch % 64 == 0
            and cfg.D % 8 == 0 and "bits=0" not in (getattr(cfg, "options", "") or ""))


def region_bytes(cfg, name: str) -> float:
    """Algorithmic HBM bytes per launch of a bandwidth-bound region: every operand read once and
    every output written once at its stored width (fp32 = 4 B; bf16 plane images = 2 B per plane,
    np planes per value: 0 in f32 mode, 1 bf16, 3 f32x). Counts follow the kernels' inputs and
    outputs in magic_amd/csrc/mvae_kernels.hip; the per-pair latent-head figure of SURVEY.md §8d
    (~80 L B/pair, the minimum of a fully fused head) is reported beside them."""
    B, D, L = cfg.batch, cfg.D, cfg.latent
    np_ = {"f32": 0, "bf16": 1, "f32x": 3}[cfg.precision]
    BL = B * L
    if name == "deinterleave":  # fp32 X read; bf16 plane 0 of 3 blocks (plane modes) or fp32 xs
        if bits_on(cfg):  # ... or the two BitMats (3 bits per pixel each) and the target's bits
            return B * D * (12.0 + 7.0 / 8.0)
        return B * D * (12.0 + (6.0 if np_ else 12.0))
    if name == "eps_rng":       # caller-given eps copied once (internal draws: no kernel)
        return 3 * BL * 8.0
    # the fused latent head (magic_amd/csrc/mvae_kernels.hip): eps regenerated from the Philox
    # stream inside the kernels, z recomputed in the backward instead of stored and re-read
    cos = cfg.metric == "cosine"
    zl = 2.0 * np_ if (np_ and L >= 64) else 4.0   # lock z in the decoder GEMMs' operand format
    if name == "latent_fwd":    # mu, s of 3 passes in; lock z (+ fp32 lock/key rows: cosine), row sums out
        return 3 * BL * 8.0 + BL * (8.0 if cos else zl) + B * 16.0
    if name == "colsq":
        return 2 * BL * 4.0
    if name == "metric_loss":   # row sums, BCE row partials, areas (+ cosine: lock/key rows); 3 row values out
        nblk = (D + 127) // 128
        return B * (16.0 + 4.0 * nblk + 4.0 + 12.0) + (2 * BL * 4.0 if cos else 0.0)
    if name == "coldot":
        return 2 * BL * 4.0 + B * 4.0
    if name == "latent_bwd":    # mu, s of 3 passes + dz_dec in; dhead (4 rows x 2L) out
        # (fp32 dhead rows only when a native-fp32 head GEMM reads them: f32 mode, or 2L < 256)
        d32 = 4.0 if (np_ == 0 or 2 * L < 256) else 0.0
        return BL * (24.0 + 4.0) + 4 * BL * 2 * (d32 + 2.0 * np_)
    if cfg.conv:  # the conv tower's per-pixel kernels (magic_amd/csrc/conv_tower.hip)
        S1 = cfg.image_size // 2
        A1 = S1 * S1 * 64.0                # elements of one image after pool 1
        F = (S1 // 2) ** 2 * 64.0          # tower features
        mf = cfg.precision == "bf16"    # MFMA conv: bf16 n1 / d a2 images instead of fp32
        if name == "conv1_fwd":         # pixels in; p1, arg1, n1 (fp32 or bf16) out
            return 3 * B * (D * 4.0 + A1 * (5.0 + (2.0 if mf else 4.0)))
        if name == "lrn2_pool2_fwd":    # a2 in; features (fp32 and/or planes) + arg2 out
            return 3 * B * (A1 * 4.0 + F * (4.0 + 2.0 * np_ + 1.0))
        if name == "pool2_bwd":         # dxf, arg2, a2 in; d a2 (fp32 or bf16) out, per backward image
            return 4 * B * (F * 5.0 + A1 * (4.0 + (2.0 if mf else 4.0)))
        if name == "conv1_wgrad":       # d n1, p1, arg1, pixels in (LRN-1 backward fused)
            return 4 * B * (A1 * 9.0 + D * 4.0)
    return 0.0


def adam_bytes(n_all: int, n_enc: int, np_: int) -> float:
    """Fused dual Adam: theta, g1, m1, v1 (+ g2, m2, v2 on the encoder slice) in, theta, m1, v1
    (+ m2, v2) and the parameter planes out."""
    return n_all * (16.0 + 12.0 + 2.0 * np_) + n_enc * (12.0 + 8.0)


# ------------------------------------------------------------------------ PMC passes
def _csv_rows(d, suffix):
    import csv
    import glob
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def _region_dispatches(d, region_ids):
    """For every region id: the lists of kernel-trace rows between each pair of its marker
    kernels (one list per bracketed launch), from one rocprofv3 output directory."""
    trace = sorted(_csv_rows(d, "kernel_trace.csv"), key=lambda r: int(r["Dispatch_Id"]))
    from magic_amd._lib import MARKER_GRID

    def wgs(r):
        g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        return g // max(1, int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1))
    out = {}
    for rid in region_ids:
        groups, open_ = [], None
        for r in trace:
            if "mvae_region_marker" in r["Kernel_Name"]:
                if wgs(r) != MARKER_GRID + rid:
                    continue
                if open_ is None:
                    open_ = (int(r["Dispatch_Id"]), r.get("Queue_Id"))
                else:
                    lo, q = open_
                    hi = int(r["Dispatch_Id"])
                    groups.append([x for x in trace if lo < int(x["Dispatch_Id"]) < hi and x.get("Queue_Id") == q
                                   and "mvae_region_marker" not in x["Kernel_Name"]])
                    open_ = None
        if groups:
            out[rid] = groups
    return out


def _region_counter(d, counter, region_ids):
    """Mean per launch of `counter` (summed over the dispatches between each pair of marker
    kernels of a region) for every region id, from one rocprofv3 output directory."""
    vals = {}
    for r in _csv_rows(d, "counter_collection.csv"):
        if r.get("Counter_Name") == counter:
            k = int(r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    out = {}
    for rid, groups in _region_dispatches(d, region_ids).items():
        sums = [sum(vals.get(int(x["Dispatch_Id"]), 0.0) for x in g) for g in groups]
        out[rid] = sum(sums) / len(sums)
    return out


def _region_ns(d, region_ids):
    """Mean summed kernel duration (ns) per bracketed launch of each region."""
    out = {}
    for rid, groups in _region_dispatches(d, region_ids).items():
        t = [sum(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in g) for g in groups]
        out[rid] = sum(t) / len(t)
    return out


N_SIMD = 1024  # 256 CUs x 4 SIMDs (MI355X)


def pmc_traffic(args, names, regions_all, config=None, mfma=()):
    """HBM bytes per step of each region in `names` (the mean per bracketed launch x the region's
    launches per child step: 2 for the BCE head split and the chunked layer-0 weight gradient): two rocprofv3 child runs of this bench
    (FETCH_SIZE and WRITE_SIZE cannot share a pass), markers around the regions; FETCH_SIZE x2
    (MI355X_MICROARCH.md: gfx950 reports half of a wide streaming read) and KB -> B. For the
    regions in `mfma`, a third pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE): the matrix-pipe
    busy fraction over the kernels' own cycles, mfma_busy = MFMA-busy cycles / (N_SIMD x
    GRBM_GUI_ACTIVE / 8) (GRBM_GUI_ACTIVE is summed over the 8 XCDs), and the clock the chip held,
    (GRBM_GUI_ACTIVE / 8) / kernel time."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not on PATH"
    ids = {n: regions_all.index(n) for n in names if n in regions_all}
    base = os.path.join(HERE, "gpurun_out") if os.path.isdir(os.path.join(HERE, "gpurun_out")) \
        else tempfile.gettempdir()
    root = tempfile.mkdtemp(prefix="bench_pmc_", dir=base)
    child_steps = 3  # every child step runs the markers
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", ",".join(str(r) for r in ids.values()),
             "--config", config or args.config, "--steps", "2", "--warmup", "1"]
    if args.batch and config is None:
        child += ["--batch", str(args.batch)]
    if args.precision and config is None:
        child += ["--precision", args.precision]
    for o in args.opt:
        child += ["--opt", o]
    passes = [("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE"])]
    if mfma:
        passes.append(("mfma", ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]))
    res, ns, nl = {}, {}, {}
    for tag, counters in passes:
        d = os.path.join(root, tag)
        cmd = [exe, "--pmc", *counters, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run",
               "--", *child]
        env = dict(os.environ, TMPDIR="/tmp")
        with open(os.path.join(root, tag + ".log"), "w") as log:
            p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT,
                                 start_new_session=True)
            try:
                rc = p.wait(timeout=150)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return None, f"{tag} pass timed out"
        if rc != 0:
            return None, f"{tag} pass rc={rc} (log {root})"
        for c in counters:
            res[c] = _region_counter(d, c, list(ids.values()))
        if tag == "fetch":
            nl = {rid: len(g) for rid, g in _region_dispatches(d, list(ids.values())).items()}
        if tag == "mfma":
            ns = _region_ns(d, list(ids.values()))
    out = {}
    for n, rid in ids.items():
        k = max(1, round(nl.get(rid, child_steps) / child_steps))
        f, w = res["FETCH_SIZE"].get(rid), res["WRITE_SIZE"].get(rid)
        if f is not None and w is not None:
            out[n] = {"hbm_bytes": round(k * (f * 1024 * 2 + w * 1024)),
                      "fetch_bytes": round(k * f * 1024 * 2), "write_bytes": round(k * w * 1024)}
            if k != 1:
                out[n]["launches_per_step"] = k
        busy, gui = res.get("SQ_VALU_MFMA_BUSY_CYCLES", {}).get(rid), res.get("GRBM_GUI_ACTIVE", {}).get(rid)
        if n in mfma and busy and gui:
            cyc = gui / 8.0
            e = out.setdefault(n, {})
            e["mfma_busy"] = round(busy / (N_SIMD * cyc), 4)
            e["mfma_busy_cycles"] = round(k * busy)
            e["kernel_cycles"] = round(k * cyc)
            if ns.get(rid):
                e["clock_ghz"] = round(cyc / ns[rid], 3)
                e["profiled_ms"] = round(k * ns[rid] / 1e6, 4)
    return out, (f"rocprofv3 child passes of this bench ({config or args.config}), marker-bracketed: "
                 f"--pmc FETCH_SIZE / WRITE_SIZE" + (" / SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE" if mfma else "")
                 + f" ({root})")


# ------------------------------------------------------------------------ CPU baseline
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(cfg, dev, seconds: float):
    """The oracle (CPU restatement of the reference maths, numpy fp32 + BLAS) on this host:
    (1) parity: one C1-shaped step (B = 64, this run's GEMM arithmetic) on the GPU and on the
    CPU from the same seeded batch, eps and parameters; (2) timings: the GPU-batch workload
    with all BLAS threads (`value`), C1 with all threads and with 1 thread."""
    import torch
    from threadpoolctl import threadpool_info, threadpool_limits

    from magic_amd import _lib
    from magic_amd.engine import Engine
    from magic_amd.overlap_input import synthetic_batch
    from oracle import mvae_oracle as O

    oc = O.OracleConfig(image_size=cfg.image_size, enc=tuple(cfg.enc), dec=tuple(cfg.dec),
                        latent=cfg.latent, act=cfg.act, deform_weight=cfg.deform_weight,
                        metric=cfg.metric, reciprocal=cfg.reciprocal, lr=tuple(cfg.lr),
                        conv=cfg.conv)
    B1 = 8 if cfg.conv else 64   # the conv oracle's im2col: 3*B*2500 x 1600 per step
    c1 = cfg.replace(batch=B1, global_batch=B1)
    x1, a1 = synthetic_batch(B1, cfg.image_size, seed=4242, device=dev)
    eps1 = torch.from_numpy(np.random.default_rng(2).standard_normal((3, B1, cfg.latent))
                            .astype(np.float32)).to(dev)
    eng = Engine(c1, dev.index)
    try:
        eng.init_params(0)
        P = {k: v.cpu().numpy().copy() for k, v in eng.params().items()}
        eng.forward(x1, eps1)
        eng.metric(a1)
        eng.backward()
        torch.cuda.synchronize(dev)
        lg = eng.losses.cpu().numpy().astype(np.float64)
        dg = eng.dist.cpu().numpy().astype(np.float64)
        g1g = {k: v.cpu().numpy().astype(np.float64) for k, v in eng.tensors(_lib.KIND_GRAD1).items()}
        g2g = {k: v.cpu().numpy().astype(np.float64) for k, v in eng.tensors(_lib.KIND_GRAD2).items()}
    finally:
        eng.close()
    X1, A1, E1 = x1.cpu().numpy(), a1.cpu().numpy(), eps1.cpu().numpy()

    def rel(a, b, mag=None):
        s = max(np.abs(b).max(), 1e-2 * np.abs(mag).max() if mag is not None else 0.0, 1e-30)
        return float(np.abs(np.asarray(a, np.float64) - b).max() / s)
    c = O.forward(P, X1, E1, oc, dtype=np.float32)
    O.metric(c, A1, oc, B1)
    lo = O.loss_sums(c, B1)
    g1o, g2o = O.backward(c, oc, B1)
    m1, m2 = O.backward(c, oc, B1, magnitude=True)
    parity = {
        "losses": float(np.max(np.abs(lg - lo) / np.maximum(np.abs(lo), 1e-3))),
        "distance": rel(dg, c["dist"]),
        "grads": max(max(rel(g1g[k], g1o[k], m1[k]) for k in g1o),
                     max(rel(g2g[k], g2o[k], m2[k]) for k in g2o)),
    }
    bar = 1e-4 if cfg.precision in ("f32", "f32x") else 5e-2

    def timed(X, A, E, budget, min_steps=2):
        st = O.adam_init(oc, P)
        Pt = dict(P)
        O.train_step(Pt, st, X, A, E, oc, dtype=np.float32)  # warm-up
        t0 = time.perf_counter()
        n = 0
        while n < min_steps or time.perf_counter() - t0 < budget:
            _, _, Pt, st, _ = O.train_step(Pt, st, X, A, E, oc, dtype=np.float32)
            n += 1
        dt = time.perf_counter() - t0
        return n * X.shape[0] / dt, n, dt
    blas = [i for i in threadpool_info() if i.get("user_api") == "blas"]
    cores = max([i.get("num_threads", 1) for i in blas] or [1])
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count()
    v_c1, n_c1, t_c1 = timed(X1, A1, E1, seconds)
    with threadpool_limits(1):
        v_c1_1, n_c1_1, t_c1_1 = timed(X1, A1, E1, seconds)
    # the GPU-batch workload (the bench's own step shape), all threads, >= 2 steps; the conv
    # oracle's im2col would hold 3*B*2500 x 1600 values: its sample is 64 pairs of that shape
    Bg = min(cfg.batch, 64) if cfg.conv else cfg.batch
    xg, ag = synthetic_batch(Bg, cfg.image_size, seed=4243, device=dev)
    Eg = np.random.default_rng(3).standard_normal((3, Bg, cfg.latent)).astype(np.float32)
    v_g, n_g, t_g = timed(xg.cpu().numpy(), ag.cpu().numpy(), Eg, seconds)
    del xg, ag
    return {"value": round(v_g, 2), "unit": "shape-pairs/s", "cores": int(cores), "kind": "port",
            "sample": f"oracle/mvae_oracle.py train_step (numpy float32 + {blas[0].get('internal_api', 'BLAS') if blas else 'BLAS'}), "
                      f"{n_g} steps x {Bg} pairs of this run's step shape ({cfg.image_size}x{cfg.image_size}, "
                      f"enc {list(cfg.enc)}, L={cfg.latent}) in {t_g:.1f} s",
            "c1_all_threads": round(v_c1, 2), "c1_one_thread": round(v_c1_1, 2),
            "c1_sample": f"{n_c1} / {n_c1_1} steps x {B1} pairs ({t_c1:.1f} / {t_c1_1:.1f} s)",
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "affinity_cpus": affinity, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "threads_note": (f"all-thread legs use the BLAS pool's {cores} threads: OMP_NUM_THREADS="
                             f"{os.environ.get('OMP_NUM_THREADS')} is this lease's CPU share (a one-GPU "
                             f"slice of the host; the process may run on {affinity} of the host's "
                             f"{os.cpu_count()} CPUs, which other leases share)"),
            "torch_threads": torch.get_num_threads(),
            "parity_c1": {"gpu_precision": cfg.precision, "bar": bar, **{k: float(f"{v:.3g}") for k, v in parity.items()},
                          "ok": all(v <= bar for v in parity.values()),
                          "what": "max-norm relative GPU vs CPU, same seeded B=64 batch, eps and params: "
                                  "5 losses, distance[B], every g1/g2 gradient (cancellation-aware)"}}


# ------------------------------------------------------------------------ dry run
class DryRunEngine:
    """Launcher rehearsal only (``--dry-run``): the DataParallelStep interface on CPU tensors,
    computing deterministic functions of the local rows (column sums / global batch) so that
    the all-reduced result of N ranks equals one rank's on the concatenated batch. Not the
    model, not a measurement."""
    N_BACKWARD_PARTS = 3

    def __init__(self, cfg):
        import torch
        self.cfg = cfg
        L = cfg.latent
        self.colsq = torch.zeros(2 * L, dtype=torch.float64)
        self.coldot = torch.zeros(L, dtype=torch.float64)
        self.grads = torch.zeros(96, dtype=torch.float64)
        self.losses = torch.zeros(5, dtype=torch.float64)
        self.dist = None

    def forward(self, x, eps=None):
        self.x = x.double()
        L = self.cfg.latent
        self.colsq.copy_((self.x[:, :2 * L] ** 2).sum(0))

    def metric(self, areas):
        inv = 1.0 / self.cfg.gbatch
        self.losses.copy_(self.x.sum() * inv * self.losses.new_tensor([1.0, 0.5, 0.25, 0.125, 2.0]))
        self.losses[1] += areas.double().sum() * inv
        self.dist = self.x[:, :4].sum(1)
        self.coldot.copy_(self.x[:, :self.cfg.latent].sum(0) * inv)

    def backward_part(self, part):
        n = self.grads.numel() // 3
        cols = self.x[:, part * n:(part + 1) * n] * torch_arange(n, part)
        self.grads[part * n:(part + 1) * n] = cols.sum(0) / self.cfg.gbatch

    def backward(self):
        for p in range(3):
            self.backward_part(p)

    def grad_ranges(self, part):
        n = self.grads.numel() // 3
        return [self.grads[part * n:(part + 1) * n]]

    def adam(self):
        pass

    def predict(self, x, eps=None):
        return x.double()[:, :4].sum(1) + 1.0

    def close(self):
        pass


def torch_arange(n, part):
    import torch
    return torch.arange(1 + part * n, 1 + (part + 1) * n, dtype=torch.float64)


def dry_run_batch(cfg, world, rank, j):
    """The global batch of draw j (seeded, identical on every rank); this rank's rows."""
    import torch
    g = torch.Generator().manual_seed(17 + j)
    B = cfg.batch
    X = (torch.rand(B * world, 3 * cfg.D, generator=g) < 0.1).float()
    A = torch.randint(296, 6427, (B * world,), generator=g).float()
    return X[rank * B:(rank + 1) * B].contiguous(), A[rank * B:(rank + 1) * B].contiguous()


# ------------------------------------------------------------------------ measurement
def allreduce_bench(eng, dev, world, dry_run, reps=5):
    """The achieved rate of one all-reduce of the step's whole gradient bucket (the [g1 | g2]
    buffer's size, fp32) on its own: mean time over reps, algorithm bandwidth and bus bandwidth
    (2 (N - 1) / N x bytes / time, the ring all-reduce's per-link traffic)."""
    import torch
    import torch.distributed as dist
    n = eng.grads.numel()
    t = torch.ones(n, dtype=eng.grads.dtype, device=dev)
    dist.all_reduce(t)
    dist.barrier()
    if dry_run:
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(t)
        ms = (time.perf_counter() - t0) * 1e3 / reps
    else:
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            dist.all_reduce(t)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / reps
    nbytes = n * t.element_size()
    return {"bytes": nbytes, "ms": round(ms, 4), "algbw_GBps": round(nbytes / (ms * 1e-3) / 1e9, 5),
            "busbw_GBps": round(2 * (world - 1) / world * nbytes / (ms * 1e-3) / 1e9, 5)}


def measure(args, cfg, world, rank, local, dev, *, timing, steps, warmup, keep=False, h2d=False,
            pipeline=False):
    """One configuration through the training step: W warm-up steps, a region pass (HIP events
    around every region, outside the timed loop), K timed steps bracketed by barrier + device
    sync (max over ranks), overlap-MSE on a held-out batch. h2d: a further timed loop in which
    every step's X first comes from pinned host memory (copied on a side stream one step ahead,
    mirroring feed_dict, 11a/vae.py:399-402). pipeline: a further timed loop fed by the input
    pipeline itself -- inputs() over uint8 pair tables resident in HBM, each step's shuffled
    draw and rotation angles on the host, the batch assembled by the HIP producer
    (11a/overlap_input.py:127-261) -- and the producer kernel's own rate. Returns a dict; the
    engine stays open with keep."""
    import torch
    import torch.distributed as dist

    from magic_amd import _lib
    from magic_amd.parallel import DataParallelStep

    if args.dry_run:
        eng = DryRunEngine(cfg)
        pool = [dry_run_batch(cfg, world, rank, j) for j in range(2)]
    else:
        from magic_amd.engine import Engine
        from magic_amd.overlap_input import synthetic_batch
        eng = Engine(cfg, local)
        for o in args.opt:
            k, v = o.split("=")
            eng.set_option(k, int(v))
        eng.init_params(0)  # identical replicas on every rank
        pool = [synthetic_batch(cfg.batch, cfg.image_size, seed=17 + 101 * rank + j, device=dev)
                for j in range(2)]
        torch.cuda.synchronize()
    stepper = DataParallelStep(eng, reduce_losses=True)

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize()

    for i in range(warmup):
        stepper.step(*pool[i % 2])
    sync()
    regions, dom = {}, None
    if timing:
        # region pass (outside the timed loop): HIP events around every region, for the
        # per-kernel table and to pick the dominant GEMM
        # (the side stream off: concurrent kernels would stretch each other's event intervals)
        eng.set_option("side_stream", 0)
        eng.timing_reset()
        eng.timing_enable(True)
        for i in range(args.region_steps):
            stepper.step(*pool[i % 2])
        sync()
        eng.timing_enable(False)
        eng.set_option("side_stream", 1 if "side_stream=0" not in args.opt else 0)
        regions = eng.timing_read()
        gemms = {k: v for k, v in regions.items() if region_flops(cfg, k) > 0}
        # the dominant GEMM by algorithmic work (ties: by time)
        dom = max(gemms, key=lambda k: (region_flops(cfg, k), gemms[k][0]))
        # timed loop: events around the dominant GEMM only (one pair per step)
        eng.timing_reset()
        eng.timing_select(dom)
        eng.timing_enable(True)
        if args.mark_dominant:
            eng.timing_marker(dom, True)

    host_t = []

    def timed(n, batch_of):
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for i in range(n):
            stepper.step(*batch_of(i))
        # host time to enqueue the steps: close to the elapsed time = launch-bound
        host_t.append(time.perf_counter() - t0)
        if world > 1:
            dist.barrier()
        sync()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    stepper.comm_timing = world > 1  # exposed collective waits of the timed steps
    elapsed = timed(steps, lambda i: pool[i % 2])
    stepper.comm_timing = False
    if timing and args.mark_dominant:
        eng.timing_marker(dom, False)
    comm = None
    if world > 1:
        comm = stepper.comm_stats()
        comm["allreduce_bench"] = allreduce_bench(eng, dev, world, args.dry_run)
    dom_timed = None
    if timing:
        eng.timing_enable(False)
        dom_timed = eng.timing_read().get(dom)
        eng.timing_select(None)
    losses = eng.losses.cpu().numpy().tolist()
    if not np.all(np.isfinite(losses)):
        raise RuntimeError(f"non-finite losses after the timed steps: {losses}")
    out = {"cfg": cfg, "elapsed": elapsed, "host_elapsed": host_t[0], "steps": steps,
           "regions": regions, "dom": dom,
           "dom_timed": dom_timed, "losses": losses, "comm": comm}
    if not args.dry_run:
        out["n_all"] = eng.buffer(_lib.BUF_PARAMS).numel()
        out["n_enc"] = eng.buffer(_lib.BUF_GRADS).numel() - out["n_all"]
        if cfg.precision == "f32x":
            out["dyn"] = int(eng.buffer(_lib.BUF_DYN).view(torch.int32).item())
    if h2d and not args.dry_run:
        # X of every step from pinned host memory: the copy of step i+1's batch runs on a copy
        # stream beside step i (two device buffers), as an input pipeline feeding the step would
        host = [pool[j][0].cpu().pin_memory() for j in range(2)]
        bufs = [torch.empty_like(pool[0][0]) for _ in range(2)]
        cs = torch.cuda.Stream(device=dev)
        ev = [torch.cuda.Event() for _ in range(2)]

        def fetch(i):
            with torch.cuda.stream(cs):
                bufs[i % 2].copy_(host[i % 2], non_blocking=True)
                ev[i % 2].record(cs)
        fetch(0)

        def batch_h2d(i):
            torch.cuda.current_stream().wait_event(ev[i % 2])
            if i + 1 < steps:
                cs.wait_stream(torch.cuda.current_stream())  # buffer (i+1)%2 no longer read
                fetch(i + 1)
            return bufs[i % 2], pool[i % 2][1]
        el_h = timed(steps, batch_h2d)
        out["h2d"] = {"value": round(cfg.batch * world * steps / el_h, 2), "unit": "shape-pairs/s",
                      "ms_per_step": round(el_h / steps * 1e3, 4),
                      "bytes_per_step": int(pool[0][0].numel() * 4),
                      "note": "PCIe-inclusive: each step's X [B, 3D] f32 copied pinned host -> HBM "
                              "(one step ahead on a copy stream), mirroring feed_dict "
                              "(11a/vae.py:399-402); never the headline value"}
    if pipeline and not args.dry_run:
        from magic_amd.overlap_input import BatchStream, make_batch
        bs = BatchStream(cfg.batch, cfg.image_size, normalize=True, seed=7 + rank, device=dev)
        for _ in range(2):
            stepper.step(*next(bs))
        el_p = timed(steps, lambda i: next(bs))
        # the producer kernel alone: HIP events around back-to-back launches on one batch's draw
        idx = torch.arange(cfg.batch, dtype=torch.int32, device=dev) % bs.locks.shape[0]
        coef = torch.from_numpy(np.tile(np.array([[0.6, 0.8, 10.0, -20.0]], np.float32),
                                        (cfg.batch, 1))).to(dev)
        xb = torch.empty(cfg.batch, 3 * cfg.D, device=dev)
        make_batch(bs.locks, bs.keys, idx, coef, out=xb)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nk = 10
        e0.record()
        for _ in range(nk):
            make_batch(bs.locks, bs.keys, idx, coef, out=xb)
        e1.record()
        e1.synchronize()
        mb_ms = e0.elapsed_time(e1) / nk
        mb_bytes = cfg.batch * cfg.D * (12 + 2)  # X written (3 fp32 / pixel) + lock and key bytes
        out["pipeline"] = {"value": round(cfg.batch * world * steps / el_p, 2), "unit": "shape-pairs/s",
                           "ms_per_step": round(el_p / steps * 1e3, 4),
                           "make_batch": {"avg_ms": round(mb_ms, 4), "bytes": mb_bytes,
                                          "gbs": round(mb_bytes / (mb_ms * 1e-3) / 1e9, 1),
                                          "frac": round(mb_bytes / (mb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                           "note": "inputs() -> partial_fit: a pool of 960 synthetic uint8 pairs in "
                                   "HBM, per step a host shuffle draw + U[0,2pi) angles (11a/overlap_"
                                   "input.py:127-261), rotation/interleave//255 by the HIP batch "
                                   "producer (mvae_make_batch), then the training step"}
    # overlap-MSE on a held-out seeded batch (11a/main.py:94-111; 1/pred for reciprocal)
    if args.dry_run:
        xe, ae = dry_run_batch(cfg, world, rank, 99)
    else:
        from magic_amd.overlap_input import synthetic_batch
        xe, ae = synthetic_batch(cfg.batch, cfg.image_size, seed=999, device=dev)
    pred = stepper.predict(xe).double()   # global-batch cosine norms under DP
    if cfg.reciprocal:
        pred = 1.0 / pred
    out["mse"] = float(((pred - ae.double()) ** 2).mean().item())
    if args.dry_run:
        w = torch.arange(1, eng.grads.numel() + 1, dtype=torch.float64)
        out["grad_checksum"] = float((eng.grads * w).sum())
    if keep:
        out["eng"] = eng
    else:
        eng.close()
    return out


def rooflines(args, m):
    """roofline (dominant GEMM) and loss_roofline (HBM-bound kernels) of one measured config."""
    cfg, regions, dom, dom_timed = m["cfg"], m["regions"], m["dom"], m["dom_timed"]
    if not regions or not dom_timed:
        return None, None
    gemms = {k: v for k, v in regions.items() if region_flops(cfg, k) > 0}
    # per step (a region may be several launches: the layer-0 weight gradient in row chunks)
    ms_avg = dom_timed[0] / m["steps"]  # HIP events over the timed loop
    flops = region_flops(cfg, dom)
    achieved = flops / (ms_avg * 1e-3) / 1e12
    peak = F32_MFMA_PEAK_TFLOPS if cfg.precision == "f32" else BF16_MFMA_PEAK_TFLOPS
    iso_ms = regions[dom][0] / args.region_steps
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None,
                "kernel": dom, "flops_per_launch": flops, "avg_ms": round(ms_avg, 4),
                "isolated_avg_ms": round(iso_ms, 4),
                "isolated_frac": round(flops / (iso_ms * 1e-3) / 1e12 / peak, 4),
                "work": "algorithmic 2*M*N*K of the region's fp32 GEMM, counted once"}
    if cfg.precision == "f32x":
        pp = plane_pairs(cfg, dom, m.get("dyn", 0) == 0)
        roofline.update({
            "arith": "f32x: fp32-accurate exact 3-term bf16 split on the bf16 MFMA pipe",
            "bf16_plane_pairs": pp,
            "mfma_pipe_tflops": round(achieved * pp, 2),
            "mfma_pipe_frac": round(achieved * pp / BF16_MFMA_PEAK_TFLOPS, 4),
            "frac_of_fp32_mfma_peak": round(achieved / F32_MFMA_PEAK_TFLOPS, 4)})
    rs = args.region_steps
    total_gemm_ms = sum(v[0] for v in gemms.values()) / rs
    gemm_flops = sum(region_flops(cfg, k) * min(v[1], rs) for k, v in gemms.items()) / rs  # (a region
    # launched in parts -- the BCE head split, the layer-0 weight gradient in row chunks -- once per step)
    roofline["all_gemms"] = {"ms_per_step": round(total_gemm_ms, 4),
                             "tflops": round(gemm_flops / total_gemm_ms / 1e9, 2)}
    # HBM-bound kernels and the fused BCE head (north_star: achieved GB/s vs peak)
    loss_roofline = {}
    np_ = {"f32": 0, "bf16": 1, "f32x": 3}[cfg.precision]
    for k in ("deinterleave", "eps_rng", "latent_fwd", "colsq", "metric_loss", "coldot",
              "latent_bwd", "adam", "conv1_fwd", "lrn2_pool2_fwd", "pool2_bwd", "conv1_wgrad"):
        if k not in regions:
            continue
        ms_k = regions[k][0] / args.region_steps
        by = adam_bytes(m["n_all"], m["n_enc"], np_) if k == "adam" else region_bytes(cfg, k)
        loss_roofline[k] = {"bytes": by, "avg_ms": round(ms_k, 4),
                            "gbs": round(by / (ms_k * 1e-3) / 1e9, 1),
                            "frac": round(by / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if "deint_fwd0" in regions:
        # the fused launch (create option deint_fuse): its bound is the larger of the
        # de-interleave's HBM time and the forward's MFMA time at the dense peaks
        ms_f = regions["deint_fwd0"][0] / args.region_steps
        by_d = region_bytes(cfg, "deinterleave")
        fl = region_flops(cfg, "enc_fwd_0") * (plane_pairs(cfg, "enc_fwd_0", m.get("dyn", 0) == 0)
                                               if cfg.precision == "f32x" else 1)
        t_hbm = by_d / (HBM_PEAK_GBS * 1e9)
        t_mfma = fl / ((F32_MFMA_PEAK_TFLOPS if cfg.precision == "f32" else BF16_MFMA_PEAK_TFLOPS) * 1e12)
        loss_roofline["deint_fwd0"] = {
            "deint_bytes": by_d, "fwd_mfma_flops": fl, "avg_ms": round(ms_f, 4),
            "hbm_bound_ms": round(t_hbm * 1e3, 4), "mfma_bound_ms": round(t_mfma * 1e3, 4),
            "frac_of_bound": round(max(t_hbm, t_mfma) / (ms_f * 1e-3), 4),
            "deint_gbs": round(by_d / (ms_f * 1e-3) / 1e9, 1),
            "note": "the de-interleave's workers beside the layer-0 forward's tiles in one launch "
                    "(DeintJob); bound = max(HBM time of the de-interleave's bytes, MFMA time of "
                    "the forward's bf16 products)"}
    lat = [k for k in ("eps_rng", "latent_fwd", "colsq", "metric_loss", "coldot", "latent_bwd")
           if k in regions]
    ms_lat = sum(regions[k][0] / args.region_steps for k in lat)
    by_lat = 80.0 * cfg.latent * cfg.batch
    loss_roofline["latent_head_total"] = {
        "kernels": lat, "avg_ms": round(ms_lat, 4), "bytes_survey": by_lat,
        "gbs_survey": round(by_lat / (ms_lat * 1e-3) / 1e9, 1),
        "frac_survey": round(by_lat / (ms_lat * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "note": "SURVEY.md §8d: ~80*L B/pair for the fused latent head fwd+bwd"}
    if "dec_fwd_out_bce" in regions:
        ms_b = regions["dec_fwd_out_bce"][0] / args.region_steps
        by_b = 12.0 * cfg.D * cfg.batch
        # what the fused kernel moves: the target (its bf16 plane for binary pixels, else fp32)
        # and dU as the next GEMMs' planes (fp32 when they run native fp32); the logits never
        # reach HBM. Its bound: max(MFMA time of the decoder-output product at the dense peak of
        # the arithmetic it runs on, HBM time of those bytes at 8 TB/s)
        np_b = 1 if cfg.precision == "bf16" else (6 if cfg.precision == "f32x" else 0)
        by_f = cfg.D * cfg.batch * ((2.0 + 2.0 * (1 if np_b == 1 else 3)) if np_b else 8.0)
        fl_b = region_flops(cfg, "dec_fwd_out_bce") * (np_b if np_b else 1)
        t_mfma = fl_b / ((BF16_MFMA_PEAK_TFLOPS if np_b else F32_MFMA_PEAK_TFLOPS) * 1e12)
        t_hbm = by_f / (HBM_PEAK_GBS * 1e9)
        loss_roofline["bce_head"] = {
            "bytes": by_b, "avg_ms": round(ms_b, 4),
            "gbs": round(by_b / (ms_b * 1e-3) / 1e9, 1),
            "frac": round(by_b / (ms_b * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "bytes_fused": by_f, "mfma_bound_ms": round(t_mfma * 1e3, 4),
            "hbm_bound_ms": round(t_hbm * 1e3, 4),
            "frac_of_bound": round(max(t_mfma, t_hbm) / (ms_b * 1e-3), 4),
            "note": "BASELINE.md §4: 12*D B/pair (logits, targets, dlogits) for the unfused head; "
                    "the fused decoder-output GEMM moves bytes_fused (target + dU planes) and is "
                    "bounded by max(mfma_bound_ms, hbm_bound_ms); frac_of_bound = that / avg_ms"}
    return roofline, loss_roofline


def print_regions(args, m, tag):
    cfg, regions, dom = m["cfg"], m["regions"], m["dom"]
    if not regions:
        return
    gemms = {k: v for k, v in regions.items() if region_flops(cfg, k) > 0}
    rs = args.region_steps
    total_gemm_ms = sum(v[0] for v in gemms.values()) / rs
    gemm_flops = sum(region_flops(cfg, k) * min(v[1], rs) for k, v in gemms.items()) / rs  # (a region
    # launched in parts -- the BCE head split, the layer-0 weight gradient in row chunks -- once per step)
    ms_dom = m["dom_timed"][0] / m["steps"] if m["dom_timed"] else float("nan")
    print(f"[bench] {tag}: region pass ({rs} steps, kernels serialised on one stream): GEMM time/step "
          f"{total_gemm_ms:.3f} ms, {gemm_flops / total_gemm_ms / 1e9:.1f} TFLOP/s over all GEMMs; timed step "
          f"{m['elapsed'] / m['steps'] * 1e3:.3f} ms; {dom} {ms_dom:.4f} ms in the timed loop", file=sys.stderr)
    _, lr = rooflines(args, m)
    for k, (ms, n) in sorted(regions.items(), key=lambda kv: -kv[1][0]):
        fl = region_flops(cfg, k)
        extra = f"  {fl / (ms / rs * 1e-3) / 1e12:7.1f} TF/s" if fl else ""
        if lr and k in lr and "gbs" in lr[k]:
            extra = f"  {lr[k]['gbs']:7.1f} GB/s"
        elif lr and k in lr and "deint_gbs" in lr[k]:
            extra = f"{extra}  {lr[k]['deint_gbs']:7.1f} GB/s of the de-interleave"
        print(f"[bench] {k:18s} {ms / rs:9.4f} ms/step ({n} launches){extra}", file=sys.stderr)


def workload(args_config, cfg):
    return (f"BASELINE {args_config}: "
            f"{'CifarNet conv tower (6b/net.py:50-60) + ' if cfg.conv else ''}preset "
            f"{ {20: '8c', 200: '8d', 2000: '8e'}.get(cfg.latent, '?') } enc "
            f"{list(cfg.enc)} L={cfg.latent} {cfg.act} "
            f"{'reciprocal ' if cfg.reciprocal else ''}{cfg.metric}")


# ------------------------------------------------------------------------ plan
def run_plan(args) -> dict:
    """What ``bench.py --gpus N`` runs on each rank (``--plan``): the headline and configs-block
    workloads with their per-rank and global batches, and the data-parallel exchange per step
    (DataParallelStep: cosine colsq / coldot, the async loss reduce, the gradient bucket in
    backward parts with the layer-0 rows in ``wgrad0_chunks`` chunks). No GPU is touched."""
    from magic_amd.config import baseline_config

    N = args.gpus
    ids = [args.config] + ([] if args.no_configs else
                           [c for c in (["C3", "C5", "C5CONV"] if N == 1 else ["C4", "C5"])
                            if c != args.config and not (c == "C4" and args.config == "C3")])
    out = {"n_gpus": N, "launcher": "torch.distributed.run, one process per GPU" if N > 1 else "one process",
           "backend": "nccl (RCCL over xGMI)" if N > 1 else None, "configs": {}}
    for cid in ids:
        cfg = baseline_config("C3" if cid == "C4" else cid)
        if cid == args.config and args.batch:
            cfg = cfg.replace(batch=args.batch)
        if cid == args.config and args.precision:
            cfg = cfg.replace(precision=args.precision)
        e, L = list(cfg.enc), cfg.latent
        widths = [cfg.D] + e
        enc = sum((widths[i] + 1) * widths[i + 1] for i in range(len(e))) + (e[-1] + 1) * 2 * L
        dec = (L + 1) * cfg.dec[0] + (cfg.dec[0] + 1) * cfg.dec[1] + (cfg.dec[1] + 1) * cfg.D
        g1, g2 = enc + dec, enc
        chunks = 4 if N > 1 else 1
        out["configs"][cid] = {
            "workload": workload("C3" if cid == "C4" else cid, cfg),
            "per_rank_batch": cfg.batch, "global_batch": cfg.batch * N, "precision": cfg.precision,
            "metric": ("reciprocal " if cfg.reciprocal else "") + cfg.metric,
            "wgrad0_chunks": chunks,
            "per_step_collectives": ([] if N == 1 else
                                     (["all_reduce colsq (%d floats, blocking)" % (2 * L),
                                       "all_reduce coldot (%d floats, blocking)" % L]
                                      if cfg.metric == "cosine" else []) +
                                     ["all_reduce losses (5 floats, async)",
                                      "all_reduce gradient bucket [g1|g2] %.1f MB fp32 in %d async parts "
                                      "(decoder; layer-0 rows x %d chunks; rest of the encoder)"
                                      % ((g1 + g2) * 4e-6, chunks + 2, chunks)]),
            "params_approx": g1,
        }
    return out


# ------------------------------------------------------------------------ main
def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.plan:
        print(json.dumps(run_plan(args)), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, argv))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    from magic_amd import _lib
    from magic_amd.config import baseline_config

    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        if args.dry_run:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    def config_of(cid, batch=0, precision="", small=False):
        cfg = baseline_config(cid)
        if batch:
            cfg = cfg.replace(batch=batch)
        if precision:
            cfg = cfg.replace(precision=precision)
        if small:  # launcher rehearsal of the configs block: a small stand-in shape
            cfg = cfg.replace(batch=min(cfg.batch, 16), image_size=12, latent=min(cfg.latent, 16))
        # one seed on every rank: each rank's internal sampler draws its own rows of the global
        # batch's eps stream (Engine.set_shard via DataParallelStep)
        return cfg.replace(global_batch=cfg.batch * world, options=",".join(args.create_opt))

    cfg = config_of(args.config, args.batch, args.precision)
    timing = not (args.no_timing or args.dry_run or args.pmc_child)

    if args.pmc_child:  # profiler child: markers around the named regions, a few steps
        from magic_amd.engine import Engine
        from magic_amd.overlap_input import synthetic_batch
        from magic_amd.parallel import DataParallelStep
        eng = Engine(cfg, local)
        eng.init_params(0)
        pool = [synthetic_batch(cfg.batch, cfg.image_size, seed=17 + j, device=dev) for j in range(2)]
        stepper = DataParallelStep(eng, reduce_losses=True)
        names = eng.timing_names()
        for rid in args.pmc_child.split(","):
            eng.timing_marker(names[int(rid)], True)
        for i in range(args.warmup + args.steps):
            stepper.step(*pool[i % 2])
        torch.cuda.synchronize()
        eng.close()
        return

    head = measure(args, cfg, world, rank, local, dev, timing=timing, steps=args.steps,
                   warmup=args.warmup, keep=True, h2d=not args.no_h2d, pipeline=not args.no_pipeline)
    eng = head.pop("eng")
    if rank == 0:
        print_regions(args, head, f"{args.config}")
    # the other BASELINE configurations in the same run (their own rooflines): C3 (the
    # north_star's L = 200 target) and C5 (L = 2000) on one GPU; with N ranks, C4 (= C3's shape
    # per rank, global batch 8192 N) and C5 at N ranks
    extra = {}
    if not args.no_configs:
        # (one GPU: also C5CONV, BASELINE config 5's conv-encoder variant -- SURVEY.md §8 f4)
        ids = ["C3", "C5", "C5CONV"] if world == 1 else ["C4", "C5"]
        for cid in ids:
            if cid == args.config or (cid == "C4" and args.config == "C3"):
                continue
            c = config_of("C3" if cid == "C4" else cid, small=args.dry_run)
            m = measure(args, c, world, rank, local, dev, timing=timing, steps=args.steps,
                        warmup=args.warmup, pipeline=not args.no_pipeline, keep=True)
            ce = m.pop("eng", None)
            names_c = ce.timing_names() if hasattr(ce, "timing_names") else []
            if ce is not None:
                ce.close()
            if rank == 0:
                print_regions(args, m, cid)
                rf, lr = rooflines(args, m)
                # the config's own HBM traffic and MFMA-busy counters (same passes as the headline)
                if rf and world == 1 and args.pmc == "auto" and not args.dry_run:
                    mf = [m["dom"]] + [k for k in PMC_REGIONS_MFMA if k in m["regions"] and k != m["dom"]]
                    want = mf + [k for k in PMC_REGIONS_BW if k in m["regions"]]
                    tr, how = pmc_traffic(args, want, names_c, config=cid, mfma=tuple(mf))
                    rf["traffic_method"] = how
                    if tr and m["dom"] in tr:
                        rf["traffic"] = tr[m["dom"]].get("hbm_bytes")
                        rf["traffic_detail"] = tr[m["dom"]]
                        if "mfma_busy" in tr[m["dom"]]:
                            rf["mfma_busy"] = tr[m["dom"]]["mfma_busy"]
                    if tr:
                        rf["pmc_regions"] = {k: tr[k] for k in mf if k in tr}
                        if "dec_fwd_out_bce" in tr and lr and "bce_head" in lr:
                            lr["bce_head"]["traffic"] = tr["dec_fwd_out_bce"].get("hbm_bytes")
                    for k in PMC_REGIONS_BW:
                        if tr and k in tr and lr and k in lr and "hbm_bytes" in tr[k]:
                            lr[k]["traffic"] = tr[k]["hbm_bytes"]
                extra[cid] = {"workload": workload("C3" if cid == "C4" else cid, c) +
                              (f" x {world} ranks" if world > 1 else ""),
                              "value": round(c.batch * world * m["steps"] / m["elapsed"], 2),
                              "unit": "shape-pairs/s", "per_gpu_value": round(c.batch * m["steps"] / m["elapsed"], 2),
                              "ms_per_step": round(m["elapsed"] / m["steps"] * 1e3, 4),
                              "host_ms_per_step": round(m["host_elapsed"] / m["steps"] * 1e3, 4),
                              "global_batch": c.batch * world, "per_gpu_batch": c.batch,
                              "dtype": c.precision, "overlap_mse": round(m["mse"], 2),
                              "comm": m.get("comm"),
                              "roofline": rf, "loss_roofline": lr, "pipeline": m.get("pipeline")}

    if rank == 0:
        pairs = cfg.batch * world * args.steps
        value = pairs / head["elapsed"]
        roofline, loss_roofline = rooflines(args, head)
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not args.dry_run:
            cpu = cpu_baseline(cfg, dev, args.cpu_seconds)
        if roofline and world == 1 and args.pmc == "auto" and not args.dry_run:
            names = eng.timing_names()
            mf = [head["dom"]] + [k for k in PMC_REGIONS_MFMA if k in head["regions"] and k != head["dom"]]
            want = mf + [k for k in PMC_REGIONS_BW if k in head["regions"]]
            tr, how = pmc_traffic(args, want, names, mfma=tuple(mf))
            roofline["traffic_method"] = how
            if tr:
                if head["dom"] in tr:
                    roofline["traffic"] = tr[head["dom"]].get("hbm_bytes")
                    roofline["traffic_detail"] = tr[head["dom"]]
                    if "mfma_busy" in tr[head["dom"]]:
                        roofline["mfma_busy"] = tr[head["dom"]]["mfma_busy"]
                roofline["pmc_regions"] = {k: tr[k] for k in mf if k in tr}
                if "dec_fwd_out_bce" in tr and "bce_head" in loss_roofline:
                    loss_roofline["bce_head"]["traffic"] = tr["dec_fwd_out_bce"].get("hbm_bytes")
                for k in PMC_REGIONS_BW:
                    if k in tr and k in loss_roofline:
                        loss_roofline[k]["traffic"] = tr[k]["hbm_bytes"]
        losses = head["losses"]
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "shape-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["elapsed"] / args.steps * 1e3, 4),
            "host_ms_per_step": round(head["host_elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"f32": "f32", "f32x": "f32 (exact 3-term bf16 split MFMA, fp32 accumulate)",
                      "bf16": "bf16 GEMM operands, fp32 accumulate"}[cfg.precision],
            "data": ("dry run: CPU stand-in engine, launcher rehearsal only (no GPU, not a measurement)"
                     if args.dry_run else
                     "synthetic 100x100 binary shape pairs (random ellipses/rectangles, nearest-"
                     "neighbour rotated lock), areas resampled from the reference's OVERLAP_AREAS; "
                     "random xavier init"),
            "config": {"workload": workload(args.config, cfg),
                       "global_batch": cfg.batch * world, "per_gpu_batch": cfg.batch,
                       "image": f"{cfg.image_size}x{cfg.image_size}", "parallelism": f"dp{world}",
                       "collective": ("gloo (dry run)" if args.dry_run else "RCCL all-reduce")
                       if world > 1 else None},
            "per_gpu_value": round(value / world, 2),
            "overlap_mse": round(head["mse"], 2),
            "losses": {"cost": losses[0], "training_loss": losses[1], "r_l": losses[2],
                       "l_l": losses[3], "d_l": losses[4]},
            "roofline": roofline,
            "loss_roofline": loss_roofline,
            "cpu_baseline": cpu,
            "h2d": head.get("h2d"),
            "pipeline": head.get("pipeline"),
            "configs": extra,
            # N > 1: per-step exposed wait of the gradient all-reduces and blocking statistics
            # all-reduces (HIP events on the step's stream), bucket bytes, and one all-reduce of
            # the bucket's size on its own (bus bandwidth)
            "comm": head.get("comm"),
            "build_id": None if args.dry_run else _lib.load().mvae_build_id().decode(),
        }
        if args.dry_run:
            line["grad_checksum"] = head["grad_checksum"]
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
