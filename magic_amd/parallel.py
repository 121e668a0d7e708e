"""Data parallelism for the metric-VAE step: one process per GPU, batch rows sharded over
ranks, full replicas of the parameters and of both Adam states.

The reference has no distributed code; this is the MI355X-native layer.
Per step and rank (``world`` ranks, local batch B, global batch N*B):

  forward(x_local)                     local encoder/decoder, 1/(N*B) loss scaling
  all_reduce(colsq)  [cosine only]     2L floats: axis-0 l2_normalize needs sum_b z^2 over
                                       the GLOBAL batch (``8c/vae.py:449-450``)
  metric(areas_local)
  all_reduce(coldot) [cosine only]     L floats: sum_b draw_b n_lock n_key (global)
  backward()                           in parts; the gradient ranges each part finishes
  all_reduce(grads)                    (decoder; the layer-0 g1/g2 rows in 4 chunks; the
                                       rest) are all-reduced asynchronously (RCCL over
                                       xGMI on MI355X) while the later parts run, then
                                       waited on
  adam()                               identical on every rank -> replicas stay bitwise equal
  all_reduce(losses) (optional)        5 floats, for logging / the NaN guard: issued async
                                       right after metric() so it runs beside the backward,
                                       waited for at the end of the step -- colsq / coldot
                                       are the only blocking collectives of a cosine step

The squared-difference metric needs no mid-step collective; the result equals the
single-process step on the concatenated batch (tests/test_parallel_gloo.py) to fp32
rounding (the rows are summed in another order across ranks). With more than one rank the
layer-0 weight gradient runs as ``wgrad0_chunks`` row chunks (engine option, set here and
restored by ``close()``); the chunk GEMMs keep the one-GEMM plan, so chunking alone changes no
bit of a rank's gradients.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist


class DataParallelStep:
    """Drives any engine exposing forward/metric/backward/adam and the tensors
    ``colsq``, ``coldot``, ``grads``, ``losses`` (the HIP ``Engine``; tests also drive a
    CPU stand-in built on the oracle)."""

    def __init__(self, engine, group=None, reduce_losses: bool = True, overlap: bool = True,
                 force_collectives: bool = False, wgrad0_chunks: int = 4, early_adam=None):
        self.e = engine
        # bucketed all-reduce overlapped with the rest of the backward (engines exposing
        # backward_part/grad_ranges); otherwise one bucket after the whole backward
        self.overlap = overlap and hasattr(engine, "backward_part")
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.reduce_losses = reduce_losses
        # force_collectives: issue the collectives even in a one-rank group (tests run the RCCL
        # path -- async all-reduces of the library's buffers on its streams -- on a 1-GPU box)
        self.coll = self.world > 1 or (force_collectives and dist.is_initialized())
        self.cosine = engine.cfg.metric == "cosine"
        if engine.cfg.gbatch != engine.cfg.batch * self.world:
            raise ValueError(f"engine global_batch {engine.cfg.gbatch} != batch {engine.cfg.batch} "
                             f"x world {self.world}")
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self._chunks_set = False
        if self.coll and self.overlap and hasattr(engine, "set_option"):
            # the layer-0 weight gradient (40 MB of the 69 MB bucket at C4) in 4 row chunks, each
            # all-reduced while the next computes, instead of one transfer after the last GEMM
            engine.set_option("wgrad0_chunks", wgrad0_chunks)
            self._chunks_set = True
        self._early_set = False
        early = engine.cfg.precision in ("f32x", "bf16") if early_adam is None else bool(early_adam)
        if not self.coll and hasattr(engine, "set_option") and early:
            # no collective between backward() and adam(): Adam of the blocks after layer 0 runs
            # on the engine's side stream beside the layer-0 weight gradient. Measured per mode:
            # C2 (f32x) 2.775 -> 2.742 ms (profiles/r4/r4ae_early_adam.txt); C3 (bf16) slower
            # with round 4's kernels (1.992 -> 2.005 ms), faster with round 5's (1.844 -> 1.837 ms
            # over 4 same-box pairs, profiles/r5/r5n_early_adam_bf16.txt); early_adam=False: one
            # Adam launch after the backward
            engine.set_option("early_adam", 1)
            self._early_set = True
        elif self.coll and hasattr(engine, "set_option"):
            # collectives between backward and adam: never Adam on the side stream (an engine an
            # earlier collective-free DataParallelStep left with the option on)
            engine.set_option("early_adam", 0)
        if hasattr(engine, "set_shard"):
            # the internal eps sampler draws this rank's rows of the global batch's stream,
            # so a sharded step without explicit eps equals the single-process step too
            engine.set_shard(self.rank * engine.cfg.batch)
        # communication timing (comm_stats): off by default; bench.py turns it on for the timed
        # loop of an N-rank run
        self.comm_timing = False
        self._marks = []          # per step: (blocking collectives [(t0, t1)], (t0, t1) of the wait)
        self._bucket_bytes = 0
        self._n_coll = 0

    # a timestamp on the step's stream: a HIP event (recorded, read after a sync) or, for the CPU
    # (gloo) path, the host clock (gloo's waits block the host)
    def _mark(self):
        if not self.comm_timing:
            return None
        if self.grads_on_gpu():
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def grads_on_gpu(self) -> bool:
        return getattr(self.e.grads, "is_cuda", False)

    @staticmethod
    def _ms(a, b) -> float:
        if isinstance(a, float):
            return (b - a) * 1e3
        return a.elapsed_time(b)

    def comm_stats(self) -> dict:
        """Per-step communication figures of the steps run with comm_timing on (call after a
        device sync): the exposed wait of the gradient all-reduces (the step's stream from the end
        of the backward's launches until every bucket's all-reduce is done), the blocking cosine
        statistics all-reduces, the bucket bytes and collective count. Clears the record."""
        n = len(self._marks)
        if n == 0:
            return {}
        wait = sum(self._ms(*m[1]) for m in self._marks) / n
        blk = sum(sum(self._ms(a, b) for a, b in m[0]) for m in self._marks) / n
        out = {"steps": n, "exposed_allreduce_wait_ms": round(wait, 4),
               "blocking_stats_allreduce_ms": round(blk, 4),
               "bucket_bytes": self._bucket_bytes, "collectives_per_step": self._n_coll,
               "world": self.world}
        self._marks = []
        return out

    def _ar_timed(self, t, blk):
        a = self._mark()
        self._ar(t)
        b = self._mark()
        if a is not None:
            blk.append((a, b))

    def _ar(self, t):
        if self.coll:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def close(self):
        """Restore the engine's one-GEMM layer-0 weight gradient (single-process rounding)."""
        if self._chunks_set:
            self.e.set_option("wgrad0_chunks", 1)
            self._chunks_set = False
        if self._early_set:
            self.e.set_option("early_adam", 0)
            self._early_set = False

    def step(self, x, areas, eps=None):
        e = self.e
        blk = []
        e.forward(x, eps)
        if self.cosine:
            self._ar_timed(e.colsq, blk)
        e.metric(areas)
        # the 5 loss sums are final after metric(): reduce them beside the backward
        h_loss = None
        if self.reduce_losses and self.coll:
            h_loss = dist.all_reduce(e.losses, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if self.cosine:
            self._ar_timed(e.coldot, blk)
        if self.coll and self.overlap:
            handles = []
            nbytes = 0
            for part in range(e.N_BACKWARD_PARTS):
                e.backward_part(part)
                for view in e.grad_ranges(part):
                    handles.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group,
                                                   async_op=True))
                    nbytes += view.numel() * view.element_size()
            w0 = self._mark()
            for h in handles:
                h.wait()
            w1 = self._mark()
            if w0 is not None:
                self._marks.append((blk, (w0, w1)))
                self._bucket_bytes, self._n_coll = nbytes, len(handles) + len(blk) + (h_loss is not None)
        else:
            e.backward()
            w0 = self._mark()
            self._ar(e.grads)
            w1 = self._mark()
            if w0 is not None and self.coll:
                self._marks.append((blk, (w0, w1)))
                self._bucket_bytes = e.grads.numel() * e.grads.element_size()
                self._n_coll = 1 + len(blk) + (h_loss is not None)
        e.adam()
        if h_loss is not None:
            h_loss.wait()
        return e.losses


    def predict(self, x, eps=None):
        """``get_predictions`` on this rank's rows with the global batch's cosine column norms
        (all-reduced ``colsq`` between the two phases); engines without the phases predict
        locally."""
        e = self.e
        if not hasattr(e, "predict_encode"):
            return e.predict(x, eps)
        e.predict_encode(x, eps)
        if self.cosine:
            self._ar(e.colsq)
        return e.predict_finish()


def shard_rows(t: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    n = t.shape[0] // world
    return t[rank * n:(rank + 1) * n]
