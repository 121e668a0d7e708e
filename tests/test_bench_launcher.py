"""bench.py's launcher, data-parallel, timing and JSON path on CPU (``--dry-run``: gloo, a
stand-in engine, no kernels). ``--gpus 2`` without a torchrun environment must start two
ranks itself and report the whole job: n_gpus 2, global batch 2B, and the same all-reduced
result as one rank on the concatenated batch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", *args],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks_and_matches_one():
    two = _run("--gpus", "2", "--batch", "8", "--steps", "3", "--warmup", "1")
    one = _run("--gpus", "1", "--batch", "16", "--steps", "3", "--warmup", "1")
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["global_batch"] == 16 and two["config"]["per_gpu_batch"] == 8
    assert two["config"]["parallelism"] == "dp2" and two["scaling"] == "weak"
    assert abs(two["grad_checksum"] - one["grad_checksum"]) <= 1e-9 * abs(one["grad_checksum"])
    for k in one["losses"]:
        assert abs(two["losses"][k] - one["losses"][k]) <= 1e-9 * max(abs(one["losses"][k]), 1.0)
    # whole-job throughput: pairs of all ranks / max-over-ranks time
    assert abs(two["value"] - 16 * 3 / (two["ms_per_step"] * 3e-3)) <= 1e-3 * two["value"]
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better",
              "vs_baseline", "dtype", "data", "roofline", "cpu_baseline", "h2d", "configs", "build_id"):
        assert k in two and k in one
    # the configs block: C3 / C5 / C5CONV on one GPU, C4 (C3's shape per rank) / C5 with N ranks, each
    # with its own value and rooflines
    assert set(one["configs"]) == {"C3", "C5", "C5CONV"} and set(two["configs"]) == {"C4", "C5"}
    for line in (one, two):
        for cid, c in line["configs"].items():
            for k in ("workload", "value", "ms_per_step", "global_batch", "per_gpu_batch", "roofline",
                      "loss_roofline"):
                assert k in c, (cid, k)
    assert two["configs"]["C4"]["global_batch"] == 2 * two["configs"]["C4"]["per_gpu_batch"]
    # communication figures with N ranks (none with one): exposed all-reduce wait per step, the
    # bucket, and the bucket-sized all-reduce's bus bandwidth
    assert one["comm"] is None
    for c in (two["comm"], two["configs"]["C4"]["comm"], two["configs"]["C5"]["comm"]):
        for k in ("exposed_allreduce_wait_ms", "blocking_stats_allreduce_ms", "bucket_bytes",
                  "collectives_per_step", "allreduce_bench"):
            assert k in c, k
        assert c["bucket_bytes"] > 0 and c["steps"] == 3 and c["world"] == 2
        assert c["allreduce_bench"]["busbw_GBps"] > 0
