"""bench.py contract on CPU: one JSON line from rank 0, whole-job value, MAX-over-ranks timing.

Runs the real serving path with a tiny shape on the CPU (gloo for world 2). The GPU numbers come
from the same script on MI355X (profiles/).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--device", "cpu", "--batch", "2", "--image-size", "64", "--steps", "2", "--warmup", "1"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(d, n):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 2 * n and d["config"]["parallelism"] == f"dp{n}"
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    # value is the whole-job aggregate derived from the (max-over-ranks) step time
    assert abs(d["value"] - 2 * n * 1e3 / d["ms_per_step"]) / d["value"] < 0.01


def _env():
    env = dict(os.environ, AI4E_KERNEL_BACKEND="torch", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    return env


def test_bench_single_process_cpu():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1"] + ARGS, cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 1)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_torchrun_ranks_gloo(world):
    """The driver's multi-GPU launch shape (torchrun, one rank per device; rank 0 = node scheduler, the other
    ranks attach as workers + ingest shards) with gloo on CPU ranks."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(world)] + ARGS
    env = dict(_env(), OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    _check(lines[0], world)
    # warmup 1 + steps 2 + the uncounted tail (inflight 2 + 1 steps) that keeps the pipeline full past t1
    w = lines[0]["window"]
    assert w["counted_images"] == 2 * world * 2 and w["first_counted_image"] == 2 * world
    assert len(lines[0]["workers"]) == world
    assert sum(x["images"] for x in lines[0]["workers"]) == 2 * world * (3 + w["tail_steps_uncounted"])


@pytest.mark.parametrize("model,extra,par", [
    ("landcover_spatial", ["--group", "3", "--size", "128", "--tile", "32", "--stride", "24"], "spatial3"),
    ("ensemble_group", ["--group", "3", "--classifiers", "1", "--size", "64", "--batch", "2"], "pipeline2:1"),
])
def test_api_bench_worker_group_forms_cpu(model, extra, par):
    """bench/api_bench.py runs configs 4 and 5 in their multi-GPU forms through the task path (one process; the
    pool spawns the group, gloo on CPU here, RCCL on the node) and labels the parallelism."""
    cmd = [sys.executable, "bench/api_bench.py", "--model", model, "--device", "cpu", "--steps", "2", "--warmup", "1",
           "--inflight", "1"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=dict(_env(), OMP_NUM_THREADS="1"), capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_lines(r.stdout)[-1]
    assert d["config"]["parallelism"] == par and d["n_gpus"] == 3 and d["value"] > 0
    if model == "ensemble_group":
        assert d["config"]["wire_dtype"] == "uint8" and d["config"]["stage_dtypes"]["classifier"] == "fp16"
