"""bench.py driver contract, multi-process: 2 ranks via torch.distributed.run (gloo
coordination, one server + closed-loop client + engine per rank, tiny model on CPU).
Rank 0 prints exactly one JSON line with the required keys; value is the whole-job
aggregate over the ranks' MAX wall time."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


@pytest.mark.timeout(600)
def test_bench_two_ranks_cpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2", VGATE_DRY_RUN="false")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29541", str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", "1", "--warmup", "1", "--model", "tiny", "--max-tokens", "4", "--requests-per-step", "4",
           "--kv-blocks", "256", "--port", "18300"]
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert REQUIRED <= set(r)
    assert r["n_gpus"] == 2 and r["steps"] == 1 and r["warmup"] == 1
    assert r["unit"] == "req/s" and r["higher_is_better"] is True and r["scaling"] == "weak"
    assert r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 16
    assert r["value"] > 0 and r["failures"] == 0
    # value = total requests over the slowest rank's wall time
    assert abs(r["value"] - 8 / (r["ms_per_step"] / 1e3)) / r["value"] < 0.02


@pytest.mark.timeout(600)
def test_bench_tensor_parallel_two_ranks_cpu(tmp_path):
    """--tp 2: ONE replica whose TP follower rank executes the serving rank's steps (shared-memory
    step ring, gloo collectives on CPU); the JSON line reports dp1xtp2 and the replica's load."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2", VGATE_DRY_RUN="false")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29543", str(ROOT / "bench.py"), "--gpus", "2", "--tp", "2",
           "--steps", "1", "--warmup", "1", "--model", "tiny-tp8", "--max-tokens", "4", "--requests-per-step", "4",
           "--kv-blocks", "256", "--port", "18310"]
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert REQUIRED <= set(r)
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp1xtp2" and r["config"]["global_batch"] == 8
    assert r["value"] > 0 and r["failures"] == 0


@pytest.mark.timeout(600)
def test_bench_forensics_account_for_the_timed_wall(tmp_path):
    """One rank on CPU: the engine thread's timed wall splits into idle + coalesce + busy and that sum
    matches the timed wall; per-step averages and the wave trace are timed-region
    fields."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2", VGATE_DRY_RUN="false")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1", "--model", "tiny",
           "--max-tokens", "8", "--requests-per-step", "16", "--kv-blocks", "512", "--port", "18340"]
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=540)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    wall, acc = r["timed_wall_ms"], r["timed_wall_ms_accounted"]
    assert wall > 0 and abs(acc - wall) / wall < 0.05, (acc, wall)
    assert r["timed_engine_busy_ms"] > 0 and r["timed_engine_coalesce_ms"] >= 0
    assert r["engine_avg_step_ms"] is not None and r["engine_avg_step_ms"] > 0
