"""Benchmark tooling: percentile method and the load generator's result schema against a
live in-process dry-run server (the reference's bench_load contract)."""
from __future__ import annotations

import asyncio
import socket
import sys
import threading
import time
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "benchmarks"))

import bench_load  # noqa: E402


def test_percentile_index_method():
    xs = [5.0, 1.0, 3.0, 2.0, 4.0]
    assert bench_load.percentile(xs, 50) == 3.0  # sorted[min(int(5*0.5), 4)] = sorted[2]
    assert bench_load.percentile(xs, 99) == 5.0
    assert bench_load.percentile(xs, 0) == 1.0
    assert bench_load.percentile([], 50) == 0.0


def test_counter_parse():
    text = "# HELP x\nvgate_stream_tokens_total 12.0\nvgate_stream_tokens_created 1.7e9\nother 3\n"
    assert bench_load.counter_value(text, "vgate_stream_tokens_total") == 12.0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def server(clean_env):
    import uvicorn

    from vgate.api.app import create_app
    from vgate.backends.base import DryRunBackend
    from vgate.config import get_config
    from vgate.engine import VGateEngine
    cfg = get_config()
    eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=DryRunBackend(), dry_run=True)
    app = create_app(cfg, engine=eng)
    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = time.time()
    while not srv.started and time.time() - t0 < 20:
        time.sleep(0.05)
    yield f"http://127.0.0.1:{port}"
    srv.should_exit = True
    th.join(timeout=10)


def test_load_generator_schema_and_stats_diff(server):
    r = asyncio.run(bench_load.run_load_test(server, 4, 12, bench_load.DEFAULT_PROMPTS, max_tokens=8))
    assert r["failures"] == 0
    assert r["config"] == {"concurrency": 4, "total_requests": 12, "unique_prompts": 4, "max_tokens": 8,
                           "stream": False}
    assert set(r["latency"]) >= {"mean_s", "p50_s", "p95_s", "p99_s", "max_s"}
    assert r["throughput"]["requests_per_second"] > 0
    # 4 distinct prompts x 3 repeats: everything after the first wave is a cache hit or coalesced
    assert r["cache"]["hits"] + r["batching"]["deduplicated"] >= 1
    assert r["batching"]["requests"] >= 1
    md = bench_load.format_markdown(r)
    assert "Throughput" in md and "req/s" in md


def test_load_generator_streaming(server):
    r = asyncio.run(bench_load.run_load_test(server, 2, 4, bench_load.DEFAULT_PROMPTS, max_tokens=8,
                                             stream=True, unique=True))
    assert r["failures"] == 0
    assert r["throughput"]["content_chunks"] > 0
    assert r["throughput"]["total_tokens"] > 0  # from the server's vgate_stream_tokens_total
    assert r["latency"]["ttft_p50_s"] > 0


@pytest.mark.timeout(300)
def test_scenario_cli_and_aggregate(tmp_path):
    """run_scenario_cli (one scenario, fresh dry-run server process) -> JSON, twice, then
    aggregate_results -> one report (reference _run_scenario_cli.py / _aggregate_results.py)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    out = tmp_path / "sc"
    for name in ("baseline", "cache_impact"):
        r = subprocess.run([sys.executable, str(root / "benchmarks/run_scenario_cli.py"), name, "--engine", "dry-run",
                            "--requests", "8", "--concurrency", "4", "--max-tokens", "4", "--port", "18770",
                            "--dry-latency-ms", "2", "--out-dir", str(out)],
                           capture_output=True, text=True, timeout=240, cwd=str(root))
        assert r.returncode == 0, r.stderr[-3000:]
        assert json.loads(r.stdout.strip().splitlines()[-1])["scenario"] == name
    r = subprocess.run([sys.executable, str(root / "benchmarks/aggregate_results.py"), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rep = json.loads((out / "report.json").read_text())
    assert list(rep) == ["baseline", "cache_impact"]
    assert rep["baseline"]["throughput"]["requests_per_second"] > 0
    assert "| baseline |" in (out / "report.md").read_text()
