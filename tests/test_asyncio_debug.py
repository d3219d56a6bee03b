"""asyncio debug pass over the async gateway suites (SURVEY.md §5.2 sanitizers: the Python side).

Runs the gateway, batcher, worker and drain tests in a child pytest with ``PYTHONASYNCIODEBUG=1``:
the event loops run in debug mode (a call_soon from a foreign thread raises, callbacks slower than
100 ms and never-retrieved task exceptions are logged, coroutines that are never awaited warn).
tests/conftest.py records every such report in that child and fails its session.
"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SUITES = ["tests/test_api.py", "tests/test_gateway_behaviour.py", "tests/test_batcher.py",
          "tests/test_workers.py", "tests/test_drain.py"]


def test_async_suites_clean_under_asyncio_debug():
    env = dict(os.environ, PYTHONASYNCIODEBUG="1", VGATE_DRY_RUN="true")
    r = subprocess.run([sys.executable, "-m", "pytest", *SUITES, "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        "-p", "no:xdist"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ASYNCIO-DEBUG FINDINGS" not in out, out[-4000:]
    assert "was never awaited" not in out, out[-4000:]
