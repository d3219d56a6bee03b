"""Shared pytest configuration.

* registers the ``gpu`` marker (tests needing a real MI355X; run with ``-m gpu``)
* runs ``async def`` tests without pytest-asyncio (not installed here): each
  coroutine test gets a fresh event loop via ``asyncio.run``
* resets global config/tracing state between tests
"""
from __future__ import annotations

import asyncio
import inspect
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
CLIENT = ROOT / "vgate-client"
if str(CLIENT) not in sys.path:
    sys.path.insert(0, str(CLIENT))

os.environ.setdefault("VGATE_DRY_RUN", "true")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (gfx950) and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")
    if os.environ.get("PYTHONASYNCIODEBUG"):
        _install_asyncio_debug_recorder()


# ---- asyncio debug pass (tests/test_asyncio_debug.py runs the async suites with
# PYTHONASYNCIODEBUG=1): every asyncio-logger warning (slow callback > 100 ms, non-threadsafe call,
# never-retrieved exception) and every "coroutine ... was never awaited" is recorded and fails the run
ASYNCIO_DEBUG_FINDINGS: list[str] = []


def _install_asyncio_debug_recorder() -> None:
    import logging
    import re
    import warnings

    class _Rec(logging.Handler):
        def emit(self, record):
            msg = record.getMessage()
            if "coro=<test_" in msg:  # a test function's own body blocking its loop: harness, not product
                return
            m = re.search(r" took ([0-9.]+) seconds", msg)
            if m and float(m.group(1)) < 0.25:  # 0.1-0.25 s: CPU contention of a loaded test host, not a
                return                          # blocking call (those take the same time on an idle one)
            ASYNCIO_DEBUG_FINDINGS.append(f"asyncio {record.levelname}: {msg}")

    lg = logging.getLogger("asyncio")
    lg.addHandler(_Rec(level=logging.WARNING))
    lg.setLevel(logging.WARNING)
    orig = warnings.showwarning

    def show(message, category, filename, lineno, file=None, line=None):
        if issubclass(category, RuntimeWarning) and "never awaited" in str(message):
            ASYNCIO_DEBUG_FINDINGS.append(f"{category.__name__}: {message} ({filename}:{lineno})")
        return orig(message, category, filename, lineno, file, line)
    warnings.showwarning = show
    warnings.filterwarnings("always", message=".*was never awaited", category=RuntimeWarning)


def pytest_sessionfinish(session, exitstatus):
    if os.environ.get("PYTHONASYNCIODEBUG") and ASYNCIO_DEBUG_FINDINGS:
        import gc
        gc.collect()
        sys.stderr.write("\nASYNCIO-DEBUG FINDINGS:\n" + "\n".join(ASYNCIO_DEBUG_FINDINGS) + "\n")
        session.exitstatus = 1


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    fn = pyfuncitem.obj
    if inspect.iscoroutinefunction(fn):
        argnames = pyfuncitem._fixtureinfo.argnames
        kwargs = {n: pyfuncitem.funcargs[n] for n in argnames if n in pyfuncitem.funcargs}
        asyncio.run(fn(**kwargs))
        return True
    return None


@pytest.fixture(autouse=True)
def _reset_globals():
    yield
    try:
        from vgate.config import reset_config
        reset_config()
    except Exception:  # noqa: BLE001
        pass
    try:
        from vgate import tracing
        tracing.shutdown_tracing()
    except Exception:  # noqa: BLE001
        pass


@pytest.fixture
def clean_env(monkeypatch):
    """Strip every VGATE_* variable so config tests see only what they set."""
    for k in list(os.environ):
        if k.startswith("VGATE_"):
            monkeypatch.delenv(k, raising=False)
    yield monkeypatch


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


# ---- GPU tests: the in-launch hand-off words are "zeroed once, self-resetting" — every launch leaves
# them zero. A test that leaves one set would poison the next kernel that shares the buffer (the GEMM
# split-K tickets and the flash K-split tickets live in the same workspace), so check after each GPU
# test and name the test that did it.
@pytest.fixture(autouse=True)
def _gpu_handoff_words_clean(request):
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    try:
        import torch

        from vgate import ops
    except Exception:  # noqa: BLE001
        return
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    dirty = []
    for name, store, n in (("workspace tickets", getattr(ops, "_WS", {}), 65536),
                           ("attention tickets", getattr(ops, "_TICKETS", {}), None)):
        for key, t in list(store.items()):
            v = t[:n] if n else t
            if v.dtype != torch.int32:
                v = v.view(torch.int32)[:n] if n else v.view(torch.int32)
            nz = int(torch.count_nonzero(v))
            if nz:
                dirty.append(f"{name} [{key}]: {nz} non-zero words")
                v.zero_()  # the next test starts clean
    assert not dirty, "in-launch hand-off words left set: " + "; ".join(dirty)
