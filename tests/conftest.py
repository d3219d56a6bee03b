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
