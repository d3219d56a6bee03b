"""ROCTx hook (vgate/utils/profiling.py): disabled -> shared no-op; enabled -> real
push/pop into the ROCm ROCTx library (a subprocess, since the switch is read at import)."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_disabled_is_shared_noop():
    from vgate.utils import profiling
    if profiling.ENABLED:
        return
    assert profiling.range_("a") is profiling.range_("b")
    with profiling.range_("x"):
        pass
    profiling.mark("m")


def test_enabled_pushes_and_pops():
    code = ("from vgate.utils import profiling as p\n"
            "assert p.ENABLED, 'roctx library not loaded'\n"
            "with p.range_('vgate.test'):\n    p.mark('inside')\n"
            "print('ok')\n")
    env = dict(os.environ, VGATE_ROCTX="1", PYTHONPATH=str(ROOT))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=60)
    if "roctx library not loaded" in r.stderr:
        import pytest
        pytest.skip("no ROCTx library in this image")
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr
