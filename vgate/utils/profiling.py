"""Opt-in ROCTx ranges around engine phases (GPU profiling hooks the
reference lacks — it only relays vLLM's TTFT/gen-time).

``VGATE_ROCTX=1`` loads the rocprofiler-sdk ROCTx library and every :func:`range_` in the
engine (``vgate.step``, ``vgate.schedule``, ``vgate.launch``, ``vgate.collect``,
``vgate.process``, graph captures) becomes a push/pop pair that
``rocprofv3 --marker-trace --kernel-trace`` records next to the kernels, so a trace shows
which host phase issued which graph replay. Disabled (the default) it is a shared no-op
context manager: no ctypes call, no allocation on the hot path.

    VGATE_ROCTX=1 rocprofv3 --marker-trace --kernel-trace -d out -- python3 bench.py --steps 2
"""
from __future__ import annotations

import contextlib
import ctypes
import logging
import os

log = logging.getLogger("vgate.profiling")

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")
_lib = None
_NULL = contextlib.nullcontext()


def _load():
    global _lib
    for name in _LIBS:
        for path in (name, os.path.join("/opt/rocm/lib", name)):
            try:
                lib = ctypes.CDLL(path)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                return True
            except (OSError, AttributeError):
                continue
    log.warning("VGATE_ROCTX=1 but no ROCTx library could be loaded; ranges disabled")
    return False


ENABLED = os.environ.get("VGATE_ROCTX", "0") not in ("", "0", "false") and _load()


class _Range:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name.encode()

    def __enter__(self):
        _lib.roctxRangePushA(self.name)
        return self

    def __exit__(self, *exc):
        _lib.roctxRangePop()
        return False


def range_(name: str):
    """Context manager: a ROCTx range when VGATE_ROCTX=1, otherwise a shared no-op."""
    return _Range(name) if ENABLED else _NULL


def mark(name: str) -> None:
    if ENABLED:
        _lib.roctxMarkA(name.encode())
