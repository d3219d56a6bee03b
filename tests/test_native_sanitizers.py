"""Sanitizer tier for the native host runtime: the C++ block allocator,
sharded LRU and the lock-free TP step ring (csrc/runtime) are compiled into a host-only test program with
AddressSanitizer + UndefinedBehaviorSanitizer, and separately with ThreadSanitizer, and
run on the CPU. (GPU sanitizers / XNACK are not available on this pool: kernels are
checked by the numerics tier against fp32 references instead.) Also: the native
ShardedLRU through its Python binding and the native result-cache backend."""
from __future__ import annotations

import asyncio
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRCS = [ROOT / "csrc/tests/host_test.cpp", ROOT / "csrc/runtime/allocator.cpp", ROOT / "csrc/runtime/lru_cache.cpp"]


def _build_and_run(tmp_path, flags, name):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    import pybind11
    py_inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION")
    exe = tmp_path / name
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, f"-I{pybind11.get_include()}",
           f"-I{py_inc}", *map(str, SRCS), "-o", str(exe), f"-L{libdir}", f"-lpython{ver}", "-lpthread"]
    cmd.append("-lrt")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                            "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
                            "TSAN_OPTIONS": "halt_on_error=1"})
    assert r.returncode == 0 and "host_test: ok" in r.stdout, (r.stdout + r.stderr)[-4000:]


@pytest.mark.timeout(600)
def test_host_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "host_asan")


@pytest.mark.timeout(600)
def test_host_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], "host_tsan")


def _native():
    try:
        from vgate import ops
        return ops.native()
    except Exception:  # noqa: BLE001
        pytest.skip("native extension not built")


def test_sharded_lru_binding():
    C = _native()
    c = C.ShardedLRU(4, 1)
    for k in "abcd":
        c.put(k, k.encode() * 3)
    assert c.get("a") == b"aaa"
    assert c.put("e", b"e") == 1 and c.get("b") is None
    assert len(c) == 4 and c.hits == 1 and c.misses == 1 and c.evictions == 1


def test_result_cache_native_backend():
    _native()
    from vgate.cache import ResultCache

    async def run():
        cache = ResultCache(maxsize=2, enabled=True, backend="native")
        k1 = ResultCache.make_key("p1", 0.7, 0.9, 16)
        await cache.put(k1, {"text": "hi", "token_ids": [1, 2], "num_tokens": 2})
        v = await cache.get(k1)
        assert v == {"text": "hi", "token_ids": [1, 2], "num_tokens": 2}
        v["text"] = "mutated"  # a hit is an independent copy
        assert (await cache.get(k1))["text"] == "hi"
        for i in range(3):
            await cache.put(ResultCache.make_key(f"q{i}", 0.7, 0.9, 16), {"text": str(i)})
        st = cache.get_stats()
        assert st["size"] <= 2 and st["evictions"] >= 1 and st["hits"] == 2

    asyncio.run(run())


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-v"]))
