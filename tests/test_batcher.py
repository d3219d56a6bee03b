"""Batcher: fan-out, in-flight dedup, admission, abandonment, error propagation, async backends."""
import asyncio
import threading
import time

import pytest

from vgate.batcher import RequestBatcher
from vgate.config import VGateConfig, set_config


class _Engine:
    def __init__(self, backend):
        self.backend = backend
        self.is_remote = False


class RecordingBackend:
    supports_concurrent_calls = True

    def __init__(self, delay=0.0, fail=False):
        self.calls = []
        self.delay = delay
        self.fail = fail
        self.active = 0
        self.peak = 0
        self._lock = threading.Lock()

    def create_sampling_params(self, temperature, top_p, max_tokens):
        return {"temperature": temperature, "top_p": top_p, "max_tokens": max_tokens}

    def generate(self, prompts, sp):
        with self._lock:
            self.active += 1
            self.peak = max(self.peak, self.active)
            self.calls.append(list(prompts))
        try:
            time.sleep(self.delay)
            if self.fail:
                raise RuntimeError("boom")
            return [{"text": f"out:{p}", "num_tokens": 3, "metrics": {"ttft": 0.01, "gen_time": 0.03}}
                    for p in prompts]
        finally:
            with self._lock:
                self.active -= 1


class AsyncBackend(RecordingBackend):
    async def agenerate(self, prompt, sp):
        self.active += 1
        self.peak = max(self.peak, self.active)
        self.calls.append([prompt])
        try:
            await asyncio.sleep(self.delay)
            if self.fail:
                raise RuntimeError("boom")
            return {"text": f"out:{prompt}", "num_tokens": 4, "prompt_tokens": 2, "finish_reason": "length",
                    "metrics": {"ttft": 0.01, "gen_time": 0.04}}
        finally:
            self.active -= 1


@pytest.fixture(autouse=True)
def cfg():
    set_config(VGateConfig(batch={"max_batch_size": 4}, cache={"enabled": True, "maxsize": 100}))
    yield


async def test_one_backend_call_per_request_and_result_shape():
    be = RecordingBackend()
    b = RequestBatcher(_Engine(be))
    await b.start()
    rs = await asyncio.gather(*(b.submit(f"p{i}", max_tokens=8) for i in range(5)))
    assert len(be.calls) == 5 and all(len(c) == 1 for c in be.calls)
    assert rs[0]["text"] == "out:p0" and rs[0]["total_tokens"] == 3
    assert rs[0]["tpot"] == pytest.approx(0.01)
    m = b.get_metrics()
    assert m["total_requests"] == 5 and m["total_batches"] == 5 and m["average_batch_size"] == 1.0


async def test_async_backend_used_directly_with_extra_fields():
    be = AsyncBackend(delay=0.01)
    b = RequestBatcher(_Engine(be))
    r = await b.submit("x", max_tokens=4)
    assert r["prompt_tokens"] == 2 and r["finish_reason"] == "length" and r["total_tokens"] == 4


async def test_dedup_only_while_inflight_and_cache_hit():
    be = AsyncBackend(delay=0.05)
    b = RequestBatcher(_Engine(be))
    rs = await asyncio.gather(*(b.submit("same", max_tokens=8) for _ in range(4)))
    assert len(be.calls) == 1 and all(r["text"] == "out:same" for r in rs)
    assert b.total_deduplicated == 3
    before = b.total_requests
    r = await b.submit("same", max_tokens=8)  # now a cache hit
    assert r["text"] == "out:same" and len(be.calls) == 1
    assert b.total_requests == before  # cache hits are not counted


async def test_admission_limit_bounds_concurrency():
    be = AsyncBackend(delay=0.03)
    b = RequestBatcher(_Engine(be), max_batch_size=2)
    await asyncio.gather(*(b.submit(f"q{i}") for i in range(8)))
    assert be.peak == 2


async def test_serial_backend_forced_to_one():
    class Serial(RecordingBackend):
        supports_concurrent_calls = False
    be = Serial(delay=0.02)
    b = RequestBatcher(_Engine(be), max_batch_size=8)
    assert b.max_concurrent_inferences == 1
    await asyncio.gather(*(b.submit(f"s{i}") for i in range(4)))
    assert be.peak == 1


async def test_errors_reach_all_waiters_and_are_not_cached():
    be = AsyncBackend(delay=0.02, fail=True)
    b = RequestBatcher(_Engine(be))
    res = await asyncio.gather(*(b.submit("bad") for _ in range(3)), return_exceptions=True)
    assert all(isinstance(r, RuntimeError) for r in res)
    assert len(be.calls) == 1
    be.fail = False
    r = await b.submit("bad")
    assert r["text"] == "out:bad" and len(be.calls) == 2


async def test_abandoned_queued_work_is_cancelled_started_survives():
    be = AsyncBackend(delay=0.2)
    b = RequestBatcher(_Engine(be), max_batch_size=1)
    t1 = asyncio.create_task(b.submit("first"))
    await asyncio.sleep(0.02)  # first is running, holds the only permit
    with pytest.raises(asyncio.TimeoutError):
        await b.submit("second", timeout=0.05)  # queued, then abandoned
    await asyncio.sleep(0.01)
    r1 = await t1
    await asyncio.sleep(0.05)
    assert r1["text"] == "out:first"
    assert [c[0] for c in be.calls] == ["first"]  # "second" never ran
    # started work survives its waiter timing out and still fills the cache
    t = asyncio.create_task(b.submit("third", timeout=0.05))
    with pytest.raises(asyncio.TimeoutError):
        await t
    await asyncio.sleep(0.3)
    hit = await b.cache.get(b.cache.make_key("third", 0.7, 0.9, 256))
    assert hit is not None


async def test_followers_hold_no_permit():
    be = AsyncBackend(delay=0.1)
    b = RequestBatcher(_Engine(be), max_batch_size=1)
    ts = [asyncio.create_task(b.submit("dup")) for _ in range(5)]
    await asyncio.sleep(0.02)
    other = asyncio.create_task(b.submit("other"))
    await asyncio.gather(*ts, other)
    assert sorted(c[0] for c in be.calls) == ["dup", "other"]


async def test_stop_drains_inflight():
    be = AsyncBackend(delay=0.05)
    b = RequestBatcher(_Engine(be))
    t = asyncio.create_task(b.submit("d"))
    await asyncio.sleep(0.01)
    await b.stop()
    assert t.done() and (await t)["text"] == "out:d"


async def test_sync_backend_runs_in_executor():
    be = RecordingBackend(delay=0.05)
    b = RequestBatcher(_Engine(be), max_batch_size=4)
    t0 = time.perf_counter()
    await asyncio.gather(*(b.submit(f"e{i}") for i in range(4)))
    assert time.perf_counter() - t0 < 0.18  # ran concurrently, not serialised
