"""Result cache (LRU, keying, disabled mode) and security (bearer parsing, sliding window, middleware)."""
import asyncio
import time

import httpx
import pytest
from fastapi import FastAPI

from vgate.cache import ResultCache
from vgate.config import SecurityConfig
from vgate.security import RateLimiter, SecurityMiddleware, parse_bearer


# ----------------------------------------------------------------------------- cache
def test_make_key_stable_and_sensitive():
    k = ResultCache.make_key("p", 0.7, 0.9, 64)
    assert k == ResultCache.make_key("p", 0.7, 0.9, 64) and len(k) == 16
    assert k != ResultCache.make_key("p", 0.7, 0.9, 65)
    assert k != ResultCache.make_key("q", 0.7, 0.9, 64)
    # same algorithm as the reference: sha256 of sorted-key JSON, first 16 hex chars
    import hashlib
    import json
    blob = json.dumps({"prompt": "p", "temperature": 0.7, "top_p": 0.9, "max_tokens": 64}, sort_keys=True)
    assert k == hashlib.sha256(blob.encode()).hexdigest()[:16]


async def test_lru_eviction_and_stats():
    c = ResultCache(maxsize=2, enabled=True)
    await c.put("a", {"v": 1})
    await c.put("b", {"v": 2})
    assert (await c.get("a"))["v"] == 1  # a becomes most recent
    await c.put("c", {"v": 3})  # evicts b
    assert await c.get("b") is None
    assert (await c.get("c"))["v"] == 3
    s = c.get_stats()
    assert s["size"] == 2 and s["evictions"] == 1 and s["hits"] == 2 and s["misses"] == 1


async def test_cache_returns_copies():
    c = ResultCache(maxsize=4, enabled=True)
    await c.put("k", {"text": "x", "n": [1]})
    got = await c.get("k")
    got["text"] = "mutated"
    got["n"].append(2)
    again = await c.get("k")
    assert again == {"text": "x", "n": [1]}


async def test_disabled_cache_noop():
    c = ResultCache(maxsize=4, enabled=False)
    await c.put("k", {"v": 1})
    assert await c.get("k") is None and len(c) == 0


# -------------------------------------------------------------------------- security
@pytest.mark.parametrize("hdr,expect", [("Bearer abc", "abc"), ("bearer abc", "abc"), ("BEARER abc", "abc"),
                                        ("Bearer", None), ("Basic abc", None), ("Bearer a b", None), ("", None),
                                        (None, None)])
def test_parse_bearer(hdr, expect):
    assert parse_bearer(hdr) == expect


def test_rate_limiter_window_and_headers():
    rl = RateLimiter(window_seconds=60)
    for i in range(3):
        ok, h = rl.is_allowed("k", 3)
        assert ok and h["X-RateLimit-Remaining"] == str(2 - i)
    ok, h = rl.is_allowed("k", 3)
    assert not ok and int(h["Retry-After"]) >= 1 and h["X-RateLimit-Limit"] == "3"
    assert abs(int(h["X-RateLimit-Reset"]) - (time.time() + 60)) < 3  # wall-clock epoch


def test_rate_limiter_uses_monotonic_clock(monkeypatch):
    rl = RateLimiter(window_seconds=60)
    assert rl.is_allowed("k", 1)[0]
    # a wall-clock jump must not reopen the window
    monkeypatch.setattr(time, "time", lambda: 10**12)
    assert not rl.is_allowed("k", 1)[0]


def test_rate_limiter_expiry(monkeypatch):
    now = [1000.0]
    monkeypatch.setattr(time, "monotonic", lambda: now[0])
    rl = RateLimiter(window_seconds=10)
    assert rl.is_allowed("k", 1)[0]
    assert not rl.is_allowed("k", 1)[0]
    now[0] += 10.5
    assert rl.is_allowed("k", 1)[0]
    assert rl.get_usage("k")["current_requests"] == 1


def _secured_app(**kw):
    cfg = SecurityConfig(enabled=True, api_keys=[{"key": "good", "name": "dev", "rate_limit": 2}], **kw)
    app = FastAPI()

    @app.get("/x")
    async def x():
        return {"ok": True}

    @app.get("/health")
    async def h():
        return {"status": "ok"}

    app.add_middleware(SecurityMiddleware, config=cfg)
    return app


async def _client(app):
    return httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t")


async def test_middleware_auth_and_limits():
    async with await _client(_secured_app()) as c:
        r = await c.get("/x")
        assert r.status_code == 401 and r.json() == {"detail": "Missing API key. Use Authorization: Bearer <api_key>"}
        r = await c.get("/x", headers={"Authorization": "Bearer bad"})
        assert r.status_code == 401 and r.json() == {"detail": "Invalid API key"}
        r = await c.get("/x", headers={"Authorization": "Bearer good"})
        assert r.status_code == 200 and r.headers["X-RateLimit-Remaining"] == "1"
        await c.get("/x", headers={"Authorization": "Bearer good"})
        r = await c.get("/x", headers={"Authorization": "Bearer good"})
        assert r.status_code == 429
        assert r.json()["detail"] == "Rate limit exceeded" and r.json()["retry_after"] >= 1
        assert "Retry-After" in r.headers
        # exempt path: exact match only
        assert (await c.get("/health")).status_code == 200
        assert (await c.get("/health/")).status_code in (401, 404, 307)


async def test_middleware_disabled_passthrough():
    cfg = SecurityConfig(enabled=False)
    app = FastAPI()

    @app.get("/x")
    async def x():
        return {"ok": True}

    app.add_middleware(SecurityMiddleware, config=cfg)
    async with await _client(app) as c:
        r = await c.get("/x")
        assert r.status_code == 200 and "X-RateLimit-Limit" not in r.headers


def test_rate_limiter_high_qps_is_fast():
    rl = RateLimiter(window_seconds=60)
    t0 = time.perf_counter()
    for _ in range(50_000):
        rl.is_allowed("k", 10**9)
    assert time.perf_counter() - t0 < 2.0  # O(1) amortised; the list-rebuild design is O(n) per call
