"""Bearer-key authentication + per-key sliding-window rate limiting.

Behavioral contract kept from the reference (``vgate/security.py:42-265``,
SURVEY.md Appendix A item 8): exact-match exempt paths; ``Authorization: Bearer
<key>`` with a case-insensitive scheme and exactly two tokens; missing key ->
401 ``Missing API key. Use Authorization: Bearer <api_key>``; unknown key -> 401
``Invalid API key``; over the limit -> 429 ``{"detail": "Rate limit exceeded",
"retry_after": n}`` + ``Retry-After``; ``X-RateLimit-Limit/Remaining/Reset``
(Reset = wall-clock epoch) on admitted responses; the window runs on the
monotonic clock.

Implementation is built for the high-QPS configuration: a pure-ASGI middleware
(no per-request task/stream wrapping like BaseHTTPMiddleware) and O(1) amortised
deque windows instead of list rebuilds.
"""
from __future__ import annotations

import contextlib
import json
import time
from collections import defaultdict, deque
from typing import Optional

from vgate.config import APIKeyConfig, SecurityConfig
from vgate.logging_config import get_logger
from vgate.tracing import _NOOP, get_tracer, is_tracing_enabled

logger = get_logger("vgate.security")
tracer = get_tracer(__name__)
_NO_SPAN = contextlib.nullcontext(_NOOP)


class RateLimiter:
    """Sliding window over monotonic timestamps, one deque per key."""

    def __init__(self, window_seconds: int = 60):
        self.window_seconds = window_seconds
        self._requests: dict[str, deque] = defaultdict(deque)

    def _cleanup(self, key: str, now: float) -> deque:
        q = self._requests[key]
        cutoff = now - self.window_seconds
        while q and q[0] <= cutoff:
            q.popleft()
        return q

    def is_allowed(self, key: str, limit: int) -> tuple[bool, dict]:
        now = time.monotonic()
        q = self._cleanup(key, now)
        count = len(q)
        remaining = max(0, limit - count)
        headers = {
            "X-RateLimit-Limit": str(limit),
            "X-RateLimit-Remaining": str(remaining),
            "X-RateLimit-Reset": str(int(time.time() + self.window_seconds)),
        }
        if count >= limit:
            if q:
                retry = int(q[0] + self.window_seconds - now) + 1
                headers["Retry-After"] = str(max(1, retry))
            else:
                headers["Retry-After"] = str(self.window_seconds)
            return False, headers
        q.append(now)
        headers["X-RateLimit-Remaining"] = str(remaining - 1)
        return True, headers

    def get_usage(self, key: str) -> dict:
        q = self._cleanup(key, time.monotonic())
        return {"current_requests": len(q), "window_seconds": self.window_seconds}


_HDR_NAMES = {k: k.lower().encode() for k in ("X-RateLimit-Limit", "X-RateLimit-Remaining", "X-RateLimit-Reset",
                                               "Retry-After")}


def parse_bearer(value: Optional[str]) -> Optional[str]:
    if not value:
        return None
    parts = value.split()
    if len(parts) != 2 or parts[0].lower() != "bearer":
        return None
    return parts[1]


def extract_api_key(request) -> Optional[str]:
    """From a Starlette/FastAPI request (or anything with ``.headers``)."""
    return parse_bearer(request.headers.get("Authorization"))


def _header(scope, name: bytes) -> Optional[str]:
    for k, v in scope.get("headers", ()):
        if k == name:
            return v.decode("latin-1")
    return None


class SecurityMiddleware:
    """Pure ASGI middleware: ``app.add_middleware(SecurityMiddleware, config=cfg.security)``."""

    def __init__(self, app, config: SecurityConfig):
        self.app = app
        self.config = config
        self.key_map: dict[str, APIKeyConfig] = {k.key: k for k in config.api_keys}
        self.exempt = set(config.exempt_paths)
        self.limiter = RateLimiter(config.rate_limiting.window_seconds)
        logger.info("Security middleware initialized", extra={"extra_data": {
            "enabled": config.enabled, "api_keys_count": len(config.api_keys),
            "rate_limiting_enabled": config.rate_limiting.enabled, "exempt_paths": config.exempt_paths}})

    async def _reject(self, send, status: int, body: dict, headers: dict | None = None):
        raw = json.dumps(body).encode()
        hdrs = [(b"content-type", b"application/json"), (b"content-length", str(len(raw)).encode())]
        for k, v in (headers or {}).items():
            hdrs.append((k.lower().encode(), str(v).encode()))
        await send({"type": "http.response.start", "status": status, "headers": hdrs})
        await send({"type": "http.response.body", "body": raw})

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http" or not self.config.enabled:
            await self.app(scope, receive, send)
            return
        path = scope.get("path", "")
        if path in self.exempt:
            await self.app(scope, receive, send)
            return
        with (tracer.start_as_current_span("security.check") if is_tracing_enabled() else _NO_SPAN) as span:
            span.set_attribute("http.path", path)
            key = parse_bearer(_header(scope, b"authorization"))
            if not key:
                logger.warning("Missing API key", extra={"extra_data": {"path": path, "method": scope.get("method")}})
                await self._reject(send, 401, {"detail": "Missing API key. Use Authorization: Bearer <api_key>"})
                return
            kc = self.key_map.get(key)
            if kc is None:
                logger.warning("Invalid API key", extra={"extra_data": {"path": path, "method": scope.get("method")}})
                await self._reject(send, 401, {"detail": "Invalid API key"})
                return
            span.set_attribute("api_key_name", kc.name)
            headers: dict = {}
            if self.config.rate_limiting.enabled:
                allowed, headers = self.limiter.is_allowed(key, kc.rate_limit)
                if not allowed:
                    logger.warning("Rate limit exceeded", extra={"extra_data": {
                        "key_name": kc.name, "path": path, "limit": kc.rate_limit}})
                    await self._reject(send, 429, {"detail": "Rate limit exceeded",
                                                   "retry_after": int(headers.get("Retry-After", 60))}, headers)
                    return
        if not headers:
            await self.app(scope, receive, send)
            return
        extra = [(_HDR_NAMES.get(k) or k.lower().encode(), v.encode()) for k, v in headers.items()]

        async def send_with_headers(msg):
            if msg["type"] == "http.response.start":
                msg = dict(msg)
                msg["headers"] = list(msg.get("headers", [])) + extra
            await send(msg)

        await self.app(scope, receive, send_with_headers)
