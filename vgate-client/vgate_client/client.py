"""Sync and async V-Gate clients.

Behavior contract:
* unary requests retry on 429 (sleeping ``Retry-After`` or ``2**attempt``) and on
  5xx (``2**attempt``), up to ``max_retries``; connection failures raise
  :class:`ConnectionError`; 401 -> AuthenticationError, 429 -> RateLimitError;
* streams are never retried (text already delivered would be duplicated); the
  response must be ``text/event-stream``; an in-band error event or a stream that
  ends without ``data: [DONE]`` raises ServerError;
* stream objects are iterators AND (async) context managers, so breaking out
  early closes the HTTP connection deterministically.

The retry/backoff decision and SSE parsing live in one place (:class:`_Policy`,
:func:`parse_sse_line`) shared by both clients.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import AsyncIterator, Iterator, Optional

import httpx

from .exceptions import AuthenticationError, ConnectionError, RateLimitError, ServerError, VGateError
from .models import (ChatCompletion, ChatCompletionChunk, ChatCompletionRequest, ChatMessage, EmbeddingRequest,
                     EmbeddingResponse, HealthResponse, RateLimitInfo)

DEFAULT_BASE_URL = "http://localhost:8000"
DEFAULT_TIMEOUT = 60.0
DEFAULT_MAX_RETRIES = 2
STREAM_DONE = object()

# indirection points so tests can skip backoff waits without patching the stdlib
_sleep = time.sleep
_asleep = asyncio.sleep


def parse_rate_limit(headers: httpx.Headers) -> RateLimitInfo:
    def num(key, cast):
        v = headers.get(key)
        try:
            return cast(v) if v is not None else None
        except ValueError:
            return None
    return RateLimitInfo(limit=num("X-RateLimit-Limit", int), remaining=num("X-RateLimit-Remaining", int),
                         reset=num("X-RateLimit-Reset", float), retry_after=num("Retry-After", float))


def raise_for_status(resp: httpx.Response) -> None:
    if resp.is_success:
        return
    try:
        body = resp.json()
    except Exception:  # noqa: BLE001
        body = {"detail": resp.text}
    detail = body.get("detail", resp.text) if isinstance(body, dict) else resp.text
    code = resp.status_code
    if code == 401:
        raise AuthenticationError(str(detail), status_code=code, body=body)
    if code == 429:
        raise RateLimitError(str(detail), retry_after=parse_rate_limit(resp.headers).retry_after,
                             status_code=code, body=body)
    if code >= 500:
        raise ServerError(str(detail), status_code=code, body=body)
    raise VGateError(str(detail), status_code=code, body=body)


def parse_sse_line(line: str):
    """None (skip) | STREAM_DONE | ChatCompletionChunk; raises ServerError on an error event."""
    if not line or not line.startswith("data:"):
        return None
    payload = line[5:].lstrip(" ")
    if payload == "[DONE]":
        return STREAM_DONE
    data = json.loads(payload)
    if isinstance(data, dict) and "error" in data:
        err = data["error"] if isinstance(data["error"], dict) else {"message": str(data["error"])}
        raise ServerError(err.get("message", "stream error"), body=data)
    return ChatCompletionChunk.model_validate(data)


def check_stream_content_type(resp: httpx.Response) -> None:
    ct = resp.headers.get("content-type", "")
    if "text/event-stream" not in ct:
        raise VGateError(f"Expected a text/event-stream response but got Content-Type: {ct or '<missing>'}",
                         status_code=resp.status_code)


class _Policy:
    """Retry decision shared by both clients: returns seconds to wait, or None to stop."""

    def __init__(self, max_retries: int):
        self.max_retries = max_retries

    def backoff(self, resp: httpx.Response, attempt: int) -> Optional[float]:
        if attempt >= self.max_retries:
            return None
        if resp.status_code == 429:
            ra = parse_rate_limit(resp.headers).retry_after
            return ra if ra is not None else float(2 ** attempt)
        if resp.status_code >= 500:
            return float(2 ** attempt)
        return None


def _headers(api_key: Optional[str]) -> dict:
    h = {"Content-Type": "application/json"}
    if api_key:
        h["Authorization"] = f"Bearer {api_key}"
    return h


def _chat_req(model, messages, temperature, top_p, max_tokens, stream=False) -> dict:
    return ChatCompletionRequest(model=model, messages=[ChatMessage(**m) for m in messages],
                                 temperature=temperature, top_p=top_p, max_tokens=max_tokens,
                                 stream=stream).model_dump()


class SyncChatStream:
    def __init__(self, gen: Iterator[ChatCompletionChunk]):
        self._gen = gen

    def __iter__(self):
        return self

    def __next__(self) -> ChatCompletionChunk:
        return next(self._gen)

    def close(self) -> None:
        self._gen.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class AsyncChatStream:
    def __init__(self, gen: AsyncIterator[ChatCompletionChunk]):
        self._gen = gen

    def __aiter__(self):
        return self

    async def __anext__(self) -> ChatCompletionChunk:
        return await self._gen.__anext__()

    async def aclose(self) -> None:
        await self._gen.aclose()

    async def __aenter__(self):
        return self

    async def __aexit__(self, *exc):
        await self.aclose()


# ------------------------------------------------------------------ sync client
class _SyncChat:
    def __init__(self, client: "VGate"):
        self._c = client

    def create(self, *, model: str, messages: list[dict], temperature: float = 0.7, top_p: float = 0.9,
               max_tokens: int = 256) -> ChatCompletion:
        data = self._c._request("POST", "/v1/chat/completions",
                                json=_chat_req(model, messages, temperature, top_p, max_tokens))
        return ChatCompletion.model_validate(data)

    def stream(self, *, model: str, messages: list[dict], temperature: float = 0.7, top_p: float = 0.9,
               max_tokens: int = 256) -> SyncChatStream:
        return SyncChatStream(self._c._stream(_chat_req(model, messages, temperature, top_p, max_tokens, True)))


class _SyncEmbeddings:
    def __init__(self, client: "VGate"):
        self._c = client

    def create(self, *, model: str, input: str) -> EmbeddingResponse:  # noqa: A002
        data = self._c._request("POST", "/v1/embeddings", json=EmbeddingRequest(model=model, input=input).model_dump())
        return EmbeddingResponse.model_validate(data)


class VGate:
    """Synchronous client: ``VGate(base_url=..., api_key=...)``; ``.chat``, ``.embeddings``."""

    def __init__(self, *, base_url: str = DEFAULT_BASE_URL, api_key: Optional[str] = None,
                 timeout: float = DEFAULT_TIMEOUT, max_retries: int = DEFAULT_MAX_RETRIES,
                 transport: Optional[httpx.BaseTransport] = None):
        self.base_url = base_url.rstrip("/")
        self.api_key = api_key
        self.max_retries = max_retries
        self._policy = _Policy(max_retries)
        kw = dict(base_url=self.base_url, headers=_headers(api_key), timeout=timeout)
        if transport is not None:
            kw["transport"] = transport
        self._http = httpx.Client(**kw)
        self._last_rate_limit = RateLimitInfo()
        self.chat = _SyncChat(self)
        self.embeddings = _SyncEmbeddings(self)

    def _request(self, method: str, path: str, **kw) -> dict:
        attempt = 0
        while True:
            try:
                resp = self._http.request(method, path, **kw)
            except httpx.ConnectError as e:
                raise ConnectionError(f"Cannot connect to {self.base_url}: {e}") from e
            self._last_rate_limit = parse_rate_limit(resp.headers)
            if resp.is_success:
                return resp.json()
            wait = self._policy.backoff(resp, attempt)
            if wait is None:
                raise_for_status(resp)
            _sleep(wait)
            attempt += 1

    def _stream(self, body: dict) -> Iterator[ChatCompletionChunk]:
        try:
            with self._http.stream("POST", "/v1/chat/completions", json=body) as resp:
                if not resp.is_success:
                    resp.read()
                    raise_for_status(resp)
                check_stream_content_type(resp)
                done = False
                for line in resp.iter_lines():
                    item = parse_sse_line(line)
                    if item is STREAM_DONE:
                        done = True
                        break
                    if item is not None:
                        yield item
                if not done:
                    raise ServerError("Stream ended without a [DONE] event "
                                      "(connection closed early or the server crashed mid-stream)")
        except httpx.ConnectError as e:
            raise ConnectionError(f"Cannot connect to {self.base_url}: {e}") from e

    def health(self) -> HealthResponse:
        return HealthResponse.model_validate(self._request("GET", "/health"))

    def stats(self) -> dict:
        return self._request("GET", "/stats")

    def rate_limit_info(self) -> RateLimitInfo:
        """Rate-limit headers of the most recent response."""
        return self._last_rate_limit

    def close(self) -> None:
        self._http.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ----------------------------------------------------------------- async client
class _AsyncChat:
    def __init__(self, client: "AsyncVGate"):
        self._c = client

    async def create(self, *, model: str, messages: list[dict], temperature: float = 0.7, top_p: float = 0.9,
                     max_tokens: int = 256) -> ChatCompletion:
        data = await self._c._request("POST", "/v1/chat/completions",
                                      json=_chat_req(model, messages, temperature, top_p, max_tokens))
        return ChatCompletion.model_validate(data)

    def stream(self, *, model: str, messages: list[dict], temperature: float = 0.7, top_p: float = 0.9,
               max_tokens: int = 256) -> AsyncChatStream:
        """Not a coroutine: returns the stream immediately (``async for`` / ``async with``)."""
        return AsyncChatStream(self._c._stream(_chat_req(model, messages, temperature, top_p, max_tokens, True)))


class _AsyncEmbeddings:
    def __init__(self, client: "AsyncVGate"):
        self._c = client

    async def create(self, *, model: str, input: str) -> EmbeddingResponse:  # noqa: A002
        data = await self._c._request("POST", "/v1/embeddings",
                                      json=EmbeddingRequest(model=model, input=input).model_dump())
        return EmbeddingResponse.model_validate(data)


class AsyncVGate:
    """Asynchronous client mirroring :class:`VGate`."""

    def __init__(self, *, base_url: str = DEFAULT_BASE_URL, api_key: Optional[str] = None,
                 timeout: float = DEFAULT_TIMEOUT, max_retries: int = DEFAULT_MAX_RETRIES,
                 transport: Optional[httpx.AsyncBaseTransport] = None):
        self.base_url = base_url.rstrip("/")
        self.api_key = api_key
        self.max_retries = max_retries
        self._policy = _Policy(max_retries)
        kw = dict(base_url=self.base_url, headers=_headers(api_key), timeout=timeout)
        if transport is not None:
            kw["transport"] = transport
        self._http = httpx.AsyncClient(**kw)
        self._last_rate_limit = RateLimitInfo()
        self.chat = _AsyncChat(self)
        self.embeddings = _AsyncEmbeddings(self)

    async def _request(self, method: str, path: str, **kw) -> dict:
        attempt = 0
        while True:
            try:
                resp = await self._http.request(method, path, **kw)
            except httpx.ConnectError as e:
                raise ConnectionError(f"Cannot connect to {self.base_url}: {e}") from e
            self._last_rate_limit = parse_rate_limit(resp.headers)
            if resp.is_success:
                return resp.json()
            wait = self._policy.backoff(resp, attempt)
            if wait is None:
                raise_for_status(resp)
            await _asleep(wait)
            attempt += 1

    async def _stream(self, body: dict) -> AsyncIterator[ChatCompletionChunk]:
        try:
            async with self._http.stream("POST", "/v1/chat/completions", json=body) as resp:
                if not resp.is_success:
                    await resp.aread()
                    raise_for_status(resp)
                check_stream_content_type(resp)
                done = False
                async for line in resp.aiter_lines():
                    item = parse_sse_line(line)
                    if item is STREAM_DONE:
                        done = True
                        break
                    if item is not None:
                        yield item
                if not done:
                    raise ServerError("Stream ended without a [DONE] event "
                                      "(connection closed early or the server crashed mid-stream)")
        except httpx.ConnectError as e:
            raise ConnectionError(f"Cannot connect to {self.base_url}: {e}") from e

    async def health(self) -> HealthResponse:
        return HealthResponse.model_validate(await self._request("GET", "/health"))

    async def stats(self) -> dict:
        return await self._request("GET", "/stats")

    def rate_limit_info(self) -> RateLimitInfo:
        return self._last_rate_limit

    async def close(self) -> None:
        await self._http.aclose()

    async def __aenter__(self):
        return self

    async def __aexit__(self, *exc):
        await self.close()
