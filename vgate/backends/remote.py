"""Gateway -> worker transport (HTTP/JSON, drop-in wire contract of ``/internal/generate``).

Re-designed vs the reference (``remote_backend.py``):
* **async**: a request awaits its worker call on the event loop instead of pinning an
  executor thread — the reference's 20-thread / ~180 req/s gateway ceiling
  (reference benchmarks/results/scaling.md:160-181) disappears by construction;
* **aiohttp connection pool** on the serving path: httpx's pool re-scans every
  connection for every queued request (``_assign_requests_to_connections``), which
  under 64+ in-flight worker calls cost the gateway ~5 ms of CPU per request and
  made throughput FALL as offered load rose (benchmarks/results/scaling.md,
  "Saturation"); aiohttp's per-host keep-alive pool is O(1) per request. httpx is
  used only when a test injects an ``httpx`` transport (ASGI/mock workers);
* **streaming pass-through**: ``stream_generate`` proxies the worker's
  ``/internal/generate_stream`` SSE stream (the reference returned 501);
* **trace propagation**: W3C ``traceparent`` header on every worker call.

Retry policy (the safe one): only a connect failure or a 503 refusal (a draining worker,
or one whose engine is not bound yet) moves to another worker (nothing ran); timeouts / mid-request errors / non-200 /
malformed results fail without retry so one client request never costs two
generations; exhausting the pool raises :class:`NoHealthyWorkersError` (503).
The sync ``generate`` is kept for protocol compatibility (runs the coroutine on
a private loop).
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import time
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple

import httpx

try:  # imported with the module, not by the first request on the event loop (~0.2 s)
    import aiohttp as _aiohttp
except ImportError:  # pragma: no cover - aiohttp is in requirements.txt
    _aiohttp = None

from vgate.config import ModelConfig, WorkerConfig
from vgate.logging_config import get_logger
from vgate.metrics import WORKER_LATENCY, WORKER_REQUESTS, WORKER_RETRIES
from vgate.tracing import get_tracer, inject_traceparent
from vgate.worker_registry import NoHealthyWorkersError, WorkerRegistry

logger = get_logger("vgate.remote")
tracer = get_tracer(__name__)


class RemoteInferenceError(RuntimeError):
    """A worker was reached but the call failed (non-retryable: it may have run)."""


class _ConnectFailed(Exception):
    """Nothing reached the worker: safe to retry on another one."""


class _Refused(Exception):
    """The worker answered 503 before running anything (draining / not ready): retry elsewhere."""


class _RequestFailed(Exception):
    """The request may have been delivered: never retried."""


class _AiohttpTransport:
    """Serving-path HTTP client: one aiohttp session (keep-alive pool) per event loop."""

    def __init__(self, cfg: WorkerConfig, headers: dict):
        if _aiohttp is None:
            raise RuntimeError("the remote backend needs aiohttp")
        aiohttp = self._aiohttp = _aiohttp
        # SSE pass-through: no bound on the stream's lifetime (a long generation is legitimate),
        # timeout_seconds bounds the silence between two chunks instead
        self._stream_timeout = aiohttp.ClientTimeout(total=None, connect=cfg.connect_timeout_seconds,
                                                     sock_read=cfg.timeout_seconds)
        self._session = aiohttp.ClientSession(
            connector=aiohttp.TCPConnector(limit=cfg.max_connections, limit_per_host=0, ttl_dns_cache=300),
            timeout=aiohttp.ClientTimeout(total=cfg.timeout_seconds, connect=cfg.connect_timeout_seconds),
            headers=headers)

    async def post_json(self, url: str, body: dict, headers: dict) -> Tuple[int, bytes]:
        a = self._aiohttp
        try:
            async with self._session.post(url, json=body, headers=headers) as r:
                return r.status, await r.read()
        except a.ClientConnectorError as e:
            raise _ConnectFailed(type(e).__name__) from e
        except (a.ClientError, asyncio.TimeoutError) as e:
            raise _RequestFailed(type(e).__name__) from e

    @contextlib.asynccontextmanager
    async def stream_lines(self, url: str, body: dict, headers: dict):
        a = self._aiohttp
        try:
            cm = self._session.post(url, json=body, headers=headers, timeout=self._stream_timeout)
            try:
                r = await cm.__aenter__()
            except a.ClientConnectorError as e:
                raise _ConnectFailed(type(e).__name__) from e

            async def lines():
                # own line splitting over raw chunks: aiohttp's readline() raises ValueError on a
                # line over its 64 KiB limit (one large SSE delta would kill the stream)
                buf = b""
                try:
                    async for chunk in r.content.iter_any():
                        buf += chunk
                        while True:
                            nl = buf.find(b"\n")
                            if nl < 0:
                                break
                            line, buf = buf[:nl], buf[nl + 1:]
                            yield line.decode("utf-8", "replace").rstrip("\r")
                    if buf:
                        yield buf.decode("utf-8", "replace").rstrip("\r")
                except (a.ClientError, asyncio.TimeoutError, ValueError) as e:
                    raise _RequestFailed(type(e).__name__) from e
            try:
                yield r.status, (await r.read() if r.status != 200 else b""), lines()
            finally:
                await cm.__aexit__(None, None, None)
        except (_ConnectFailed, _RequestFailed, RemoteInferenceError):
            raise
        except (a.ClientError, asyncio.TimeoutError) as e:
            raise _RequestFailed(type(e).__name__) from e

    async def aclose(self) -> None:
        await self._session.close()


class _HttpxTransport:
    """Test-path HTTP client over an injected httpx transport (ASGI app / mock handler)."""

    def __init__(self, cfg: WorkerConfig, headers: dict, transport: httpx.AsyncBaseTransport):
        self._c = httpx.AsyncClient(
            transport=transport, headers=headers,
            timeout=httpx.Timeout(cfg.timeout_seconds, connect=cfg.connect_timeout_seconds))

    async def post_json(self, url: str, body: dict, headers: dict) -> Tuple[int, bytes]:
        try:
            r = await self._c.post(url, json=body, headers=headers)
        except httpx.ConnectError as e:
            raise _ConnectFailed(type(e).__name__) from e
        except httpx.RequestError as e:
            raise _RequestFailed(type(e).__name__) from e
        return r.status_code, r.content

    @contextlib.asynccontextmanager
    async def stream_lines(self, url: str, body: dict, headers: dict):
        try:
            async with self._c.stream("POST", url, json=body, headers=headers) as r:
                async def lines():
                    try:
                        async for ln in r.aiter_lines():
                            yield ln
                    except httpx.RequestError as e:
                        raise _RequestFailed(type(e).__name__) from e
                yield r.status_code, (await r.aread() if r.status_code != 200 else b""), lines()
        except httpx.ConnectError as e:
            raise _ConnectFailed(type(e).__name__) from e
        except httpx.RequestError as e:
            raise _RequestFailed(type(e).__name__) from e

    async def aclose(self) -> None:
        await self._c.aclose()


class RemoteBackend:
    supports_concurrent_calls = True
    supports_streaming = True

    def __init__(self, worker_config: WorkerConfig, registry: Optional[WorkerRegistry] = None,
                 transport: Optional[httpx.AsyncBaseTransport] = None):
        discovering = bool(worker_config.discovery.dns_name)
        if not worker_config.endpoints and not discovering:
            raise ValueError("RemoteBackend requires worker.endpoints or worker.discovery.dns_name")
        self.config = worker_config
        self.registry = registry or WorkerRegistry(
            worker_config.endpoints, failure_threshold=worker_config.failure_threshold,
            success_threshold=worker_config.success_threshold, allow_empty=discovering,
            routing=worker_config.routing)
        self._headers = {"Authorization": f"Bearer {worker_config.api_key}"} if worker_config.api_key else {}
        self._transport = transport
        self._clients: dict = {}  # one AsyncClient per event loop
        logger.info("Remote backend initialized", extra={"extra_data": {
            "endpoints": worker_config.endpoints, "discovery_dns_name": worker_config.discovery.dns_name,
            "timeout_seconds": worker_config.timeout_seconds, "authenticated": bool(worker_config.api_key),
            "routing": worker_config.routing}})

    def _client(self):
        loop = asyncio.get_running_loop()
        c = self._clients.get(loop)
        if c is None:
            c = (_HttpxTransport(self.config, self._headers, self._transport) if self._transport is not None
                 else _AiohttpTransport(self.config, self._headers))
            self._clients[loop] = c
        return c

    def load_model(self, model_config: ModelConfig) -> None:
        """No-op: workers own their models."""

    def create_sampling_params(self, temperature: float, top_p: float, max_tokens: int) -> Any:
        return {"temperature": temperature, "top_p": top_p, "max_tokens": max_tokens}

    # ------------------------------------------------------------------ unary
    async def agenerate_batch(self, prompts: List[str], sampling_params: Any) -> List[Dict[str, Any]]:
        with tracer.start_as_current_span("remote.generate") as span:
            span.set_attribute("num_prompts", len(prompts))
            tried: set = set()
            last_connect: Optional[Exception] = None
            client = self._client()
            headers = inject_traceparent({})
            for attempt in range(max(1, len(self.registry.endpoints()))):
                try:
                    ep = self.registry.pick(exclude=tried)
                except NoHealthyWorkersError:
                    break
                if attempt > 0:
                    WORKER_RETRIES.labels(worker=ep).inc()
                    span.set_attribute("retried", True)
                t0 = time.perf_counter()
                self.registry.begin(ep)
                try:
                    status, raw = await client.post_json(f"{ep}/internal/generate",
                                                         {"prompts": prompts, "sampling_params": sampling_params},
                                                         headers)
                except _ConnectFailed as e:
                    self.registry.record_failure(ep)
                    WORKER_REQUESTS.labels(worker=ep, outcome="connect_error").inc()
                    tried.add(ep)
                    last_connect = e
                    continue
                except _RequestFailed as e:
                    self.registry.record_failure(ep)
                    WORKER_REQUESTS.labels(worker=ep, outcome="request_error").inc()
                    span.set_attribute("error", True)
                    raise RemoteInferenceError(f"worker at {ep} failed mid-request: {e}") from e
                finally:
                    self.registry.end(ep)
                    WORKER_LATENCY.labels(worker=ep).observe(time.perf_counter() - t0)
                if status == 503:
                    # 503 = the worker refused before running anything (draining on SIGTERM, engine
                    # not bound yet): like a refused connection, safe to send to another worker
                    self.registry.record_failure(ep)
                    WORKER_REQUESTS.labels(worker=ep, outcome="http_error").inc()
                    tried.add(ep)
                    continue
                if status != 200:
                    self.registry.record_failure(ep)
                    WORKER_REQUESTS.labels(worker=ep, outcome="http_error").inc()
                    span.set_attribute("error", True)
                    raise RemoteInferenceError(f"worker at {ep} returned {status}: "
                                               f"{raw[:200].decode('utf-8', 'replace')}")
                try:
                    results = json.loads(raw).get("results")
                except (ValueError, AttributeError):
                    results = None
                if not isinstance(results, list) or len(results) != len(prompts):
                    self.registry.record_failure(ep)
                    WORKER_REQUESTS.labels(worker=ep, outcome="bad_response").inc()
                    raise RemoteInferenceError(
                        f"worker at {ep} returned {len(results) if isinstance(results, list) else 'no'} results "
                        f"for {len(prompts)} prompts")
                self.registry.record_success(ep)
                WORKER_REQUESTS.labels(worker=ep, outcome="success").inc()
                span.set_attribute("endpoint", ep)
                return results
            span.set_attribute("error", True)
            detail = f"last error: {type(last_connect).__name__}" if last_connect else "none reachable"
            raise NoHealthyWorkersError(f"no healthy worker served the request after {len(tried)} attempt(s); {detail}")

    async def agenerate(self, prompt: str, sampling_params: Any) -> Dict[str, Any]:
        return (await self.agenerate_batch([prompt], sampling_params))[0]

    def generate(self, prompts: List[str], sampling_params: Any) -> List[Dict[str, Any]]:
        loop = asyncio.new_event_loop()
        try:
            return loop.run_until_complete(self.agenerate_batch(prompts, sampling_params))
        finally:
            c = self._clients.pop(loop, None)
            if c is not None:
                loop.run_until_complete(c.aclose())
            loop.close()

    # -------------------------------------------------------------- streaming
    async def stream_generate(self, prompt: str, sampling_params: Any) -> AsyncIterator[Dict[str, Any]]:
        """Proxy the worker's SSE stream. Retries only a ConnectError before any byte flowed."""
        tried: set = set()
        client = self._client()
        headers = inject_traceparent({})
        for attempt in range(max(1, len(self.registry.endpoints()))):
            try:
                ep = self.registry.pick(exclude=tried)
            except NoHealthyWorkersError:
                break
            if attempt > 0:
                WORKER_RETRIES.labels(worker=ep).inc()
            self.registry.begin(ep)
            try:
                async with client.stream_lines(f"{ep}/internal/generate_stream",
                                               {"prompt": prompt, "sampling_params": sampling_params},
                                               headers) as (status, err_body, lines):
                    if status == 503:  # refused before anything ran (draining): try another worker
                        raise _Refused()
                    if status != 200:
                        self.registry.record_failure(ep)
                        WORKER_REQUESTS.labels(worker=ep, outcome="http_error").inc()
                        raise RemoteInferenceError(f"worker at {ep} returned {status}: {err_body[:200]!r}")
                    async for line in lines:
                        if not line.startswith("data:"):
                            continue
                        data = line[5:].strip()
                        if data == "[DONE]":
                            break
                        chunk = json.loads(data)
                        if "error" in chunk:
                            raise RemoteInferenceError(f"worker at {ep}: {chunk['error']}")
                        yield chunk
                self.registry.record_success(ep)
                WORKER_REQUESTS.labels(worker=ep, outcome="success").inc()
                return
            except _ConnectFailed:
                self.registry.record_failure(ep)
                WORKER_REQUESTS.labels(worker=ep, outcome="connect_error").inc()
                tried.add(ep)
                continue
            except _Refused:
                self.registry.record_failure(ep)
                WORKER_REQUESTS.labels(worker=ep, outcome="http_error").inc()
                tried.add(ep)
                continue
            except _RequestFailed as e:
                self.registry.record_failure(ep)
                WORKER_REQUESTS.labels(worker=ep, outcome="request_error").inc()
                raise RemoteInferenceError(f"worker at {ep} failed mid-stream: {e}") from e
            finally:
                self.registry.end(ep)
        raise NoHealthyWorkersError("no healthy worker available for streaming")

    async def aclose(self) -> None:
        for c in list(self._clients.values()):
            try:
                await c.aclose()
            except Exception:  # noqa: BLE001
                pass
        self._clients.clear()

    def shutdown(self) -> None:
        self._clients.clear()
