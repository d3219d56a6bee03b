"""Background worker health probing + DNS membership refresh for the gateway.

Semantics (reference ``vgate/health_checker.py``): the first pass (resolve, then
probe) completes before ``start()`` returns, bounded by ``startup_resolve_timeout``;
each tick starts a NON-blocking membership refresh (skipped while the previous
one is still running) and then probes ``GET /health`` of every member
concurrently (only HTTP 200 is healthy); DNS runs on a dedicated single-thread
executor (``vgate-dns``) with its own timeout; resolver errors/timeouts never
count as an empty answer; only ``empty_resolve_threshold`` consecutive
authoritative-empty answers empty the pool.
"""
from __future__ import annotations

import asyncio
from concurrent.futures import ThreadPoolExecutor
from typing import Optional

import httpx

from vgate.logging_config import get_logger
from vgate.worker_discovery import DnsWorkerDiscovery, TransientResolutionError
from vgate.worker_registry import WorkerRegistry

logger = get_logger("vgate.health")


class WorkerHealthChecker:
    def __init__(self, registry: WorkerRegistry, interval_seconds: float = 5.0, timeout_seconds: float = 2.0,
                 api_key: Optional[str] = None, transport: Optional[httpx.AsyncBaseTransport] = None,
                 discovery: Optional[DnsWorkerDiscovery] = None, empty_resolve_threshold: int = 3,
                 startup_resolve_timeout: float = 5.0, resolve_timeout: float = 5.0):
        self.registry = registry
        self.interval_seconds = interval_seconds
        self.timeout_seconds = timeout_seconds
        self.discovery = discovery
        self.empty_resolve_threshold = max(1, empty_resolve_threshold)
        self.startup_resolve_timeout = startup_resolve_timeout
        self.resolve_timeout = resolve_timeout
        self._empty_resolves = 0
        self._headers = {"Authorization": f"Bearer {api_key}"} if api_key else {}
        self._transport = transport
        self._task: Optional[asyncio.Task] = None
        self._refresh_task: Optional[asyncio.Task] = None
        self._dns_executor: Optional[ThreadPoolExecutor] = None
        self._first_pass: Optional[asyncio.Event] = None
        self._running = False
        self.ticks = 0

    async def start(self) -> None:
        if self._running:
            return
        self._running = True
        self._first_pass = asyncio.Event()
        self._task = asyncio.create_task(self._loop())
        try:
            await asyncio.wait_for(self._first_pass.wait(), timeout=self.startup_resolve_timeout)
        except asyncio.TimeoutError:
            logger.warning("First discovery/probe pass did not finish before startup; continuing in background",
                           extra={"extra_data": {"timeout_seconds": self.startup_resolve_timeout}})
        logger.info("Worker health checker started", extra={"extra_data": {
            "workers": self.registry.endpoints(), "interval_seconds": self.interval_seconds}})

    async def stop(self) -> None:
        self._running = False
        for t in (self._task, self._refresh_task):
            if t is None:
                continue
            t.cancel()
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._task = self._refresh_task = None
        if self._dns_executor is not None:
            self._dns_executor.shutdown(wait=False, cancel_futures=True)
            self._dns_executor = None
        logger.info("Worker health checker stopped")

    async def _loop(self) -> None:
        kw = dict(timeout=self.timeout_seconds, headers=self._headers)
        if self._transport is not None:
            kw["transport"] = self._transport
        else:
            # the client's TLS context (CA bundle parse, ~0.1 s) is built off the event loop: the
            # asyncio debug pass flags it as a slow callback otherwise (tests/test_asyncio_debug.py)
            kw["verify"] = await asyncio.to_thread(httpx.create_ssl_context)
        async with httpx.AsyncClient(**kw) as client:
            try:
                await self.refresh_members()
                await self.probe_once(client)
            finally:
                self._first_pass.set()
            while self._running:
                await asyncio.sleep(self.interval_seconds)
                if not self._running:
                    break
                self._begin_refresh()
                await self.probe_once(client)
                self.ticks += 1

    def _begin_refresh(self) -> None:
        if self.discovery is None:
            return
        if self._refresh_task is not None and not self._refresh_task.done():
            logger.warning("Previous worker discovery has not finished; skipping this tick",
                           extra={"extra_data": {"dns_name": self.discovery.dns_name}})
            return
        self._refresh_task = asyncio.create_task(self.refresh_members())

    async def refresh_members(self) -> None:
        if self.discovery is None:
            return
        loop = asyncio.get_running_loop()
        if self._dns_executor is None:
            self._dns_executor = ThreadPoolExecutor(max_workers=1, thread_name_prefix="vgate-dns")
        try:
            eps = await asyncio.wait_for(loop.run_in_executor(self._dns_executor, self.discovery.resolve),
                                         timeout=self.resolve_timeout)
        except asyncio.TimeoutError:
            logger.warning("Worker discovery did not answer in time; keeping the current member set",
                           extra={"extra_data": {"dns_name": self.discovery.dns_name}})
            return
        except TransientResolutionError as e:
            logger.warning("Worker discovery could not resolve; keeping the current member set",
                           extra={"extra_data": {"error": str(e)}})
            return
        except Exception as e:  # noqa: BLE001 - never kill the loop
            logger.warning("Worker discovery failed; keeping the current member set",
                           extra={"extra_data": {"error": str(e), "error_type": type(e).__name__}})
            return
        if eps:
            self._empty_resolves = 0
            self.registry.set_members(eps)
            return
        if not self.registry.endpoints():
            return
        self._empty_resolves += 1
        if self._empty_resolves < self.empty_resolve_threshold:
            logger.warning("Worker discovery returned no endpoints; awaiting confirmation",
                           extra={"extra_data": {"consecutive_empty": self._empty_resolves,
                                                 "threshold": self.empty_resolve_threshold}})
            return
        logger.warning("Worker discovery empty on %d consecutive ticks; emptying the pool" % self._empty_resolves)
        self.registry.set_members([])

    async def probe_once(self, client: httpx.AsyncClient) -> None:
        eps = self.registry.endpoints()
        res = await asyncio.gather(*(self._probe(client, ep) for ep in eps), return_exceptions=True)
        for ep, ok in zip(eps, res):
            if ok is True:
                self.registry.record_success(ep)
            else:
                self.registry.record_failure(ep)

    async def _probe(self, client: httpx.AsyncClient, endpoint: str) -> bool:
        try:
            r = await client.get(f"{endpoint}/health")
        except httpx.RequestError:
            return False
        return r.status_code == 200
