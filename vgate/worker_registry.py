"""Worker membership + health bookkeeping for the gateway (reference ``vgate/worker_registry.py``).

Semantics kept:
* static endpoints start healthy; discovered arrivals start ``pending`` (out of
  rotation) and are admitted on their FIRST success;
* a worker is demoted after ``failure_threshold`` consecutive failures and a
  demoted worker needs ``success_threshold`` consecutive successes to recover;
* transitions are labelled removed / admitted / recovered; the per-worker
  health gauge is removed when a worker departs; survivors keep their state
  across membership refreshes.

Additions: ``least_inflight`` routing (the reference roadmap's load-aware
policy) using per-worker in-flight counters maintained by the remote backend.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import List, Optional

from vgate.logging_config import get_logger
from vgate.metrics import WORKER_HEALTHY, WORKER_STATE_CHANGES

logger = get_logger("vgate.registry")


@dataclass
class WorkerState:
    endpoint: str
    healthy: bool = True
    consecutive_failures: int = 0
    consecutive_successes: int = 0
    last_change_at: float = field(default_factory=time.monotonic)
    total_failures: int = 0
    pending: bool = False
    inflight: int = 0
    total_requests: int = 0


class NoHealthyWorkersError(RuntimeError):
    """Every known worker is out of rotation (or none is known yet)."""


class WorkerRegistry:
    def __init__(self, endpoints: List[str], failure_threshold: int = 2, success_threshold: int = 2,
                 allow_empty: bool = False, routing: str = "round_robin"):
        if not endpoints and not allow_empty:
            raise ValueError("WorkerRegistry requires at least one endpoint")
        self.failure_threshold = failure_threshold
        self.success_threshold = success_threshold
        self.routing = routing
        self._lock = threading.Lock()
        self._order = list(dict.fromkeys(endpoints))
        self._states = {ep: WorkerState(endpoint=ep) for ep in self._order}
        self._cursor = 0
        for ep in self._order:
            WORKER_HEALTHY.labels(worker=ep).set(1)

    # -------------------------------------------------------------- membership
    def set_members(self, endpoints: List[str]) -> tuple[list, list]:
        with self._lock:
            incoming = list(dict.fromkeys(endpoints))
            wanted = set(incoming)
            added = [ep for ep in incoming if ep not in self._states]
            removed = [ep for ep in self._order if ep not in wanted]
            if not added and not removed:
                return [], []
            for ep in removed:
                del self._states[ep]
                try:
                    WORKER_HEALTHY.remove(ep)
                except KeyError:
                    pass
            for ep in added:
                self._states[ep] = WorkerState(endpoint=ep, healthy=False, pending=True)
                WORKER_HEALTHY.labels(worker=ep).set(0)
            self._order = incoming
            self._cursor = self._cursor % len(incoming) if incoming else 0
        logger.info("Worker membership changed", extra={"extra_data": {
            "added": added, "removed": removed, "total": len(incoming)}})
        return added, removed

    # ----------------------------------------------------------------- routing
    def pick(self, exclude: Optional[set] = None) -> str:
        exclude = exclude or set()
        with self._lock:
            n = len(self._order)
            if self.routing == "least_inflight":
                best, best_load = None, None
                for off in range(n):
                    ep = self._order[(self._cursor + off) % n]
                    st = self._states[ep]
                    if ep in exclude or not st.healthy:
                        continue
                    if best_load is None or st.inflight < best_load:
                        best, best_load = ep, st.inflight
                if best is not None:
                    self._cursor = (self._order.index(best) + 1) % n
                    return best
            else:
                for off in range(n):
                    ep = self._order[(self._cursor + off) % n]
                    if ep in exclude:
                        continue
                    if self._states[ep].healthy:
                        self._cursor = (self._cursor + off + 1) % n
                        return ep
        raise NoHealthyWorkersError(f"no healthy worker available ({len(exclude)} excluded this request)")

    def begin(self, endpoint: str) -> None:
        with self._lock:
            st = self._states.get(endpoint)
            if st is not None:
                st.inflight += 1
                st.total_requests += 1

    def end(self, endpoint: str) -> None:
        with self._lock:
            st = self._states.get(endpoint)
            if st is not None and st.inflight > 0:
                st.inflight -= 1

    # ------------------------------------------------------------------ health
    def record_failure(self, endpoint: str) -> None:
        with self._lock:
            st = self._states.get(endpoint)
            if st is None:
                return
            st.total_failures += 1
            st.consecutive_successes = 0
            st.consecutive_failures += 1
            if st.healthy and st.consecutive_failures >= self.failure_threshold:
                st.healthy = False
                st.last_change_at = time.monotonic()
                self._on_change(endpoint, healthy=False)

    def record_success(self, endpoint: str) -> None:
        with self._lock:
            st = self._states.get(endpoint)
            if st is None:
                return
            st.consecutive_failures = 0
            if st.healthy:
                st.consecutive_successes = 0
                return
            st.consecutive_successes += 1
            need = 1 if st.pending else self.success_threshold
            if st.consecutive_successes >= need:
                st.healthy = True
                st.last_change_at = time.monotonic()
                self._on_change(endpoint, healthy=True, admitted=st.pending)
                st.pending = False

    def _on_change(self, endpoint: str, healthy: bool, admitted: bool = False) -> None:
        WORKER_HEALTHY.labels(worker=endpoint).set(1 if healthy else 0)
        transition = "removed" if not healthy else ("admitted" if admitted else "recovered")
        WORKER_STATE_CHANGES.labels(worker=endpoint, transition=transition).inc()
        logger.info("Worker %s" % transition, extra={"extra_data": {"worker": endpoint, "healthy": healthy}})

    # ----------------------------------------------------------------- queries
    def endpoints(self) -> List[str]:
        with self._lock:
            return list(self._order)

    def healthy_endpoints(self) -> List[str]:
        with self._lock:
            return [ep for ep in self._order if self._states[ep].healthy]

    def has_healthy(self) -> bool:
        with self._lock:
            return any(self._states[ep].healthy for ep in self._order)

    def snapshot(self) -> List[dict]:
        with self._lock:
            now = time.monotonic()
            return [{"endpoint": ep, "healthy": s.healthy, "pending": s.pending,
                     "consecutive_failures": s.consecutive_failures, "total_failures": s.total_failures,
                     "seconds_in_state": round(now - s.last_change_at, 1), "inflight": s.inflight}
                    for ep, s in ((e, self._states[e]) for e in self._order)]
