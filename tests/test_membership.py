"""Worker membership behaviour of the split deployment, expressed against this code base:
DNS discovery (stable names, authoritative-empty vs transient failures, IPv6), registry
membership refreshes (survivor state, pending arrivals, removed workers), the health checker's
refresh / probe loop (empty-answer confirmation, resolver timeouts, dedicated DNS executor,
startup bounds) and the remote backend's retry surface.

Behavioural parity targets: reference tests/test_worker_discovery.py, test_worker_registry.py
(SURVEY.md Appendix A item 9). No network: every resolver and worker is injected.
"""
import asyncio
import json
import socket
import threading
import time

import httpx
import pytest

from vgate.backends.remote import RemoteBackend, RemoteInferenceError
from vgate.config import WorkerConfig
from vgate.health_checker import WorkerHealthChecker
from vgate.metrics import WORKER_HEALTHY, WORKER_STATE_CHANGES
from vgate.worker_discovery import DnsWorkerDiscovery, TransientResolutionError, host_for_url
from vgate.worker_registry import NoHealthyWorkersError, WorkerRegistry

A, B, C = "http://a:8000", "http://b:8000", "http://c:8000"


def _gai(errno):
    return socket.gaierror(errno, "resolver says so")


# ---------------------------------------------------------------------------- discovery
def test_discovery_resolves_pods_to_stable_names():
    names = {"10.0.0.1": "w-0.workers.ns.svc.cluster.local.", "10.0.0.2": "w-1.workers.ns.svc.cluster.local."}
    d = DnsWorkerDiscovery("workers", 8000, forward_resolver=lambda h, p: list(names),
                           reverse_resolver=lambda a: names[a])
    assert d.resolve() == ["http://w-0.workers.ns.svc.cluster.local:8000",
                           "http://w-1.workers.ns.svc.cluster.local:8000"]


def test_discovery_falls_back_to_address_when_reverse_fails():
    def rev(a):
        raise socket.herror(1, "no PTR")
    d = DnsWorkerDiscovery("workers", 8000, forward_resolver=lambda h, p: ["10.0.0.7"], reverse_resolver=rev)
    assert d.resolve() == ["http://10.0.0.7:8000"]
    assert d.resolve() == ["http://10.0.0.7:8000"]  # logged once, still answered
    assert d._logged_fallbacks == {"10.0.0.7"}


@pytest.mark.parametrize("name", ["EAI_NONAME", "EAI_NODATA"])
def test_authoritative_no_such_name_is_empty(name):
    if not hasattr(socket, name):
        pytest.skip(f"{name} not on this platform")

    def fwd(h, p):
        raise _gai(getattr(socket, name))
    assert DnsWorkerDiscovery("workers", forward_resolver=fwd).resolve() == []


@pytest.mark.parametrize("name", ["EAI_AGAIN", "EAI_FAIL", "EAI_SYSTEM"])
def test_resolver_that_cannot_answer_is_transient(name):
    if not hasattr(socket, name):
        pytest.skip(f"{name} not on this platform")

    def fwd(h, p):
        raise _gai(getattr(socket, name))
    with pytest.raises(TransientResolutionError):
        DnsWorkerDiscovery("workers", forward_resolver=fwd).resolve()


def test_os_error_is_transient():
    def fwd(h, p):
        raise OSError("socket table full")
    with pytest.raises(TransientResolutionError):
        DnsWorkerDiscovery("workers", forward_resolver=fwd).resolve()


def test_ptr_naming_the_service_is_not_an_identity():
    d = DnsWorkerDiscovery("workers.ns.svc", 9000, forward_resolver=lambda h, p: ["10.1.1.1"],
                           reverse_resolver=lambda a: "workers.ns.svc.")
    assert d.resolve() == ["http://10.1.1.1:9000"]


def test_scheme_and_port_are_configurable():
    d = DnsWorkerDiscovery("w", 9443, scheme="https", forward_resolver=lambda h, p: ["10.0.0.3"],
                           reverse_resolver=lambda a: "pod-3.w.")
    assert d.resolve() == ["https://pod-3.w:9443"]


def test_ipv6_addresses_are_bracketed_and_names_are_not():
    def rev(a):
        raise socket.herror(1, "x")
    d = DnsWorkerDiscovery("w", 8000, forward_resolver=lambda h, p: ["fd00::5"], reverse_resolver=rev)
    assert d.resolve() == ["http://[fd00::5]:8000"]
    d2 = DnsWorkerDiscovery("w", 8000, forward_resolver=lambda h, p: ["fd00::5"], reverse_resolver=lambda a: "pod-v6.w.")
    assert d2.resolve() == ["http://pod-v6.w:8000"]
    assert host_for_url("[fd00::1]") == "[fd00::1]" and host_for_url("10.0.0.1") == "10.0.0.1"


def test_forward_resolution_is_not_ipv4_only_and_deduplicates():
    seen = {}

    def fwd(h, p):
        seen["called"] = (h, p)
        return ["10.0.0.1", "fd00::1", "10.0.0.1"]
    d = DnsWorkerDiscovery("w", 8000, forward_resolver=fwd, reverse_resolver=lambda a: {"10.0.0.1": "p1.w",
                                                                                         "fd00::1": "p2.w"}[a])
    assert d.resolve() == ["http://p1.w:8000", "http://p2.w:8000"]
    assert seen["called"] == ("w", 8000)


# ---------------------------------------------------------------------------- registry
def test_set_members_adds_and_removes():
    r = WorkerRegistry([A, B])
    added, removed = r.set_members([B, C])
    assert added == [C] and removed == [A]
    assert r.endpoints() == [B, C]
    assert r.set_members([B, C]) == ([], [])


def test_rediscovery_does_not_reset_a_worker_being_demoted():
    r = WorkerRegistry([A, B], failure_threshold=3)
    r.record_failure(A)
    r.record_failure(A)
    r.set_members([A, B, C])
    r.record_failure(A)
    assert A not in r.healthy_endpoints()


def test_removed_worker_is_never_picked():
    r = WorkerRegistry([A, B, C])
    r.set_members([A, C])
    picks = {r.pick() for _ in range(10)}
    assert picks == {A, C}
    r.record_failure(B)  # a late probe result for a departed worker is ignored
    assert r.endpoints() == [A, C]


def test_returning_worker_does_not_inherit_old_verdict():
    r = WorkerRegistry([A, B], failure_threshold=1)
    r.record_failure(A)
    assert A not in r.healthy_endpoints()
    r.set_members([B])
    r.set_members([A, B])
    snap = {s["endpoint"]: s for s in r.snapshot()}
    assert snap[A]["pending"] and snap[A]["consecutive_failures"] == 0
    r.record_success(A)  # a fresh arrival is admitted on its first success
    assert A in r.healthy_endpoints()


def test_discovered_arrival_waits_for_a_probe():
    r = WorkerRegistry([A])
    r.set_members([A, B])
    assert [r.pick() for _ in range(4)] == [A, A, A, A]
    r.record_success(B)
    assert B in {r.pick() for _ in range(4)}


def test_demoted_worker_needs_sustained_recovery_even_after_refresh():
    r = WorkerRegistry([A, B], failure_threshold=1, success_threshold=3)
    r.record_failure(A)
    r.set_members([A, B, C])
    r.record_success(A)
    r.record_success(A)
    assert A not in r.healthy_endpoints()
    r.record_success(A)
    assert A in r.healthy_endpoints()


def test_configured_endpoints_start_healthy():
    r = WorkerRegistry([A, B])
    assert r.healthy_endpoints() == [A, B]
    assert all(not s["pending"] for s in r.snapshot())


def test_round_robin_follows_the_new_member_set():
    r = WorkerRegistry([A, B, C])
    r.pick()
    r.set_members([B, C])
    got = [r.pick() for _ in range(4)]
    assert set(got) == {B, C} and got[0] != got[1]


def test_discovered_registry_may_start_empty_and_static_may_not():
    r = WorkerRegistry([], allow_empty=True)
    assert r.endpoints() == [] and not r.has_healthy()
    with pytest.raises(NoHealthyWorkersError):
        r.pick()
    with pytest.raises(ValueError):
        WorkerRegistry([])


def test_failure_threshold_tolerates_one_blip_and_success_resets_streak():
    r = WorkerRegistry([A], failure_threshold=2)
    r.record_failure(A)
    r.record_success(A)
    r.record_failure(A)
    assert r.healthy_endpoints() == [A]
    r.record_failure(A)
    assert r.healthy_endpoints() == []


def test_failure_during_recovery_restarts_the_count():
    r = WorkerRegistry([A], failure_threshold=1, success_threshold=2)
    r.record_failure(A)
    r.record_success(A)
    r.record_failure(A)
    r.record_success(A)
    assert r.healthy_endpoints() == []
    r.record_success(A)
    assert r.healthy_endpoints() == [A]


def test_pick_raises_when_everything_is_excluded_or_unhealthy():
    r = WorkerRegistry([A, B], failure_threshold=1)
    with pytest.raises(NoHealthyWorkersError):
        r.pick(exclude={A, B})
    r.record_failure(A)
    r.record_failure(B)
    with pytest.raises(NoHealthyWorkersError):
        r.pick()


def test_transition_labels_and_gauge_lifecycle():
    r = WorkerRegistry(["http://lbl:1"], failure_threshold=1, success_threshold=1)

    def count(t):
        return WORKER_STATE_CHANGES.labels(worker="http://lbl:1", transition=t)._value.get()
    before = {t: count(t) for t in ("removed", "recovered", "admitted")}
    r.record_failure("http://lbl:1")
    r.record_success("http://lbl:1")
    assert count("removed") == before["removed"] + 1 and count("recovered") == before["recovered"] + 1
    r.set_members(["http://lbl:1", "http://lbl:2"])
    r.record_success("http://lbl:2")
    assert WORKER_STATE_CHANGES.labels(worker="http://lbl:2", transition="admitted")._value.get() >= 1
    r.set_members(["http://lbl:2"])
    names = {s.labels.get("worker") for m in WORKER_HEALTHY.collect() for s in m.samples}
    assert "http://lbl:1" not in names  # a departed worker's gauge is removed


def test_snapshot_reports_inflight_and_failures():
    r = WorkerRegistry([A, B])
    r.begin(A)
    r.record_failure(B)
    snap = {s["endpoint"]: s for s in r.snapshot()}
    assert snap[A]["inflight"] == 1 and snap[B]["total_failures"] == 1
    r.end(A)
    r.end(A)  # never negative
    assert {s["endpoint"]: s for s in r.snapshot()}[A]["inflight"] == 0


def test_least_inflight_breaks_ties_round_robin():
    r = WorkerRegistry([A, B, C], routing="least_inflight")
    assert [r.pick() for _ in range(3)] == [A, B, C]


# ---------------------------------------------------------------------- health checker
class _Res:
    """Scripted resolver: a queue of answers (list = endpoints, Exception = raise, 'hang' = sleep)."""

    def __init__(self, *answers):
        self.answers = list(answers)
        self.calls = 0
        self.threads = set()

    def resolve(self):
        self.calls += 1
        self.threads.add(threading.current_thread().name)
        a = self.answers.pop(0) if len(self.answers) > 1 else self.answers[0]
        if a == "hang":
            time.sleep(0.5)
            return [A]
        if isinstance(a, Exception):
            raise a
        return a


def _ok_transport():
    return httpx.MockTransport(lambda req: httpx.Response(200, json={"status": "healthy"}))


def _checker(reg, res, **kw):
    disc = DnsWorkerDiscovery("workers")
    disc.resolve = res.resolve
    kw.setdefault("interval_seconds", 0.02)
    return WorkerHealthChecker(reg, transport=_ok_transport(), discovery=disc, **kw)


async def test_refresh_applies_discovered_membership():
    reg = WorkerRegistry([], allow_empty=True)
    hc = _checker(reg, _Res([A, B]))
    await hc.refresh_members()
    assert reg.endpoints() == [A, B]


async def test_one_empty_resolve_does_not_empty_the_pool_but_a_streak_does():
    reg = WorkerRegistry([A, B])
    hc = _checker(reg, _Res([], [], []), empty_resolve_threshold=3)
    await hc.refresh_members()
    await hc.refresh_members()
    assert reg.endpoints() == [A, B]
    await hc.refresh_members()
    assert reg.endpoints() == []


async def test_successful_resolve_resets_the_empty_streak():
    reg = WorkerRegistry([A])
    hc = _checker(reg, _Res([], [], [A], [], []), empty_resolve_threshold=3)
    for _ in range(5):
        await hc.refresh_members()
    assert reg.endpoints() == [A]


async def test_dns_outage_never_empties_a_healthy_pool():
    reg = WorkerRegistry([A, B])
    hc = _checker(reg, _Res(TransientResolutionError("down")), empty_resolve_threshold=1)
    for _ in range(5):
        await hc.refresh_members()
    assert reg.endpoints() == [A, B]


async def test_resolver_exception_does_not_kill_the_loop():
    reg = WorkerRegistry([A])
    res = _Res(RuntimeError("boom"))
    hc = _checker(reg, res)
    await hc.start()
    await asyncio.sleep(0.15)
    assert hc._task is not None and not hc._task.done()
    assert res.calls >= 2
    await hc.stop()


async def test_start_resolves_before_returning():
    reg = WorkerRegistry([], allow_empty=True)
    hc = _checker(reg, _Res([A]), interval_seconds=10)
    await hc.start()
    assert reg.endpoints() == [A]
    assert reg.healthy_endpoints() == [A]  # first probe pass done too: pending arrival admitted
    await hc.stop()


async def test_start_does_not_hang_on_a_stalled_resolver():
    reg = WorkerRegistry([], allow_empty=True)
    hc = _checker(reg, _Res("hang"), startup_resolve_timeout=0.05, resolve_timeout=2.0, interval_seconds=10)
    t0 = time.perf_counter()
    await hc.start()
    assert time.perf_counter() - t0 < 0.4
    await hc.stop()


async def test_dns_runs_on_its_dedicated_executor():
    reg = WorkerRegistry([], allow_empty=True)
    res = _Res([A])
    hc = _checker(reg, res)
    await hc.refresh_members()
    assert res.threads and all(t.startswith("vgate-dns") for t in res.threads)
    await hc.stop()


async def test_resolve_timeout_keeps_members_and_is_not_empty():
    reg = WorkerRegistry([A])
    hc = _checker(reg, _Res("hang"), resolve_timeout=0.05, empty_resolve_threshold=1)
    for _ in range(3):
        await hc.refresh_members()
    assert reg.endpoints() == [A] and hc._empty_resolves == 0
    await hc.stop()


async def test_refresh_in_flight_is_skipped_not_queued():
    reg = WorkerRegistry([A])
    res = _Res("hang")
    hc = _checker(reg, res, resolve_timeout=2.0)
    hc._begin_refresh()
    first = hc._refresh_task
    hc._begin_refresh()
    hc._begin_refresh()
    assert hc._refresh_task is first
    await first
    await hc.stop()
    assert res.calls == 1


async def test_refresh_is_a_noop_without_discovery():
    reg = WorkerRegistry([A])
    hc = WorkerHealthChecker(reg, transport=_ok_transport())
    await hc.refresh_members()
    assert reg.endpoints() == [A]


async def test_probe_demotes_failing_and_restores_recovered_worker():
    state = {"a_ok": False}

    def handler(req):
        if req.url.host == "a":
            return httpx.Response(200 if state["a_ok"] else 503)
        return httpx.Response(200)
    reg = WorkerRegistry([A, B], failure_threshold=2, success_threshold=2)
    hc = WorkerHealthChecker(reg, transport=httpx.MockTransport(handler))
    async with httpx.AsyncClient(transport=httpx.MockTransport(handler)) as c:
        await hc.probe_once(c)
        await hc.probe_once(c)
        assert reg.healthy_endpoints() == [B]
        state["a_ok"] = True
        await hc.probe_once(c)
        assert reg.healthy_endpoints() == [B]
        await hc.probe_once(c)
        assert reg.healthy_endpoints() == [A, B]


async def test_probe_treats_connection_error_as_unhealthy_and_sends_api_key():
    seen = []

    def handler(req):
        seen.append(req.headers.get("authorization"))
        raise httpx.ConnectError("refused", request=req)
    reg = WorkerRegistry([A], failure_threshold=1)
    hc = WorkerHealthChecker(reg, api_key="sekret", transport=httpx.MockTransport(handler), interval_seconds=10)
    await hc.start()
    await hc.stop()
    assert reg.healthy_endpoints() == [] and seen == ["Bearer sekret"]


# ------------------------------------------------------------------ remote backend retries
def _mt(script):
    def handler(request):
        return script[f"{request.url.scheme}://{request.url.host}:{request.url.port}"](request)
    return httpx.MockTransport(handler)


def _ok(request):
    body = json.loads(request.content)
    return httpx.Response(200, json={"results": [{"text": p, "num_tokens": 1} for p in body["prompts"]]})


def _refuse(request):
    raise httpx.ConnectError("refused", request=request)


async def test_retry_count_is_bounded_by_worker_count():
    calls = []

    def refuse(request):
        calls.append(request.url.host)
        raise httpx.ConnectError("refused", request=request)
    be = RemoteBackend(WorkerConfig(endpoints=[A, B, C]), transport=_mt({A: refuse, B: refuse, C: refuse}))
    with pytest.raises(NoHealthyWorkersError):
        await be.agenerate("x", {"max_tokens": 1})
    assert sorted(calls) == ["a", "b", "c"]
    await be.aclose()


async def test_success_marks_worker_healthy_again():
    reg = WorkerRegistry([A], failure_threshold=1, success_threshold=1)
    reg.record_failure(A)
    reg.record_success(A)  # recovered by a probe
    be = RemoteBackend(WorkerConfig(endpoints=[A]), registry=reg, transport=_mt({A: _ok}))
    assert (await be.agenerate("hi", {"max_tokens": 1}))["text"] == "hi"
    assert reg.healthy_endpoints() == [A]
    await be.aclose()


async def test_result_count_mismatch_is_rejected_without_retry():
    calls = []

    def short(request):
        calls.append(1)
        return httpx.Response(200, json={"results": []})
    be = RemoteBackend(WorkerConfig(endpoints=[A, B]), transport=_mt({A: short, B: short}))
    with pytest.raises(RemoteInferenceError):
        await be.agenerate("x", {"max_tokens": 1})
    assert len(calls) == 1
    await be.aclose()


async def test_malformed_json_is_a_remote_error():
    be = RemoteBackend(WorkerConfig(endpoints=[A]), transport=_mt({A: lambda r: httpx.Response(200, text="<html>")}))
    with pytest.raises(RemoteInferenceError):
        await be.agenerate("x", {"max_tokens": 1})
    await be.aclose()


async def test_traceparent_and_sampling_params_are_forwarded():
    seen = {}

    def handler(request):
        seen["body"] = json.loads(request.content)
        seen["tp"] = request.headers.get("traceparent")
        return _ok(request)
    be = RemoteBackend(WorkerConfig(endpoints=[A]), transport=_mt({A: handler}))
    sp = be.create_sampling_params(0.3, 0.8, 17)
    await be.agenerate("p", sp)
    assert seen["body"]["sampling_params"] == {"temperature": 0.3, "top_p": 0.8, "max_tokens": 17}
    await be.aclose()


def test_sync_generate_runs_on_a_private_loop():
    be = RemoteBackend(WorkerConfig(endpoints=[A]), transport=_mt({A: _ok}))
    out = be.generate(["u", "v"], {"max_tokens": 1})
    assert [o["text"] for o in out] == ["u", "v"]
    assert be._clients == {}  # the private loop's client was closed with it


async def test_stream_connect_error_moves_to_next_worker():
    def sse(request):
        return httpx.Response(200, text='data: {"delta": "x", "num_tokens": 1}\n\ndata: [DONE]\n\n')
    be = RemoteBackend(WorkerConfig(endpoints=[A, B]), transport=_mt({A: _refuse, B: sse}))
    pieces = [c async for c in be.stream_generate("p", {"max_tokens": 2})]
    assert pieces == [{"delta": "x", "num_tokens": 1}]
    await be.aclose()


async def test_stream_error_chunk_is_raised():
    def sse(request):
        return httpx.Response(200, text='data: {"error": "engine fault"}\n\n')
    be = RemoteBackend(WorkerConfig(endpoints=[A]), transport=_mt({A: sse}))
    with pytest.raises(RemoteInferenceError, match="engine fault"):
        _ = [c async for c in be.stream_generate("p", {"max_tokens": 2})]
    await be.aclose()


def test_remote_backend_requires_endpoints_or_discovery():
    with pytest.raises(ValueError):
        RemoteBackend(WorkerConfig())
    be = RemoteBackend(WorkerConfig(discovery={"dns_name": "workers"}))
    assert be.registry.endpoints() == []


def test_worker_endpoint_validation():
    with pytest.raises(ValueError):
        WorkerConfig(endpoints=["w1:8000"])
    assert WorkerConfig(endpoints=["http://w1:8000/"]).endpoints == ["http://w1:8000"]
    with pytest.raises(ValueError):
        WorkerConfig(routing="random")
