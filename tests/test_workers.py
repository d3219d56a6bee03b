"""Gateway <-> worker: registry semantics, async remote retry policy, streaming pass-through,
DNS discovery semantics, health checker membership/probing — no cluster needed."""
import asyncio
import socket
import threading

import httpx
import pytest

from vgate.api.app import create_app
from vgate.backends.base import DryRunBackend
from vgate.backends.remote import RemoteBackend, RemoteInferenceError
from vgate.config import VGateConfig, WorkerConfig
from vgate.engine import VGateEngine
from vgate.health_checker import WorkerHealthChecker
from vgate.worker_discovery import DnsWorkerDiscovery, TransientResolutionError
from vgate.worker_registry import NoHealthyWorkersError, WorkerRegistry

W1, W2, W3 = "http://w1:8000", "http://w2:8000", "http://w3:8000"


# ------------------------------------------------------------------------ registry
def test_registry_round_robin_and_exclude():
    r = WorkerRegistry([W1, W2, W3])
    assert [r.pick() for _ in range(4)] == [W1, W2, W3, W1]
    assert r.pick(exclude={W2}) == W3


def test_registry_demote_and_recover_thresholds():
    r = WorkerRegistry([W1, W2], failure_threshold=2, success_threshold=2)
    r.record_failure(W1)
    assert W1 in r.healthy_endpoints()
    r.record_failure(W1)
    assert r.healthy_endpoints() == [W2]
    r.record_success(W1)
    assert r.healthy_endpoints() == [W2]
    r.record_success(W1)
    assert set(r.healthy_endpoints()) == {W1, W2}


def test_registry_pending_admitted_on_first_success_and_survivor_state():
    r = WorkerRegistry([W1], allow_empty=True)
    r.record_failure(W1)
    added, removed = r.set_members([W1, W2])
    assert added == [W2] and removed == []
    snap = {s["endpoint"]: s for s in r.snapshot()}
    assert snap[W2]["pending"] and not snap[W2]["healthy"]
    assert snap[W1]["consecutive_failures"] == 1  # survivor keeps its state
    r.record_success(W2)
    assert W2 in r.healthy_endpoints()


def test_registry_no_healthy_raises_and_empty_allowed():
    with pytest.raises(ValueError):
        WorkerRegistry([])
    r = WorkerRegistry([], allow_empty=True)
    with pytest.raises(NoHealthyWorkersError):
        r.pick()


def test_registry_least_inflight():
    r = WorkerRegistry([W1, W2, W3], routing="least_inflight")
    r.begin(W1)
    r.begin(W1)
    r.begin(W2)
    assert r.pick() == W3
    r.begin(W3)
    r.begin(W3)
    assert r.pick() == W2


def test_registry_thread_hammer():
    r = WorkerRegistry([W1, W2, W3], failure_threshold=3)

    def work():
        for i in range(2000):
            try:
                ep = r.pick()
            except NoHealthyWorkersError:
                ep = W1
            (r.record_success if i % 3 else r.record_failure)(ep)
            r.set_members([W1, W2, W3] if i % 50 else [W1, W2])

    ts = [threading.Thread(target=work) for _ in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert set(r.endpoints()) <= {W1, W2, W3}


# ------------------------------------------------------------------ remote backend
def _transport(script):
    """script: endpoint -> callable(request) -> httpx.Response or raise."""
    def handler(request: httpx.Request):
        base = f"{request.url.scheme}://{request.url.host}:{request.url.port}"
        return script[base](request)
    return httpx.MockTransport(handler)


def _ok(request):
    body = __import__("json").loads(request.content)
    return httpx.Response(200, json={"results": [{"text": "ok:" + p, "num_tokens": 2} for p in body["prompts"]]})


def _refuse(request):
    raise httpx.ConnectError("refused", request=request)


def _timeout(request):
    raise httpx.ReadTimeout("slow", request=request)


async def test_remote_connect_error_retries_other_worker():
    be = RemoteBackend(WorkerConfig(endpoints=[W1, W2]), transport=_transport({W1: _refuse, W2: _ok}))
    r = await be.agenerate("p", {"max_tokens": 2})
    assert r["text"] == "ok:p"
    await be.aclose()


@pytest.mark.parametrize("fn,exc", [(_timeout, RemoteInferenceError),
                                    (lambda rq: httpx.Response(500, text="bad"), RemoteInferenceError),
                                    (lambda rq: httpx.Response(200, json={"results": []}), RemoteInferenceError)])
async def test_remote_no_retry_after_delivery(fn, exc):
    calls = []

    def counted(rq):
        calls.append(1)
        return fn(rq)

    be = RemoteBackend(WorkerConfig(endpoints=[W1, W2]), transport=_transport({W1: counted, W2: counted}))
    with pytest.raises(exc):
        await be.agenerate("p", {"max_tokens": 2})
    assert len(calls) == 1
    await be.aclose()


async def test_remote_all_refused_no_healthy():
    be = RemoteBackend(WorkerConfig(endpoints=[W1, W2]), transport=_transport({W1: _refuse, W2: _refuse}))
    with pytest.raises(NoHealthyWorkersError):
        await be.agenerate("p", {})
    await be.aclose()


def test_remote_sync_generate_and_bearer():
    seen = {}

    def h(rq):
        seen["auth"] = rq.headers.get("authorization")
        return _ok(rq)

    be = RemoteBackend(WorkerConfig(endpoints=[W1], api_key="sek"), transport=_transport({W1: h}))
    assert be.generate(["a", "b"], {})[1]["text"] == "ok:b"
    assert seen["auth"] == "Bearer sek"


def _worker_app(backend=None):
    cfg = VGateConfig(role="worker")
    eng = VGateEngine(model_config=cfg.model, worker_config=cfg.worker, backend=backend or DryRunBackend(),
                      dry_run=True)
    return create_app(cfg, engine=eng)


async def test_gateway_to_real_worker_app_unary_and_stream():
    wapp = _worker_app()
    async with wapp.router.lifespan_context(wapp):
        be = RemoteBackend(WorkerConfig(endpoints=[W1]), transport=httpx.ASGITransport(app=wapp))
        r = await be.agenerate("hello there", {"temperature": 0.7, "top_p": 0.9, "max_tokens": 8})
        assert r["text"] == "[dry-run] echo: hello there" and r["num_tokens"] == 8
        pieces = [p async for p in be.stream_generate("one two three", {"max_tokens": 8})]
        assert "".join(p["delta"] for p in pieces) == "[dry-run] echo: one two three"
        await be.aclose()


def _free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


async def test_remote_backend_aiohttp_path_over_real_sockets():
    """The serving path (no injected transport): aiohttp pool against a real uvicorn worker —
    unary, SSE stream, a refused endpoint skipped (connect failure is the one retried case) and
    a non-200 surfaced without retry."""
    import time as _time

    import uvicorn
    wapp = _worker_app()
    port, dead = _free_port(), _free_port()
    srv = uvicorn.Server(uvicorn.Config(wapp, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = _time.time()
    while not srv.started and _time.time() - t0 < 20:
        await asyncio.sleep(0.05)
    try:
        live, refused = f"http://127.0.0.1:{port}", f"http://127.0.0.1:{dead}"
        be = RemoteBackend(WorkerConfig(endpoints=[refused, live], routing="round_robin"))
        rs = await asyncio.gather(*(be.agenerate(f"p{i}", {"max_tokens": 4}) for i in range(16)))
        assert all(r["text"] == f"[dry-run] echo: p{i}" for i, r in enumerate(rs))
        pieces = [c async for c in be.stream_generate("one two three", {"max_tokens": 8})]
        assert "".join(c["delta"] for c in pieces) == "[dry-run] echo: one two three"
        assert be.registry.healthy_endpoints() == [live]  # refused one demoted by the retries
        bad = RemoteBackend(WorkerConfig(endpoints=[live + "/nope"]))
        with pytest.raises(RemoteInferenceError, match="404"):
            await bad.agenerate("x", {"max_tokens": 1})
        await be.aclose()
        await bad.aclose()
    finally:
        srv.should_exit = True
        th.join(timeout=10)


async def test_full_gateway_over_worker_streaming_end_to_end():
    wapp = _worker_app()
    async with wapp.router.lifespan_context(wapp):
        gcfg = VGateConfig(worker={"endpoints": [W1]})
        be = RemoteBackend(gcfg.worker, transport=httpx.ASGITransport(app=wapp))
        geng = VGateEngine(model_config=gcfg.model, worker_config=gcfg.worker, backend=be)
        geng.is_remote = True
        gapp = create_app(gcfg, engine=geng)
        async with gapp.router.lifespan_context(gapp):
            async with httpx.AsyncClient(transport=httpx.ASGITransport(app=gapp), base_url="http://g") as c:
                body = {"model": "m", "messages": [{"role": "user", "content": "hi"}]}
                r = await c.post("/v1/chat/completions", json=body)
                assert r.status_code == 200 and "echo" in r.json()["choices"][0]["message"]["content"]
                r = await c.post("/v1/chat/completions", json={**body, "stream": True})
                assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
                s = (await c.get("/stats")).json()
                assert s["workers"][0]["endpoint"] == W1


async def test_worker_503_before_engine_bound():
    from fastapi import FastAPI
    from vgate import worker_api
    worker_api._engine = None
    app = FastAPI()
    app.include_router(worker_api.router)
    async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://w") as c:
        assert (await c.post("/internal/generate", json={"prompts": ["x"]})).status_code == 503


# ----------------------------------------------------------------------- discovery
def _gai(errno):
    e = socket.gaierror(errno, "x")
    return e


def test_discovery_reverse_names_and_ipv6():
    names = {"10.0.0.1": "w-0.svc.ns.", "10.0.0.2": "w-1.svc.ns"}

    def rev(a):
        if a not in names:
            raise socket.herror(1, "no PTR")
        return names[a]

    d = DnsWorkerDiscovery("svc.ns", 8000, forward_resolver=lambda h, p: ["10.0.0.2", "fd00::1", "10.0.0.1"],
                           reverse_resolver=rev)
    assert d.resolve() == ["http://[fd00::1]:8000", "http://w-0.svc.ns:8000", "http://w-1.svc.ns:8000"]


def test_discovery_ptr_equal_to_service_is_not_identity():
    d = DnsWorkerDiscovery("svc.ns", 9000, forward_resolver=lambda h, p: ["10.0.0.9"],
                           reverse_resolver=lambda a: "svc.ns.")
    assert d.resolve() == ["http://10.0.0.9:9000"]


def test_discovery_authoritative_empty_vs_transient():
    def empty(h, p):
        raise _gai(socket.EAI_NONAME)

    def broken(h, p):
        raise _gai(socket.EAI_AGAIN)

    assert DnsWorkerDiscovery("s", forward_resolver=empty).resolve() == []
    with pytest.raises(TransientResolutionError):
        DnsWorkerDiscovery("s", forward_resolver=broken).resolve()


# ------------------------------------------------------------------- health checker
async def test_health_checker_probes_and_membership():
    answers = {"n": 0}
    state = {"eps": ["10.0.0.1"]}

    def fwd(h, p):
        answers["n"] += 1
        if state["eps"] is None:
            raise _gai(socket.EAI_NONAME)
        return state["eps"]

    disc = DnsWorkerDiscovery("svc", 8000, forward_resolver=fwd, reverse_resolver=lambda a: f"pod-{a[-1]}")
    reg = WorkerRegistry([], allow_empty=True)
    health = {"http://pod-1:8000": 200, "http://pod-2:8000": 500}
    tr = httpx.MockTransport(lambda rq: httpx.Response(health.get(f"http://{rq.url.host}:{rq.url.port}", 404)))
    hc = WorkerHealthChecker(reg, interval_seconds=0.02, timeout_seconds=0.5, transport=tr, discovery=disc,
                             empty_resolve_threshold=3)
    await hc.start()
    assert reg.healthy_endpoints() == ["http://pod-1:8000"]  # admitted on first successful probe
    state["eps"] = ["10.0.0.1", "10.0.0.2"]
    await asyncio.sleep(0.15)
    assert "http://pod-2:8000" in reg.endpoints() and "http://pod-2:8000" not in reg.healthy_endpoints()
    state["eps"] = None  # authoritative empty: needs 3 ticks before the pool is emptied
    await asyncio.sleep(0.3)
    assert reg.endpoints() == []
    await hc.stop()


async def test_health_checker_transient_dns_keeps_pool():
    def broken(h, p):
        raise _gai(socket.EAI_AGAIN)

    reg = WorkerRegistry([W1])
    tr = httpx.MockTransport(lambda rq: httpx.Response(200))
    hc = WorkerHealthChecker(reg, interval_seconds=0.02, transport=tr,
                             discovery=DnsWorkerDiscovery("svc", forward_resolver=broken))
    await hc.start()
    await asyncio.sleep(0.1)
    assert reg.endpoints() == [W1] and reg.healthy_endpoints() == [W1]
    await hc.stop()


async def test_health_checker_stalled_resolver_does_not_block_probes():
    import time

    def stall(h, p):
        time.sleep(0.5)
        return ["10.0.0.1"]

    reg = WorkerRegistry([W1, W2], failure_threshold=1)
    probes = []
    tr = httpx.MockTransport(lambda rq: (probes.append(1), httpx.Response(500 if rq.url.host == "w2" else 200))[1])
    hc = WorkerHealthChecker(reg, interval_seconds=0.02, transport=tr, startup_resolve_timeout=0.1,
                             resolve_timeout=0.05, discovery=DnsWorkerDiscovery("svc", forward_resolver=stall,
                                                                               reverse_resolver=lambda a: "x"))
    t0 = asyncio.get_running_loop().time()
    await hc.start()
    assert asyncio.get_running_loop().time() - t0 < 0.4  # startup bounded
    await asyncio.sleep(0.2)
    assert len(probes) >= 3  # probing kept ticking while DNS was wedged
    await hc.stop()


# ---------------------------------------------------------------- engine-aware health
class _FaultyBackend(DryRunBackend):
    """Dry-run backend with the native backend's health hook (fault injection)."""

    def __init__(self):
        super().__init__()
        self.ok = True

    def healthy(self) -> bool:
        return self.ok


async def test_worker_health_fails_when_engine_faults_and_gateway_demotes():
    be = _FaultyBackend()
    wapp = _worker_app(be)
    async with wapp.router.lifespan_context(wapp):
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=wapp), base_url="http://w") as c:
            r = await c.get("/health")
            assert r.status_code == 200 and r.json()["status"] == "ok" and r.json()["role"] == "worker"
        reg = WorkerRegistry([W1], failure_threshold=2, success_threshold=2)
        hc = WorkerHealthChecker(reg, interval_seconds=0.02, timeout_seconds=0.5,
                                 transport=httpx.ASGITransport(app=wapp))
        await hc.start()
        assert reg.healthy_endpoints() == [W1]
        be.ok = False  # inject an engine fault: the worker's /health turns 503
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=wapp), base_url="http://w") as c:
            r = await c.get("/health")
            assert r.status_code == 503 and r.json()["status"] == "unhealthy"
        for _ in range(100):
            if not reg.healthy_endpoints():
                break
            await asyncio.sleep(0.02)
        assert reg.healthy_endpoints() == []  # demoted within failure_threshold probes
        be.ok = True  # recovery needs success_threshold probes
        for _ in range(100):
            if reg.healthy_endpoints():
                break
            await asyncio.sleep(0.02)
        assert reg.healthy_endpoints() == [W1]
        await hc.stop()


def test_native_backend_watchdog_is_configurable():
    import time
    from vgate.backends.native import NativeBackend

    class _Eng:
        healthy = True
        last_step_wall = time.monotonic() - 5.0

        def has_unfinished(self):
            return True

    nb = NativeBackend(_Eng(), watchdog_seconds=10.0)
    assert nb.healthy()
    nb.watchdog_seconds = 2.0  # work pending and no step for 5 s: a hung queue
    assert not nb.healthy()
    _Eng.has_unfinished = lambda self: False  # idle engines are never flagged
    assert nb.healthy()


async def test_aiohttp_stream_outlives_timeout_and_carries_long_lines():
    """ROUND-2 ADVICE (medium): an SSE pass-through is bounded by the silence between chunks
    (worker.timeout_seconds), not by its total lifetime, and a delta line over aiohttp's 64 KiB
    readline limit is delivered instead of raising. The mock worker streams for ~3x the timeout."""
    import json as _json
    import time as _time

    import uvicorn
    from fastapi import FastAPI
    from fastapi.responses import StreamingResponse

    app = FastAPI()
    big = "x" * (100 * 1024)

    @app.post("/internal/generate_stream")
    async def gen_stream():
        async def body():
            for i in range(12):
                await asyncio.sleep(0.25)
                yield f"data: {_json.dumps({'delta': str(i), 'num_tokens': i + 1})}\n\n"
            yield f"data: {_json.dumps({'delta': big, 'num_tokens': 13})}\n\n"
            yield "data: [DONE]\n\n"
        return StreamingResponse(body(), media_type="text/event-stream")

    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    t0 = _time.time()
    while not srv.started and _time.time() - t0 < 20:
        await asyncio.sleep(0.05)
    try:
        be = RemoteBackend(WorkerConfig(endpoints=[f"http://127.0.0.1:{port}"], timeout_seconds=1.0))
        t1 = _time.time()
        pieces = [c async for c in be.stream_generate("p", {"max_tokens": 13})]
        assert _time.time() - t1 > 2.5  # longer than timeout_seconds, still served
        assert [c["delta"] for c in pieces[:12]] == [str(i) for i in range(12)]
        assert pieces[-1]["delta"] == big
        await be.aclose()
    finally:
        srv.should_exit = True
        th.join(timeout=10)
