"""The engine core in its own process (``model.engine_process: true``).

In-process, the engine thread shares one GIL with the HTTP event loop (uvicorn/h11
parsing, pydantic validation, batcher, cache, metrics) and a fault in the engine takes the
API server with it. Here the :class:`vgate.runtime.engine.LLMEngine` runs in a child
process (spawned before the
parent touches the GPU) and the API process talks to it over one duplex pipe:

  parent -> child   ("add", rid, prompt, prompt_ids, params, stream) | ("abort", rid)
                    ("call", id, "embed", args) | ("stop",)
  child  -> parent  ("tok", rid, n, delta) | ("fin", rid, kind, fields, error)
                    ("snap", snapshot) every 0.25 s | ("ret", id, ok, value)

:class:`EngineProcessClient` exposes the subset of the LLMEngine interface the backends
use (add_request with callbacks, abort, embed, snapshot, healthy, stop), so
:class:`vgate.backends.native.NativeBackend` is unchanged. Callbacks receive a
:class:`SeqView` carrying the fields the backend reads. This mirrors the reference's
vLLM deployment, whose EngineCore also runs in a separate process
(reference benchmarks/run_report.py:89-93). TP > 1 keeps the in-process engine (rank 0
drives its followers directly). Measured on MI355X (profiles/r1_bench_concurrency_sweep.log):
equal throughput at the headline's 8 concurrent clients, +6% at 64 and +28% at 128
(372 -> 477 req/s) — at high request rates the HTTP side's Python work holds the shared
GIL long enough to stall the engine's step loop.
"""
from __future__ import annotations

import itertools
import logging
import threading
import time
import traceback
from concurrent.futures import Future

log = logging.getLogger("vgate.engine")


class SeqView:
    """What a completion callback may read from a sequence (NativeBackend._result)."""

    __slots__ = ("request_id", "text", "output_ids", "prompt_ids", "finish_reason", "first_token_time",
                 "arrival", "finish_time")

    def __init__(self, request_id: str):
        self.request_id = request_id
        self.text = ""
        self.output_ids: list[int] = []
        self.prompt_ids: list[int] = []
        self.finish_reason = None
        self.first_token_time = None
        self.arrival = time.perf_counter()
        self.finish_time = None


def _fields(seq) -> dict:
    return {"text": seq.text, "output_ids": list(seq.output_ids), "prompt_len": len(seq.prompt_ids),
            "finish_reason": seq.finish_reason, "first_token_time": seq.first_token_time, "arrival": seq.arrival,
            "finish_time": seq.finish_time}


def _core_main(cfg, conn, snap_period: float = 0.25) -> None:
    """Child process: build the engine, run its thread, serve the pipe."""
    logging.basicConfig(level=logging.WARNING)
    try:
        from vgate.runtime.engine import LLMEngine
        eng = LLMEngine(cfg)
        eng.start()
    except BaseException:  # noqa: BLE001 - reported to the parent, which raises it
        conn.send(("fatal", traceback.format_exc()))
        return
    lock = threading.Lock()

    def send(msg) -> None:
        with lock:
            conn.send(msg)

    def snap() -> dict:
        s = eng.snapshot()
        s["healthy"] = bool(eng.healthy)
        s["has_work"] = bool(eng.has_unfinished())
        s["last_step_age_s"] = time.monotonic() - eng.last_step_wall
        return s

    def make_cb(rid: str):
        def cb(kind, seq, payload):
            if kind == "token":
                send(("tok", rid, len(seq.output_ids), payload))
            else:
                send(("fin", rid, kind, _fields(seq), payload))
        return cb

    stop = threading.Event()

    def pusher():
        while not stop.wait(snap_period):
            try:
                send(("snap", snap()))
            except (OSError, EOFError, BrokenPipeError):
                return

    threading.Thread(target=pusher, name="vgate-core-snap", daemon=True).start()
    send(("ready", snap()))
    try:
        while True:
            try:
                msg = conn.recv()
            except (EOFError, OSError):
                break
            op = msg[0]
            if op == "add":
                _, rid, prompt, ids, params, stream = msg
                eng.add_request(rid, prompt, params, make_cb(rid), stream=stream, prompt_ids=ids)
            elif op == "abort":
                eng.abort(msg[1])
            elif op == "call":
                _, cid, name, args = msg
                try:
                    if name == "embed":
                        val = eng.embed(*args)
                    elif name == "snapshot":
                        val = snap()
                    else:
                        raise ValueError(f"unknown call {name}")
                    send(("ret", cid, True, val))
                except Exception as e:  # noqa: BLE001
                    send(("ret", cid, False, f"{type(e).__name__}: {e}"))
            elif op == "stop":
                break
    finally:
        stop.set()
        eng.stop()
        try:
            send(("stopped",))
        except (OSError, EOFError, BrokenPipeError):
            pass


class _Sched:
    def __init__(self, client: "EngineProcessClient"):
        self._c = client

    def has_work(self) -> bool:
        return bool(self._c._snap.get("has_work", False))


class EngineProcessClient:
    """LLMEngine-compatible proxy to the engine core process (see module docstring)."""

    def __init__(self, cfg, boot_timeout: float = 1800.0):
        import multiprocessing as mp

        from vgate.parallel.comm import TPGroup

        if cfg.tensor_parallel_size > 1:
            raise ValueError("engine_process requires tensor_parallel_size == 1")
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe(duplex=True)
        self._proc = ctx.Process(target=_core_main, args=(cfg, child), name="vgate-engine-core", daemon=True)
        self._proc.start()
        child.close()
        if not self._conn.poll(boot_timeout):
            self._proc.kill()
            raise RuntimeError("engine core process did not start in time")
        msg = self._conn.recv()
        if msg[0] == "fatal":
            self._proc.join(timeout=10)
            raise RuntimeError(f"engine core process failed to start:\n{msg[1]}")
        self.cfg = cfg
        self.tp = TPGroup()
        self._snap = msg[1]
        self._snap_t = time.monotonic()
        self._send_lock = threading.Lock()
        self._seqs: dict[str, tuple[SeqView, object]] = {}
        self._calls: dict[int, Future] = {}
        self._ids = itertools.count()
        self._running = True
        self._dead = None
        self.scheduler = _Sched(self)
        self._reader = threading.Thread(target=self._read_loop, name="vgate-core-reader", daemon=True)
        self._reader.start()

    # --------------------------------------------------------------- transport
    def _send(self, msg) -> None:
        with self._send_lock:
            self._conn.send(msg)

    def _read_loop(self) -> None:
        try:
            while True:
                msg = self._conn.recv()
                op = msg[0]
                if op == "tok":
                    _, rid, n, delta = msg
                    ent = self._seqs.get(rid)
                    if ent is not None:
                        sv, cb = ent
                        if sv.first_token_time is None:
                            sv.first_token_time = time.perf_counter()
                        sv.output_ids.extend([0] * (n - len(sv.output_ids)))
                        sv.text += delta
                        if cb is not None:
                            cb("token", sv, delta)
                elif op == "fin":
                    _, rid, kind, f, err = msg
                    ent = self._seqs.pop(rid, None)
                    if ent is not None:
                        sv, cb = ent
                        sv.text = f["text"]
                        sv.output_ids = f["output_ids"]
                        sv.prompt_ids = [0] * f["prompt_len"]
                        sv.finish_reason = f["finish_reason"]
                        # perf_counter is CLOCK_MONOTONIC: comparable across processes
                        sv.first_token_time, sv.arrival, sv.finish_time = (f["first_token_time"], f["arrival"],
                                                                           f["finish_time"])
                        if cb is not None:
                            cb(kind, sv, err)
                elif op == "snap":
                    self._snap, self._snap_t = msg[1], time.monotonic()
                elif op == "ret":
                    _, cid, ok, val = msg
                    fut = self._calls.pop(cid, None)
                    if fut is not None:
                        if ok:
                            fut.set_result(val)
                        else:
                            fut.set_exception(RuntimeError(val))
                elif op == "stopped":
                    break
        except (EOFError, OSError) as e:
            self._dead = f"engine core process exited ({type(e).__name__})"
        finally:
            self._running = False
            err = self._dead or "engine core stopped"
            for rid, (sv, cb) in list(self._seqs.items()):
                self._seqs.pop(rid, None)
                if cb is not None:
                    cb("error", sv, err)
            for fut in list(self._calls.values()):
                if not fut.done():
                    fut.set_exception(RuntimeError(err))

    def _call(self, name: str, *args, timeout: float = 300.0):
        cid = next(self._ids)
        fut: Future = Future()
        self._calls[cid] = fut
        self._send(("call", cid, name, args))
        return fut.result(timeout=timeout)

    # --------------------------------------------------------- engine surface
    def start(self) -> None:  # the core starts its engine thread itself
        return None

    def add_request(self, request_id: str, prompt: str | None = None, params=None, callback=None,
                    stream: bool = False, prompt_ids: list[int] | None = None) -> SeqView:
        from vgate.runtime.sampling_params import SamplingParams

        sv = SeqView(request_id)
        self._seqs[request_id] = (sv, callback)
        if not self._running:
            self._seqs.pop(request_id, None)
            if callback is not None:
                callback("error", sv, self._dead or "engine core stopped")
            return sv
        self._send(("add", request_id, prompt, prompt_ids, params or SamplingParams(), stream))
        return sv

    def abort(self, request_id: str) -> None:
        if self._running:
            self._send(("abort", request_id))

    def embed(self, text: str | None = None, prompt_ids: list[int] | None = None):
        return tuple(self._call("embed", text, prompt_ids))

    def snapshot(self) -> dict:
        return dict(self._snap)

    def has_unfinished(self) -> bool:
        return bool(self._seqs) or bool(self._snap.get("has_work"))

    @property
    def healthy(self) -> bool:
        return self._running and self._proc.is_alive() and bool(self._snap.get("healthy", True))

    @property
    def last_step_wall(self) -> float:
        return self._snap_t - float(self._snap.get("last_step_age_s", 0.0))

    def run_until_idle(self, max_steps: int = 0) -> None:
        raise RuntimeError("the engine core process steps itself; wait on the request callbacks")

    def stop(self) -> None:
        if self._proc.is_alive():
            try:
                self._send(("stop",))
            except (OSError, BrokenPipeError):
                pass
            self._proc.join(timeout=60)
            if self._proc.is_alive():
                self._proc.kill()
                self._proc.join(timeout=10)
        self._running = False

    def shutdown_followers(self) -> None:
        return None
