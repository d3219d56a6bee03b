"""Distributed tracing (OpenTelemetry when installed, a built-in tracer otherwise).

The OpenTelemetry SDK is not installed in this environment, so the module ships
a small self-contained tracer with the same surface the rest of the code uses:
``get_tracer().start_as_current_span(name, attributes=...)`` context managers,
W3C ``traceparent`` inject/extract for gateway->worker propagation, 32/16-hex
trace/span ids for log correlation, ratio sampling, and an in-memory exporter
(tests, ``/stats`` debugging). When ``opentelemetry`` IS importable and tracing
is enabled, spans go to the real SDK with an OTLP exporter instead.

Span names match the reference (security.check, batcher.submit,
batcher.inference, cache.get/put, engine.chat_completions, remote.generate,
worker.generate) plus engine-side ones (engine.step).
"""
from __future__ import annotations

import contextlib
import contextvars
import random
import threading
import time
from dataclasses import dataclass, field

_enabled = False
_sample_rate = 1.0
_service = "vgate"
_otel_tracer = None
_finished: list = []
_lock = threading.Lock()
_MAX_FINISHED = 10_000

_current: contextvars.ContextVar = contextvars.ContextVar("vgate_span", default=None)


@dataclass
class Span:
    name: str
    trace_id: int
    span_id: int
    parent_id: int | None
    sampled: bool
    start: float = field(default_factory=time.time)
    end: float | None = None
    attributes: dict = field(default_factory=dict)
    status: str = "OK"

    def set_attribute(self, k, v):
        self.attributes[k] = v

    def set_attributes(self, d: dict):
        self.attributes.update(d)

    def record_exception(self, e: BaseException):
        self.attributes["exception.type"] = type(e).__name__
        self.attributes["exception.message"] = str(e)

    def set_status(self, status, description: str | None = None):
        self.status = str(status)

    def is_recording(self) -> bool:
        return self.sampled

    def get_span_context(self):
        return self


class _NoopSpan:
    trace_id = 0
    span_id = 0
    sampled = False

    def set_attribute(self, *a):
        pass

    def set_attributes(self, *a):
        pass

    def record_exception(self, *a):
        pass

    def set_status(self, *a, **k):
        pass

    def is_recording(self):
        return False


_NOOP = _NoopSpan()


class Tracer:
    def __init__(self, name: str):
        self.name = name

    @contextlib.contextmanager
    def start_as_current_span(self, name: str, attributes: dict | None = None, **_kw):
        if _otel_tracer is not None:
            with _otel_tracer.start_as_current_span(name, attributes=attributes) as s:
                yield s
            return
        if not _enabled:
            yield _NOOP
            return
        parent = _current.get()
        if parent is not None:
            trace_id, sampled, pid = parent.trace_id, parent.sampled, parent.span_id
        else:
            trace_id, sampled, pid = random.getrandbits(128) or 1, random.random() < _sample_rate, None
        span = Span(name, trace_id, random.getrandbits(64) or 1, pid, sampled, attributes=dict(attributes or {}))
        tok = _current.set(span)
        try:
            yield span
        except BaseException as e:
            span.record_exception(e)
            span.status = "ERROR"
            raise
        finally:
            span.end = time.time()
            _current.reset(tok)
            if span.sampled:
                with _lock:
                    _finished.append(span)
                    if len(_finished) > _MAX_FINISHED:
                        del _finished[: len(_finished) - _MAX_FINISHED]


def init_tracing(config=None) -> bool:
    """Enable tracing per ``config.tracing``. Returns True when spans will be recorded."""
    global _enabled, _sample_rate, _service, _otel_tracer
    tc = getattr(config, "tracing", None)
    if tc is None or not tc.enabled:
        _enabled = False
        return False
    _sample_rate = float(tc.sample_rate)
    _service = tc.service_name
    try:  # real SDK when available
        from opentelemetry import trace  # type: ignore
        from opentelemetry.exporter.otlp.proto.grpc.trace_exporter import OTLPSpanExporter  # type: ignore
        from opentelemetry.sdk.resources import Resource  # type: ignore
        from opentelemetry.sdk.trace import TracerProvider  # type: ignore
        from opentelemetry.sdk.trace.export import BatchSpanProcessor  # type: ignore
        from opentelemetry.sdk.trace.sampling import TraceIdRatioBased  # type: ignore
        version = getattr(config, "version", "0")
        provider = TracerProvider(resource=Resource.create({"service.name": tc.service_name,
                                                            "service.version": version}),
                                  sampler=TraceIdRatioBased(tc.sample_rate))
        provider.add_span_processor(BatchSpanProcessor(OTLPSpanExporter(endpoint=tc.otlp_endpoint,
                                                                        insecure=tc.otlp_insecure)))
        trace.set_tracer_provider(provider)
        _otel_tracer = trace.get_tracer("vgate")
    except Exception:  # noqa: BLE001 - SDK absent: built-in tracer
        _otel_tracer = None
    _enabled = True
    return True


def shutdown_tracing() -> None:
    global _enabled, _otel_tracer
    _enabled = False
    _otel_tracer = None
    with _lock:
        _finished.clear()


def is_tracing_enabled() -> bool:
    return _enabled


def get_tracer(name: str = "vgate") -> Tracer:
    return Tracer(name)


def current_span():
    return _current.get()


def current_ids() -> tuple[str, str]:
    s = _current.get()
    if s is None or not s.trace_id:
        if _otel_tracer is not None:
            try:
                from opentelemetry import trace  # type: ignore
                ctx = trace.get_current_span().get_span_context()
                if ctx.trace_id:
                    return format(ctx.trace_id, "032x"), format(ctx.span_id, "016x")
            except Exception:  # noqa: BLE001
                pass
        return "", ""
    return format(s.trace_id, "032x"), format(s.span_id, "016x")


def get_current_trace_id() -> str:
    return current_ids()[0]


def finished_spans() -> list[Span]:
    with _lock:
        return list(_finished)


# ---- context propagation -------------------------------------------------------------
def capture_context():
    """Snapshot of the current span context (to re-attach on another thread)."""
    return contextvars.copy_context()


def inject_traceparent(headers: dict) -> dict:
    s = _current.get()
    if s is not None and s.trace_id:
        headers["traceparent"] = f"00-{s.trace_id:032x}-{s.span_id:016x}-{'01' if s.sampled else '00'}"
    return headers


@contextlib.contextmanager
def attach_traceparent(value: str | None):
    """Make a remote parent (W3C traceparent) the current context for the block."""
    if not value or not _enabled:
        yield
        return
    try:
        _, tid, sid, flags = value.split("-")
        parent = Span("remote", int(tid, 16), int(sid, 16), None, flags == "01")
    except ValueError:
        yield
        return
    tok = _current.set(parent)
    try:
        yield
    finally:
        _current.reset(tok)

