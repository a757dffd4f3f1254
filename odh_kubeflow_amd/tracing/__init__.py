"""Minimal OpenTelemetry-shaped tracing (spans, attributes, span events).

The reference instruments only the admission webhook: a root span ``handleFunc``
with ``notebook`` / ``namespace`` / ``operation`` attributes, a child span
``maybeRestartRunningNotebook`` and the span events ``imagestream-not-found`` /
``imagestream-tag-not-found`` (``odh/controllers/notebook_webhook.go:70-72,89-90,
360-365,509-510,834,850,883``).  In production the global provider is a no-op; the
tests install an in-memory exporter and use span events as an oracle for which code
path ran (``odh/controllers/opentelemetry_test.go:26-77``).

``opentelemetry`` is not installed in this image, so this module provides the same
shape: a global provider (no-op by default), ``tracer.start_span(...)`` as a context
manager, ``current_span()`` via ``contextvars`` and :class:`InMemoryExporter`.  The
reconcilers also open spans (``reconcile`` with controller/name attributes) so a
provider installed in production traces the whole create→Ready path.
"""

from __future__ import annotations

import contextlib
import contextvars
import itertools
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional

_ids = itertools.count(1)


@dataclass
class SpanEvent:
    name: str
    timestamp: float
    attributes: Dict[str, Any] = field(default_factory=dict)


@dataclass
class Span:
    name: str
    tracer: str
    trace_id: int
    span_id: int
    parent_id: Optional[int]
    attributes: Dict[str, Any] = field(default_factory=dict)
    events: List[SpanEvent] = field(default_factory=list)
    start: float = 0.0
    end: Optional[float] = None
    status: str = "UNSET"
    recording: bool = True

    def add_event(self, name: str, attributes: Optional[Dict[str, Any]] = None) -> None:
        if self.recording:
            self.events.append(SpanEvent(name, time.time(), dict(attributes or {})))

    def set_attribute(self, key: str, value: Any) -> None:
        if self.recording:
            self.attributes[key] = value

    def set_status(self, status: str) -> None:
        if self.recording:
            self.status = status

    def record_exception(self, exc: BaseException) -> None:
        self.add_event("exception", {"exception.type": type(exc).__name__, "exception.message": str(exc)})

    @property
    def duration(self) -> float:
        return (self.end or time.time()) - self.start


_NOOP = Span("noop", "", 0, 0, None, recording=False)
_current: contextvars.ContextVar[Optional[Span]] = contextvars.ContextVar("odh_current_span", default=None)


class InMemoryExporter:
    """Collects finished spans (``tracetest.InMemoryExporter``)."""

    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._spans: List[Span] = []

    def export(self, span: Span) -> None:
        with self._lock:
            self._spans.append(span)

    def get_finished_spans(self) -> List[Span]:
        with self._lock:
            return list(self._spans)

    def reset(self) -> None:
        with self._lock:
            self._spans.clear()

    def events(self, name: Optional[str] = None) -> List[str]:
        return [e.name for s in self.get_finished_spans() if name is None or s.name == name for e in s.events]


class TracerProvider:
    def __init__(self, exporter: Optional[InMemoryExporter] = None):
        self.exporter = exporter

    def tracer(self, name: str) -> "Tracer":
        return Tracer(name, self)


class _NoopProvider(TracerProvider):
    def __init__(self) -> None:
        super().__init__(None)


_provider: TracerProvider = _NoopProvider()


def set_tracer_provider(p: Optional[TracerProvider]) -> None:
    global _provider
    _provider = p if p is not None else _NoopProvider()


def get_tracer_provider() -> TracerProvider:
    return _provider


class Tracer:
    def __init__(self, name: str, provider: Optional[TracerProvider] = None):
        self.name = name
        self._provider = provider

    @property
    def provider(self) -> TracerProvider:
        # resolved lazily, like the reference's sync.OnceValue(otel.GetTracerProvider().Tracer(..))
        return self._provider if self._provider is not None else _provider

    @contextlib.contextmanager
    def start_span(self, name: str, attributes: Optional[Dict[str, Any]] = None,
                   new_root: bool = False) -> Iterator[Span]:
        prov = self.provider
        if prov.exporter is None:
            tok = _current.set(_NOOP)
            try:
                yield _NOOP
            finally:
                _current.reset(tok)
            return
        parent = None if new_root else _current.get()
        if parent is not None and not parent.recording:
            parent = None
        sid = next(_ids)
        span = Span(name, self.name, parent.trace_id if parent else sid, sid, parent.span_id if parent else None,
                    dict(attributes or {}), start=time.time())
        tok = _current.set(span)
        try:
            yield span
        except BaseException as e:
            span.record_exception(e)
            span.set_status("ERROR")
            raise
        finally:
            span.end = time.time()
            _current.reset(tok)
            prov.exporter.export(span)


def get_tracer(name: str) -> Tracer:
    return Tracer(name)


def current_span() -> Span:
    s = _current.get()
    return s if s is not None else _NOOP
