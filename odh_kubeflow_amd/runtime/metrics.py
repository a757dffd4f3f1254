"""controller-runtime's built-in Prometheus metrics (reconcile counters/latency and
workqueue gauges), served on the manager's ``/metrics`` endpoint.

Names follow controller-runtime so existing dashboards keep working:
``controller_runtime_reconcile_total``, ``controller_runtime_reconcile_errors_total``,
``controller_runtime_reconcile_time_seconds``, ``controller_runtime_max_concurrent_reconciles``,
``controller_runtime_active_workers``, ``workqueue_depth``, ``workqueue_adds_total``,
``workqueue_queue_duration_seconds``, ``workqueue_retries_total``.

These are updated several times per reconcile on the event loop, so they are plain
attribute arithmetic (``prometheus_client``'s metric objects take a lock and validate
arguments on every update); a collector registered with the manager's
``CollectorRegistry`` turns them into metric families at scrape time only.
"""

from __future__ import annotations

from bisect import bisect_left
from typing import Dict, List, Sequence, Tuple

from prometheus_client import CollectorRegistry
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily

_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60)


class _Value:
    __slots__ = ("v",)

    def __init__(self):
        self.v = 0.0

    def inc(self, amount: float = 1.0) -> None:
        self.v += amount

    def dec(self, amount: float = 1.0) -> None:
        self.v -= amount

    def set(self, value: float) -> None:
        self.v = float(value)


class _Histo:
    __slots__ = ("bounds", "counts", "sum")

    def __init__(self, bounds: Sequence[float]):
        self.bounds = bounds
        self.counts = [0] * (len(bounds) + 1)  # last slot: +Inf
        self.sum = 0.0

    def observe(self, x: float) -> None:
        self.sum += x
        self.counts[bisect_left(self.bounds, x)] += 1  # first bound >= x: Prometheus "le"


class _Metric:
    def __init__(self, kind: str, name: str, doc: str, labelnames: Sequence[str], buckets=None):
        self.kind, self.name, self.doc, self.labelnames = kind, name, doc, tuple(labelnames)
        self.buckets = tuple(float(b) for b in buckets) if buckets else None
        self.children: Dict[Tuple[str, ...], object] = {}

    def labels(self, *values) -> object:
        c = self.children.get(values)
        if c is None:
            if len(values) != len(self.labelnames):
                raise ValueError(f"{self.name}: expected labels {self.labelnames}, got {values}")
            key = tuple(str(v) for v in values)
            c = self.children.get(key)
            if c is None:
                c = _Histo(self.buckets) if self.kind == "histogram" else _Value()
                self.children[key] = c
            self.children[values] = c  # memoised under the caller's exact key too
        return c

    def _series(self):
        seen = set()
        for k, c in list(self.children.items()):
            if id(c) not in seen:
                seen.add(id(c))
                yield tuple(str(v) for v in k), c

    def family(self):
        if self.kind == "counter":
            fam = CounterMetricFamily(self.name, self.doc, labels=self.labelnames)
            for k, c in self._series():
                fam.add_metric(k, c.v)
        elif self.kind == "gauge":
            fam = GaugeMetricFamily(self.name, self.doc, labels=self.labelnames)
            for k, c in self._series():
                fam.add_metric(k, c.v)
        else:
            fam = HistogramMetricFamily(self.name, self.doc, labels=self.labelnames)
            for k, h in self._series():
                acc, buckets = 0, []
                for b, n in zip(self.buckets, h.counts):
                    acc += n
                    buckets.append((repr(b), acc))
                buckets.append(("+Inf", acc + h.counts[-1]))
                fam.add_metric(k, buckets, h.sum)
        return fam


class _Collector:
    def __init__(self, metrics: List[_Metric]):
        self.metrics = metrics

    def collect(self):
        for m in self.metrics:
            yield m.family()

    def describe(self):
        return [m.family() for m in self.metrics]


class RuntimeMetrics:
    def __init__(self, registry: CollectorRegistry):
        self.registry = registry
        self.reconcile_total = _Metric("counter", "controller_runtime_reconcile_total",
                                       "Total number of reconciliations per controller", ["controller", "result"])
        self.reconcile_errors = _Metric("counter", "controller_runtime_reconcile_errors_total",
                                        "Total number of reconciliation errors per controller", ["controller"])
        self.reconcile_time = _Metric("histogram", "controller_runtime_reconcile_time_seconds",
                                      "Length of time per reconciliation per controller", ["controller"],
                                      buckets=_BUCKETS)
        self.max_concurrent = _Metric("gauge", "controller_runtime_max_concurrent_reconciles",
                                      "Maximum number of concurrent reconciles per controller", ["controller"])
        self.active_workers = _Metric("gauge", "controller_runtime_active_workers",
                                      "Number of currently used workers per controller", ["controller"])
        self.depth = _Metric("gauge", "workqueue_depth", "Current depth of workqueue", ["name"])
        self.adds = _Metric("counter", "workqueue_adds_total", "Total number of adds handled by workqueue", ["name"])
        self.queue_latency = _Metric("histogram", "workqueue_queue_duration_seconds",
                                     "How long in seconds an item stays in workqueue before being requested",
                                     ["name"], buckets=_BUCKETS)
        self.retries = _Metric("counter", "workqueue_retries_total", "Total number of retries handled by workqueue",
                               ["name"])
        # not in controller-runtime: what queued each reconcile (the watched kind whose event
        # first queued the request, or "requeue"), and own-write watch echoes not queued
        self.reconcile_trigger = _Metric("counter", "odh_controller_reconcile_trigger_total",
                                         "Reconciles per controller by the watched kind that queued them",
                                         ["controller", "trigger"])
        self.echoes_skipped = _Metric("counter", "odh_controller_own_write_echoes_skipped_total",
                                      "Watch events of a controller's own writes that did not requeue the writer",
                                      ["controller"])
        registry.register(_Collector([self.reconcile_total, self.reconcile_errors, self.reconcile_time,
                                      self.max_concurrent, self.active_workers, self.depth, self.adds,
                                      self.queue_latency, self.retries, self.reconcile_trigger,
                                      self.echoes_skipped]))

    @staticmethod
    def child(metric: _Metric, *labels):
        """``metric.labels(*labels)`` (children are memoised by the metric)."""
        return metric.labels(*labels)

    # workqueue hooks
    def on_add(self, name: str, depth: int) -> None:
        self.adds.labels(name).v += 1.0
        self.depth.labels(name).v = float(depth)

    def on_get(self, name: str, depth: int, latency: float) -> None:
        self.depth.labels(name).v = float(depth)
        self.queue_latency.labels(name).observe(latency)

    def on_retry(self, name: str) -> None:
        self.retries.labels(name).v += 1.0
