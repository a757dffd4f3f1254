"""controller-runtime's built-in Prometheus metrics (reconcile counters/latency and
workqueue gauges), served on the manager's ``/metrics`` endpoint.

Names follow controller-runtime so existing dashboards keep working:
``controller_runtime_reconcile_total``, ``controller_runtime_reconcile_errors_total``,
``controller_runtime_reconcile_time_seconds``, ``controller_runtime_max_concurrent_reconciles``,
``controller_runtime_active_workers``, ``workqueue_depth``, ``workqueue_adds_total``,
``workqueue_queue_duration_seconds``, ``workqueue_retries_total``.
"""

from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram

_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60)


class RuntimeMetrics:
    def __init__(self, registry: CollectorRegistry):
        self.registry = registry
        self.reconcile_total = Counter("controller_runtime_reconcile_total", "Total number of reconciliations per controller",
                                       ["controller", "result"], registry=registry)
        self.reconcile_errors = Counter("controller_runtime_reconcile_errors_total",
                                        "Total number of reconciliation errors per controller", ["controller"],
                                        registry=registry)
        self.reconcile_time = Histogram("controller_runtime_reconcile_time_seconds",
                                        "Length of time per reconciliation per controller", ["controller"],
                                        buckets=_BUCKETS, registry=registry)
        self.max_concurrent = Gauge("controller_runtime_max_concurrent_reconciles",
                                    "Maximum number of concurrent reconciles per controller", ["controller"],
                                    registry=registry)
        self.active_workers = Gauge("controller_runtime_active_workers",
                                    "Number of currently used workers per controller", ["controller"], registry=registry)
        self.depth = Gauge("workqueue_depth", "Current depth of workqueue", ["name"], registry=registry)
        self.adds = Counter("workqueue_adds_total", "Total number of adds handled by workqueue", ["name"],
                            registry=registry)
        self.queue_latency = Histogram("workqueue_queue_duration_seconds",
                                       "How long in seconds an item stays in workqueue before being requested",
                                       ["name"], buckets=_BUCKETS, registry=registry)
        self.retries = Counter("workqueue_retries_total", "Total number of retries handled by workqueue", ["name"],
                               registry=registry)

        self._children = {}

    def child(self, metric, *labels):
        """Memoised ``metric.labels(*labels)`` (label lookup is the hot part of a metric update)."""
        k = (id(metric), labels)
        c = self._children.get(k)
        if c is None:
            c = self._children[k] = metric.labels(*labels)
        return c

    # workqueue hooks
    def on_add(self, name: str, depth: int) -> None:
        self.child(self.adds, name).inc()
        self.child(self.depth, name).set(depth)

    def on_get(self, name: str, depth: int, latency: float) -> None:
        self.child(self.depth, name).set(depth)
        self.child(self.queue_latency, name).observe(latency)

    def on_retry(self, name: str) -> None:
        self.child(self.retries, name).inc()
