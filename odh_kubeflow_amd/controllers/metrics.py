"""Notebook controller Prometheus metrics (``kf/pkg/metrics/metrics.go``).

``notebook_running{namespace}`` is recomputed on every scrape from the StatefulSets
whose pod template carries ``notebook-name == sts.name`` (metrics.go:82-99), read from
the cache rather than a cluster-wide live List.  ``notebook_culling_total`` and
``last_notebook_culling_timestamp_seconds`` are registered and exported too — the
reference defines them but leaves them out of Describe/Collect (metrics.go:67-79),
so they never reach ``/metrics``; that is treated as a bug here.
Two MI355X additions: ``notebook_gpus_allocated{namespace}`` (``amd.com/gpu`` limits
of running notebooks) and ``notebook_pod_ready_seconds`` (start→Ready latency, observed
by the kf reconciler when a Notebook's status turns Ready: from the Notebook's creation
for its first pod, from the pod's creation for a resumed or restarted one).
"""

from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram
from prometheus_client.core import GaugeMetricFamily

from ..models import kinds
from ..models.notebook import NOTEBOOK_NAME_LABEL, gpu_request
from ..utils.timeutil import now as _now
from ..utils.timeutil import parse_rfc3339

# a pod created within this long of its Notebook is the Notebook's first pod (admission,
# lock removal and StatefulSet creation take seconds; a resumed notebook's pod comes later)
FIRST_POD_WINDOW_S = 300.0


class _RunningCollector:
    def __init__(self, reader):
        self.reader = reader

    def describe(self):
        return [GaugeMetricFamily("notebook_running", "Current running notebooks in the cluster", labels=["namespace"]),
                GaugeMetricFamily("notebook_gpus_allocated", "amd.com/gpu requested by running notebooks",
                                  labels=["namespace"])]

    def collect(self):
        running = GaugeMetricFamily("notebook_running", "Current running notebooks in the cluster",
                                    labels=["namespace"])
        gpus = GaugeMetricFamily("notebook_gpus_allocated", "amd.com/gpu requested by running notebooks",
                                 labels=["namespace"])
        per_ns, per_ns_gpu = {}, {}
        try:
            items = self.reader.list(kinds.STATEFUL_SET)
        except Exception:
            items = []
        for sts in items:
            tmpl = ((sts.get("spec") or {}).get("template") or {})
            name = ((tmpl.get("metadata") or {}).get("labels") or {}).get(NOTEBOOK_NAME_LABEL)
            if name and name == sts["metadata"]["name"]:
                ns = sts["metadata"].get("namespace", "")
                per_ns[ns] = per_ns.get(ns, 0) + 1
                if (sts.get("spec") or {}).get("replicas", 1):
                    per_ns_gpu[ns] = per_ns_gpu.get(ns, 0) + gpu_request(tmpl.get("spec") or {})
        for ns, v in sorted(per_ns.items()):
            running.add_metric([ns], v)
        for ns, v in sorted(per_ns_gpu.items()):
            gpus.add_metric([ns], v)
        yield running
        yield gpus


class CullerMetrics:
    """The two culling metrics alone: a process that runs only the culler (``--controllers
    culler``) exports these and leaves the notebook metrics to the kf process."""

    def __init__(self, registry: CollectorRegistry):
        self.registry = registry
        self.notebook_culling_count = Counter("notebook_culling", "Total times of culling notebooks",
                                              ["namespace", "name"], registry=registry)
        self.notebook_culling_timestamp = Gauge("last_notebook_culling_timestamp_seconds",
                                                "Timestamp of the last notebook culling in seconds",
                                                ["namespace", "name"], registry=registry)


class NotebookMetrics(CullerMetrics):
    def __init__(self, reader, registry: CollectorRegistry):
        super().__init__(registry)
        registry.register(_RunningCollector(reader))
        self.notebook_creation = Counter("notebook_create", "Total times of creating notebooks", ["namespace"],
                                         registry=registry)
        self.notebook_fail_creation = Counter("notebook_create_failed", "Total failure times of creating notebooks",
                                              ["namespace"], registry=registry)
        self.pod_ready_seconds = Histogram("notebook_pod_ready_seconds",
                                           "Seconds from Notebook creation (first pod) or pod creation "
                                           "(resume/restart) to the Notebook reporting Ready",
                                           ["namespace"], registry=registry,
                                           buckets=(0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10, 30, 60, 120, 300))

    def observe_ready(self, nb: dict, pod, now=None) -> float:
        """Record one start→Ready latency (called on the Notebook's transition to Ready)."""
        md = nb.get("metadata") or {}
        nb_t = parse_rfc3339(md.get("creationTimestamp"))
        pod_t = parse_rfc3339(((pod or {}).get("metadata") or {}).get("creationTimestamp"))
        start = nb_t if (pod_t is None or (nb_t is not None and pod_t - nb_t < FIRST_POD_WINDOW_S)) else pod_t
        if start is None:
            return -1.0
        dt = max(0.0, (_now() if now is None else now) - start)
        self.pod_ready_seconds.labels(md.get("namespace", "")).observe(dt)
        return dt
