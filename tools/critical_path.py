"""Create → Ready critical path of each Notebook, from an apiserver audit log.

    DEBUG_WRITE_AUDITLOG=/tmp/audit.jsonl python bench.py ...
    python tools/critical_path.py /tmp/audit.jsonl [--namespace-prefix bench-] > path.json

Both test apiservers write kube-apiserver audit events with microsecond
``requestReceivedTimestamp`` / ``stageTimestamp`` and the client's user agent (the
program: ``control_plane``, ``scheduler``, ``bench`` …).  For every Notebook the requests
on its Ready path are picked out in order:

    notebook create (admission webhook inside) → StatefulSet create (kf reconciler)
    → lock release (odh reconciler; optional) → StatefulSet scale-up (kf reconciler;
    optional) → Pod create (StatefulSet controller) → Pod bind (scheduler) → Pod status Ready (node
    agent, start-up probe inside) → StatefulSet status → Notebook status (kf reconciler)

and each hop is split into ``gap`` (previous request answered → this one received: watch
delivery, queueing, the controller's own work) and ``serve`` (this request inside the
apiserver, admission included).  Medians and p95 over the Notebooks are printed as JSON,
with the user agent that issued each step, and every successful write per notebook by
client, verb and resource (``writes_per_notebook``).  This is where the create→Ready milliseconds
of ``bench.py`` go, hop by hop (the reference's envtest audit-log aid,
``odh/controllers/suite_test.go:125-137``, put to a latency use).
"""

from __future__ import annotations

import argparse
import json
import sys
from collections import defaultdict
from datetime import datetime, timezone

OPTIONAL = {"lock_release", "sts_scale"}  # odh lock path (absent for kf-only / unlocked notebooks)
STEPS = (
    ("notebook_create", "create", "notebooks", "", "{nb}"),
    ("sts_create", "create", "statefulsets", "", "{nb}"),
    # odh: the webhook's image-pull lock (kubeflow-resource-stopped) holds replicas at 0
    # until the reconciler sees the workbench ServiceAccount and removes it
    ("lock_release", "patch", "notebooks", "", "{nb}"),
    ("sts_scale", "update", "statefulsets", "", "{nb}"),
    ("pod_create", "create", "pods", "", "{nb}-0"),
    ("pod_bind", ("patch", "update", "create"), "pods", ("", "binding"), "{nb}-0"),
    ("pod_ready", "patch", "pods", "status", "{nb}-0"),
    ("sts_status", ("patch", "update"), "statefulsets", "status", "{nb}"),
    ("notebook_status", ("patch", "update"), "notebooks", "status", "{nb}"),
)


def _ts(s: str) -> float:
    return datetime.strptime(s, "%Y-%m-%dT%H:%M:%S.%fZ").replace(tzinfo=timezone.utc).timestamp()


def _match(want, got) -> bool:
    return got in want if isinstance(want, tuple) else got == want


def pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))]


def analyse(lines, ns_prefix: str = "", name_prefix: str = "") -> dict:
    by_obj = defaultdict(list)  # (ns, resource, name) -> events in order
    for line in lines:
        e = json.loads(line)
        if e.get("stage") != "ResponseComplete" or e.get("verb") in ("watch", "get", "list"):
            continue
        ref = e.get("objectRef") or {}
        ns = ref.get("namespace", "")
        if ns_prefix and not ns.startswith(ns_prefix):
            continue
        code = (e.get("responseStatus") or {}).get("code", 0)
        if code >= 300:
            continue
        by_obj[(ns, ref.get("resource"), ref.get("name", ""))].append(
            (_ts(e["requestReceivedTimestamp"]), _ts(e["stageTimestamp"]), e["verb"], ref.get("subresource", ""),
             e.get("userAgent", "").split("/")[0]))
    notebooks = [(ns, name) for (ns, res, name) in by_obj if res == "notebooks" and name and
                 name.startswith(name_prefix) and any(v == "create" for _, _, v, _, _ in by_obj[(ns, res, name)])]
    # every successful write, attributed to its client and target: who spends the writes
    writes = defaultdict(int)
    for (ns, res, name), evs in by_obj.items():
        for _, _, v, sub, ua in evs:
            writes[(ua or "?", v, res + ("/" + sub if sub else ""))] += 1
    hops = defaultdict(lambda: {"gap": [], "serve": [], "agents": defaultdict(int)})
    totals = []
    for evs in by_obj.values():
        evs.sort(key=lambda e: e[0])  # by arrival: the log is in completion order

    def find(ns, nb, i, after):
        """The first request of hop ``i`` that arrived after ``after`` (the previous hop's
        arrival).  Not after its completion: the apiserver commits — and the watchers see
        the write — before it stamps the response, so under load the next hop can arrive
        before the previous one's completion stamp."""
        _, verb, res, sub, name = STEPS[i]
        evs = by_obj.get((ns, res, name.format(nb=nb)), [])
        return next(((r, d, ua) for r, d, v, s, ua in evs
                     if _match(verb, v) and _match(sub, s) and (after is None or r > after)), None)

    for ns, nb in notebooks:
        prev_done = prev_at = None
        t0 = None
        ok = True
        for i, (step, *_) in enumerate(STEPS):
            hit = find(ns, nb, i, prev_at)
            if hit is not None and step in OPTIONAL:
                # an optional hop is on the path only if the next required hop follows it: a
                # notebook whose lock was gone before kf created its StatefulSet has no
                # lock-release / scale-up hop, and a later patch (finalizers) must not pose as one
                nxt = next(j for j in range(i + 1, len(STEPS)) if STEPS[j][0] not in OPTIONAL)
                if find(ns, nb, nxt, hit[0]) is None and find(ns, nb, nxt, prev_at) is not None:
                    hit = None
            if hit is None:
                if step in OPTIONAL:
                    continue
                ok = False
                break
            r, d, ua = hit
            if t0 is None:
                t0 = r
            h = hops[step]
            h["serve"].append((d - r) * 1e3)
            if prev_done is not None:
                h["gap"].append(max(0.0, r - prev_done) * 1e3)
            h["agents"][ua] += 1
            prev_done, prev_at = d, r
        if ok:
            totals.append((prev_done - t0) * 1e3)
    out = {"notebooks": len(totals), "create_to_notebook_status_ms": {"p50": pct(totals, .5), "p95": pct(totals, .95)},
           "hops": {}}
    for step, *_ in STEPS:
        h = hops.get(step)
        if not h:
            continue
        out["hops"][step] = {
            "gap_ms_p50": round(pct(h["gap"], .5), 3) if h["gap"] else None,
            "gap_ms_p95": round(pct(h["gap"], .95), 3) if h["gap"] else None,
            "serve_ms_p50": round(pct(h["serve"], .5), 3), "serve_ms_p95": round(pct(h["serve"], .95), 3),
            "by": dict(h["agents"]),
        }
    out["teardown"] = _teardown(by_obj, notebooks)
    n_created = max(1, len(notebooks))
    out["writes_per_notebook"] = {
        "total": round(sum(writes.values()) / n_created, 2),
        "by_client": {f"{ua} {v} {res}": round(c / n_created, 2)
                      for (ua, v, res), c in sorted(writes.items(), key=lambda kv: (kv[0][0], -kv[1], kv[0]))}}
    for k in ("p50", "p95"):
        v = out["create_to_notebook_status_ms"][k]
        out["create_to_notebook_status_ms"][k] = round(v, 3) if v is not None else None
    return out


def _teardown(by_obj, notebooks) -> dict:
    """Delete → finalizer removed, per Notebook: the delete's service time, then the gap to the
    write that removes the odh finalizer (the reconciler's wake-up and its deletes of the
    exposure children — auth-delegator CRB, central HTTPRoute, ReferenceGrant — are in it) and
    that write's service time (the admission webhook inside).  The garbage collector's cascade
    after it (StatefulSet, then Pod) runs inside the apiserver and is not in the audit log."""
    dserve, gap, fserve, total = [], [], [], []
    for ns, nb in notebooks:
        evs = by_obj.get((ns, "notebooks", nb), [])
        dels = [e for e in evs if e[2] == "delete"]
        if not dels:
            continue
        r0, d0 = dels[-1][0], dels[-1][1]
        fin = next((e for e in evs if e[0] > r0 and e[2] in ("patch", "update") and not e[3]), None)
        if fin is None:
            continue
        dserve.append((d0 - r0) * 1e3)
        gap.append(max(0.0, fin[0] - d0) * 1e3)
        fserve.append((fin[1] - fin[0]) * 1e3)
        total.append((fin[1] - r0) * 1e3)

    def q(xs):
        return {"p50": round(pct(xs, .5), 3), "p95": round(pct(xs, .95), 3)} if xs else None
    return {"notebooks": len(total), "delete_to_finalizer_removed_ms": q(total), "delete_serve_ms": q(dserve),
            "gap_to_finalizer_write_ms": q(gap), "finalizer_write_serve_ms": q(fserve)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("audit_log")
    ap.add_argument("--namespace-prefix", default="")
    ap.add_argument("--name-prefix", default="", help="only Notebooks whose name starts with this (nb-s: the timed "
                                                      "window; nb-res-: the notebooks created on top of --resident)")
    a = ap.parse_args(argv)
    with open(a.audit_log) as f:
        print(json.dumps(analyse(f, a.namespace_prefix, a.name_prefix), indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
