"""kube-apiserver audit logging for the test apiservers (``audit.k8s.io/v1``).

The reference's envtest suite turns on kube-apiserver's audit log when
``DEBUG_WRITE_AUDITLOG=<path>`` is set, with the policy ``odh/envtest-audit-policy.yaml``
(``odh/controllers/suite_test.go:125-137``), to inspect what the controllers did.  Both
test apiservers here do the same (the Python REST server through this module, the native
C++ server with ``--audit-log-path`` / ``--audit-policy``), and the test cluster enables it
from the same environment variable; ``config/debug/audit-policy.yaml`` is the default
policy.

Supported policy subset (first matching rule wins; no match → ``None``): ``level``
(``None`` / ``Metadata`` / ``Request`` / ``RequestResponse``), ``users``, ``verbs``,
``namespaces``, ``resources`` (``group`` + ``resources``, ``resource/subresource`` form
included), ``omitStages`` (only ``ResponseComplete`` / ``ResponseStarted`` are emitted).
Events are JSON lines in kube-apiserver's ``--audit-log-format=json`` shape.
"""

from __future__ import annotations

import json
import os
import threading
import time
import uuid
from typing import List, Optional

import yaml

LEVELS = ("None", "Metadata", "Request", "RequestResponse")
DEFAULT_POLICY = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))),
                              "config", "debug", "audit-policy.yaml")


def _now() -> str:
    t = time.time()
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + ".%06dZ" % int((t % 1) * 1e6)


class AuditPolicy:
    def __init__(self, rules: List[dict], omit_stages: Optional[List[str]] = None):
        self.rules = rules
        self.omit_stages = set(omit_stages or [])

    @classmethod
    def load(cls, path: str) -> "AuditPolicy":
        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        if doc.get("kind") != "Policy":
            raise ValueError(f"{path}: not an audit.k8s.io Policy")
        return cls(doc.get("rules") or [], doc.get("omitStages"))

    def to_json(self) -> dict:
        return {"rules": self.rules, "omitStages": sorted(self.omit_stages)}

    def level(self, user: str, verb: str, namespace: str, group: str, resource: str, subresource: str = "") -> str:
        for r in self.rules:
            if r.get("users") and user not in r["users"]:
                continue
            if r.get("verbs") and verb not in r["verbs"]:
                continue
            if r.get("namespaces") is not None and namespace not in r["namespaces"]:
                continue
            if r.get("resources"):
                full = f"{resource}/{subresource}" if subresource else resource
                if not any((gr.get("group", "") == group) and (not gr.get("resources") or resource in gr["resources"]
                                                               or full in gr["resources"])
                           for gr in r["resources"]):
                    continue
            lv = r.get("level", "None")
            return lv if lv in LEVELS else "None"
        return "None"


def verb_of(method: str, name: str, watch: bool) -> str:
    if method == "GET":
        return "watch" if watch else ("get" if name else "list")
    return {"POST": "create", "PUT": "update", "PATCH": "patch",
            "DELETE": "delete" if name else "deletecollection"}.get(method, method.lower())


class AuditLogger:
    def __init__(self, path: str, policy: AuditPolicy):
        self.path = path
        self.policy = policy
        self._lock = threading.Lock()
        self.events = 0

    def log(self, *, verb: str, uri: str, user: str, user_agent: str, group: str, version: str, resource: str,
            namespace: str, name: str, subresource: str, code: int, request_obj=None, response_obj=None,
            received: Optional[str] = None, stage: str = "ResponseComplete") -> None:
        lv = self.policy.level(user, verb, namespace, group, resource, subresource)
        if lv == "None" or stage in self.policy.omit_stages:
            return
        ref = {"resource": resource, "apiGroup": group, "apiVersion": version}
        if namespace:
            ref["namespace"] = namespace
        if name:
            ref["name"] = name
        if subresource:
            ref["subresource"] = subresource
        ev = {"kind": "Event", "apiVersion": "audit.k8s.io/v1", "level": lv, "auditID": str(uuid.uuid4()),
              "stage": stage, "requestURI": uri, "verb": verb,
              "user": {"username": user, "groups": ["system:masters", "system:authenticated"]},
              "sourceIPs": ["127.0.0.1"], "userAgent": user_agent, "objectRef": ref,
              "responseStatus": {"metadata": {}, "code": code},
              "requestReceivedTimestamp": received or _now(), "stageTimestamp": _now()}
        if lv in ("Request", "RequestResponse") and request_obj is not None:
            ev["requestObject"] = request_obj
        if lv == "RequestResponse" and response_obj is not None and stage == "ResponseComplete":
            ev["responseObject"] = response_obj
        line = json.dumps(ev, separators=(",", ":")) + "\n"
        with self._lock:
            with open(self.path, "a") as f:
                f.write(line)
            self.events += 1
