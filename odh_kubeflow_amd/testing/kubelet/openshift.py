"""OpenShift platform stand-in: the ServiceAccount image-pull-secret controller.

On OpenShift, openshift-controller-manager gives every ServiceAccount a
``<sa>-dockercfg-<suffix>`` Secret (type ``kubernetes.io/dockercfg``, credentials for the
internal registry) and lists it in the SA's ``imagePullSecrets`` shortly after the SA is
created.  The reference's odh controller depends on it: its reconciliation-lock removal
waits for the notebook ServiceAccount's ``imagePullSecrets`` with a blocking 1 s + 5 s
backoff (``odh/controllers/notebook_controller.go:143-174``), so on OpenShift — its target
platform — the stall is about one backoff step (≈1 s), and only on vanilla Kubernetes,
where nothing ever adds the secret, does it reach the full 6 s.

``delay_s`` is how long after the SA appears the secret is added (default 0.2 s; the
benchmark's ``--openshift-pull-secret-ms``).  Together with the OpenShift APIs served by the
apiserver this is the "OpenShift-like" regime of the fair reference comparison (README,
"Reference baseline").
"""

from __future__ import annotations

import base64
import logging
import random
import string
import time
from typing import Dict

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_not_found
from ...runtime.controller import Request, Result, pred_funcs

log = logging.getLogger("testing.openshift")

DOCKERCFG_SECRET_TYPE = "kubernetes.io/dockercfg"


def _suffix(n: int = 5) -> str:
    return "".join(random.choice(string.ascii_lowercase + string.digits) for _ in range(n))


class PullSecretController:
    """Adds a dockercfg pull secret to every ServiceAccount that has none, ``delay_s`` after
    this controller first saw the SA."""

    def __init__(self, client, reader, delay_s: float = 0.2):
        self.client = client
        self.reader = reader
        self.delay_s = float(delay_s)
        self.added = 0
        self._seen: Dict[str, float] = {}

    @staticmethod
    def wants(sa: dict) -> bool:
        return not sa.get("imagePullSecrets") and not m.is_deleting(sa)

    async def reconcile(self, req: Request) -> Result:
        key = str(req)
        sa = self.reader.get(kinds.SERVICE_ACCOUNT, req.name, req.namespace)
        if sa is None or not self.wants(sa):
            self._seen.pop(key, None)
            return Result()
        t0 = self._seen.setdefault(key, time.monotonic())
        left = self.delay_s - (time.monotonic() - t0)
        if left > 0:
            return Result(requeue_after=left)
        name = f"{req.name}-dockercfg-{_suffix()}"
        secret = {"apiVersion": "v1", "kind": "Secret", "type": DOCKERCFG_SECRET_TYPE,
                  "metadata": {"name": name, "namespace": req.namespace, "annotations": {
                      "kubernetes.io/service-account.name": req.name,
                      "openshift.io/internal-registry-auth-token.service-account": req.name},
                      "ownerReferences": [{"apiVersion": "v1", "kind": "ServiceAccount", "name": req.name,
                                           "uid": m.uid(sa), "controller": True, "blockOwnerDeletion": True}]},
                  "data": {".dockercfg": base64.b64encode(b"{}").decode()}}
        try:
            await self.client.create(secret)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            if not is_already_exists(e):
                raise
        try:
            await self.client.patch(kinds.SERVICE_ACCOUNT, {"metadata": {"resourceVersion": m.resource_version(sa)},
                                                            "imagePullSecrets": [{"name": name}],
                                                            "secrets": [{"name": name}]},
                                    name=req.name, namespace=req.namespace)
        except ApiError as e:
            if is_not_found(e):
                return Result()
            raise  # a conflict: the SA changed, decide again
        self._seen.pop(key, None)
        self.added += 1
        return Result()

    def setup_with_manager(self, mgr, max_concurrent: int = 8):
        pred = pred_funcs(create=self.wants, update=lambda o, old: self.wants(o), delete=lambda o: False)
        return (mgr.builder().named("serviceaccount-pull-secrets").for_(kinds.SERVICE_ACCOUNT, [pred])
                .with_options(max_concurrent_reconciles=max_concurrent).complete(self))
