"""NetworkPolicies per notebook (reference ``odh/controllers/notebook_network.go``).

* ``<nb>-ctrl-np``: TCP 8888 only from the controller's namespace (:132-174);
* ``<nb>-kube-rbac-proxy-np``: TCP 8443 from anywhere (:177-211).

Both are owned by the Notebook and drift-corrected (labels + spec) under
``RetryOnConflict`` (:68-122).
"""

from __future__ import annotations

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_already_exists, is_not_found
from ...runtime.retry import retry_on_conflict
from .constants import CTRL_NP_SUFFIX, KUBE_RBAC_PROXY_NP_SUFFIX, KUBE_RBAC_PROXY_PORT, NOTEBOOK_PORT


def new_notebook_network_policy(nb: dict, controller_namespace: str) -> dict:
    return {
        "apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
        "metadata": {"name": m.name(nb) + CTRL_NP_SUFFIX, "namespace": m.namespace(nb)},
        "spec": {
            "podSelector": {"matchLabels": {"notebook-name": m.name(nb)}},
            "ingress": [{
                "ports": [{"protocol": "TCP", "port": NOTEBOOK_PORT}],
                "from": [{"namespaceSelector": {"matchLabels": {"kubernetes.io/metadata.name": controller_namespace}}}],
            }],
            "policyTypes": ["Ingress"],
        },
    }


def new_kube_rbac_proxy_network_policy(nb: dict) -> dict:
    return {
        "apiVersion": "networking.k8s.io/v1", "kind": "NetworkPolicy",
        "metadata": {"name": m.name(nb) + KUBE_RBAC_PROXY_NP_SUFFIX, "namespace": m.namespace(nb)},
        "spec": {
            "podSelector": {"matchLabels": {"notebook-name": m.name(nb)}},
            "ingress": [{"ports": [{"protocol": "TCP", "port": KUBE_RBAC_PROXY_PORT}]}],
            "policyTypes": ["Ingress"],
        },
    }


def _same(desired: dict, found: dict) -> bool:
    return (m.labels(desired) or {}) == (m.labels(found) or {}) and desired.get("spec") == found.get("spec")


async def reconcile_network_policy(client, nb: dict, desired: dict) -> None:
    ns, name = m.namespace(nb), m.name(desired)
    try:
        found = await client.get(kinds.NETWORK_POLICY, name, ns)
    except ApiError as e:
        if not is_not_found(e):
            raise
        m.set_controller_reference(nb, desired)
        try:
            await client.create(desired)
        except ApiError as e2:
            if not is_already_exists(e2):
                raise
        return
    if _same(desired, found):
        return

    async def update():
        cur = await client.get(kinds.NETWORK_POLICY, name, ns)
        cur["spec"] = desired["spec"]
        labels = m.labels(desired)
        if labels:
            cur["metadata"]["labels"] = dict(labels)
        else:
            cur["metadata"].pop("labels", None)
        await client.update(cur)

    await retry_on_conflict(update)


async def reconcile_all_network_policies(client, nb: dict, controller_namespace: str) -> None:
    await reconcile_network_policy(client, nb, new_notebook_network_policy(nb, controller_namespace))
    await reconcile_network_policy(client, nb, new_kube_rbac_proxy_network_policy(nb))
