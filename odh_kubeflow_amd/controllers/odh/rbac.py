"""Elyra / Data Science Pipelines RoleBinding (reference ``odh/controllers/notebook_rbac.go``).

With ``SET_PIPELINE_RBAC=true`` and Role ``ds-pipeline-user-access-dspa`` present in the
notebook namespace, RoleBinding ``elyra-pipelines-<name>`` binds it to the notebook's
ServiceAccount.  The reference's update path sends a fresh object without a
resourceVersion (``notebook_rbac.go:130-133``), which a real apiserver rejects; here
the subjects are written onto the live object instead (internal bug fixed, observable
result unchanged).
"""

from __future__ import annotations

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_not_found
from .constants import DSPA_ROLE_NAME


def new_role_binding(nb: dict, name: str, role_kind: str, role_name: str) -> dict:
    return {
        "apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
        "metadata": {"name": name, "namespace": m.namespace(nb), "labels": {"notebook-name": m.name(nb)}},
        "subjects": [{"kind": "ServiceAccount", "name": m.name(nb), "namespace": m.namespace(nb)}],
        "roleRef": {"kind": role_kind, "name": role_name, "apiGroup": "rbac.authorization.k8s.io"},
    }


async def role_exists(client, kind: str, name: str, namespace: str) -> bool:
    try:
        if kind == "ClusterRole":
            await client.get(kinds.CLUSTER_ROLE, name)
        else:
            await client.get(kinds.ROLE, name, namespace)
        return True
    except ApiError as e:
        if is_not_found(e):
            return False
        raise


async def reconcile_role_binding(client, nb: dict, rb_name: str, role_kind: str, role_name: str) -> None:
    if not await role_exists(client, role_kind, role_name, m.namespace(nb)):
        return
    desired = new_role_binding(nb, rb_name, role_kind, role_name)
    try:
        found = await client.get(kinds.ROLE_BINDING, rb_name, m.namespace(nb))
    except ApiError as e:
        if not is_not_found(e):
            raise
        m.set_controller_reference(nb, desired)
        await client.create(desired)
        return
    if found.get("subjects") != desired["subjects"]:
        found["subjects"] = desired["subjects"]
        await client.update(found)


async def reconcile_role_bindings(client, nb: dict) -> None:
    await reconcile_role_binding(client, nb, "elyra-pipelines-" + m.name(nb), "Role", DSPA_ROLE_NAME)
