"""The reference envtest suite's debug aids (``odh/controllers/suite_test.go:125-155``):
``DEBUG_WRITE_AUDITLOG`` (apiserver audit log, ``audit.k8s.io/v1`` JSON lines, policy
``config/debug/audit-policy.yaml``) and ``DEBUG_WRITE_KUBECONFIG`` (a kubeconfig for the
test apiserver), over both network apiservers."""

import json

import pytest
import yaml

from odh_kubeflow_amd.testing.apiserver.audit import AuditPolicy
from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.runtime.rest import RestClient, RestConfig


@pytest.mark.parametrize("transport", ["http", "native"])
def test_audit_log_and_kubeconfig(run, tmp_path, transport):
    log, kcfg = tmp_path / "audit.log", tmp_path / "kubeconfig"

    async def go():
        cfg = ClusterConfig(transport=transport, audit_log_path=str(log), kubeconfig_path=str(kcfg))
        async with LocalCluster(cfg) as cl:
            # the kubeconfig reaches the test apiserver: the notebooks are created through it
            k = yaml.safe_load(kcfg.read_text())
            assert k["users"][0]["name"] == "MasterOfTheSystems"
            rc = RestClient(RestConfig.load(None, str(kcfg)))
            try:
                for ns in ("developer", "other"):
                    await cl.ensure_namespace(ns)
                    await rc.create(notebook("nb", ns))
                assert await cl.wait_for(lambda: cl.notebook_ready("nb", "developer") and
                                         cl.notebook_ready("nb", "other"), 15)
                assert (await rc.get(kinds.NOTEBOOK, "nb", "developer"))["metadata"]["name"] == "nb"
            finally:
                await rc.close()
    run(go())
    events = [json.loads(line) for line in log.read_text().splitlines()]
    assert events and all(e["apiVersion"] == "audit.k8s.io/v1" and e["kind"] == "Event" for e in events)
    assert {e["objectRef"]["namespace"] for e in events} == {"developer"}  # the policy's namespace only
    create = [e for e in events if e["verb"] == "create" and e["objectRef"]["resource"] == "notebooks"]
    assert len(create) == 1 and create[0]["level"] == "RequestResponse"
    c = create[0]
    assert c["objectRef"]["apiGroup"] == "kubeflow.org" and c["responseStatus"]["code"] == 201
    assert c["requestObject"]["metadata"]["name"] == "nb" and c["responseObject"]["metadata"]["uid"]
    assert c["objectRef"]["name"] == "nb"  # kube-apiserver names the created object
    # client-go's default user agent: the program, so the log tells the processes apart
    assert c["userAgent"].split("/")[0] not in ("", "odh-kubeflow-amd") and "odh-kubeflow-amd" in c["userAgent"]
    sts = [e for e in events if e["verb"] == "create" and e["objectRef"]["resource"] == "statefulsets"]
    assert sts[0]["objectRef"]["name"] == "nb"
    verbs = {(e["verb"], e["objectRef"]["resource"]) for e in events}
    assert ("create", "statefulsets") in verbs  # what the controllers did in that namespace
    assert any(e["verb"] == "patch" and e["objectRef"].get("subresource") == "status" for e in events)
    # watches are logged at ResponseStarted; the controllers' caches watch cluster-wide, which
    # a namespaces: [developer] rule does not select
    assert all(e["stage"] == "ResponseComplete" for e in events if e["verb"] != "watch")


def test_audit_policy_rules():
    p = AuditPolicy([{"level": "None", "users": ["system:kube-proxy"]},
                     {"level": "Metadata", "resources": [{"group": "", "resources": ["secrets"]}]},
                     {"level": "Request", "verbs": ["create", "update"], "namespaces": ["a"]},
                     {"level": "RequestResponse", "resources": [{"group": "kubeflow.org",
                                                                 "resources": ["notebooks/status"]}]}])
    assert p.level("system:kube-proxy", "get", "a", "", "secrets") == "None"
    assert p.level("u", "get", "a", "", "secrets") == "Metadata"
    assert p.level("u", "create", "a", "", "configmaps") == "Request"
    assert p.level("u", "create", "b", "", "configmaps") == "None"
    assert p.level("u", "patch", "b", "kubeflow.org", "notebooks", "status") == "RequestResponse"
    assert p.level("u", "patch", "b", "kubeflow.org", "notebooks") == "None"
