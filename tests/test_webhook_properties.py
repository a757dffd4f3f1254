"""Property tests of the odh mutating webhook (``webhook/notebook_webhook.py``) over
generated Notebooks: odd containers, resources (valid and invalid quantities, any
``amd.com/gpu`` value), the auth / sidecar-resource / image-selection / stop annotations.

* the handler always answers an AdmissionReview — an allow with a patch or a deny with a
  status — and never raises (an exception would be an HTTP 500 and, with
  ``failurePolicy: Fail``, an opaque refusal);
* the JSONPatch it returns turns the request object into exactly the object it mutated;
* admitting the admitted object again changes nothing (kube-apiserver may re-invoke
  mutating webhooks, ``reinvocationPolicy: IfNeeded``): no second sidecar, volume or mount.
"""

import asyncio
import base64
import json

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from odh_kubeflow_amd.testing.apiserver.store import ObjectStore
from odh_kubeflow_amd.testing.apiserver.inprocess import InProcessClient
from odh_kubeflow_amd.utils.jsonpatch import apply_patch
from odh_kubeflow_amd.webhook.notebook_webhook import NotebookWebhook

PROXY_IMAGE = "quay.io/brancz/kube-rbac-proxy:v0.18.1"
QTY = st.sampled_from(["100m", "0.5", "1", "2Gi", "64Mi", "", "abc", "-1", "1e3", " 200m "])
GPU = st.sampled_from(["1", "2", "8", "0", "9", "x", "1.5", "-1", ""])
ANNOTATIONS = st.dictionaries(
    st.sampled_from(["notebooks.opendatahub.io/inject-auth",
                     "notebooks.opendatahub.io/auth-sidecar-cpu-request",
                     "notebooks.opendatahub.io/auth-sidecar-memory-limit",
                     "notebooks.opendatahub.io/last-image-selection",
                     "kubeflow-resource-stopped", "notebooks.kubeflow.org/last-activity"]),
    st.sampled_from(["true", "false", "yes", "", "100m", "2Gi", "nope", "img:tag", "odh-notebook-controller-lock"]),
    max_size=4)


@st.composite
def notebooks(draw):
    names = draw(st.lists(st.sampled_from(["nb", "side", "kube-rbac-proxy", "helper"]), min_size=1, max_size=3,
                          unique=True))
    containers = []
    for n in names:
        c = {"name": n, "image": draw(st.sampled_from(["rocm/pytorch:latest", "img", ""]))}
        res = {}
        for section in ("requests", "limits"):
            if draw(st.booleans()):
                r = {}
                if draw(st.booleans()):
                    r["cpu"] = draw(QTY)
                if draw(st.booleans()):
                    r["amd.com/gpu"] = draw(GPU)
                res[section] = r
        if res:
            c["resources"] = res
        if draw(st.booleans()):
            c["env"] = [{"name": draw(st.sampled_from(["A", "NB_PREFIX", "JUPYTER_IMAGE"])), "value": "v"}]
        if draw(st.booleans()):
            c["volumeMounts"] = [{"name": "data", "mountPath": "/data"}]
        containers.append(c)
    spec = {"containers": containers}
    if draw(st.booleans()):
        spec["volumes"] = [{"name": "data", "emptyDir": {}}]
    return {"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
            "metadata": {"name": names[0] if names[0] != "kube-rbac-proxy" else "nbx", "namespace": "user",
                         "annotations": draw(ANNOTATIONS)},
            "spec": {"template": {"spec": spec}}}


def _review(op, obj, old=None):
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
            "request": {"uid": "u", "operation": op, "name": obj["metadata"]["name"], "namespace": "user",
                        "object": obj, "oldObject": old}}


async def _admit(wh, op, obj, old=None):
    out = (await wh.handle(_review(op, obj, old)))["response"]
    assert isinstance(out["allowed"], bool)
    if not out["allowed"]:
        assert out["status"]["code"] in (400, 403, 422, 500) and out["status"]["message"]
        return None
    if "patch" not in out:
        return obj
    ops = json.loads(base64.b64decode(out["patch"]))
    return apply_patch(obj, ops)


def _make_webhook():
    store = ObjectStore()
    admin = InProcessClient(store)

    async def setup():
        for ns in ("opendatahub", "user"):
            await admin.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    asyncio.run(setup())
    return NotebookWebhook(InProcessClient(store), "opendatahub", PROXY_IMAGE, env={})


WH = None


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(notebooks())
def test_webhook_answers_patch_is_exact_and_reinvocation_is_stable(nb):
    global WH
    if WH is None:
        WH = _make_webhook()

    async def go():
        first = await _admit(WH, "CREATE", json.loads(json.dumps(nb)))
        if first is None:
            return
        # the patch reproduces the mutation exactly
        again = await WH.mutate("CREATE", json.loads(json.dumps(nb)), None, nb["metadata"]["name"], "user")
        assert json.loads(json.dumps(again)) == json.loads(json.dumps(first))
        # re-invocation on the admitted object changes nothing
        second = await _admit(WH, "CREATE", json.loads(json.dumps(first)))
        assert second is not None, "the admitted object is refused on re-invocation"
        assert second["spec"] == first["spec"], (first["spec"], second["spec"])
        assert second["metadata"].get("annotations") == first["metadata"].get("annotations")
        # an UPDATE that changes nothing is admitted and is stable too
        upd = await _admit(WH, "UPDATE", json.loads(json.dumps(first)), json.loads(json.dumps(first)))
        assert upd is not None and upd["spec"] == first["spec"]
    asyncio.run(go())


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.one_of(
    st.recursive(st.one_of(st.none(), st.booleans(), st.integers(), st.text(max_size=5)),
                 lambda kids: st.one_of(st.lists(kids, max_size=3), st.dictionaries(st.text(max_size=5), kids,
                                                                                    max_size=3)), max_leaves=8),
    st.fixed_dictionaries({"request": st.fixed_dictionaries(
        {"uid": st.one_of(st.text(max_size=3), st.integers()),
         "operation": st.sampled_from(["CREATE", "UPDATE", "DELETE", "CONNECT", "", 5]),
         "object": st.one_of(st.none(), st.integers(), st.dictionaries(st.sampled_from(["metadata", "spec"]),
                                                                       st.one_of(st.none(), st.integers(),
                                                                                 st.dictionaries(st.text(max_size=3),
                                                                                                 st.none(), max_size=2)),
                                                                       max_size=2))})})))
def test_webhook_never_raises_on_garbage_reviews(review):
    """Any JSON body at the webhook endpoint gets an AdmissionReview answer (allow or deny),
    never an exception (which would be a 500 and a connection error at the apiserver)."""
    global WH
    if WH is None:
        WH = _make_webhook()
    out = asyncio.run(WH.handle(review))
    assert out["kind"] == "AdmissionReview" and isinstance(out["response"]["allowed"], bool)
