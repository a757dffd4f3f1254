"""``matchConditions`` of the MutatingWebhookConfiguration: the CEL subset both test apiservers
evaluate (``utils/celmatch.py``, ``apiserver.cpp`` ``cel_*``), and the webhook left out of a
terminating Notebook's writes on every transport."""

import pytest

from odh_kubeflow_amd.models import kinds
from odh_kubeflow_amd.models.notebook import notebook
from odh_kubeflow_amd.testing.cluster import ClusterConfig, LocalCluster
from odh_kubeflow_amd.utils.celmatch import CelError, compile_condition, conditions_allow
from odh_kubeflow_amd.webhook.notebook_webhook import MATCH_CONDITIONS

LIVE = {"metadata": {"name": "a"}}
DYING = {"metadata": {"name": "a", "deletionTimestamp": "2026-10-18T00:00:00Z"}}


def test_the_shipped_condition():
    c = compile_condition(MATCH_CONDITIONS[0]["expression"])
    assert c(LIVE, None) is True and c(DYING, LIVE) is False
    assert c({"metadata": {"deletionTimestamp": None}}, None) is True  # null is not set


def test_operators_roots_and_errors():
    ev = lambda e, o=LIVE, old=None: compile_condition(e)(o, old)  # noqa: E731
    assert ev("has(object.metadata.name) && !(false || has(object.metadata.labels))")
    assert ev("has(oldObject.metadata.name)", LIVE, DYING)
    with pytest.raises(CelError):
        ev("has(oldObject.metadata.name)")  # oldObject is null on CREATE
    with pytest.raises(CelError):
        ev("has(object.spec.template)")  # no such key: spec
    # CEL's logical operators absorb an error on either side
    assert ev("has(object.spec.x) || true") is True and ev("true || has(object.spec.x)") is True
    assert ev("has(object.spec.x) && false") is False
    with pytest.raises(CelError):
        ev("has(object.spec.x) && true")


@pytest.mark.parametrize("expr", ["object.metadata.name == 'a'", "has(request.name)", "has(object)",
                                  "has(object.metadata.name", "size(object.metadata) > 0", "true true"])
def test_expressions_outside_the_subset_do_not_compile(expr):
    with pytest.raises(CelError):
        compile_condition(expr)


def test_any_false_skips_errors_follow_the_failure_policy():
    t, f = compile_condition("true"), compile_condition("false")
    err = compile_condition("has(object.spec.x)")
    assert conditions_allow([t, t], LIVE, None, True) is True
    assert conditions_allow([err, f], LIVE, None, True) is False  # a false one wins over an error
    assert conditions_allow([t, err], LIVE, None, False) is False  # Ignore: the webhook is skipped
    with pytest.raises(CelError):
        conditions_allow([t, err], LIVE, None, True)  # Fail: the request is refused


@pytest.mark.parametrize("transport", ["inprocess", "http", "native"])
def test_a_terminating_notebook_never_reaches_the_webhook(run, transport):
    """The odh finalizer's removal (and any other write to a Notebook being deleted) is not
    sent to the webhook; creates and live updates still are."""
    async def go():
        cfg = ClusterConfig(odh=True, webhook=True, transport=transport, gc=True,
                            env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("user")
            await cl.admin.create(notebook("nb", "user", annotations={"notebooks.opendatahub.io/inject-auth": "true"}))
            assert await cl.wait_for(lambda: cl.notebook_ready("nb", "user"), 20)
            assert await cl.settle(10)
            before = cl.webhook.requests
            assert before >= 2  # the create and the odh lock release
            live = await cl.admin.get(kinds.NOTEBOOK, "nb", "user")
            assert live["metadata"].get("finalizers")  # the odh cleanup finalizers: removed while terminating
            await cl.admin.delete(kinds.NOTEBOOK, "nb", "user")
            assert await cl.wait_for(lambda: cl.store.peek(kinds.NOTEBOOK, "nb", "user") is None, 10)
            assert cl.webhook.requests == before, "a write to the terminating Notebook was admitted by the webhook"
    run(go(), timeout=90)


def test_native_apiserver_refuses_on_a_condition_error_when_failing_closed(run):
    """An expression the native apiserver cannot evaluate, with failurePolicy Fail: the write
    is refused with the condition's error; with Ignore the webhook is skipped."""
    from odh_kubeflow_amd.models.errors import ApiError
    from odh_kubeflow_amd.testing.apiserver import native

    if not native.available():
        pytest.skip("native apiserver not built")

    async def go():
        cfg = ClusterConfig(odh=True, webhook=True, transport="native",
                            env={"SET_PIPELINE_RBAC": "false", "SET_PIPELINE_SECRET": "false"})
        async with LocalCluster(cfg) as cl:
            await cl.ensure_namespace("user")
            mwcs = await cl.admin.list(kinds.MUTATING_WEBHOOK_CONFIGURATION)
            assert mwcs and all(w.get("matchConditions") == MATCH_CONDITIONS for c in mwcs for w in c["webhooks"])
            cfg0 = mwcs[0]
            cfg0["webhooks"][0]["matchConditions"] = [{"name": "bad", "expression": "has(object.spec.nothing.here)"}]
            await cl.admin.update(cfg0)
            with pytest.raises(ApiError) as e:
                await cl.admin.create(notebook("nb", "user"))
            assert "matchConditions" in str(e.value) and "no such key" in str(e.value)
            cfg1 = await cl.admin.get(kinds.MUTATING_WEBHOOK_CONFIGURATION, cfg0["metadata"]["name"])
            cfg1["webhooks"][0]["failurePolicy"] = "Ignore"
            before = cl.webhook.requests
            await cl.admin.update(cfg1)
            await cl.admin.create(notebook("nb", "user"))
            assert cl.webhook.requests == before
    run(go(), timeout=60)
