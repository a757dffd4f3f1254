"""The ``BeMatchingK8sResource`` counterpart (``tests/k8s_match.py``) with the controllers'
own comparators, as the reference's envtest suite uses it (``odh/controllers/
matchers_test.go``, ``notebook_controller_test.go`` route / NetworkPolicy checks)."""

import pytest

from odh_kubeflow_amd.controllers.odh import network, route
from odh_kubeflow_amd.models.notebook import notebook

from k8s_match import assert_matching_k8s_resource, diff_paths, minimized_diff


def _live(obj):
    """What an apiserver hands back: server-set metadata the comparators ignore."""
    o = {**obj, "metadata": {**obj["metadata"], "uid": "u-1", "resourceVersion": "42", "generation": 1,
                             "managedFields": [{"manager": "odh"}], "creationTimestamp": "2026-01-01T00:00:00Z"}}
    o["status"] = {"parents": []}
    return o


def test_server_metadata_does_not_fail_the_match():
    nb = notebook("nb", "user")
    want = route.new_notebook_httproute(nb, "opendatahub", env={})
    assert_matching_k8s_resource(_live(want), want, route._same_route)
    np = network.new_notebook_network_policy(nb, "opendatahub")
    assert_matching_k8s_resource(_live(np), np, network._same)


def test_mismatch_reports_full_and_minimized_diff():
    nb = notebook("nb", "user")
    want = route.new_notebook_httproute(nb, "opendatahub", env={})
    got = _live(want)
    got["spec"] = {**got["spec"], "rules": [{**got["spec"]["rules"][0], "backendRefs": [
        {**got["spec"]["rules"][0]["backendRefs"][0], "port": 8888}]}]}
    with pytest.raises(AssertionError) as e:
        assert_matching_k8s_resource(got, want, route._same_route)
    msg = str(e.value)
    full, minimized = msg.split("minimized diff")
    assert "metadata.uid" in full and "metadata.resourceVersion" in full  # everything that differs...
    assert "spec.rules.0.backendRefs.0.port: -8888 +80" in minimized     # ...and what the comparator saw
    assert "uid" not in minimized and "resourceVersion" not in minimized and "status" not in minimized


def test_diff_paths_and_minimization_units():
    a = {"metadata": {"labels": {"x": "1"}, "uid": "a"}, "spec": {"p": [1, 2]}}
    b = {"metadata": {"labels": {"x": "2"}}, "spec": {"p": [1, 3]}}
    paths = [p for p, _, _ in diff_paths(a, b)]
    assert paths == [("metadata", "labels", "x"), ("metadata", "uid"), ("spec", "p", 1)]
    same_spec = lambda e, x: e.get("spec") == x.get("spec")  # noqa: E731
    assert [p for p, _, _ in minimized_diff(a, b, same_spec)] == [("spec", "p", 1)]
