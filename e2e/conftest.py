"""Options of the e2e suite (the reference's ``odh/e2e/notebook_controller_setup_test.go:121-128``
flags, plus where to run).

    python -m pytest e2e                                   # local processes, no cluster
    python -m pytest e2e --kubeconfig ~/.kube/config \\
        --nb-namespace e2e-notebook-controller [--skip-deletion]   # a deployed overlay
"""

import os

import pytest


def pytest_addoption(parser):
    g = parser.getgroup("odh e2e")
    g.addoption("--kubeconfig", default=None,
                help="run against this cluster (else $E2E_KUBECONFIG; neither: the local dev processes)")
    g.addoption("--in-cluster", action="store_true",
                help="run against the cluster this pod runs in (its ServiceAccount; config/conformance)")
    g.addoption("--nb-namespace", default="e2e-notebook-controller",
                help="namespace the test notebooks are created in")
    g.addoption("--controller-namespace", default="opendatahub", help="namespace the controllers are deployed in")
    g.addoption("--name-prefix", default="odh-kubeflow-amd-", help="kustomize namePrefix of the deployed overlay")
    g.addoption("--skip-deletion", action="store_true", help="leave the notebooks in place at the end")
    g.addoption("--notebook-image", default="quay.io/thoth-station/s2i-minimal-notebook:v0.2.2",
                help="workbench image of the test notebooks")
    g.addoption("--updated-image",
                default="quay.io/opendatahub/workbench-images:jupyter-minimal-ubi9-python-3.11-20241119-3ceb400",
                help="image the update step rolls the first notebook to")


@pytest.fixture(scope="session")
def opts(request):
    return request.config.option


@pytest.fixture(scope="session")
def harness(opts, tmp_path_factory):
    from .harness import ClusterHarness, LocalHarness

    kc = opts.kubeconfig or os.environ.get("E2E_KUBECONFIG")
    if opts.in_cluster:
        h = ClusterHarness(opts.nb_namespace, opts.controller_namespace, None, opts.name_prefix, in_cluster=True)
    elif kc:
        h = ClusterHarness(opts.nb_namespace, opts.controller_namespace, kc, opts.name_prefix)
    else:
        h = LocalHarness(opts.nb_namespace, opts.controller_namespace, str(tmp_path_factory.mktemp("e2e")))
    yield h
    h.close()
