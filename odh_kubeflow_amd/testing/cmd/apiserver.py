"""Development apiserver (the envtest substitute as a process) + kube-controller-manager stand-ins.

    python -m odh_kubeflow_amd.testing.cmd.apiserver --port 6443 --kubeconfig-out /tmp/kc.yaml

Serves the in-memory store over the Kubernetes REST/watch API.  With ``--controllers``
it also runs the StatefulSet controller, the scheduler / ``amd.com/gpu`` allocator and
ownerReference GC that a real cluster provides (envtest has none of these;
``kf/controllers/notebook_controller_bdd_test.go:73-76``).  ``--tls`` serves HTTPS with a
generated CA; ``--token`` requires a bearer token.
"""

from __future__ import annotations

import argparse
import asyncio
import base64
import logging
import sys

import yaml

log = logging.getLogger("apiserver")


def parse(argv=None):
    p = argparse.ArgumentParser(prog="odh-dev-apiserver")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=6443)
    p.add_argument("--token", default=None)
    p.add_argument("--tls", action="store_true")
    p.add_argument("--kubeconfig-out", default=None)
    p.add_argument("--controllers", action="store_true", help="run STS controller + scheduler + GC")
    p.add_argument("--no-openshift-apis", action="store_true")
    p.add_argument("--debug-log", action="store_true")
    return p.parse_args(argv)


def write_kubeconfig(path: str, server: str, token=None, ca_pem=None) -> None:
    cluster = {"server": server}
    if ca_pem:
        cluster["certificate-authority-data"] = base64.b64encode(ca_pem.encode()).decode()
    user = {"token": token} if token else {}
    kc = {"apiVersion": "v1", "kind": "Config", "current-context": "odh",
          "clusters": [{"name": "odh", "cluster": cluster}], "users": [{"name": "odh", "user": user}],
          "contexts": [{"name": "odh", "context": {"cluster": "odh", "user": "odh"}}]}
    with open(path, "w") as f:
        yaml.safe_dump(kc, f)


async def amain(argv=None) -> int:
    from ..apiserver.http import ApiServer
    from ..apiserver.store import ObjectStore
    from ..kubelet.node import SchedulerController
    from ..kubelet.statefulset import StatefulSetController
    from ...models import kinds
    from ...runtime.manager import Manager
    from ...cmd.common import setup_logging, signal_event

    args = parse(argv)
    setup_logging(debug=args.debug_log)
    store = ObjectStore(gc=args.controllers)
    if args.no_openshift_apis:
        for crd in (kinds.IMAGE_STREAM, kinds.PROXY, kinds.ROUTE, kinds.OAUTH_CLIENT):
            store.uninstall_crd(crd)
    ctx = None
    ca = None
    if args.tls:
        import ssl

        from ...webhook.certs import generate

        certs = generate((args.host, "localhost"))
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(certs.cert_file, certs.key_file)
        ca = certs.ca_pem
    srv = await ApiServer(store, token=args.token).start(args.host, args.port, ctx)
    log.info("serving on %s", srv.url)
    if args.kubeconfig_out:
        write_kubeconfig(args.kubeconfig_out, srv.url, args.token, ca)
    mgr = None
    if args.controllers:
        from ..apiserver.inprocess import in_process_manager

        mgr = in_process_manager(store, name="kube-controller-manager")
        StatefulSetController(mgr.client, mgr.reader, mgr.get_event_recorder_for("statefulset-controller")) \
            .setup_with_manager(mgr)
        SchedulerController(mgr.client, mgr.reader, mgr.get_event_recorder_for("default-scheduler")) \
            .setup_with_manager(mgr)
        await mgr.start()
    await signal_event().wait()
    if mgr is not None:
        await mgr.stop()
    await srv.stop()
    return 0


def main(argv=None) -> int:
    return asyncio.run(amain(argv))


if __name__ == "__main__":
    sys.exit(main())
