"""Test platform (never deployed, not part of the production wheel).

The stand-ins a notebook control plane needs around it when there is no cluster — what
envtest, kind and a GPU node provide to the reference's test suites:

* ``apiserver/`` — in-process object store, Python REST/watch server, audit log, and the
  wrapper of the native C++ apiserver (``native/apiserver``, built into ``native/bin``);
* ``kubelet/`` — StatefulSet controller, ``amd.com/gpu`` scheduler / device allocator,
  kubelet stand-in (init containers, container runtimes), Gateway resolver;
* ``notebook_server/`` — Jupyter REST stand-in and the PyTorch-ROCm workbench process;
* ``cluster.py`` — all of it wired into one in-process cluster for tests;
* ``cmd/`` — the dev apiserver, scheduler and fake kubelet as processes.

No production entry point (``cmd/control_plane``, ``kf_manager``, ``odh_manager``,
``node_agent``, ``webhook_certs``) imports this package; ``tests/test_packaging.py`` enforces it.
"""
