"""Native (C++) runtime core: JSON-tree operations on the control plane's hot path.

``_objcore`` (``objcore.cpp``, CPython C API, built in-tree by
``odh_kubeflow_amd.ops.build``) provides ``deepcopy`` and ``semantic_equal`` for
Kubernetes objects held as plain dict/list trees.  Every apiserver read/write, every
cache read and every desired-vs-found diff goes through these, so they are the
equivalent of the Go runtime's generated ``DeepCopy`` and ``equality.Semantic``.
"""
