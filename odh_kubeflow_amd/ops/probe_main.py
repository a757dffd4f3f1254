"""MI355X start-up probe runner without torch: ``python -m odh_kubeflow_amd.ops.probe_main``.

The notebook pod's init container (``amd.com/gpu-probe: "true"``, injected by
:func:`odh_kubeflow_amd.controllers.notebook.gpu_probe_init_container`) runs the native
``odh-gpu-probe`` program; this module is the same probe for images that carry the Python
package instead of the binary.  Both call ``odh_probe_cli`` in ``libodh_gpu_probe.so``
(``csrc/probe_cli.cpp``): hipMalloc'd operands, the MFMA bf16 GEMM verified in registers, the
HBM3E pattern sweep, and with 2+ visible GPUs the xGMI ring — one JSON result on stdout and in
``/dev/termination-log``, exit status 0 healthy / 1 check failed / 2 no GPU or HIP error /
3 watchdog / 64 usage.

Nothing here imports torch: loading the library costs only the HIP runtime it links.
"""

from __future__ import annotations

import ctypes
import json
import os
import sys
from typing import List, Optional, Sequence

from .build import PROBE_EXE, lib_path

PROBE_LIB = "libodh_gpu_probe.so"
# exit statuses of odh_probe_cli
OK, CHECK_FAILED, NO_GPU, TIMEOUT, USAGE = 0, 1, 2, 3, 64


def executable() -> str:
    """Path of the native ``odh-gpu-probe`` program built in-tree (``ops/_lib``)."""
    return lib_path(PROBE_EXE)


def command(args: Sequence[str] = ()) -> List[str]:
    """argv that runs the probe: the native program when built, else this module."""
    exe = executable()
    if os.path.exists(exe):
        return [exe, *args]
    return [sys.executable, "-m", "odh_kubeflow_amd.ops.probe_main", *args]


def parse_result(text: str) -> Optional[dict]:
    """The probe's JSON result from its output (last line that parses as a JSON object)."""
    for line in reversed((text or "").strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def run(argv: Sequence[str]) -> int:
    path = lib_path(PROBE_LIB)
    if not os.path.exists(path):
        sys.stderr.write(f"{path} not built; run `python -m odh_kubeflow_amd.ops.build`\n")
        return NO_GPU
    lib = ctypes.CDLL(path)
    lib.odh_probe_cli.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
    lib.odh_probe_cli.restype = ctypes.c_int
    args = ["odh-gpu-probe", *argv]
    arr = (ctypes.c_char_p * (len(args) + 1))(*[a.encode() for a in args], None)
    sys.stdout.flush()
    return int(lib.odh_probe_cli(len(args), arr))


def main(argv: Optional[Sequence[str]] = None) -> int:
    return run(list(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    sys.exit(main())
