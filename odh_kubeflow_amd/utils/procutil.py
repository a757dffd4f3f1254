"""Child-process hygiene for the processes the benchmark and the test platform launch."""

from __future__ import annotations

import ctypes
import signal

_PR_SET_PDEATHSIG = 1


def die_with_parent() -> None:
    """``preexec_fn``: the child gets SIGTERM when the process that started it dies.

    The benchmark's ranks and the test platform start helper processes (apiserver,
    scheduler, kubelet, control planes) whose stdout they read; a rank killed by a time
    limit or a crash must not leave them running — on a shared GPU box they would outlive
    the job, and they keep the launching shell's pipes open.  Linux-only (prctl); a no-op
    elsewhere."""
    try:
        ctypes.CDLL(None, use_errno=True).prctl(_PR_SET_PDEATHSIG, int(signal.SIGTERM), 0, 0, 0)
    except (OSError, AttributeError):
        pass
