"""Child-process hygiene for the processes the benchmark and the test platform launch.

The benchmark's ranks and the test platform start helper processes (apiserver, scheduler,
kubelet, control planes, workbenches) whose stdout they read; a rank killed by a time limit
or a crash must not leave them running — on a shared GPU box they would outlive the job,
and they keep the launching shell's pipes open.  Linux's ``PR_SET_PDEATHSIG`` gives a child
SIGTERM when its parent dies.

It is armed by the CHILD, not through ``preexec_fn``: a ``preexec_fn`` forces CPython's
``subprocess`` from vfork/posix_spawn onto a full ``fork()``, which for a parent holding a
HIP context and torch's mappings blocks the parent's event loop for ~17 ms per child
(measured: 8 workbench spawns added 137 ms to the control-plane time of the real-pods
benchmark).  The parent puts its pid in ``ODH_PDEATHSIG_PARENT`` (:func:`child_env`); the
child calls :func:`arm_from_env` first thing (``odh_kubeflow_amd/__init__.py`` does it for
every Python child; the native apiserver does the same in ``main``).
"""

from __future__ import annotations

import ctypes
import os
import signal
from typing import Dict, Optional

ENV = "ODH_PDEATHSIG_PARENT"
_PR_SET_PDEATHSIG = 1


def child_env(env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """``env`` (default: this process's) asking the child to die with this process."""
    out = dict(os.environ if env is None else env)
    out[ENV] = str(os.getpid())
    return out


def proc_cpu_ns(pid: Optional[int], proc: str = "/proc") -> Optional[int]:
    """CPU time of process ``pid`` in nanoseconds: the scheduler's ``sum_exec_runtime`` of each
    of its threads (first field of ``/proc/<pid>/task/<tid>/schedstat``), summed.  Exact to the
    nanosecond, where ``utime + stime`` of ``/proc/<pid>/stat`` counts 10 ms clock ticks — over a
    20-step window that quantised every per-step figure to 0.5 ms.  A thread that has exited
    takes its time with it, so a caller measuring a window needs threads that outlive it
    (the control plane's and the platform's do; the native apiserver reports its own
    ``CLOCK_PROCESS_CPUTIME_ID`` instead).  Falls back to the tick count when schedstat is not
    available (``CONFIG_SCHEDSTATS`` off); ``None`` if the process is gone."""
    if pid is None:
        return None
    try:
        total = 0
        for tid in os.listdir(f"{proc}/{pid}/task"):
            try:
                with open(f"{proc}/{pid}/task/{tid}/schedstat") as f:
                    total += int(f.read().split()[0])
            except FileNotFoundError:  # the thread exited between listdir and open
                continue
        return total
    except (OSError, IndexError, ValueError):
        pass
    try:
        with open(f"{proc}/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return (int(fields[11]) + int(fields[12])) * 1_000_000_000 // os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return None


def arm_from_env() -> None:
    """In a child started with :func:`child_env`: SIGTERM when the parent dies.  The
    variable is consumed, so this process's own children are not tied to its parent."""
    parent = os.environ.pop(ENV, None)
    if not parent:
        return
    try:
        ctypes.CDLL(None, use_errno=True).prctl(_PR_SET_PDEATHSIG, int(signal.SIGTERM), 0, 0, 0)
    except (OSError, AttributeError):
        return
    if str(os.getppid()) != parent:  # the parent died before the signal was armed
        os.kill(os.getpid(), signal.SIGTERM)


# ------------------------------------------------------------------ listen ports for children

_port_seq = [0]


def _ephemeral_range() -> tuple:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo, hi = (int(x) for x in f.read().split())
            return lo, hi
    except (OSError, ValueError):
        return 32768, 60999


def listen_port(host: str = "127.0.0.1") -> int:
    """A free TCP port for a child process to listen on once it has started.

    Chosen below the kernel's ephemeral range: a port picked with ``bind(0)`` is an ephemeral
    one, and in the second or two before the child binds it, any process's outgoing
    connection can take it as its local port (a 4-rank benchmark run lost a control-plane
    process to that, ``profiles/r5_f7``).  Each process walks the range from its own
    pid-derived offset, so concurrent ranks pick from different places."""
    import socket

    lo, top = 20000, _ephemeral_range()[0]
    if top - lo < 1000:
        lo, top = 10000, max(top, 11000)
    span = top - lo
    start = (os.getpid() * 7919) % span
    for _ in range(span):
        port = lo + (start + _port_seq[0]) % span
        _port_seq[0] += 1
        with socket.socket() as s:
            try:
                s.bind((host, port))
            except OSError:
                continue
            return port
    with socket.socket() as s:  # the whole range in use: fall back to the kernel's choice
        s.bind((host, 0))
        return s.getsockname()[1]
