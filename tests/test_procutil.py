"""Children started by the benchmark / test platform die with their launcher (utils/procutil.py)."""

import os
import signal
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie is dead for our purposes
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return False


def test_child_gets_sigterm_when_launcher_is_killed():
    # the child arms the signal itself (importing the package), so the launcher keeps
    # subprocess's vfork/posix_spawn path (no preexec_fn)
    launcher = textwrap.dedent("""
        import subprocess, sys, time
        from odh_kubeflow_amd.utils.procutil import child_env
        c = subprocess.Popen([sys.executable, "-c", "import odh_kubeflow_amd, os, time; "
                              "assert 'ODH_PDEATHSIG_PARENT' not in os.environ; time.sleep(60)"], env=child_env())
        print(c.pid, flush=True)
        time.sleep(60)
    """)
    parent = subprocess.Popen([sys.executable, "-c", launcher], cwd=ROOT, stdout=subprocess.PIPE, text=True,
                              env=dict(os.environ, PYTHONPATH=ROOT))
    child = int(parent.stdout.readline())
    try:
        assert _alive(child)
        parent.send_signal(signal.SIGKILL)  # a crash / time limit: no cleanup code runs
        parent.wait(10)
        deadline = time.monotonic() + 10
        while _alive(child) and time.monotonic() < deadline:
            time.sleep(0.05)
        assert not _alive(child), "the child outlived its killed launcher"
    finally:
        if _alive(child):
            os.kill(child, signal.SIGKILL)
