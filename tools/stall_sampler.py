"""Scheduling-stall sampler (diagnostics for the burst pause, README "A fair reference baseline").

A process of its own that sleeps 1 ms at a time and prints every iteration that took at least
``--ms`` milliseconds, with its wall-clock end (the apiserver audit log's clock), until killed
or ``--seconds`` pass.  A pause that this process sees too is the box's (the container
descheduled, a host hiccup), not a control-plane process's; the apiserver's own watchdog
(``ODH_STALL_WATCHDOG_MS``) tells a stall of the apiserver process apart.

    python tools/stall_sampler.py --ms 20 --seconds 300 > gaps.txt
"""

from __future__ import annotations

import argparse
import signal
import sys
import time


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--ms", type=float, default=20.0)
    p.add_argument("--seconds", type=float, default=600.0)
    a = p.parse_args(argv)
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(0))
    end = time.monotonic() + a.seconds
    worst, n = 0.0, 0
    print(f"stall-sampler: start {time.time():.6f} threshold {a.ms} ms", flush=True)
    try:
        while time.monotonic() < end:
            t0 = time.monotonic()
            time.sleep(0.001)
            ms = (time.monotonic() - t0) * 1000.0
            n += 1
            worst = max(worst, ms)
            if ms >= a.ms:
                print(f"stall-sampler: {ms:.1f} ms ending at {time.time():.6f}", flush=True)
    finally:
        print(f"stall-sampler: end {time.time():.6f} iterations {n} worst {worst:.1f} ms", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
