"""``odh-gpu-probe`` run K times, each started GAP seconds after the previous one exited:
process wall time (spawn to exit), the time from its verdict line to its exit, and the
probe's own timings, medians per variant.

    python tools/probe_chain.py K GAP [NAME=VALUE...] [probe args...]
"""

import json
import os
import re
import statistics
import subprocess
import sys
import time

EXE = "./odh_kubeflow_amd/ops/_lib/odh-gpu-probe"


def main() -> None:
    k, gap, rest = int(sys.argv[1]), float(sys.argv[2]), sys.argv[3:]
    env = dict(os.environ, **dict(a.split("=", 1) for a in rest if re.match(r"^[A-Z_]+=", a)))
    extra = [a for a in rest if not re.match(r"^[A-Z_]+=", a)]
    walls, exits, runs = [], [], []
    for _ in range(k):
        time.sleep(gap)
        env["ODH_PROBE_T0_NS"] = str(time.time_ns())  # the probe reports process start + linking as "exec"
        t0 = time.perf_counter()
        p = subprocess.Popen(["timeout", "-k", "10", "60", EXE, "--json", "-", "--quiet", *extra],
                             stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env)
        line = p.stdout.readline()  # the verdict, written just before the process leaves
        t_line = time.perf_counter()
        tail = p.stdout.read()
        rc = p.wait(timeout=90)
        t1 = time.perf_counter()
        walls.append((t1 - t0) * 1e3)
        exits.append((t1 - t_line) * 1e3)
        if rc != 0:
            print(f"probe failed rc={rc}: {(line + tail)[-300:]}")
            sys.exit(1)
        runs.append(json.loads(line))

    def med(f):
        return round(statistics.median(f(x) for x in runs), 2)

    print(f"gap={gap}s args={' '.join(rest) or '-'} runs={k} wall_p50={statistics.median(walls):.1f} "
          f"walls={[round(w) for w in walls]} verdict_to_exit_p50={statistics.median(exits):.1f} hip_init={med(lambda x: x['timings_ms']['hip_init'])} "
          f"alloc_fill={med(lambda x: x['timings_ms']['alloc_fill'])} total={med(lambda x: x['timings_ms']['total'])} "
          f"exec={med(lambda x: x['timings_ms']['exec'])}")


if __name__ == "__main__":
    main()
