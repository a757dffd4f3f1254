"""Medians of ``odh-gpu-probe`` runs grouped by ``--streams`` (``tools/gpu_pass.sh probestreams``)."""

import json
import statistics
import sys
from collections import defaultdict


def main(path: str) -> None:
    by = defaultdict(list)
    for line in open(path):
        if line.startswith("{"):
            r = json.loads(line)
            by[r["setup_ms"]["n_streams"]].append(r)
    for ns in sorted(by, reverse=True):
        rs = by[ns]

        def med(f):
            return round(statistics.median(f(r) for r in rs), 3)

        print(f"streams={ns} runs={len(rs)} ok={all(r['ok'] for r in rs)} "
              f"setup_streams={med(lambda r: r['setup_ms']['streams'])} first_op={med(lambda r: r['setup_ms'].get('first_op', 0))} "
              f"alloc={med(lambda r: r['timings_ms']['alloc'])} code_load={med(lambda r: r['timings_ms']['code_load'])} "
              f"fill={med(lambda r: r['timings_ms']['fill'])} probe={med(lambda r: r['timings_ms']['probe'])} "
              f"hip_init={med(lambda r: r['timings_ms']['hip_init'])} total={med(lambda r: r['timings_ms']['total'])} "
              f"gemm_tflops={med(lambda r: r['results'][0]['gemm_tflops'])} "
              f"hbm_gbps={med(lambda r: r['results'][0]['hbm_gbps'])}")


if __name__ == "__main__":
    main(sys.argv[1])
