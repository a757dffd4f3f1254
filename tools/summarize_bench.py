#!/usr/bin/env python3
"""One line per bench log: the headline, CPU per step and the resident block.

    python tools/summarize_bench.py gpurun_out/r5_p2/*.log
"""

from __future__ import annotations

import json
import sys


def last_json(path: str):
    for line in reversed(open(path, errors="replace").read().splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                return None
    return None


def summary(path: str) -> str:
    d = last_json(path)
    if d is None:
        return f"{path}: no JSON"
    cpu = {k.replace("control_plane_", "cp_"): v for k, v in (d.get("cpu_ms_per_step") or {}).items()}
    out = [f"{path.rsplit('/', 1)[-1]}: N={d.get('n_gpus')} nb/s={d.get('notebooks_ready_per_s')} "
           f"rec/s={d.get('value')} p50={d.get('p50_ready_ms')} p95={d.get('p95_ready_ms')} "
           f"rec/nb={d.get('reconciles_per_notebook')} cpu/step={json.dumps(cpu)}"]
    prof = d.get("apiserver_profile_per_step") or {}
    w = (d.get("writes_per_notebook") or {}).get("total")
    if prof.get("process_cpu_ms") is not None and w:
        out.append(f"  apiserver cpu/write={prof['process_cpu_ms'] / (w * (d.get('n_gpus') or 1)):.4f} ms "
                   f"(cpu/step {prof['process_cpu_ms']} ms, {w} writes/notebook)"
                   + (f" namespaces/rank={(d.get('config') or {}).get('namespaces_per_rank')}"))
    r = d.get("resident")
    if r:
        a = r.get("at_rest") or {}
        top = r.get("new_notebooks_on_top") or {}
        out.append(f"  resident R={r.get('notebooks')} ok={r.get('all_ok')} fill={r.get('fill_s')}s "
                   f"on-top p50/p99={top.get('ready_ms', {}).get('p50')}/{top.get('ready_ms', {}).get('p99')} "
                   f"(x{top.get('p50_vs_empty')} of empty {top.get('empty_cluster_p50_ms')}) "
                   f"checks/s={a.get('culler_checks_per_s')} kf+odh NB-triggered={a.get('notebook_triggered_reconciles_kf_odh')}")
        out.append(f"  at rest cpu ms/s={json.dumps({k.replace('control_plane_', 'cp_'): v for k, v in (a.get('cpu_ms_per_s') or {}).items()})}")
        out.append(f"  at rest rss MiB={json.dumps({k.replace('control_plane_', 'cp_'): v for k, v in (a.get('rss_mib') or {}).items()})}")
    if r:
        a = r.get("at_rest") or {}
        out.append(f"  webhook heartbeats/s fast={a.get('webhook_heartbeat_fast_path_per_s')} "
                   f"full={a.get('webhook_heartbeat_full_pipeline_per_s')} admissions/s={a.get('admissions_per_s')}")
    for k, st in sorted(d.items()):
        if k.startswith("storage_") and isinstance(st, dict):
            out.append(f"  {k}: {st.get('notebooks_ready_per_s')} nb/s (x{st.get('notebooks_per_s_vs_headline')}), "
                       f"ready p50/p95={(st.get('ready_ms') or {}).get('p50')}/{(st.get('ready_ms') or {}).get('p95')} "
                       f"rec/s={st.get('reconciles_per_s')}" + (f" errors={st['errors']}" if st.get("errors") else ""))
    b = d.get("burst")
    if b:
        out.append(f"  burst {b.get('notebooks')}: {b.get('notebooks_per_s')} nb/s, ready p50/p99 "
                   f"{(b.get('ready_ms') or {}).get('p50')}/{(b.get('ready_ms') or {}).get('p99')}, adm p99 "
                   f"{(b.get('admission_ms') or {}).get('p99')}")
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(summary(p))
