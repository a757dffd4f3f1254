"""A/B timings of the node-agent kernels on one MI355X (run on the GPU box).

GEMM 4096³ / 8192³: 128² register-staged kernel vs 256² LDS-DMA kernel vs torch (hipBLASLt);
fused-verify probe GEMM; HBM pattern write with plain vs non-temporal stores; HBM check.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from odh_kubeflow_amd.ops import gpu  # noqa: E402


def timeit(fn, iters=20, warm_s=0.25):
    """Median of ``iters`` event-timed calls after ``warm_s`` seconds of back-to-back calls:
    MI355X clocks ramp under load (DVFS), so a few warm-up calls time a cold chip."""
    import time

    t_end = time.perf_counter() + warm_s
    while time.perf_counter() < t_end:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    out = {}
    lib = gpu.load_library()
    dev = torch.device("cuda", 0)
    for n in (4096, 8192):
        g = torch.Generator(device=dev).manual_seed(n)
        a = (torch.rand((n, n), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand((n, n), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty((n, n), dtype=torch.float32, device=dev)
        fl = 2.0 * n ** 3
        import ctypes

        lib.odh_gemm_bf16_256_variant.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
        st = torch.cuda.current_stream().cuda_stream
        ref = a.float() @ bt.float().t()
        for v in (0, 1, 2, 3):  # 2-buffer BK=64 (v0 / v1 fragment-pipelined) vs deep BK=32 4-buffer ring (v2, v3 cross-barrier prefetch)
            ms = timeit(lambda: lib.odh_gemm_bf16_256_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), n, n, n, v, st))
            c.zero_()
            lib.odh_gemm_bf16_256_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), n, n, n, v, st)
            out[f"gemm256_v{v}_{n}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                                        "maxerr": float((c - ref).abs().max().item())}
        for name, fn in (("gemm128", lambda: gpu.gemm_bf16(a, bt, out=c, tile=128)),
                         ("gemm256", lambda: gpu.gemm_bf16(a, bt, out=c)),
                         ("torch_bf16_out", lambda: torch.mm(a, bt.t()))):
            ms = timeit(fn)
            out[f"{name}_{n}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
        gpu.gemm_bf16(a, bt, out=c)
        out[f"gemm256_{n}_maxerr"] = float((c - ref).abs().max().item())
        del a, bt, c, ref
        torch.cuda.empty_cache()
    import ctypes

    p = gpu.GpuProbe(0, 4096, 4096, 4096, hbm_bytes=1 << 30)  # the round-1 probe size: kernel A/B numbers
    s = torch.cuda.current_stream().cuda_stream
    cnt = p.counters.data_ptr()
    ms = timeit(lambda: lib.odh_probe_gemm_verify(p.a.data_ptr(), p.bt.data_ptr(), p.m, p.n, p.k,
                                                  p.tile_xcd.data_ptr(), cnt, cnt + 64, cnt + 32, s))
    out["probe_gemm_fused_verify_4096"] = {"ms": round(ms, 4), "tflops": round(2.0 * 4096 ** 3 / ms / 1e9, 1)}
    ms = timeit(lambda: lib.odh_probe_gemm_verify_2buf(p.a.data_ptr(), p.bt.data_ptr(), p.m, p.n, p.k,
                                                       p.tile_xcd.data_ptr(), cnt, cnt + 64, cnt + 32, s))
    out["probe_gemm_fused_verify_2buf_4096"] = {"ms": round(ms, 4), "tflops": round(2.0 * 4096 ** 3 / ms / 1e9, 1)}
    for rep in range(1):
        for v in range(8):  # bit 0 XB, bits 1-2 tile grouping GM = 1/2/4/8
            p.counters.zero_()
            ms = timeit(lambda: lib.odh_probe_gemm_verify_deep(p.a.data_ptr(), p.bt.data_ptr(), p.m, p.n, p.k,
                                                               p.tile_xcd.data_ptr(), cnt, cnt + 64, cnt + 32, v, s))
            torch.cuda.synchronize()
            out[f"probe_gemm_fused_verify_deep_v{v}_r{rep}_4096"] = {
                "ms": round(ms, 4), "tflops": round(2.0 * 4096 ** 3 / ms / 1e9, 1),
                "errors": int(p.counters[16].item())}
    for nt in (0, 1):
        ms = timeit(lambda: lib.odh_hbm_write(p.hbm.data_ptr(), p.hbm_bytes, 7, nt, s))
        out[f"hbm_write_nt{nt}_1GiB"] = {"ms": round(ms, 4), "gbps": round(p.hbm_bytes / ms / 1e6, 1)}
    import ctypes

    lib.odh_hbm_write_variant.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_void_p]
    for v in (1, 2, 3):
        for blocks in (1024, 2048, 4096, 8192):
            ms = timeit(lambda: lib.odh_hbm_write_variant(p.hbm.data_ptr(), p.hbm_bytes, 7, v, blocks, s))
            out[f"hbm_write_v{v}_b{blocks}"] = {"ms": round(ms, 4), "gbps": round(p.hbm_bytes / ms / 1e6, 1)}
    big = torch.empty((4 << 30) // 4, dtype=torch.int32, device=dev)
    for v in (1, 3):
        ms = timeit(lambda: lib.odh_hbm_write_variant(big.data_ptr(), 4 << 30, 7, v, 4096, s), iters=5, warm_s=0.05)
        out[f"hbm_write_v{v}_4GiB"] = {"ms": round(ms, 4), "gbps": round((4 << 30) / ms / 1e6, 1)}
    ms = timeit(lambda: big.fill_(3), iters=5, warm_s=0.05)
    out["torch_fill_4GiB"] = {"ms": round(ms, 4), "gbps": round((4 << 30) / ms / 1e6, 1)}
    del big
    lib.odh_hbm_write(p.hbm.data_ptr(), p.hbm_bytes, 7, 0, s)  # check against a matching pattern (the probe's case)
    ms = timeit(lambda: lib.odh_hbm_check(p.hbm.data_ptr(), p.hbm_bytes, 7, cnt + 72, s))
    out["hbm_check_1GiB"] = {"ms": round(ms, 4), "gbps": round(p.hbm_bytes / ms / 1e6, 1)}
    lib.odh_hbm_write(p.hbm.data_ptr(), p.hbm_bytes, 7, 0, s)
    for v in (0, 1, 2, 3):
        for blocks in (1024, 2048, 4096, 8192):
            p.counters.zero_()
            ms = timeit(lambda: lib.odh_hbm_check_variant(p.hbm.data_ptr(), p.hbm_bytes, 7, cnt + 72, v, blocks, s))
            torch.cuda.synchronize()
            out[f"hbm_check_v{v}_b{blocks}"] = {"ms": round(ms, 4), "gbps": round(p.hbm_bytes / ms / 1e6, 1),
                                                "errors": int(p.counters[18].item())}
    ms = timeit(lambda: p.hbm.sum())
    out["torch_sum_1GiB"] = {"ms": round(ms, 4), "gbps": round(p.hbm_bytes / ms / 1e6, 1)}
    for ov in (False, True):
        p.overlap = ov
        rs = [p.run() for _ in range(12)][2:]
        rs.sort(key=lambda r: r["gpu_ms"])
        r = rs[len(rs) // 2]
        out[f"probe_run_overlap{int(ov)}"] = {k: (round(r[k], 4) if isinstance(r[k], float) else r[k]) for k in
                                              ("ok", "gpu_ms", "wall_ms", "gemm_ms", "hbm_ms", "gemm_tflops",
                                               "hbm_gbps", "xcds", "fused_verify")}
    print(json.dumps(out, indent=1))


def startup():
    """The start-up probe as the node agent runs it (``gpu.PROBE_SHAPE``,
    ``gpu.PROBE_HBM_BYTES``): eager launches vs the hipGraph replay, 200 runs each
    (after 20 warm-up), medians and p95 of host wall time and GPU time."""
    out = {}
    p = gpu.GpuProbe(0)
    probes = {"eager": p, "graph": p, "serial": gpu.GpuProbe(0, graph="serial")}
    for key in ("eager", "graph", "serial") * 2:  # interleaved: clock drift shows up as A≠A
        q = probes[key]
        q.graph = {"eager": False, "graph": True, "serial": "serial"}[key]
        for _ in range(20):
            q.run()
        rs = [q.run() for _ in range(200)]
        assert all(r["ok"] and r["graph"] is (key != "eager") for r in rs), rs[-1]
        row = {}
        for k in ("wall_ms", "gpu_ms", "gemm_ms", "hbm_ms"):
            v = sorted(r[k] for r in rs)
            row[k + "_p50"] = round(v[len(v) // 2], 4)
            row[k + "_p95"] = round(v[int(len(v) * 0.95)], 4)
        out.setdefault(key, []).append(row)
    p.close()
    probes["serial"].close()
    print(json.dumps(out, indent=1))


def pmc_pass():
    """A short, fixed workload for ``rocprofv3 --pmc`` passes: the node agent's start-up
    probe as it runs on the notebook path (fused-verify bf16 MFMA GEMM of
    ``gpu.PROBE_SHAPE`` + HBM pattern write/check of ``gpu.PROBE_HBM_BYTES``) ×10, and the
    standalone 256² GEMM at 8192³ ×3."""
    p = gpu.GpuProbe(0)  # the start-up probe as it runs on the notebook path
    for _ in range(10):
        assert p.run()["ok"]
    dev = torch.device("cuda", 0)
    n = 8192
    a = torch.ones((n, n), device=dev, dtype=torch.bfloat16)
    bt = torch.ones((n, n), device=dev, dtype=torch.bfloat16)
    c = torch.empty((n, n), dtype=torch.float32, device=dev)
    for _ in range(3):
        gpu.gemm_bf16(a, bt, out=c)
    torch.cuda.synchronize()
    print("pmc pass ok")


if __name__ == "__main__":
    if "--pmc-pass" in sys.argv:
        pmc_pass()
    elif "--startup" in sys.argv:
        startup()
    else:
        main()
