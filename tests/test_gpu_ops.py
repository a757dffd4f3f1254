"""HIP kernels of the node agent on a real MI355X (numerics vs PyTorch fp32 references)."""

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    from odh_kubeflow_amd.ops import gpu

    gpu.load_library()  # loud failure if the in-tree .so is missing
    return torch.device("cuda", 0)


@pytest.mark.parametrize("tile", [None, 128])
@pytest.mark.parametrize("m,n,k", [(128, 128, 32), (256, 384, 96), (512, 768, 192), (1024, 512, 4096),
                                   (2048, 2048, 1024)])
def test_gemm_bf16_matches_fp32_reference(dev, m, n, k, tile):
    """Both kernels (256² LDS-DMA where it divides the shape, 128² register-staged) vs fp32 torch."""
    from odh_kubeflow_amd.ops.gpu import gemm_bf16

    g = torch.Generator(device=dev).manual_seed(m + n + k)
    a = torch.randn((m, k), generator=g, device=dev).to(torch.bfloat16)
    bt = torch.randn((n, k), generator=g, device=dev).to(torch.bfloat16)
    c = gemm_bf16(a, bt, tile=tile)
    ref = a.float() @ bt.float().t()
    torch.cuda.synchronize()
    err = (c - ref).abs().max().item()
    assert err <= 1e-3 * (k ** 0.5) + 1e-3, err


def test_gemm_bf16_identity_asymmetric(dev):
    from odh_kubeflow_amd.ops.gpu import gemm_bf16

    m = n = k = 256
    a = torch.eye(m, device=dev, dtype=torch.bfloat16)
    b = (torch.arange(k, device=dev).view(k, 1) * 3 - torch.arange(n, device=dev).view(1, n) * 2) % 97
    bt = b.t().contiguous().to(torch.bfloat16)
    c = gemm_bf16(a, bt)
    assert torch.equal(c, b.float())


def test_gemm_bf16_rejects_bad_shapes(dev):
    from odh_kubeflow_amd.ops.gpu import gemm_bf16

    a = torch.zeros((100, 64), device=dev, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        gemm_bf16(a, torch.zeros((128, 64), device=dev, dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        gemm_bf16(torch.zeros((128, 64), device=dev, dtype=torch.bfloat16),
                  torch.zeros((128, 32), device=dev, dtype=torch.bfloat16))


def test_startup_probe_passes_and_sees_all_xcds(dev):
    from odh_kubeflow_amd.ops.gpu import GpuProbe

    for shape, fused in (((2048, 2048, 2048), True), ((1024, 1152, 512), False)):
        p = GpuProbe(0, *shape, hbm_bytes=256 << 20, overlap=False)  # phases timed in isolation
        r = p.run()
        r = p.run()
        assert r["ok"], r
        p.overlap = True  # GEMM and HBM sweep concurrently on two streams: same verdict
        assert p.run()["ok"] and p.run()["ok"]
        p.overlap = False
        assert r["fused_verify"] is fused
        assert r["gemm_errors"] == 0 and r["hbm_errors"] == 0
        assert r["xcds"] == 8, r["xcd_blocks"]
        assert sum(r["xcd_blocks"]) == p.tiles == (shape[0] // (256 if fused else 128)) * (
            shape[1] // (256 if fused else 128))
        # sanity floors, far below the MFMA rates (a non-MFMA fallback would sit near 1 TFLOP/s):
        # the 1.2 GFLOP shape runs ~25 us, so its rate is launch- and clock-ramp-bound
        assert r["gemm_tflops"] > (50 if fused else 15) and r["hbm_gbps"] > 500, r


def test_fused_probe_verify_detects_corrupted_operand(dev):
    """The in-register check of the 256² kernel counts every wrong output element."""
    from odh_kubeflow_amd.ops import gpu

    p = gpu.GpuProbe(0, m=1024, n=1024, k=512, hbm_bytes=16 << 20)
    assert p.fused and p.run()["ok"]
    # A[5][7] += 1 changes C[5][j] by Bt[j][7] for every j: wrong wherever Bt[j][7] != 0
    expect_bad = int((p.bt[:, 7].float() != 0).sum().item())
    p.a[5, 7] = (p.a[5, 7].float() + 1).to(torch.bfloat16)
    r = p.run()
    assert not r["ok"] and r["gemm_errors"] == expect_bad and sum(r["err_xcd"]) == expect_bad
    p.a[5, 7] = (p.a[5, 7].float() - 1).to(torch.bfloat16)
    assert p.run()["ok"]


def test_graph_probe_replays_and_detects_corruption(dev):
    """The start-up probe replays as one hipGraph: same verdicts as the eager launches, a
    fresh HBM pattern per replay (device-side seed), and spans timed inside the kernels."""
    from odh_kubeflow_amd.ops import gpu

    p = gpu.GpuProbe(0, m=1024, n=1024, k=512, hbm_bytes=16 << 20)
    rs = [p.run() for _ in range(3)]
    assert all(r["ok"] and r["graph"] for r in rs), rs
    assert rs[-1]["graph_error"] is None
    r = rs[-1]
    assert r["xcds"] == 8 and sum(r["xcd_blocks"]) == p.tiles
    assert 0 < r["gemm_ms"] < r["gpu_ms"] + 0.05 and 0 < r["hbm_ms"] < r["gpu_ms"] + 0.05, r
    seeds = set()
    for _ in range(2):
        p.run()
        seeds.add(int(p.seed_dev.item()))
    assert len(seeds) == 2  # each replay advanced the on-device pattern seed
    expect_bad = int((p.bt[:, 7].float() != 0).sum().item())
    p.a[5, 7] = (p.a[5, 7].float() + 1).to(torch.bfloat16)
    r = p.run()
    assert r["graph"] and not r["ok"] and r["gemm_errors"] == expect_bad and sum(r["err_xcd"]) == expect_bad
    p.a[5, 7] = (p.a[5, 7].float() - 1).to(torch.bfloat16)
    assert p.run()["ok"]
    p.graph = False  # the eager launches: same verdict
    r = p.run()
    assert r["ok"] and not r["graph"]
    p.close()


def test_probe_verify_detects_corruption(dev):
    from odh_kubeflow_amd.ops import gpu

    p = gpu.GpuProbe(0, m=1024, n=1152, k=512, hbm_bytes=16 << 20)  # not 256-divisible: store + check kernel
    assert not p.fused and p.run()["ok"]
    lib = gpu.load_library()
    s = torch.cuda.current_stream().cuda_stream
    p.counters.zero_()
    p.c[5, 7] += 1.0
    p.c[700, 900] = float("nan")
    gpu._check(lib.odh_probe_verify(p.c.data_ptr(), p.m, p.n, p.k, p.tile_xcd.data_ptr(),
                                    p.counters.data_ptr() + 64, p.counters.data_ptr() + 32, s))
    torch.cuda.synchronize()
    h = p.counters.cpu().tolist()
    assert h[16] == 2 and sum(h[8:16]) == 2
    # HBM: flip one word after the pattern write
    p.counters.zero_()
    gpu._check(lib.odh_hbm_write(p.hbm.data_ptr(), p.hbm_bytes, 1234, 0, s))
    p.hbm[12345] ^= 1
    gpu._check(lib.odh_hbm_check(p.hbm.data_ptr(), p.hbm_bytes, 1234, p.counters.data_ptr() + 72, s))
    torch.cuda.synchronize()
    assert p.counters.cpu().tolist()[18] == 1


def test_load_generator_runs(dev):
    import time

    from odh_kubeflow_amd.ops.gpu import LoadGenerator

    lg = LoadGenerator(0, duty=1.0, chunk_ms=2.0).start()
    time.sleep(0.5)
    lg.stop()
    assert lg.launches > 5


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 768, 192), (1024, 512, 4096), (2048, 2048, 1024)])
def test_gemm256_variants_match_fp32_reference(dev, variant, m, n, k):
    """256² kernels: 2-buffer BK=64 (v0, v1 fragment-pipelined) and the deep BK=32 4-buffer ring (v2)."""
    from odh_kubeflow_amd.ops import gpu

    lib = gpu.load_library()
    g = torch.Generator(device=dev).manual_seed(7 * m + n + k + variant)
    a = torch.randn((m, k), generator=g, device=dev).to(torch.bfloat16)
    bt = torch.randn((n, k), generator=g, device=dev).to(torch.bfloat16)
    c = torch.full((m, n), float("nan"), device=dev)
    gpu._check(lib.odh_gemm_bf16_256_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, variant,
                                             torch.cuda.current_stream().cuda_stream))
    ref = a.float() @ bt.float().t()
    torch.cuda.synchronize()
    err = (c - ref).abs().max().item()
    assert err <= 1e-3 * (k ** 0.5) + 1e-3, err


@pytest.mark.parametrize("xb", [0, 1, 4, 5])
def test_deep_fused_probe_verify_counts_errors(dev, xb):
    """The deep-pipelined probe GEMM checks in registers exactly like the 2-buffer one."""
    from odh_kubeflow_amd.ops import gpu

    lib = gpu.load_library()
    p = gpu.GpuProbe(0, m=1024, n=1024, k=1024, hbm_bytes=16 << 20)
    s = torch.cuda.current_stream().cuda_stream

    def run_deep():
        p.counters.zero_()
        cnt = p.counters.data_ptr()
        gpu._check(lib.odh_probe_gemm_verify_deep(p.a.data_ptr(), p.bt.data_ptr(), p.m, p.n, p.k,
                                                  p.tile_xcd.data_ptr(), cnt, cnt + 64, cnt + 32, xb, s))
        torch.cuda.synchronize()
        h = p.counters.cpu().tolist()
        return h[16], sum(h[8:16]), sum(h[0:8])

    assert run_deep() == (0, 0, 16)
    expect_bad = int((p.bt[:, 7].float() != 0).sum().item())
    p.a[5, 7] = (p.a[5, 7].float() + 1).to(torch.bfloat16)
    assert run_deep() == (expect_bad, expect_bad, 16)
    p.a[5, 7] = (p.a[5, 7].float() - 1).to(torch.bfloat16)
    assert run_deep()[0] == 0


def test_single_gpu_pod_has_no_xgmi_links(dev):
    from odh_kubeflow_amd.ops import gpu

    assert gpu.xgmi_ring_check([0]) == []
    r = gpu.probe_devices([0])
    assert r["ok"] and "links" not in r
    assert gpu.load_library().odh_peer_enable(0, 0) == 0  # self: nothing to enable


def test_multi_gpu_pod_xgmi_ring(dev):
    """Multi-GPU pod: every link of the ring over its GPUs is read and verified over xGMI."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs 2+ MI355X (xGMI peers)")
    from odh_kubeflow_amd.ops import gpu

    devs = list(range(min(n, 4)))
    r = gpu.probe_devices(devs)
    assert r["ok"], r
    assert len(r["links"]) == (2 if len(devs) == 2 else len(devs))
    for lk in r["links"]:
        assert lk["errors"] == 0 and lk["gbps"] > 10, lk
