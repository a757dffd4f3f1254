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


@pytest.mark.parametrize("m,n,k", [(128, 128, 32), (256, 384, 96), (1024, 512, 4096), (2048, 2048, 1024)])
def test_gemm_bf16_matches_fp32_reference(dev, m, n, k):
    from odh_kubeflow_amd.ops.gpu import gemm_bf16

    g = torch.Generator(device=dev).manual_seed(m + n + k)
    a = torch.randn((m, k), generator=g, device=dev).to(torch.bfloat16)
    bt = torch.randn((n, k), generator=g, device=dev).to(torch.bfloat16)
    c = gemm_bf16(a, bt)
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

    p = GpuProbe(0, m=2048, n=2048, k=2048, hbm_bytes=256 << 20)
    r = p.run()
    r = p.run()
    assert r["ok"], r
    assert r["gemm_errors"] == 0 and r["hbm_errors"] == 0
    assert r["xcds"] == 8, r["xcd_blocks"]
    assert sum(r["xcd_blocks"]) == (2048 // 128) ** 2
    assert r["gemm_tflops"] > 50 and r["hbm_gbps"] > 500, r


def test_probe_verify_detects_corruption(dev):
    from odh_kubeflow_amd.ops import gpu

    p = gpu.GpuProbe(0, m=1024, n=1024, k=512, hbm_bytes=16 << 20)
    assert p.run()["ok"]
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
    gpu._check(lib.odh_hbm_write(p.hbm.data_ptr(), p.hbm_bytes, 1234, s))
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


def test_startup_probe_async_hook(dev):
    import asyncio

    from odh_kubeflow_amd.ops.gpu import startup_probe

    r = asyncio.run(startup_probe([0]))
    assert r["ok"], r
    assert r["results"][0]["xcds"] == 8
