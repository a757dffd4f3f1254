"""Python side of the MI355X node-agent kernels (``csrc/gpu_probe.hip``).

* :func:`gemm_bf16` — the MFMA bf16 GEMM (``C = A · Btᵀ``, fp32 out) on torch tensors.
* :class:`GpuProbe` — the notebook start-up probe: a resident bf16 GEMM whose
  integer-valued operands make every output element checkable bit-exactly on the GPU,
  plus an HBM3E pattern write/verify sweep.  Sized as a health check on the create →
  Ready path (:data:`PROBE_SHAPE`, :data:`PROBE_HBM_BYTES`): 4096×4096 outputs are 256
  tiles of 256², one workgroup per CU of the 256-CU chip, so every CU of every XCD runs
  MFMA work; K=1024 keeps the GEMM at ≈30 µs, and the 256 MiB sweep, interleaved over every
  HBM3E stack and channel, tests them all (round 1 ran K=4096 and 1 GiB: ≈0.5 ms of GPU
  time per pod start for the same coverage).  The probe is captured once into a hipGraph
  (sweep and GEMM on two forked streams, counter reset, 128-byte read-back) and replayed
  with ONE launch per pod start; the kernels time themselves (``wall_clock64`` spans), since
  events cannot split a graph launch.  Reports matrix-core
  TFLOP/s, HBM GB/s, mismatches (attributed to the XCD that computed them) and how many
  of the 8 XCDs ran workgroups.
* :func:`probe_devices` / :func:`xgmi_ring_check` — the same probe in a torch process over
  several GPUs (kernel tests, microbenchmarks).  The shipped start-up probe is the
  torch-free ``odh-gpu-probe`` init container (``csrc/probe_cli.cpp``, :mod:`.probe_main`),
  which launches these same kernels from plain hipMalloc'd buffers.
* :class:`LoadGenerator` — synthetic MFMA load at a given duty cycle (culler benchmarks).

The library is loaded with ctypes **after** ``import torch`` so it binds to the HIP
runtime torch already loaded.  If the ``.so`` is missing on a machine with a GPU the
calls raise :class:`NativeLibraryMissing` instead of silently falling back.
"""

from __future__ import annotations

import ctypes
import os
import threading
import time
from typing import Dict, List, Optional, Sequence

from .build import lib_path

PROBE_LIB = "libodh_gpu_probe.so"
BM = BN = 128
BK = 32
N_XCD = 8
PROBE_SHAPE = (4096, 4096, 1024)  # M, N, K of the start-up probe GEMM (256 tiles of 256²)
PROBE_HBM_BYTES = 256 << 20


class NativeLibraryMissing(RuntimeError):
    pass


class HipError(RuntimeError):
    pass


_lib = None
_lib_lock = threading.Lock()


def load_library(build_if_missing: bool = False):
    """Load (once) and return the ctypes handle of ``libodh_gpu_probe.so``."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  -- must own libamdhip64.so.7 before we dlopen

        path = lib_path(PROBE_LIB)
        if not os.path.exists(path):
            if build_if_missing:
                from .build import build

                build(verbose=False)
            if not os.path.exists(path):
                raise NativeLibraryMissing(f"{path} not built; run `python -m odh_kubeflow_amd.ops.build`")
        lib = ctypes.CDLL(path)
        vp, i, u32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_size_t
        lib.odh_gemm_shape_ok.argtypes = [i, i, i]
        lib.odh_gemm_shape_ok.restype = i
        lib.odh_error_string.argtypes = [i]
        lib.odh_error_string.restype = ctypes.c_char_p
        lib.odh_probe_fill.argtypes = [vp, vp, i, i, i, vp]
        lib.odh_gemm_tiles.argtypes = [i, i, i]
        lib.odh_gemm_tiles.restype = i
        lib.odh_gemm_bf16.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp]
        lib.odh_gemm_bf16_128.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp]
        lib.odh_probe_verify.argtypes = [vp, i, i, i, vp, vp, vp, vp]
        lib.odh_probe_gemm_verify.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp]
        lib.odh_hbm_write.argtypes = [vp, sz, u32, i, vp]
        lib.odh_hbm_check.argtypes = [vp, sz, u32, vp, vp]
        lib.odh_busy.argtypes = [vp, i, i, vp]
        lib.odh_peer_enable.argtypes = [i, i]
        # A/B entry points (microbenchmarks, kernel numerics tests)
        lib.odh_gemm_bf16_256_variant.argtypes = [vp, vp, vp, i, i, i, i, vp]
        lib.odh_probe_gemm_verify_2buf.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, vp]
        lib.odh_probe_gemm_verify_deep.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp, i, vp]
        lib.odh_hbm_write_variant.argtypes = [vp, sz, u32, i, i, vp]
        lib.odh_hbm_check_variant.argtypes = [vp, sz, u32, vp, i, i, vp]
        lib.odh_probe_graph_create.argtypes = [vp, vp, i, i, i, vp, vp, vp, sz, vp, vp, i, ctypes.POINTER(vp)]
        lib.odh_probe_graph_launch.argtypes = [vp, vp]
        lib.odh_probe_graph_destroy.argtypes = [vp]
        lib.odh_probe_graph_destroy.restype = None
        lib.odh_wall_clock_khz.argtypes = [i]
        lib.odh_wall_clock_khz.restype = i
        for f in ("odh_probe_fill", "odh_gemm_bf16", "odh_gemm_bf16_128", "odh_probe_verify", "odh_probe_gemm_verify",
                  "odh_hbm_write", "odh_hbm_check", "odh_busy", "odh_gemm_bf16_256_variant",
                  "odh_probe_gemm_verify_2buf", "odh_probe_gemm_verify_deep", "odh_hbm_write_variant",
                  "odh_hbm_check_variant", "odh_peer_enable", "odh_probe_graph_create", "odh_probe_graph_launch"):
            getattr(lib, f).restype = i
        _lib = lib
        return lib


def _check(rc: int) -> None:
    if rc != 0:
        msg = load_library().odh_error_string(rc)
        raise HipError(f"HIP error {rc}: {msg.decode() if msg else '?'}")


def _stream_ptr(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def gemm_shape_ok(m: int, n: int, k: int) -> bool:
    return m > 0 and n > 0 and k > 0 and m % BM == 0 and n % BN == 0 and k % BK == 0


def gemm_tiles(m: int, n: int, k: int) -> int:
    """Workgroups the GEMM launches for this shape (256² tiles when they divide it, else 128²)."""
    return load_library().odh_gemm_tiles(m, n, k)


def fused_verify_ok(m: int, n: int, k: int) -> bool:
    return gemm_shape_ok(m, n, k) and m % 256 == 0 and n % 256 == 0 and k % 64 == 0


def gemm_bf16(a, bt, out=None, tile_xcd=None, xcd_blocks=None, tile: Optional[int] = None):
    """``C[M,N] = A[M,K] · Bt[N,K]ᵀ`` in fp32 on the matrix cores.

    Shapes must be multiples of the 128×128×32 tile (checked here, before launch); the
    256×256×64 LDS-DMA kernel runs when it divides the shape (``tile=128`` forces the
    smaller kernel, for A/B measurements).
    """
    import torch

    if a.dtype != torch.bfloat16 or bt.dtype != torch.bfloat16:
        raise TypeError("gemm_bf16 expects bfloat16 operands")
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError(f"shape mismatch: A{tuple(a.shape)} Bt{tuple(bt.shape)}")
    if not (a.is_cuda and bt.is_cuda) or a.device != bt.device:
        raise ValueError("operands must live on the same GPU")
    m, k = a.shape
    n = bt.shape[0]
    if not gemm_shape_ok(m, n, k):
        raise ValueError(f"M,N must be multiples of {BM}/{BN} and K of {BK}; got {m},{n},{k}")
    a = a.contiguous()
    bt = bt.contiguous()
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous fp32 [M,N] tensor")
    if tile_xcd is not None and tile_xcd.numel() < (m // BM) * (n // BN):
        raise ValueError("tile_xcd too small")
    if xcd_blocks is not None and xcd_blocks.numel() < N_XCD:
        raise ValueError("xcd_blocks too small")
    lib = load_library()
    fn = lib.odh_gemm_bf16_128 if tile == 128 else lib.odh_gemm_bf16
    _check(fn(a.data_ptr(), bt.data_ptr(), out.data_ptr(), m, n, k,
                             tile_xcd.data_ptr() if tile_xcd is not None else None,
                             xcd_blocks.data_ptr() if xcd_blocks is not None else None, _stream_ptr(a.device)))
    return out


class GpuProbe:
    """Resident start-up probe for one GPU (allocate + fill once, then ~1 ms per run)."""

    def __init__(self, device: int = 0, m: int = PROBE_SHAPE[0], n: int = PROBE_SHAPE[1], k: int = PROBE_SHAPE[2],
                 hbm_bytes: int = PROBE_HBM_BYTES,
                 hbm_nontemporal: bool = False, overlap: bool = True, graph=True):
        import torch

        if not gemm_shape_ok(m, n, k):
            raise ValueError("probe GEMM shape must be tile aligned")
        if hbm_bytes < 16 or hbm_bytes % 16:
            raise ValueError("hbm_bytes must be a positive multiple of 16")
        self.device = torch.device("cuda", device)
        self.m, self.n, self.k = m, n, k
        self.hbm_bytes = hbm_bytes
        lib = load_library()
        with torch.cuda.device(self.device):
            self.a = torch.empty((m, k), dtype=torch.bfloat16, device=self.device)
            self.bt = torch.empty((n, k), dtype=torch.bfloat16, device=self.device)
            # the 256² kernel checks C in registers; other shapes store C and run the check kernel
            self.fused = fused_verify_ok(m, n, k)
            self.c = None if self.fused else torch.empty((m, n), dtype=torch.float32, device=self.device)
            self.tiles = lib.odh_gemm_tiles(m, n, k)
            self.tile_xcd = torch.full(((m // BM) * (n // BN),), -1, dtype=torch.int32, device=self.device)
            self.hbm = torch.empty((hbm_bytes // 4,), dtype=torch.int32, device=self.device)
            # counters: [0:8] xcd_blocks, [8:16] err_xcd, [16] gemm err, [18:20] hbm err (u64)
            self.counters = torch.zeros((32,), dtype=torch.int32, device=self.device)
            self.host = torch.zeros((32,), dtype=torch.int32).pin_memory()
            self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            self.streams = (torch.cuda.Stream(self.device), torch.cuda.Stream(self.device))
            _check(lib.odh_probe_fill(self.a.data_ptr(), self.bt.data_ptr(), m, n, k, _stream_ptr(self.device)))
            torch.cuda.current_stream(self.device).synchronize()
        self.hbm_nontemporal = hbm_nontemporal
        self.overlap = overlap
        # graph replay: fused + overlapped probes (the start-up probe) — one launch per run
        self.graph = graph
        self._graph = None
        self._graph_error: Optional[str] = None
        self.runs = 0
        self.seed = 0x9E3779B9
        # one probe in flight per GPU: runs share the counters, events and pinned host buffer
        # (two pods probing the same device — ranks sharing a GPU in a rehearsal — take turns)
        self._lock = threading.Lock()

    def run(self) -> dict:
        """One probe.  With ``overlap`` (default) the memory-bound HBM sweep and the
        MFMA-bound GEMM run concurrently on two streams of the probe: their waves co-reside
        on the CUs (the GEMM's 1 workgroup/CU leaves VGPRs and wave slots free), so the
        GEMM hides under the sweep instead of adding to it.  With ``graph`` (default) that
        whole sequence is one hipGraph launch."""
        with self._lock:
            if self.graph and self.fused and self.overlap:
                g = self._graph_handle()
                if g is not None:
                    return self._run_graph(g)
            return self._run()

    def _graph_handle(self):
        """Capture the probe graph once (``None`` if capture failed: the eager launches run
        instead and the error is kept in ``graph_error`` of every result)."""
        if self._graph is not None or self._graph_error is not None:
            return self._graph
        import torch

        lib = load_library()
        with torch.cuda.device(self.device):
            self.seed_dev = torch.full((1,), 0x1E3779B9, dtype=torch.int32, device=self.device)
            torch.cuda.current_stream(self.device).synchronize()
            h = ctypes.c_void_p()
            rc = lib.odh_probe_graph_create(self.a.data_ptr(), self.bt.data_ptr(), self.m, self.n, self.k,
                                            self.tile_xcd.data_ptr(), self.counters.data_ptr(), self.hbm.data_ptr(),
                                            self.hbm_bytes, self.seed_dev.data_ptr(), self.host.data_ptr(),
                                            int(self.graph == "serial"), ctypes.byref(h))
        if rc != 0:
            msg = lib.odh_error_string(rc)
            self._graph_error = f"HIP error {rc}: {msg.decode() if msg else '?'}"
            return None
        self._graph = h
        self._tick_khz = lib.odh_wall_clock_khz(self.device.index) or 100000
        return h

    def close(self) -> None:
        with self._lock:
            if self._graph is not None:
                load_library().odh_probe_graph_destroy(self._graph)
                self._graph = None

    def _span_ms(self, h: List[int], i: int) -> float:
        begin = ~((h[i] & 0xFFFFFFFF) | ((h[i + 1] & 0xFFFFFFFF) << 32)) & 0xFFFFFFFFFFFFFFFF
        end = (h[i + 2] & 0xFFFFFFFF) | ((h[i + 3] & 0xFFFFFFFF) << 32)
        return max(0.0, (end - begin) / self._tick_khz) if end and begin != 0xFFFFFFFFFFFFFFFF else 0.0

    def _launch_graph(self, graph) -> None:
        import torch

        with torch.cuda.device(self.device):
            sg = self.streams[0]
            sg.wait_stream(torch.cuda.current_stream(self.device))  # caller's writes to a / bt / hbm
            self.ev[0].record(sg)
            _check(load_library().odh_probe_graph_launch(graph, sg.cuda_stream))
            self.ev[4].record(sg)

    def _graph_result(self, t0: float) -> dict:
        h = self.host.tolist()
        return self._result(h, self._span_ms(h, 20), self._span_ms(h, 24), self.ev[0].elapsed_time(self.ev[4]), t0,
                            graph=True)

    def _run_graph(self, graph) -> dict:
        t0 = time.perf_counter()
        self._launch_graph(graph)
        self.ev[4].synchronize()
        return self._graph_result(t0)

    def _run(self) -> dict:
        import torch

        lib = load_library()
        t0 = time.perf_counter()
        with torch.cuda.device(self.device):
            sg, sh = self.streams
            cnt = self.counters
            base = cnt.data_ptr()
            self.seed = (self.seed * 1664525 + 1013904223) & 0xFFFFFFFF
            sg.wait_stream(torch.cuda.current_stream(self.device))  # caller's writes to a / bt / hbm
            with torch.cuda.stream(sg):
                cnt.zero_()
                self.ev[0].record(sg)
            g, h_ = sg.cuda_stream, (sh.cuda_stream if self.overlap else sg.cuda_stream)
            if self.overlap:
                sh.wait_event(self.ev[0])
            hs = sh if self.overlap else sg

            def sweep():
                self.ev[2].record(hs)
                _check(lib.odh_hbm_write(self.hbm.data_ptr(), self.hbm_bytes, self.seed, int(self.hbm_nontemporal),
                                         h_))
                _check(lib.odh_hbm_check(self.hbm.data_ptr(), self.hbm_bytes, self.seed, base + 18 * 4, h_))
                self.ev[3].record(hs)

            if self.overlap:
                sweep()  # the longer, memory-bound part first: both are in flight together
            if self.fused:
                _check(lib.odh_probe_gemm_verify(self.a.data_ptr(), self.bt.data_ptr(), self.m, self.n, self.k,
                                                 self.tile_xcd.data_ptr(), base, base + 16 * 4, base + 8 * 4, g))
                self.ev[1].record(sg)
            else:
                _check(lib.odh_gemm_bf16(self.a.data_ptr(), self.bt.data_ptr(), self.c.data_ptr(), self.m, self.n,
                                         self.k, self.tile_xcd.data_ptr(), base, g))
                self.ev[1].record(sg)
                _check(lib.odh_probe_verify(self.c.data_ptr(), self.m, self.n, self.k, self.tile_xcd.data_ptr(),
                                            base + 16 * 4, base + 8 * 4, g))
            if not self.overlap:
                sweep()
            else:
                sg.wait_event(self.ev[3])
            with torch.cuda.stream(sg):
                self.host.copy_(cnt, non_blocking=True)
                self.ev[4].record(sg)
            self.ev[4].synchronize()
        h = self.host.tolist()
        return self._result(h, self.ev[0].elapsed_time(self.ev[1]), self.ev[2].elapsed_time(self.ev[3]),
                            self.ev[0].elapsed_time(self.ev[4]), t0, graph=False)

    def _result(self, h: List[int], gemm_ms: float, hbm_ms: float, probe_ms: float, t0: float, graph: bool) -> dict:
        xcd_blocks = h[0:8]
        err_xcd = h[8:16]
        gemm_err = h[16] & 0xFFFFFFFF
        hbm_err = (h[18] & 0xFFFFFFFF) | ((h[19] & 0xFFFFFFFF) << 32)
        flops = 2.0 * self.m * self.n * self.k
        self.runs += 1
        ok = gemm_err == 0 and hbm_err == 0 and sum(xcd_blocks) == self.tiles
        return {
            "ok": bool(ok), "device": self.device.index, "gemm_ms": gemm_ms, "hbm_ms": hbm_ms,
            "gpu_ms": probe_ms, "fused_verify": self.fused, "overlap": self.overlap,
            "gemm_tflops": flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0,
            "hbm_gbps": 2.0 * self.hbm_bytes / (hbm_ms * 1e-3) / 1e9 if hbm_ms > 0 else 0.0,
            "gemm_errors": gemm_err, "hbm_errors": hbm_err, "xcd_blocks": xcd_blocks, "err_xcd": err_xcd,
            "xcds": sum(1 for x in xcd_blocks if x > 0), "wall_ms": (time.perf_counter() - t0) * 1e3,
            "graph": graph, "graph_error": self._graph_error,
        }


_probes: Dict[int, GpuProbe] = {}
_probe_lock = threading.Lock()


def get_probe(device: int, **kw) -> GpuProbe:
    with _probe_lock:
        p = _probes.get(device)
        if p is None:
            p = _probes[device] = GpuProbe(device, **kw)
        return p


XGMI_CHECK_BYTES = 64 << 20


def ring_pairs(devices: Sequence[int]) -> List[tuple]:
    """(reader, source) per xGMI link the multi-GPU probe checks: a ring over the pod's
    GPUs, so with k GPUs k links are read (MI355X: every GPU pair has a direct link)."""
    ds = list(dict.fromkeys(devices))
    if len(ds) < 2:
        return []
    if len(ds) == 2:
        return [(ds[1], ds[0]), (ds[0], ds[1])]
    return [(ds[(n + 1) % len(ds)], ds[n]) for n in range(len(ds))]


def xgmi_ring_check(devices: Sequence[int], nbytes: int = XGMI_CHECK_BYTES) -> List[dict]:
    """Peer-read check of a multi-GPU pod's xGMI links.

    Each GPU's probe has just written its seeded pattern into its HBM buffer; GPU
    ``reader`` now streams the first ``nbytes`` of GPU ``source``'s buffer over xGMI and
    verifies every word (``odh_hbm_check`` with a peer pointer).  One link failing fails
    the pod, like an XCD failing the GEMM check.  The reference has no equivalent: a
    multi-GPU notebook there starts on GPUs whose interconnect nobody has looked at.
    """
    import torch

    lib = load_library()
    out = []
    for reader, source in ring_pairs(devices):
        r = {"reader": reader, "source": source, "ok": False}
        try:
            pr, ps = get_probe(reader), get_probe(source)
            n = min(nbytes, ps.hbm_bytes) & ~15
            first, second = sorted((pr, ps), key=lambda p: p.device.index)
            with first._lock, second._lock:
                _check(lib.odh_peer_enable(reader, source))
                dev = pr.device
                with torch.cuda.device(dev):
                    err = torch.zeros((2,), dtype=torch.int32, device=dev)
                    s = pr.streams[0]
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.wait_stream(torch.cuda.current_stream(dev))
                    torch.cuda.current_stream(ps.device).synchronize()  # source pattern is in HBM
                    ev0.record(s)
                    _check(lib.odh_hbm_check(ps.hbm.data_ptr(), n, ps.seed, err.data_ptr(), s.cuda_stream))
                    ev1.record(s)
                    ev1.synchronize()
                    e = err.cpu().tolist()
                ms = ev0.elapsed_time(ev1)
            errors = (e[0] & 0xFFFFFFFF) | ((e[1] & 0xFFFFFFFF) << 32)
            r.update(ok=errors == 0, errors=errors, bytes=n, ms=ms, gbps=n / (ms * 1e-3) / 1e9 if ms > 0 else 0.0)
        except Exception as ex:  # a link that cannot be checked fails the pod, not the agent
            r["error"] = repr(ex)
        out.append(r)
    return out


def probe_devices(devices: Sequence[int]) -> dict:
    results = []
    for d in devices:
        try:
            results.append(get_probe(d).run())
        except Exception as e:  # a failed probe fails the pod, it must not crash the agent
            results.append({"ok": False, "device": d, "error": repr(e)})
    links = xgmi_ring_check(devices) if all(r.get("ok") for r in results) else []
    error = next((r.get("error") or f"probe failed on GPU {r['device']}" for r in results if not r.get("ok")), None)
    if error is None:
        error = next((lk.get("error") or f"xGMI check failed reading GPU {lk['source']} from GPU {lk['reader']}"
                      for lk in links if not lk.get("ok")), None)
    out = {"ok": error is None, "devices": list(devices), "results": results, "error": error}
    if links:
        out["links"] = links
    return out


class LoadGenerator:
    """Keeps a GPU's matrix cores busy at ``duty`` (0..1) until :meth:`stop`."""

    def __init__(self, device: int = 0, duty: float = 1.0, chunk_ms: float = 5.0, blocks: int = 1024):
        self.device = device
        self.duty = max(0.0, min(1.0, duty))
        self.chunk_ms = chunk_ms
        self.blocks = blocks
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None
        self.launches = 0
        self.iters = 2048

    def _loop(self) -> None:
        import torch

        lib = load_library()
        dev = torch.device("cuda", self.device)
        with torch.cuda.device(dev):
            out = torch.empty((self.blocks * 256,), dtype=torch.float32, device=dev)
            s = _stream_ptr(dev)
            # calibrate iterations so one launch lasts ~chunk_ms
            t0 = time.perf_counter()
            _check(lib.odh_busy(out.data_ptr(), self.blocks, self.iters, s))
            torch.cuda.current_stream(dev).synchronize()
            dt = max(1e-4, time.perf_counter() - t0)
            self.iters = max(64, min(1 << 22, int(self.iters * (self.chunk_ms * 1e-3) / dt)))
            while not self._stop.is_set():
                t0 = time.perf_counter()
                _check(lib.odh_busy(out.data_ptr(), self.blocks, self.iters, s))
                torch.cuda.current_stream(dev).synchronize()
                self.launches += 1
                busy = time.perf_counter() - t0
                if self.duty < 1.0:
                    idle = busy * (1.0 - self.duty) / max(self.duty, 1e-3)
                    self._stop.wait(idle)

    def start(self) -> "LoadGenerator":
        self._thr = threading.Thread(target=self._loop, name=f"gpu-load-{self.device}", daemon=True)
        self._thr.start()
        return self

    def wait_running(self, timeout: float = 60.0) -> bool:
        """Block until the load is on the GPU (the first calibrated launch finished): the thread
        first initialises the HIP runtime, which takes from a few hundred ms to seconds."""
        deadline = time.monotonic() + timeout
        while self.launches < 1 and time.monotonic() < deadline:
            if self._thr is not None and not self._thr.is_alive():
                return False
            time.sleep(0.005)
        return self.launches >= 1

    def stop(self) -> None:
        self._stop.set()
        if self._thr is not None:
            self._thr.join(timeout=30)


def available() -> bool:
    """True when a GPU is visible (does not initialise HIP: device_count only)."""
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def loaded_libraries() -> List[str]:
    """Native libraries of this package mapped into the process (for smoke/bench logs)."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "odh_kubeflow_amd" in line and line.rstrip().endswith(".so"):
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
