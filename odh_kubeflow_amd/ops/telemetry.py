"""ctypes binding of ``libodh_gpu_telemetry.so`` (amdgpu busy / VRAM sampler).

The culler's ``amdgpu`` activity source (``controllers/culling.py``) asks
:meth:`Telemetry.window` for the mean/max busy percentage of a GPU over the last
``W`` seconds; the native background thread keeps the per-device sample rings filled.
:func:`write_fake_sysfs` builds a synthetic ``/sys`` tree with the same layout for
CPU-only tests.
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional

from .build import lib_path

TEL_LIB = "libodh_gpu_telemetry.so"


class _Info(ctypes.Structure):
    _fields_ = [("node", ctypes.c_int), ("render_minor", ctypes.c_int), ("physical", ctypes.c_int),
                ("reserved", ctypes.c_int), ("unique_id", ctypes.c_uint64), ("location_id", ctypes.c_uint64),
                ("vram_total", ctypes.c_int64)]


class _Sample(ctypes.Structure):
    _fields_ = [("t_ns", ctypes.c_int64), ("busy", ctypes.c_int), ("reserved", ctypes.c_int),
                ("vram_used", ctypes.c_int64)]


class _Window(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("unavailable", ctypes.c_int), ("busy_mean", ctypes.c_double),
                ("busy_max", ctypes.c_int), ("reserved", ctypes.c_int), ("vram_used_mean", ctypes.c_double),
                ("span_ns", ctypes.c_int64)]


@dataclass
class DeviceInfo:
    index: int
    node: int
    render_minor: int
    physical: int
    unique_id: int
    location_id: int
    vram_total: int


@dataclass
class WindowStats:
    n: int
    unavailable: int
    busy_mean: float  # -1 when no readable sample
    busy_max: int
    vram_used_mean: float
    span_s: float


_lib = None


def _load():
    global _lib
    if _lib is None:
        path = lib_path(TEL_LIB)
        if not os.path.exists(path):
            from .build import build

            build(verbose=False)
        lib = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        lib.odh_tel_open.argtypes = [ctypes.c_char_p]
        lib.odh_tel_open.restype = vp
        lib.odh_tel_count.argtypes = [vp]
        lib.odh_tel_info_get.argtypes = [vp, ctypes.c_int, ctypes.POINTER(_Info)]
        lib.odh_tel_read.argtypes = [vp, ctypes.c_int, ctypes.POINTER(_Sample)]
        lib.odh_tel_start.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        lib.odh_tel_sweeps.argtypes = [vp]
        lib.odh_tel_sweeps.restype = ctypes.c_uint64
        lib.odh_tel_push.argtypes = [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int64]
        lib.odh_tel_window_get.argtypes = [vp, ctypes.c_int, ctypes.c_double, ctypes.POINTER(_Window)]
        lib.odh_tel_stop.argtypes = [vp]
        lib.odh_tel_stop.restype = None
        lib.odh_tel_close.argtypes = [vp]
        lib.odh_tel_close.restype = None
        _lib = lib
    return _lib


class Telemetry:
    def __init__(self, root: str = "/sys"):
        self._lib = _load()
        self.root = root
        self._h = self._lib.odh_tel_open(root.encode())

    def __len__(self) -> int:
        return self._lib.odh_tel_count(self._h)

    def devices(self) -> List[DeviceInfo]:
        out = []
        for i in range(len(self)):
            inf = _Info()
            self._lib.odh_tel_info_get(self._h, i, ctypes.byref(inf))
            out.append(DeviceInfo(i, inf.node, inf.render_minor, inf.physical, inf.unique_id, inf.location_id,
                                  inf.vram_total))
        return out

    def read(self, idx: int) -> Optional[dict]:
        s = _Sample()
        if self._lib.odh_tel_read(self._h, idx, ctypes.byref(s)) != 0:
            return None
        return {"t_ns": s.t_ns, "busy": s.busy, "vram_used": s.vram_used}

    def start(self, interval_ms: int = 100, capacity: int = 3000) -> "Telemetry":
        self._lib.odh_tel_start(self._h, int(interval_ms), int(capacity))
        return self

    def sweeps(self) -> int:
        return int(self._lib.odh_tel_sweeps(self._h))

    def push(self, idx: int, busy: int, vram_used: int = -1, t_ns: int = 0) -> None:
        self._lib.odh_tel_push(self._h, idx, int(t_ns), int(busy), int(vram_used))

    def window(self, idx: int, seconds: float) -> Optional[WindowStats]:
        w = _Window()
        if self._lib.odh_tel_window_get(self._h, idx, float(seconds), ctypes.byref(w)) != 0:
            return None
        return WindowStats(w.n, w.unavailable, w.busy_mean, w.busy_max, w.vram_used_mean, w.span_ns / 1e9)

    def stop(self) -> None:
        if self._h:
            self._lib.odh_tel_stop(self._h)

    def close(self) -> None:
        if self._h:
            self._lib.odh_tel_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ synthetic sysfs (tests)


def write_fake_sysfs(root: str, gpus: int = 8, partitions: int = 1, vram_total: int = 288 * 10 ** 9) -> List[int]:
    """Create a KFD-topology + DRM tree for ``gpus`` MI355X (× ``partitions`` nodes each).

    Returns the render minors, in device order.  Node 0 is the CPU node, as on real hosts.
    """
    nodes = os.path.join(root, "class", "kfd", "kfd", "topology", "nodes")
    os.makedirs(os.path.join(nodes, "0"), exist_ok=True)
    with open(os.path.join(nodes, "0", "properties"), "w") as f:
        f.write("cpu_cores_count 128\nsimd_count 0\ndrm_render_minor 0\n")
    minors = []
    nid = 1
    for g in range(gpus):
        for p in range(partitions):
            minor = 128 + len(minors)
            d = os.path.join(nodes, str(nid))
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "properties"), "w") as f:
                f.write(f"cpu_cores_count 0\nsimd_count {1024 // partitions}\ndrm_render_minor {minor}\n"
                        f"location_id {0x1000 * (g + 1)}\nunique_id {0xABC000 + g}\n")
            dev = os.path.join(root, "class", "drm", f"renderD{minor}", "device")
            os.makedirs(dev, exist_ok=True)
            for name, val in (("gpu_busy_percent", 0), ("mem_info_vram_used", 0),
                              ("mem_info_vram_total", vram_total // partitions)):
                with open(os.path.join(dev, name), "w") as f:
                    f.write(f"{val}\n")
            minors.append(minor)
            nid += 1
    return minors


def set_fake_counter(root: str, minor: int, busy: Optional[int] = None, vram_used: Optional[int] = None) -> None:
    dev = os.path.join(root, "class", "drm", f"renderD{minor}", "device")
    if busy is not None:
        tmp = os.path.join(dev, ".busy.tmp")
        with open(tmp, "w") as f:
            f.write(f"{busy}\n")
        os.replace(tmp, os.path.join(dev, "gpu_busy_percent"))
    if vram_used is not None:
        tmp = os.path.join(dev, ".vram.tmp")
        with open(tmp, "w") as f:
            f.write(f"{vram_used}\n")
        os.replace(tmp, os.path.join(dev, "mem_info_vram_used"))
