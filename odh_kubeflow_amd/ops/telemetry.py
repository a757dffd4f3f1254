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
                ("domain", ctypes.c_int), ("unique_id", ctypes.c_uint64), ("location_id", ctypes.c_uint64),
                ("vram_total", ctypes.c_int64), ("gpu_id", ctypes.c_int64)]


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
    domain: int = 0
    gpu_id: int = 0

    @property
    def pci_bdf(self) -> str:
        """``dddd:bb:dd.f`` — the device ID the AMD device plugin advertises for a whole GPU
        (KFD ``location_id`` = bus << 8 | device << 3 | function)."""
        loc = self.location_id
        return f"{self.domain:04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 0x7:x}"


@dataclass
class KfdProcess:
    pid: int
    gpu_id: int
    vram_bytes: int
    pod_uid: Optional[str]


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
        lib.odh_tel_kfd_procs.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64]
        lib.odh_tel_kfd_procs.restype = ctypes.c_int64
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
                                  inf.vram_total, inf.domain, inf.gpu_id))
        return out

    def kfd_processes(self, proc_root: str = "/proc") -> List[KfdProcess]:
        """Processes holding GPU memory, from KFD's per-process sysfs, with their pod UID."""
        cap = 1 << 16
        while True:
            buf = ctypes.create_string_buffer(cap)
            need = self._lib.odh_tel_kfd_procs(self._h, proc_root.encode(), buf, cap)
            if need <= cap:
                break
            cap = int(need) + 4096
        out = []
        for line in buf.raw[:max(need, 0)].decode().splitlines():
            pid, gpu_id, vram, uid = line.split()
            out.append(KfdProcess(int(pid), int(gpu_id), int(vram), None if uid == "-" else uid))
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
                        f"location_id {0x1000 * (g + 1)}\ndomain 0\nunique_id {0xABC000 + g}\n")
            with open(os.path.join(d, "gpu_id"), "w") as f:
                f.write(f"{fake_gpu_id(len(minors))}\n")
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


def fake_gpu_id(index: int) -> int:
    """KFD gpu_id of device ``index`` in :func:`write_fake_sysfs` trees (real ids are hashes)."""
    return 40000 + 1111 * index


def fake_bdf(gpu: int) -> str:
    """PCI address of GPU ``gpu`` in :func:`write_fake_sysfs` trees (``location_id`` 0x1000·(g+1))."""
    loc = 0x1000 * (gpu + 1)
    return f"0000:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 0x7:x}"


def set_fake_kfd_process(sys_root: str, proc_root: str, pid: int, vram_by_gpu_id: dict,
                         pod_uid: Optional[str] = None, systemd: bool = True) -> None:
    """A process holding VRAM (``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>``) inside the pod
    cgroup of ``pod_uid`` (``/proc/<pid>/cgroup``, systemd or cgroupfs naming)."""
    d = os.path.join(sys_root, "class", "kfd", "kfd", "proc", str(pid))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pasid"), "w") as f:
        f.write(f"{32768 + pid}\n")
    for gid, b in vram_by_gpu_id.items():
        with open(os.path.join(d, f"vram_{gid}"), "w") as f:
            f.write(f"{b}\n")
    p = os.path.join(proc_root, str(pid))
    os.makedirs(p, exist_ok=True)
    if pod_uid is None:
        line = "0::/system.slice/some-daemon.service\n"
    elif systemd:
        u = pod_uid.replace("-", "_")
        line = (f"0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{u}.slice/"
                f"cri-containerd-{pid:064x}.scope\n")
    else:
        line = f"12:memory:/kubepods/besteffort/pod{pod_uid}/{pid:064x}\n"
    with open(os.path.join(p, "cgroup"), "w") as f:
        f.write(line)


def remove_fake_kfd_process(sys_root: str, proc_root: str, pid: int) -> None:
    import shutil

    shutil.rmtree(os.path.join(sys_root, "class", "kfd", "kfd", "proc", str(pid)), ignore_errors=True)
    shutil.rmtree(os.path.join(proc_root, str(pid)), ignore_errors=True)
