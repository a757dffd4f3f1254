"""The kubelet device manager's checkpoint (``/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint``).

The kubelet persists every device-plugin allocation there so it survives kubelet restarts::

    {"Data": {"PodDeviceEntries": [{"PodUID": "<uid>", "ContainerName": "notebook",
                                    "ResourceName": "amd.com/gpu",
                                    "DeviceIDs": {"0": ["0000:c1:00.0"]},      # NUMA node -> IDs (k8s >= 1.20)
                                    "AllocResp": "<base64>"}],
              "RegisteredDevices": {"amd.com/gpu": ["0000:c1:00.0", ...]}},
     "Checksum": 1234567}

Older kubelets wrote ``DeviceIDs`` as a flat list; both shapes are accepted.  The file is
an internal kubelet format, so the node agent prefers the pod-resources API
(:mod:`.podresources`) and uses this as a fallback when the socket is not mounted; it
is keyed by pod UID, which the culler has.
"""

from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

DEFAULT_PATH = "/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint"


def _ids(raw) -> List[str]:
    if isinstance(raw, dict):
        return [str(x) for k in sorted(raw) for x in raw[k] or []]
    if isinstance(raw, list):
        return [str(x) for x in raw]
    return []


def read_checkpoint(path: str = DEFAULT_PATH, resource: str = "amd.com/gpu") -> Optional[Dict[str, List[str]]]:
    """Pod UID → device IDs of ``resource``; ``None`` when the file is missing or unreadable."""
    try:
        with open(path, "rb") as f:
            doc = json.loads(f.read())
    except (OSError, ValueError):
        return None
    out: Dict[str, List[str]] = {}
    for e in ((doc.get("Data") or {}).get("PodDeviceEntries") or []):
        if e.get("ResourceName") != resource or not e.get("PodUID"):
            continue
        out.setdefault(e["PodUID"], []).extend(_ids(e.get("DeviceIDs")))
    return out


class CheckpointWriter:
    """Writes the checkpoint the way the kubelet device manager does (fake kubelet side of the
    test harness; the production agent only reads it).  Writes are atomic renames."""

    def __init__(self, path: str, resource: str = "amd.com/gpu", registered: Optional[List[str]] = None):
        self.path = path
        self.resource = resource
        self.registered = list(registered or [])
        self.entries: Dict[str, dict] = {}
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._write()

    def allocate(self, pod_uid: str, container: str, device_ids: List[str], numa: int = 0) -> None:
        self.entries[pod_uid] = {"PodUID": pod_uid, "ContainerName": container, "ResourceName": self.resource,
                                 "DeviceIDs": {str(numa): list(device_ids)}, "AllocResp": ""}
        self._write()

    def release(self, pod_uid: str) -> None:
        if self.entries.pop(pod_uid, None) is not None:
            self._write()

    def _write(self) -> None:
        doc = {"Data": {"PodDeviceEntries": list(self.entries.values()),
                        "RegisteredDevices": {self.resource: self.registered}}, "Checksum": 0}
        tmp = f"{self.path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(doc, f)
        os.replace(tmp, self.path)
