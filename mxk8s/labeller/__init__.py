"""Node labeller: ``amd.com/gpu.*`` node labels from the native discovery core.

MI355X counterpart of GPU Feature Discovery + the NFD PCI labels the
reference's GPU Operator applies (the reference greps
them at /root/reference/README.md:288-293).  Labels (values sanitised to the
Kubernetes label-value grammar):

  amd.com/gpu.present=true        amd.com/gpu.count=8
  amd.com/gpu.arch=gfx950         amd.com/gpu.family=CDNA4
  amd.com/gpu.product=MI355X      amd.com/gpu.device-id=75a3
  amd.com/gpu.vram=288G           amd.com/gpu.cu-count=256
  amd.com/gpu.simd-count=1024     amd.com/gpu.max-sclk-mhz=2400
  amd.com/gpu.xgmi=true           amd.com/gpu.xgmi-links=7
  amd.com/gpu.xgmi-hive=<hex>     amd.com/gpu.numa-nodes=2
  amd.com/gpu.driver-version=...  amd.com/gpu.rocm-version=7.2.0
  amd.com/gpu.compute-partitioning-mode=spx|dpx|qpx|cpx|mixed
  amd.com/gpu.memory-partitioning-mode=nps1|nps2|nps4|mixed

The partition modes (the MI355X counterpart of the MIG-mode facts GFD
publishes) come from amdgpu's
``current_{compute,memory}_partition`` sysfs files; they are omitted when the
driver does not expose them.

Also writes an NFD ``features.d`` file so a stock Node Feature Discovery
(local source) publishes the same facts under feature.node.kubernetes.io/.
"""
from __future__ import annotations

import os
import re
from typing import Iterable, Optional

from ..native.node import GpuInfo

PREFIX = "amd.com/gpu."
_LABEL_VALUE = re.compile(r"^[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?$")

FAMILY = {"gfx950": "CDNA4", "gfx942": "CDNA3", "gfx90a": "CDNA2", "gfx908": "CDNA"}


def sanitize(value: str) -> str:
    """Coerce to a valid label value: <=63 chars, [A-Za-z0-9-_.], alnum ends."""
    v = re.sub(r"[^-A-Za-z0-9_.]+", "-", str(value)).strip("-_.")
    v = v[:63].strip("-_.")
    return v


def _vram_label(nbytes: int) -> str:
    gib = nbytes / 2 ** 30
    return f"{int(round(gib))}G"


def rocm_version(root: str = "") -> str:
    for p in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        full = os.path.join(root, p.lstrip("/")) if root else p
        try:
            with open(full) as f:
                return f.read().strip().split("-")[0]
        except OSError:
            continue
    return ""


def partition_modes(gpus: Iterable[GpuInfo], root: str = "") -> dict:
    """{"compute": mode, "memory": mode} from amdgpu's per-device sysfs files,
    lower-cased; "mixed" when GPUs disagree; a key is absent when no GPU has it."""
    out = {}
    for kind in ("compute", "memory"):
        seen = set()
        for g in gpus:
            path = os.path.join(root or "/", "sys/bus/pci/devices", g.bdf,
                                f"current_{kind}_partition")
            try:
                with open(path) as f:
                    seen.add(f.read().strip().lower())
            except OSError:
                continue
        seen.discard("")
        if seen:
            out[kind] = seen.pop() if len(seen) == 1 else "mixed"
    return out


def compute_labels(gpus: Iterable[GpuInfo], driver_version: str = "", rocm: str = "",
                   partitions: Optional[dict] = None) -> dict:
    gpus = list(gpus)
    if not gpus:
        return {PREFIX + "present": "false", PREFIX + "count": "0"}
    g = gpus[0]
    labels = {
        "present": "true",
        "count": str(len(gpus)),
        "arch": g.arch,
        "family": FAMILY.get(g.arch, "unknown"),
        "product": g.product or f"device-{g.device_id:04x}",
        "device-id": f"{g.device_id:04x}",
        "vram": _vram_label(g.vram_bytes),
        "cu-count": str(g.cu_count),
        "simd-count": str(g.simd_count),
        "max-sclk-mhz": str(g.max_sclk_mhz),
        "xgmi": "true" if any(x.xgmi_links > 0 for x in gpus) else "false",
        "xgmi-links": str(max(x.xgmi_links for x in gpus)),
        "numa-nodes": str(len({x.numa_node for x in gpus})),
    }
    hives = {x.hive_id for x in gpus if x.hive_id}
    if len(hives) == 1:
        labels["xgmi-hive"] = f"{next(iter(hives)):x}"
    elif len(hives) > 1:
        labels["xgmi-hives"] = str(len(hives))
    if len({(x.arch, x.device_id) for x in gpus}) > 1:
        labels["mixed"] = "true"
    if driver_version:
        labels["driver-version"] = driver_version
    if rocm:
        labels["rocm-version"] = rocm
    for kind, mode in (partitions or {}).items():
        labels[f"{kind}-partitioning-mode"] = mode
    out = {}
    for k, v in labels.items():
        s = sanitize(v)
        if s and _LABEL_VALUE.match(s):
            out[PREFIX + k] = s
    return out


def nfd_feature_file(labels: dict) -> str:
    """NFD local-source features.d content (default feature namespace)."""
    lines = ["# written by mxk8s labeller"]
    for k, v in sorted(labels.items()):
        lines.append(f"amd-gpu.{k[len(PREFIX):]}={v}")
    lines.append("pci-1002.present=true")
    return "\n".join(lines) + "\n"


def label_patch(current: dict, desired: dict) -> dict:
    """Merge-patch labels: set desired, delete stale amd.com/gpu.* keys."""
    patch = {k: v for k, v in desired.items() if current.get(k) != v}
    for k in current:
        if k.startswith(PREFIX) and k not in desired:
            patch[k] = None
    return patch


def run_once(client, node_name: str, gpus, driver: str = "", rocm: str = "",
             nfd_dir: Optional[str] = None, sysfs_root: str = "") -> dict:
    gpus = list(gpus)
    desired = compute_labels(gpus, driver, rocm, partition_modes(gpus, sysfs_root))
    node = client.get_node(node_name)
    current = node.get("metadata", {}).get("labels", {}) or {}
    patch = label_patch(current, desired)
    if patch:
        client.patch_node_labels(node_name, patch)
    if nfd_dir:
        os.makedirs(nfd_dir, exist_ok=True)
        tmp = os.path.join(nfd_dir, ".amd-gpu.tmp")
        with open(tmp, "w") as f:
            f.write(nfd_feature_file(desired))
        os.replace(tmp, os.path.join(nfd_dir, "amd-gpu"))
    return patch
