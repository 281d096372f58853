"""ctypes binding to ``libmxnode.so`` (``native/libmxnode``).

Python front ends (device plugin, labeller, exporter, doctor) call the C++
core through these wrappers.  Every function takes ``root`` so it can run
against a fake sysfs tree.
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import os
import threading
from typing import Optional

NODE_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "_lib", "libmxnode.so")
MAX_GPUS = 64
MAX_LINKS = 64

HEALTHY = 0
UNHEALTHY_NO_KFD_NODE = 1
UNHEALTHY_NO_RENDER_NODE = 2
UNHEALTHY_FAULT_INJECTED = 3
UNHEALTHY_SMI_EVENT = 4
UNHEALTHY_ECC = 5

LINK_PCIE = 2
LINK_XGMI = 11


class _GpuInfo(ctypes.Structure):
    _fields_ = [
        ("index", ctypes.c_int), ("kfd_node", ctypes.c_int), ("gpu_id", ctypes.c_uint32),
        ("gfx_target_version", ctypes.c_uint32), ("gfx_arch", ctypes.c_char * 16),
        ("drm_render_minor", ctypes.c_int), ("drm_card", ctypes.c_int),
        ("vendor_id", ctypes.c_uint32), ("device_id", ctypes.c_uint32),
        ("domain", ctypes.c_uint32), ("location_id", ctypes.c_uint32),
        ("pci_bdf", ctypes.c_char * 20), ("numa_node", ctypes.c_int),
        ("simd_count", ctypes.c_uint32), ("simd_per_cu", ctypes.c_uint32),
        ("cu_count", ctypes.c_uint32), ("vram_bytes", ctypes.c_uint64),
        ("unique_id", ctypes.c_uint64), ("hive_id", ctypes.c_uint64),
        ("max_engine_clk_mhz", ctypes.c_uint32), ("num_xgmi_links", ctypes.c_int),
        ("product", ctypes.c_char * 48), ("uuid", ctypes.c_char * 40),
    ]


class _Link(ctypes.Structure):
    _fields_ = [("from_index", ctypes.c_int), ("to_index", ctypes.c_int), ("type", ctypes.c_int),
                ("weight", ctypes.c_uint32), ("min_bandwidth_mbps", ctypes.c_uint32),
                ("max_bandwidth_mbps", ctypes.c_uint32)]


class _Sample(ctypes.Structure):
    _fields_ = [
        ("index", ctypes.c_int), ("valid", ctypes.c_int),
        ("gfx_activity_pct", ctypes.c_uint32), ("umc_activity_pct", ctypes.c_uint32),
        ("vram_used_bytes", ctypes.c_uint64), ("vram_total_bytes", ctypes.c_uint64),
        ("temp_edge_mc", ctypes.c_int64), ("temp_hotspot_mc", ctypes.c_int64),
        ("temp_mem_mc", ctypes.c_int64), ("power_w", ctypes.c_uint64),
        ("power_limit_w", ctypes.c_uint32), ("sclk_mhz", ctypes.c_uint32),
        ("mclk_mhz", ctypes.c_uint32), ("ecc_correctable", ctypes.c_uint64),
        ("ecc_uncorrectable", ctypes.c_uint64), ("num_processes", ctypes.c_uint32),
        ("bdf", ctypes.c_char * 20),
    ]


@dataclasses.dataclass(frozen=True)
class GpuInfo:
    index: int
    kfd_node: int
    gpu_id: int
    gfx_target_version: int
    arch: str
    render_minor: int
    card: int
    vendor_id: int
    device_id: int
    bdf: str
    numa_node: int
    simd_count: int
    cu_count: int
    vram_bytes: int
    unique_id: int
    hive_id: int
    max_sclk_mhz: int
    xgmi_links: int
    product: str
    uuid: str

    @property
    def render_path(self) -> str:
        return f"/dev/dri/renderD{self.render_minor}"

    @property
    def card_path(self) -> Optional[str]:
        return None if self.card < 0 else f"/dev/dri/card{self.card}"

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


@dataclasses.dataclass(frozen=True)
class Link:
    from_index: int
    to_index: int
    type: int
    weight: int
    max_bandwidth_mbps: int

    @property
    def is_xgmi(self) -> bool:
        return self.type == LINK_XGMI


@dataclasses.dataclass
class GpuSample:
    index: int
    valid: bool
    gfx_activity_pct: int
    umc_activity_pct: int
    vram_used_bytes: int
    vram_total_bytes: int
    temp_edge_c: Optional[float]
    temp_hotspot_c: Optional[float]
    temp_mem_c: Optional[float]
    power_w: int
    power_limit_w: int
    sclk_mhz: int
    mclk_mhz: int
    ecc_correctable: int
    ecc_uncorrectable: int
    num_processes: int
    bdf: str


class NodeLibraryMissing(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(NODE_LIB_PATH):
                raise NodeLibraryMissing(f"{NODE_LIB_PATH} not built: run `make node`")
            L = ctypes.CDLL(NODE_LIB_PATH)
            cp, sz, i = ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int
            ip = ctypes.POINTER(ctypes.c_int)
            L.mx_version.restype = cp
            L.mx_enumerate.argtypes = [cp, ctypes.POINTER(_GpuInfo), i, cp, sz]
            L.mx_enumerate.restype = i
            L.mx_links.argtypes = [cp, ctypes.POINTER(_Link), i, cp, sz]
            L.mx_links.restype = i
            L.mx_cdi_spec.argtypes = [cp, cp, cp, sz, cp, sz]
            L.mx_cdi_spec.restype = ctypes.c_long
            L.mx_preferred_allocation.argtypes = [cp, ip, i, ip, i, i, ip, cp, sz]
            L.mx_preferred_allocation.restype = i
            L.mx_preferred_allocation_topo.argtypes = [i, ip, ctypes.POINTER(ctypes.c_uint64), ip,
                                                       ip, i, ip, i, i, ip]
            L.mx_preferred_allocation_topo.restype = i
            L.mx_health_check.argtypes = [cp, i, cp]
            L.mx_health_check.restype = i
            L.mx_health_reason.argtypes = [i]
            L.mx_health_reason.restype = cp
            L.mx_smi_open.argtypes = [cp, sz]
            L.mx_smi_open.restype = i
            L.mx_smi_count.restype = i
            L.mx_smi_sample.argtypes = [i, ctypes.POINTER(_Sample)]
            L.mx_smi_sample.restype = i
            L.mx_smi_wait_events.argtypes = [i, ip, ip, i]
            L.mx_smi_wait_events.restype = i
            L.mx_smi_driver_version.restype = cp
            _lib = L
    return _lib


def _root(root: Optional[str]) -> bytes:
    return (root or "").encode()


def version() -> str:
    return lib().mx_version().decode()


def enumerate_gpus(root: Optional[str] = None) -> list[GpuInfo]:
    arr = (_GpuInfo * MAX_GPUS)()
    err = ctypes.create_string_buffer(512)
    n = lib().mx_enumerate(_root(root), arr, MAX_GPUS, err, len(err))
    if n < 0:
        raise RuntimeError(err.value.decode())
    out = []
    for k in range(min(n, MAX_GPUS)):
        g = arr[k]
        out.append(GpuInfo(
            index=g.index, kfd_node=g.kfd_node, gpu_id=g.gpu_id,
            gfx_target_version=g.gfx_target_version, arch=g.gfx_arch.decode(),
            render_minor=g.drm_render_minor, card=g.drm_card, vendor_id=g.vendor_id,
            device_id=g.device_id, bdf=g.pci_bdf.decode(), numa_node=g.numa_node,
            simd_count=g.simd_count, cu_count=g.cu_count, vram_bytes=g.vram_bytes,
            unique_id=g.unique_id, hive_id=g.hive_id, max_sclk_mhz=g.max_engine_clk_mhz,
            xgmi_links=g.num_xgmi_links, product=g.product.decode(), uuid=g.uuid.decode()))
    return out


def links(root: Optional[str] = None) -> list[Link]:
    cap = MAX_GPUS * MAX_LINKS
    arr = (_Link * cap)()
    err = ctypes.create_string_buffer(512)
    n = lib().mx_links(_root(root), arr, cap, err, len(err))
    if n < 0:
        raise RuntimeError(err.value.decode())
    return [Link(arr[k].from_index, arr[k].to_index, arr[k].type, arr[k].weight,
                 arr[k].max_bandwidth_mbps) for k in range(n)]


def cdi_spec(root: Optional[str] = None, kind: str = "amd.com/gpu") -> dict:
    err = ctypes.create_string_buffer(512)
    need = lib().mx_cdi_spec(_root(root), kind.encode(), None, 0, err, len(err))
    if need < 0:
        raise RuntimeError(err.value.decode())
    buf = ctypes.create_string_buffer(need + 1)
    lib().mx_cdi_spec(_root(root), kind.encode(), buf, need + 1, err, len(err))
    return json.loads(buf.value.decode())


def _iarr(vals):
    vals = list(vals)
    return (ctypes.c_int * max(1, len(vals)))(*vals), len(vals)


def preferred_allocation(available, must_include, size: int, root: Optional[str] = None) -> list[int]:
    a, na = _iarr(available)
    m, nm = _iarr(must_include)
    out = (ctypes.c_int * max(1, size))()
    err = ctypes.create_string_buffer(512)
    r = lib().mx_preferred_allocation(_root(root), a, na, m, nm, size, out, err, len(err))
    if r < 0:
        raise ValueError(err.value.decode() or "invalid allocation request")
    return list(out[:size])


def preferred_allocation_topo(numa, hive, xgmi_adj, available, must_include, size: int) -> list[int]:
    n = len(numa)
    na_, _ = _iarr(numa)
    hv = (ctypes.c_uint64 * max(1, n))(*hive)
    flat = [int(bool(xgmi_adj[i][j])) for i in range(n) for j in range(n)]
    adj, _ = _iarr(flat)
    a, na = _iarr(available)
    m, nm = _iarr(must_include)
    out = (ctypes.c_int * max(1, size))()
    r = lib().mx_preferred_allocation_topo(n, na_, hv, adj, a, na, m, nm, size, out)
    if r < 0:
        raise ValueError("invalid allocation request")
    return list(out[:size])


def health_check(index: int, root: Optional[str] = None, fault_file: Optional[str] = None) -> int:
    return lib().mx_health_check(_root(root), index, (fault_file or "").encode())


def health_reason(code: int) -> str:
    return lib().mx_health_reason(code).decode()


# ---- amd-smi ----

def smi_open() -> tuple[bool, str]:
    err = ctypes.create_string_buffer(512)
    ok = bool(lib().mx_smi_open(err, len(err)))
    return ok, err.value.decode()


def smi_count() -> int:
    return lib().mx_smi_count()


def smi_driver_version() -> str:
    return lib().mx_smi_driver_version().decode()


def smi_sample(i: int) -> GpuSample:
    s = _Sample()
    lib().mx_smi_sample(i, ctypes.byref(s))

    def t(v):
        return None if v == -(2 ** 63) else v / 1000.0
    return GpuSample(index=s.index, valid=bool(s.valid), gfx_activity_pct=s.gfx_activity_pct,
                     umc_activity_pct=s.umc_activity_pct, vram_used_bytes=s.vram_used_bytes,
                     vram_total_bytes=s.vram_total_bytes, temp_edge_c=t(s.temp_edge_mc),
                     temp_hotspot_c=t(s.temp_hotspot_mc), temp_mem_c=t(s.temp_mem_mc),
                     power_w=s.power_w, power_limit_w=s.power_limit_w, sclk_mhz=s.sclk_mhz,
                     mclk_mhz=s.mclk_mhz, ecc_correctable=s.ecc_correctable,
                     ecc_uncorrectable=s.ecc_uncorrectable, num_processes=s.num_processes,
                     bdf=s.bdf.decode())


def smi_wait_events(timeout_ms: int, max_events: int = 32) -> list[tuple[int, int]]:
    g = (ctypes.c_int * max_events)()
    e = (ctypes.c_int * max_events)()
    n = lib().mx_smi_wait_events(timeout_ms, g, e, max_events)
    if n < 0:
        return []
    return [(g[k], e[k]) for k in range(n)]
