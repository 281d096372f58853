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
        ("partition", ctypes.c_int), ("partitions", ctypes.c_int), ("num_xcc", ctypes.c_uint32),
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
        ("bdf", ctypes.c_char * 20), ("partition_id", ctypes.c_int),
        ("energy_j", ctypes.c_double),
    ]


class _HealthOpts(ctypes.Structure):
    _fields_ = [("root", ctypes.c_char_p), ("fault_file", ctypes.c_char_p),
                ("state_dir", ctypes.c_char_p), ("boot_id_file", ctypes.c_char_p),
                ("event_quarantine_ms", ctypes.c_int), ("ecc_quarantine_ms", ctypes.c_int),
                ("use_smi", ctypes.c_int)]


class _HealthStatus(ctypes.Structure):
    _fields_ = [("index", ctypes.c_int), ("code", ctypes.c_int), ("smi_index", ctypes.c_int),
                ("ecc_valid", ctypes.c_int), ("ecc_uncorrectable", ctypes.c_uint64),
                ("ecc_baseline", ctypes.c_uint64), ("vm_faults", ctypes.c_uint64),
                ("thermal_throttles", ctypes.c_uint64), ("resets", ctypes.c_uint64),
                ("quarantine_left_ms", ctypes.c_int64), ("bdf", ctypes.c_char * 20)]


class _HealthEvent(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_uint64), ("index", ctypes.c_int), ("kind", ctypes.c_int),
                ("value", ctypes.c_int64), ("unix_ms", ctypes.c_int64),
                ("message", ctypes.c_char * 96)]


class _XgmiLink(ctypes.Structure):
    _fields_ = [("link", ctypes.c_int), ("status", ctypes.c_int), ("link_type", ctypes.c_int),
                ("has_traffic", ctypes.c_int), ("peer_bdf", ctypes.c_char * 20),
                ("bit_rate_gbps", ctypes.c_uint32), ("max_bandwidth_gbps", ctypes.c_uint32),
                ("read_kb", ctypes.c_uint64), ("write_kb", ctypes.c_uint64)]


class _Proc(ctypes.Structure):
    _fields_ = [("pid", ctypes.c_uint32), ("cu_occupancy", ctypes.c_uint32),
                ("name", ctypes.c_char * 64), ("container", ctypes.c_char * 64),
                ("vram_bytes", ctypes.c_uint64), ("gtt_bytes", ctypes.c_uint64)]


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
    partition: int = 0          # compute partition of its PCI device (DPX..CPX), 0 in SPX
    partitions: int = 1         # partitions the PCI device is split into
    num_xcc: int = 0

    @property
    def key(self) -> str:
        """Stable per-device key: the BDF, plus the partition in DPX..CPX mode."""
        return self.bdf if self.partition == 0 else f"{self.bdf}#{self.partition}"

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
    partition_id: int = 0
    energy_j: Optional[float] = None    # accumulated since driver load; None if unsupported

    @property
    def key(self) -> str:
        return self.bdf if self.partition_id == 0 else f"{self.bdf}#{self.partition_id}"


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
            L.mx_smi_xgmi_links.argtypes = [i, ctypes.POINTER(_XgmiLink), i]
            L.mx_smi_xgmi_links.restype = i
            L.mx_smi_processes.argtypes = [i, ctypes.POINTER(_Proc), i]
            L.mx_smi_processes.restype = i
            L.mx_smi_close.restype = None
            L.mx_smi_reset.restype = None
            L.mx_smi_reinit.argtypes = [cp, sz]
            L.mx_smi_reinit.restype = i
            L.mx_smi_generation.restype = ctypes.c_uint64
            vp = ctypes.c_void_p
            L.mx_hm_create.argtypes = [ctypes.POINTER(_HealthOpts), cp, sz]
            L.mx_hm_create.restype = vp
            L.mx_hm_destroy.argtypes = [vp]
            L.mx_hm_destroy.restype = None
            L.mx_hm_smi_active.argtypes = [vp]
            L.mx_hm_smi_active.restype = i
            L.mx_hm_step.argtypes = [vp, i]
            L.mx_hm_step.restype = i
            L.mx_hm_status.argtypes = [vp, ctypes.POINTER(_HealthStatus), i]
            L.mx_hm_status.restype = i
            L.mx_hm_events.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(_HealthEvent), i]
            L.mx_hm_events.restype = i
            L.mx_hm_write_state.argtypes = [vp, cp]
            L.mx_hm_write_state.restype = i
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
            xgmi_links=g.num_xgmi_links, product=g.product.decode(), uuid=g.uuid.decode(),
            partition=g.partition, partitions=g.partitions, num_xcc=g.num_xcc))
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


def cdi_spec_text(root: Optional[str] = None, kind: str = "amd.com/gpu") -> str:
    """The CDI spec exactly as ``mx-cdi-gen`` writes it."""
    err = ctypes.create_string_buffer(512)
    need = lib().mx_cdi_spec(_root(root), kind.encode(), None, 0, err, len(err))
    if need < 0:
        raise RuntimeError(err.value.decode())
    buf = ctypes.create_string_buffer(need + 1)
    lib().mx_cdi_spec(_root(root), kind.encode(), buf, need + 1, err, len(err))
    return buf.value.decode()


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
                     bdf=s.bdf.decode(), partition_id=s.partition_id,
                     energy_j=s.energy_j if s.energy_j >= 0 else None)


def smi_wait_events(timeout_ms: int, max_events: int = 32) -> list[tuple[int, int]]:
    g = (ctypes.c_int * max_events)()
    e = (ctypes.c_int * max_events)()
    n = lib().mx_smi_wait_events(timeout_ms, g, e, max_events)
    if n < 0:
        return []
    return [(g[k], e[k]) for k in range(n)]


def smi_close() -> None:
    """Release one reference on the process's amd-smi session."""
    lib().mx_smi_close()


def smi_reset() -> None:
    """End the amd-smi session whatever its reference count (tests)."""
    lib().mx_smi_reset()


def smi_reinit() -> tuple[bool, str]:
    """amdsmi_shut_down + amdsmi_init on the open session: new handles for a
    changed GPU set (compute-partition change, driver reload)."""
    err = ctypes.create_string_buffer(512)
    ok = bool(lib().mx_smi_reinit(err, len(err)))
    return ok, err.value.decode()


def smi_generation() -> int:
    """Changes on every amd-smi (re)init; cached amd-smi indices are void then."""
    return int(lib().mx_smi_generation())


@dataclasses.dataclass(frozen=True)
class XgmiLink:
    link: int
    status: str                   # "up" / "down" / "disabled" / "unknown"
    link_type: int
    peer_bdf: str
    bit_rate_gbps: int
    max_bandwidth_gbps: int
    read_bytes: Optional[int]     # cumulative; None when amd-smi has no traffic counters
    write_bytes: Optional[int]


_LINK_STATUS = {0: "down", 1: "up", 2: "disabled"}


def smi_xgmi_links(i: int) -> Optional[list[XgmiLink]]:
    """xGMI link state + cumulative traffic of amd-smi GPU ``i``; None when
    amd-smi supports neither query here."""
    arr = (_XgmiLink * 64)()
    n = lib().mx_smi_xgmi_links(i, arr, 64)
    if n < 0:
        return None
    out = []
    for k in range(n):
        a = arr[k]
        out.append(XgmiLink(link=a.link, status=_LINK_STATUS.get(a.status, "unknown"),
                            link_type=a.link_type, peer_bdf=a.peer_bdf.decode(),
                            bit_rate_gbps=a.bit_rate_gbps, max_bandwidth_gbps=a.max_bandwidth_gbps,
                            read_bytes=a.read_kb * 1024 if a.has_traffic else None,
                            write_bytes=a.write_kb * 1024 if a.has_traffic else None))
    return out


@dataclasses.dataclass(frozen=True)
class GpuProcess:
    pid: int
    name: str
    container: str
    vram_bytes: int
    gtt_bytes: int
    cu_occupancy: int


def smi_processes(i: int, max_procs: int = 256) -> list[GpuProcess]:
    arr = (_Proc * max_procs)()
    n = lib().mx_smi_processes(i, arr, max_procs)
    return [GpuProcess(pid=arr[k].pid, name=arr[k].name.decode(errors="replace"),
                       container=arr[k].container.decode(errors="replace"),
                       vram_bytes=arr[k].vram_bytes, gtt_bytes=arr[k].gtt_bytes,
                       cu_occupancy=arr[k].cu_occupancy) for k in range(max(0, n))]


# ---- N02 health monitor ----

EVT_VMFAULT = 1
EVT_THERMAL_THROTTLE = 2
EVT_GPU_PRE_RESET = 3
EVT_GPU_POST_RESET = 4
EVT_ECC_UNCORRECTABLE = 100
EVT_HEALTH_CHANGE = 101
EVENT_NAMES = {EVT_VMFAULT: "vm_fault", EVT_THERMAL_THROTTLE: "thermal_throttle",
               EVT_GPU_PRE_RESET: "gpu_pre_reset", EVT_GPU_POST_RESET: "gpu_post_reset",
               EVT_ECC_UNCORRECTABLE: "ecc_uncorrectable", EVT_HEALTH_CHANGE: "health_change"}


@dataclasses.dataclass(frozen=True)
class HealthStatus:
    index: int
    code: int
    reason: str
    smi_index: int
    ecc_valid: bool
    ecc_uncorrectable: int
    ecc_baseline: int
    vm_faults: int
    thermal_throttles: int
    resets: int
    quarantine_left_ms: int
    bdf: str

    @property
    def healthy(self) -> bool:
        return self.code == HEALTHY


@dataclasses.dataclass(frozen=True)
class HealthEvent:
    seq: int
    index: int
    kind: int
    value: int
    unix_ms: int
    message: str

    @property
    def name(self) -> str:
        return EVENT_NAMES.get(self.kind, f"event_{self.kind}")


class HealthMonitor:
    """The C++ N02 state machine (``native/libmxnode/monitor.cc``)."""

    def __init__(self, root: Optional[str] = None, fault_file: Optional[str] = None,
                 state_dir: Optional[str] = None, event_quarantine_s: float = 60.0,
                 ecc_quarantine_s: float = 0.0, use_smi: bool = True,
                 boot_id_file: Optional[str] = None):
        self._keep = [(root or "").encode(), (fault_file or "").encode(),
                      (state_dir or "").encode(), (boot_id_file or "").encode()]
        opts = _HealthOpts(self._keep[0], self._keep[1], self._keep[2] or None,
                           self._keep[3] or None, int(event_quarantine_s * 1000),
                           int(ecc_quarantine_s * 1000), int(use_smi))
        err = ctypes.create_string_buffer(512)
        self._h = lib().mx_hm_create(ctypes.byref(opts), err, len(err))
        if not self._h:
            raise RuntimeError(err.value.decode() or "mx_hm_create failed")
        self._seq = 0

    @property
    def smi_active(self) -> bool:
        return bool(lib().mx_hm_smi_active(self._h))

    def step(self, wait_ms: int = 0) -> int:
        return lib().mx_hm_step(self._h, int(wait_ms))

    def status(self) -> list[HealthStatus]:
        arr = (_HealthStatus * MAX_GPUS)()
        n = lib().mx_hm_status(self._h, arr, MAX_GPUS)
        return [HealthStatus(index=a.index, code=a.code, reason=health_reason(a.code),
                             smi_index=a.smi_index, ecc_valid=bool(a.ecc_valid),
                             ecc_uncorrectable=a.ecc_uncorrectable, ecc_baseline=a.ecc_baseline,
                             vm_faults=a.vm_faults, thermal_throttles=a.thermal_throttles,
                             resets=a.resets, quarantine_left_ms=a.quarantine_left_ms,
                             bdf=a.bdf.decode()) for a in arr[:max(0, n)]]

    def new_events(self) -> list[HealthEvent]:
        """Events since the previous call (oldest first)."""
        arr = (_HealthEvent * 256)()
        n = lib().mx_hm_events(self._h, self._seq, arr, 256)
        out = [HealthEvent(seq=a.seq, index=a.index, kind=a.kind, value=a.value,
                           unix_ms=a.unix_ms, message=a.message.decode(errors="replace"))
               for a in arr[:max(0, n)]]
        if out:
            self._seq = out[-1].seq
        return out

    def write_state(self, path: str) -> bool:
        return lib().mx_hm_write_state(self._h, path.encode()) == 0

    def close(self) -> None:
        if self._h:
            lib().mx_hm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
