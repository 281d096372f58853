"""amd-smi Prometheus exporter on :9400 — the DCGM-exporter counterpart.

The reference stack's GPU Operator runs dcgm-exporter (DCGM_FI_DEV_GPU_UTIL,
_FB_USED, _GPU_TEMP, _POWER_USAGE, ... [ext]).  This exporter
samples amd-smi through ``libmxnode`` (C++, dlopen'ed amd-smi) on a
background thread and serves the latest snapshot, so scrapes never touch the
driver:

  amd_gpu_utilization_percent            amd_gpu_memory_activity_percent
  amd_gpu_memory_used_bytes              amd_gpu_memory_total_bytes
  amd_gpu_temperature_celsius{sensor}    amd_gpu_power_watts / _power_limit_watts
  amd_gpu_clock_mhz{type=sclk|mclk}      amd_gpu_ecc_errors_total{type}
  amd_gpu_processes                      amd_gpu_xgmi_links
  amd_gpu_topology_link{peer,type}       amd_gpu_link_max_bandwidth_bytes{peer,type}
  amd_gpu_xgmi_link_up{link,status}     (live amd-smi xGMI link state)
  amd_gpu_xgmi_read_bytes_total / _write_bytes_total{peer_bdf}
  amd_gpu_xgmi_link_bitrate_gbps{peer_bdf}
  amd_gpu_process_memory_bytes{pid,process,pod_uid,...}  (per-process VRAM)
  amd_gpu_pod_info{namespace,pod,container}  amd_gpu_pods (time-sliced owners)
  amd_gpu_device_healthy{source,reason}  (the device plugin's own verdict)
  amd_gpu_vm_faults_total / _resets_total / _thermal_throttle_events_total
  amd_gpu_info{arch,product,uuid,bdf,...}
  amd_gpu_stack_component_up{component}  amd_gpu_exporter_sample_seconds

Per-GPU labels: gpu, bdf, uuid and — through the kubelet PodResources API —
namespace, pod, container of the workload the GPU is allocated to (when a
time-sliced GPU has several owners, one amd_gpu_pod_info series per owner).
Health is read from the device plugin's ``health.json`` (same verdicts as
ListAndWatch, including amd-smi quarantines and ECC) when it is fresh, and
falls back to the stateless sysfs check otherwise.
"""
from __future__ import annotations

import dataclasses
import http.server
import json
import logging
import os
import threading
import time
from typing import Callable, Optional

from ..native import node

log = logging.getLogger("mxk8s.exporter")


def _esc(v) -> str:
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


class MetricWriter:
    def __init__(self):
        self.lines: list[str] = []
        self._declared = set()

    def add(self, name: str, mtype: str, help_: str, value, labels: Optional[dict] = None):
        if value is None:
            return
        if name not in self._declared:
            self.lines.append(f"# HELP {name} {help_}")
            self.lines.append(f"# TYPE {name} {mtype}")
            self._declared.add(name)
        lab = ""
        if labels:
            lab = "{" + ",".join(f'{k}="{_esc(v)}"' for k, v in labels.items()) + "}"
        if isinstance(value, float):
            val = repr(value)
        else:
            val = str(int(value)) if isinstance(value, bool) else str(value)
        self.lines.append(f"{name}{lab} {val}")

    def text(self) -> str:
        return "\n".join(self.lines) + "\n"


class SmiBackend:
    """Real backend: libmxnode topology + amd-smi samples, matched by BDF (and
    partition id: the partitions of a device share its BDF).

    amd-smi enumerates at init, so after a compute-partition change (SPX ->
    CPX: 8 -> 64 KFD GPUs) or a driver reload the open session still lists
    the old handles: when the KFD and amd-smi GPU counts disagree the backend
    re-initialises amd-smi, and it re-maps its indices whenever the session's
    generation changes (re-initialised by this or another user)."""

    def __init__(self, sysfs_root: str = ""):
        self.sysfs_root = sysfs_root
        self.ok, self.err = node.smi_open()
        self.driver = node.smi_driver_version() if self.ok else ""
        self._smi_index: dict[str, int] = {}
        self._gen = node.smi_generation() if self.ok else 0
        self.reinits = 0

    def gpus(self) -> list[node.GpuInfo]:
        return node.enumerate_gpus(self.sysfs_root)

    def _refresh(self) -> None:
        n_kfd = len(node.enumerate_gpus(self.sysfs_root))
        if node.smi_count() != n_kfd:
            ok, err = node.smi_reinit()
            self.reinits += 1
            if not ok:
                self.err = err
            self.driver = node.smi_driver_version()
        gen = node.smi_generation()
        if gen != self._gen:
            self._gen = gen
            self._smi_index.clear()

    def samples(self) -> dict[str, node.GpuSample]:
        if not self.ok:
            return {}
        self._refresh()
        out = {}
        for i in range(max(0, node.smi_count())):
            s = node.smi_sample(i)
            if s.valid:
                out[s.key] = s
                self._smi_index[s.key] = i
        return out

    def xgmi(self, key: str) -> Optional[list]:
        i = self._smi_index.get(key)
        return None if i is None else node.smi_xgmi_links(i)

    def processes(self, key: str) -> list:
        i = self._smi_index.get(key)
        return [] if i is None else node.smi_processes(i)

    def close(self) -> None:
        if self.ok:
            node.smi_close()
            self.ok = False

    def health(self, index: int) -> int:
        return node.health_check(index, self.sysfs_root, os.environ.get("MXK8S_FAULT_FILE"))

    def links(self) -> list:
        return node.links(self.sysfs_root)


def pod_uid_of(pid: int, proc_root: str = "/proc") -> Optional[str]:
    """Kubernetes pod UID of a host PID from its cgroup path
    (``.../kubepods-besteffort-pod<uid>.slice/...`` or ``.../pod<uid>/...``)."""
    try:
        with open(os.path.join(proc_root, str(pid), "cgroup")) as f:
            text = f.read()
    except OSError:
        return None
    for part in text.replace("\n", "/").split("/"):
        seg = part.rsplit("-", 1)[-1] if part.endswith(".slice") else part
        seg = seg[:-6] if seg.endswith(".slice") else seg
        if seg.startswith("pod") and len(seg) >= 35:
            return seg[3:].replace("_", "-")
    return None


def load_health_state(path: Optional[str], max_age_s: float = 120.0) -> Optional[dict]:
    """The device plugin's verdicts (``<state_dir>/health.json``), by BDF, or
    None when missing or stale (plugin down: fall back to sysfs)."""
    if not path:
        return None
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    if time.time() * 1000 - float(doc.get("unix_ms", 0)) > max_age_s * 1000:
        return None
    return {(g["bdf"] if not g.get("partition") else f'{g["bdf"]}#{g["partition"]}'): g
            for g in doc.get("gpus", [])}


def _owner_list(v) -> list:
    if not v:
        return []
    return [tuple(v)] if isinstance(v, tuple) else [tuple(o) for o in v]


def render_metrics(gpus, samples: dict, health: Callable[[int], int], owners: dict,
                   driver: str, components: dict, sample_seconds: float,
                   links: Optional[list] = None, plugin_health: Optional[dict] = None,
                   xgmi: Optional[Callable[[str], Optional[list]]] = None,
                   processes: Optional[Callable[[str], list]] = None,
                   pod_uid: Callable[[int], Optional[str]] = pod_uid_of) -> str:
    w = MetricWriter()
    by_gpu: dict = {}
    for l in links or []:
        by_gpu.setdefault(l.from_index, []).append(l)
    for g in gpus:
        base = {"gpu": str(g.index), "bdf": g.bdf, "uuid": g.uuid}
        if g.partitions > 1:
            base["partition"] = str(g.partition)
        own = _owner_list(owners.get(str(g.index)))
        if len(own) == 1:     # unambiguous: label every series (dcgm-exporter style)
            base.update(namespace=own[0][0], pod=own[0][1], container=own[0][2])
        for ns, pod, ctr in own:
            w.add("amd_gpu_pod_info", "gauge", "One series per container the GPU is allocated to.",
                  1, {"gpu": str(g.index), "bdf": g.bdf, "uuid": g.uuid, "namespace": ns,
                      "pod": pod, "container": ctr})
        w.add("amd_gpu_pods", "gauge", "Containers the GPU is allocated to (time-slicing: > 1).",
              len(own), {"gpu": str(g.index), "bdf": g.bdf, "uuid": g.uuid})
        w.add("amd_gpu_info", "gauge", "Static GPU facts (value is always 1).", 1,
              {**base, "arch": g.arch, "product": g.product, "device_id": f"0x{g.device_id:04x}",
               "driver_version": driver, "numa_node": str(g.numa_node)})
        ph = (plugin_health or {}).get(g.key)
        if ph is not None:
            w.add("amd_gpu_device_healthy", "gauge",
                  "1 if the device plugin reports the GPU Healthy in ListAndWatch.",
                  1 if ph.get("healthy") else 0,
                  {**base, "source": "device-plugin", "reason": ph.get("reason", "")})
            for key, name, help_ in (("vm_faults", "amd_gpu_vm_faults_total", "amd-smi VM-fault events."),
                                     ("resets", "amd_gpu_resets_total", "amd-smi GPU pre-reset events."),
                                     ("thermal_throttles", "amd_gpu_thermal_throttle_events_total",
                                      "amd-smi thermal-throttle events.")):
                w.add(name, "counter", help_ + " (device plugin, this boot)", int(ph.get(key, 0)), base)
            w.add("amd_gpu_quarantine_seconds", "gauge",
                  "Time left in the device plugin's event/ECC quarantine (s).",
                  float(ph.get("quarantine_left_ms", 0)) / 1000.0, base)
        else:
            h = health(g.index)
            w.add("amd_gpu_device_healthy", "gauge",
                  "1 if the device plugin reports the GPU Healthy in ListAndWatch.",
                  1 if h == 0 else 0, {**base, "source": "sysfs", "reason": node.health_reason(h)})
        w.add("amd_gpu_xgmi_links", "gauge", "xGMI links of the GPU (KFD topology).", g.xgmi_links, base)
        for l in by_gpu.get(g.index, []):
            kind = "xgmi" if l.is_xgmi else "pcie" if l.type == node.LINK_PCIE else str(l.type)
            peer = str(l.to_index) if l.to_index >= 0 else "cpu"
            lab = {**base, "peer": peer, "type": kind}
            w.add("amd_gpu_topology_link", "gauge", "1 for every GPU link in the KFD topology.", 1, lab)
            if l.max_bandwidth_mbps:
                w.add("amd_gpu_link_max_bandwidth_bytes", "gauge",
                      "Link bandwidth advertised by KFD (bytes/s).",
                      int(l.max_bandwidth_mbps) * 125000, lab)
        live = xgmi(g.key) if xgmi else None
        # amd-smi reports link state per link slot and traffic per peer; the
        # two lists are not aligned (a slot can be disabled, the metrics can
        # carry an all-ones placeholder peer), so each series keeps its own key
        for x in live or []:
            if x.status != "unknown":
                w.add("amd_gpu_xgmi_link_up", "gauge",
                      "Live xGMI link state from amd-smi (1 up, 0 down or disabled).",
                      1 if x.status == "up" else 0, {**base, "link": str(x.link), "status": x.status})
            if x.read_bytes is None or not x.peer_bdf or x.peer_bdf.startswith("ffff"):
                continue
            lab = {**base, "peer_bdf": x.peer_bdf}
            w.add("amd_gpu_xgmi_read_bytes_total", "counter",
                  "Bytes received from the peer over xGMI (amd-smi link metrics).", x.read_bytes, lab)
            w.add("amd_gpu_xgmi_write_bytes_total", "counter",
                  "Bytes sent to the peer over xGMI (amd-smi link metrics).", x.write_bytes, lab)
            if x.bit_rate_gbps:
                w.add("amd_gpu_xgmi_link_bitrate_gbps", "gauge", "Current xGMI link speed (Gb/s).",
                      x.bit_rate_gbps, lab)
        for pr in (processes(g.key) if processes else []):
            lab = {**base, "pid": str(pr.pid), "process": pr.name}
            uid = pod_uid(pr.pid)
            if uid:
                lab["pod_uid"] = uid
            w.add("amd_gpu_process_memory_bytes", "gauge", "VRAM held by a process (bytes).",
                  pr.vram_bytes, lab)
        s = samples.get(g.key)
        if s is None:
            continue
        w.add("amd_gpu_utilization_percent", "gauge", "GFX engine activity (%).", s.gfx_activity_pct, base)
        w.add("amd_gpu_memory_activity_percent", "gauge", "Memory controller activity (%).",
              s.umc_activity_pct, base)
        w.add("amd_gpu_memory_used_bytes", "gauge", "VRAM in use (bytes).", s.vram_used_bytes, base)
        w.add("amd_gpu_memory_total_bytes", "gauge", "VRAM size (bytes).", s.vram_total_bytes, base)
        for sensor, val in (("edge", s.temp_edge_c), ("hotspot", s.temp_hotspot_c), ("memory", s.temp_mem_c)):
            if val is not None:
                w.add("amd_gpu_temperature_celsius", "gauge", "Temperature by sensor (C).",
                      float(val), {**base, "sensor": sensor})
        w.add("amd_gpu_power_watts", "gauge", "Socket power (W).", s.power_w, base)
        w.add("amd_gpu_power_limit_watts", "gauge", "Power cap (W).", s.power_limit_w, base)
        if getattr(s, "energy_j", None) is not None:
            w.add("amd_gpu_energy_joules_total", "counter",
                  "Energy consumed since the driver loaded (J, amd-smi accumulator).",
                  round(s.energy_j, 3), base)
        w.add("amd_gpu_clock_mhz", "gauge", "Current clock (MHz).", s.sclk_mhz, {**base, "type": "sclk"})
        w.add("amd_gpu_clock_mhz", "gauge", "Current clock (MHz).", s.mclk_mhz, {**base, "type": "mclk"})
        w.add("amd_gpu_ecc_errors_total", "counter", "Accumulated ECC errors.", s.ecc_correctable,
              {**base, "type": "correctable"})
        w.add("amd_gpu_ecc_errors_total", "counter", "Accumulated ECC errors.", s.ecc_uncorrectable,
              {**base, "type": "uncorrectable"})
        w.add("amd_gpu_processes", "gauge", "Processes with a KFD context on the GPU.",
              s.num_processes, base)
    for comp, up in sorted(components.items()):
        w.add("amd_gpu_stack_component_up", "gauge", "1 if the stack component is healthy.",
              1 if up else 0, {"component": comp})
    w.add("amd_gpu_exporter_sample_seconds", "gauge", "Time the last sample took (s).",
          float(sample_seconds))
    return w.text()


@dataclasses.dataclass
class ExporterConfig:
    port: int = 9400
    interval: float = 5.0
    pod_resources_socket: Optional[str] = None
    plugin_socket: str = "/var/lib/kubelet/device-plugins/amd-gpu.sock"
    cdi_spec: str = "/etc/cdi/amd.com-gpu.json"
    resource_name: str = "amd.com/gpu"
    health_state_file: Optional[str] = None   # the device plugin's <state_dir>/health.json
    sysfs_root: str = ""
    pod_resources: bool = True
    state_dir: Optional[str] = None            # node-validator markers: <state_dir>/validations
    validation_steps: tuple = ("driver", "cdi", "vectoradd", "plugin")


class Exporter:
    def __init__(self, cfg: ExporterConfig, backend=None):
        self.cfg = cfg
        self.backend = backend or SmiBackend(cfg.sysfs_root)
        self._text = "# no sample yet\n"
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._httpd: Optional[http.server.ThreadingHTTPServer] = None
        self.samples_taken = 0

    def validations(self) -> dict:
        """{step: marker valid for this boot + driver instance} (empty when
        no state dir is configured)."""
        if not self.cfg.state_dir:
            return {}
        from ..validate import node as vnode
        return vnode.status(self.cfg.state_dir, self.cfg.sysfs_root, self.cfg.validation_steps)

    def components(self) -> dict:
        c = {"amd_smi": bool(getattr(self.backend, "ok", True))}
        c["device_plugin"] = os.path.exists(self.cfg.plugin_socket)
        c["cdi_spec"] = os.path.exists(self.cfg.cdi_spec)
        v = self.validations()
        if v:
            c["validation"] = all(v.values())
        return c

    def sample_once(self) -> str:
        t0 = time.perf_counter()
        gpus = self.backend.gpus()
        samples = self.backend.samples()
        owners = {}
        if (self.cfg.pod_resources and self.cfg.pod_resources_socket
                and os.path.exists(self.cfg.pod_resources_socket)):
            try:
                from .podresources import gpu_owners
                owners = gpu_owners(self.cfg.pod_resources_socket, self.cfg.resource_name)
            except Exception as e:   # kubelet busy/old: metrics without pod labels
                log.debug("pod-resources unavailable: %s", e)
        links_fn = getattr(self.backend, "links", None)
        links = links_fn() if links_fn else []
        text = render_metrics(gpus, samples, self.backend.health, owners,
                              getattr(self.backend, "driver", ""), self.components(),
                              time.perf_counter() - t0, links,
                              plugin_health=load_health_state(self.cfg.health_state_file),
                              xgmi=getattr(self.backend, "xgmi", None),
                              processes=getattr(self.backend, "processes", None))
        v = self.validations()
        if v:
            w = MetricWriter()
            for step, ok in v.items():
                w.add("amd_gpu_validation_ready", "gauge",
                      "1 if the node validator's <step>-ready marker is valid for this boot and "
                      "driver instance.", 1 if ok else 0, {"step": step})
            text += w.text()
        with self._lock:
            self._text = text
        self.samples_taken += 1
        return text

    def metrics(self) -> str:
        with self._lock:
            return self._text

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.sample_once()
            except Exception:
                log.exception("sampling failed")
            self._stop.wait(self.cfg.interval)

    def start(self) -> "Exporter":
        self.sample_once()
        self._thread = threading.Thread(target=self._loop, name="mxk8s-exporter", daemon=True)
        self._thread.start()
        exporter = self

        class Handler(http.server.BaseHTTPRequestHandler):
            def do_GET(self):
                if self.path.startswith("/metrics"):
                    body = exporter.metrics().encode()
                    ctype = "text/plain; version=0.0.4; charset=utf-8"
                elif self.path.startswith("/healthz"):
                    body, ctype = b"ok\n", "text/plain"
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        self._httpd = http.server.ThreadingHTTPServer(("", self.cfg.port), Handler)
        threading.Thread(target=self._httpd.serve_forever, name="mxk8s-exporter-http",
                         daemon=True).start()
        return self

    @property
    def port(self) -> int:
        return self._httpd.server_address[1] if self._httpd else self.cfg.port

    def stop(self):
        self._stop.set()
        if self._httpd:
            self._httpd.shutdown()
            self._httpd.server_close()
