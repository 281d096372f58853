"""``amd.com/gpu`` device plugin (kubelet Device Plugin API v1beta1).

MI355X-native counterpart of the NVIDIA device plugin DaemonSet that the
reference installs through the GPU Operator (/root/reference/README.md:264-272,
checked at README.md:288-296 and README.md:341-345).  Behaviour:

* discovery: ``libmxnode`` enumerates GPUs from the KFD topology (no ROCm
  runtime in the plugin container); device IDs are the GPU indices "0".."N-1";
  each Device carries its NUMA node for the kubelet Topology Manager;
* ``ListAndWatch``: sends the device list, then re-sends on every health
  change (HOT loop = a blocking wait on a condition variable, no polling of
  the stream);
* health: a checker thread re-runs ``mx_health_check`` (KFD node present,
  render node present, fault-injection file) every ``health_interval`` s and,
  when amd-smi is available, an event thread marks a GPU unhealthy on reset /
  VM-fault events for ``event_quarantine_s``;
* ``Allocate``: CDI device names ``amd.com/gpu=<id>`` (containerd resolves them
  with /etc/cdi/amd.com-gpu.json; no runtime shim) plus, as a fallback when CDI
  is off, explicit DeviceSpecs for /dev/kfd and /dev/dri/renderD<m> (+card<n>);
* ``GetPreferredAllocation``: the native xGMI-hive / NUMA aware policy;
* time-slicing (``replicas`` > 1): the GPU Operator's device-plugin sharing
  config [ext, SURVEY.md §2.1 R26d] re-designed for KFD: each GPU is advertised
  as ``<i>::<r>`` replicas that share one render node; Allocate de-duplicates
  replicas to physical GPUs, GetPreferredAllocation spreads replicas over the
  least-loaded GPUs, health is per physical GPU, and
  ``fail_requests_greater_than_one`` rejects multi-replica requests (a second
  replica of the same GPU buys no extra compute);
* kubelet restarts: the kubelet wipes the plugin directory when it restarts,
  so a watcher re-creates our socket and re-registers when it vanishes or
  kubelet.sock is re-created.
"""
from __future__ import annotations

import concurrent.futures
import dataclasses
import logging
import os
import threading
import time
from typing import Callable, Iterable, Optional

import grpc

from . import api
from ..native import node

log = logging.getLogger("mxk8s.deviceplugin")

RESOURCE_NAME = "amd.com/gpu"
CDI_KIND = "amd.com/gpu"


@dataclasses.dataclass
class PluginConfig:
    resource_name: str = RESOURCE_NAME
    plugin_dir: str = api.DEVICE_PLUGIN_PATH
    socket_name: str = "amd-gpu.sock"
    sysfs_root: str = ""                     # "" = real host; fixtures in tests
    dev_root: str = ""                       # prefix for device-node existence checks
    fault_file: Optional[str] = os.environ.get("MXK8S_FAULT_FILE") or None
    health_interval: float = 5.0
    use_cdi: bool = True
    use_device_specs: bool = True
    cdi_kind: str = CDI_KIND
    watch_interval: float = 1.0
    event_quarantine_s: float = 60.0
    use_smi_events: bool = True
    register: bool = True
    replicas: int = 1                        # time-slicing: >1 advertises <i>::<r> IDs
    fail_requests_greater_than_one: bool = False
    rename_shared: bool = False              # replicas>1: advertise <resource>.shared

    def __post_init__(self):
        if self.replicas < 1:
            raise ValueError(f"replicas must be >= 1, got {self.replicas}")
        if self.replicas > 1 and self.rename_shared and not self.resource_name.endswith(".shared"):
            self.resource_name += ".shared"

    @property
    def socket_path(self) -> str:
        return os.path.join(self.plugin_dir, self.socket_name)

    @property
    def kubelet_socket(self) -> str:
        return os.path.join(self.plugin_dir, api.KUBELET_SOCKET_NAME)


class DeviceState:
    """Thread-safe device list + health with change notification."""

    def __init__(self, gpus: list[node.GpuInfo], replicas: int = 1):
        self._cv = threading.Condition()
        self.replicas = replicas
        self.gpus = {str(g.index): g for g in gpus}
        self.health = {i: api.HEALTHY for i in self.gpus}
        self.reasons = {i: "healthy" for i in self.gpus}
        self.generation = 0
        self.closed = False

    def set_health(self, dev_id: str, healthy: bool, reason: str) -> bool:
        with self._cv:
            new = api.HEALTHY if healthy else api.UNHEALTHY
            if self.health.get(dev_id) == new:
                return False
            self.health[dev_id] = new
            self.reasons[dev_id] = reason
            self.generation += 1
            self._cv.notify_all()
            return True

    def devices(self) -> list:
        with self._cv:
            out = []
            for i in sorted(self.gpus, key=int):
                g = self.gpus[i]
                for did in self.replica_ids(i):
                    d = api.Device(ID=did, health=self.health[i])
                    if g.numa_node >= 0:
                        d.topology.nodes.add(ID=g.numa_node)
                    out.append(d)
            return out

    def replica_ids(self, phys: str) -> list[str]:
        if self.replicas == 1:
            return [phys]
        return [f"{phys}::{r}" for r in range(self.replicas)]

    def physical(self, dev_id: str) -> Optional[str]:
        """Advertised ID -> physical GPU index, or None when not one of ours."""
        if self.replicas == 1:
            return dev_id if dev_id in self.gpus else None
        phys, sep, rep = dev_id.partition("::")
        if not sep or phys not in self.gpus or not rep.isdigit() or int(rep) >= self.replicas:
            return None
        return phys

    def wait_change(self, seen: int, timeout: float) -> int:
        with self._cv:
            if self.generation == seen and not self.closed:
                self._cv.wait(timeout)
            return self.generation

    def close(self) -> None:
        with self._cv:
            self.closed = True
            self._cv.notify_all()


class AmdGpuDevicePlugin:
    """gRPC servicer + lifecycle (serve, register, health, kubelet-restart watch)."""

    def __init__(self, config: PluginConfig | None = None,
                 gpus: Optional[list[node.GpuInfo]] = None):
        self.cfg = config or PluginConfig()
        self.gpus = gpus if gpus is not None else node.enumerate_gpus(self.cfg.sysfs_root)
        self.state = DeviceState(self.gpus, self.cfg.replicas)
        self._server: Optional[grpc.Server] = None
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._smi_quarantine: dict[str, float] = {}
        self.registrations = 0
        self._socket_ino: Optional[int] = None
        self._kubelet_ino: Optional[int] = None

    # ------------------------------------------------------------------ RPCs
    def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False,
                                       get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        seen = -1
        while not self._stop.is_set() and context.is_active():
            gen = self.state.generation
            if gen != seen:
                seen = gen
                yield api.ListAndWatchResponse(devices=self.state.devices())
            self.state.wait_change(seen, timeout=1.0)
            if self.state.closed:
                return

    def GetPreferredAllocation(self, request, context):
        resp = api.PreferredAllocationResponse()
        if self.cfg.replicas > 1:
            for creq in request.container_requests:
                try:
                    ids = self.preferred_replicas(list(creq.available_deviceIDs),
                                                  list(creq.must_include_deviceIDs),
                                                  creq.allocation_size)
                except ValueError as e:
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
                resp.container_responses.add(deviceIDs=ids)
            return resp
        for creq in request.container_requests:
            avail = [int(x) for x in creq.available_deviceIDs]
            must = [int(x) for x in creq.must_include_deviceIDs]
            try:
                ids = node.preferred_allocation(avail, must, creq.allocation_size,
                                                self.cfg.sysfs_root)
            except ValueError as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
            resp.container_responses.add(deviceIDs=[str(i) for i in ids])
        return resp

    def Allocate(self, request, context):
        resp = api.AllocateResponse()
        for creq in request.container_requests:
            requested = list(creq.devices_ids)
            if (self.cfg.replicas > 1 and self.cfg.fail_requests_greater_than_one
                    and len(requested) > 1):
                context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                              f"time-sliced {self.cfg.resource_name}: request for "
                              f"{len(requested)} replicas refused (limit 1 per container)")
            ids: list[str] = []
            for did in requested:
                i = self.state.physical(did)
                if i is None:
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown device id {did!r}")
                if self.state.health.get(i) != api.HEALTHY:
                    context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                                  f"device {i} is unhealthy: {self.state.reasons.get(i)}")
                if i not in ids:
                    ids.append(i)
            resp.container_responses.append(self.container_response(ids))
        return resp

    def PreStartContainer(self, request, context):
        return api.PreStartContainerResponse()

    # -------------------------------------------------------------- helpers
    def preferred_replicas(self, avail: list[str], must: list[str], size: int) -> list[str]:
        """Replica choice under time-slicing: keep ``must``, then take one replica
        at a time from the physical GPU with the most free replicas that this
        request does not use yet (spread before stacking; ties -> lowest index),
        so co-scheduled pods land on the least-shared GPUs."""
        free: dict[str, list[str]] = {}
        for did in avail:
            phys = self.state.physical(did)
            if phys is None:
                raise ValueError(f"unknown device id {did!r}")
            free.setdefault(phys, []).append(did)
        if len(must) > size or size > len(avail):
            raise ValueError(f"cannot pick {size} of {len(avail)} (must include {len(must)})")
        chosen, used = [], {}
        for did in must:
            phys = self.state.physical(did)
            if phys is None or did not in free.get(phys, []):
                raise ValueError(f"must-include id {did!r} is not available")
            free[phys].remove(did)
            chosen.append(did)
            used[phys] = used.get(phys, 0) + 1
        while len(chosen) < size:
            phys = min((p for p in free if free[p]),
                       key=lambda p: (used.get(p, 0), -len(free[p]), int(p)))
            did = sorted(free[phys], key=lambda x: int(x.partition("::")[2]))[0]
            free[phys].remove(did)
            chosen.append(did)
            used[phys] = used.get(phys, 0) + 1
        return chosen

    def container_response(self, ids: list[str]):
        c = api.ContainerAllocateResponse()
        gpus = [self.state.gpus[i] for i in sorted(ids, key=int)]
        c.envs["AMD_GPU_DEVICE_IDS"] = ",".join(str(g.index) for g in gpus)
        c.envs["AMD_GPU_BDFS"] = ",".join(g.bdf for g in gpus)
        c.envs["AMD_GPU_ARCH"] = gpus[0].arch if gpus else ""
        c.annotations["amd.com/gpu.devices"] = ",".join(g.uuid for g in gpus)
        if self.cfg.use_cdi:
            for g in gpus:
                c.cdi_devices.add(name=f"{self.cfg.cdi_kind}={g.index}")
        if self.cfg.use_device_specs:
            c.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            for g in gpus:
                c.devices.add(container_path=g.render_path, host_path=g.render_path,
                              permissions="rw")
                if g.card_path:
                    c.devices.add(container_path=g.card_path, host_path=g.card_path,
                                  permissions="rw")
        return c

    def check_health_once(self) -> None:
        now = time.monotonic()
        for i, g in self.state.gpus.items():
            code = node.health_check(g.index, self.cfg.sysfs_root or self.cfg.dev_root,
                                     self.cfg.fault_file)
            if code == node.HEALTHY and self._smi_quarantine.get(i, 0) > now:
                code = node.UNHEALTHY_SMI_EVENT
            changed = self.state.set_health(i, code == node.HEALTHY, node.health_reason(code))
            if changed:
                log.warning("device %s -> %s (%s)", i, self.state.health[i],
                            node.health_reason(code))

    # ------------------------------------------------------------ lifecycle
    def serve(self) -> None:
        os.makedirs(self.cfg.plugin_dir, exist_ok=True)
        try:
            os.unlink(self.cfg.socket_path)
        except FileNotFoundError:
            pass
        server = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=8))
        server.add_generic_rpc_handlers((api.generic_handler("DevicePlugin", self),))
        server.add_insecure_port("unix:" + self.cfg.socket_path)
        server.start()
        self._server = server
        self._socket_ino = _inode(self.cfg.socket_path)
        log.info("serving %s on %s (%d GPUs)", self.cfg.resource_name, self.cfg.socket_path,
                 len(self.gpus))

    def register(self, timeout: float = 10.0) -> None:
        with grpc.insecure_channel("unix:" + self.cfg.kubelet_socket) as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            stub = api.Stub(ch, "Registration")
            stub.Register(api.RegisterRequest(
                version=api.API_VERSION, endpoint=self.cfg.socket_name,
                resource_name=self.cfg.resource_name,
                options=api.DevicePluginOptions(pre_start_required=False,
                                                get_preferred_allocation_available=True)),
                timeout=timeout)
        self.registrations += 1
        self._kubelet_ino = _inode(self.cfg.kubelet_socket)
        log.info("registered %s with kubelet (%d)", self.cfg.resource_name, self.registrations)

    def start(self) -> "AmdGpuDevicePlugin":
        self.serve()
        if self.cfg.register:
            self.register()
        self._spawn(self._health_loop, "health")
        self._spawn(self._watch_loop, "kubelet-watch")
        if self.cfg.use_smi_events:
            self._spawn(self._smi_event_loop, "smi-events")
        return self

    def stop(self) -> None:
        self._stop.set()
        self.state.close()
        if self._server is not None:
            self._server.stop(grace=0.5).wait()
            self._server = None
        for t in self._threads:
            t.join(timeout=5)
        try:
            os.unlink(self.cfg.socket_path)
        except FileNotFoundError:
            pass

    def _spawn(self, fn: Callable[[], None], name: str) -> None:
        t = threading.Thread(target=fn, name=f"mxk8s-dp-{name}", daemon=True)
        t.start()
        self._threads.append(t)

    def _health_loop(self) -> None:
        while not self._stop.is_set():
            try:
                self.check_health_once()
            except Exception:   # keep serving; a failed probe is logged, not fatal
                log.exception("health check failed")
            self._stop.wait(self.cfg.health_interval)

    def _smi_event_loop(self) -> None:
        ok, err = node.smi_open()
        if not ok:
            log.info("amd-smi events unavailable: %s", err)
            return
        # amd-smi enumeration order vs our KFD order: match by BDF
        by_bdf = {g.bdf: str(g.index) for g in self.gpus}
        smi_to_id = {}
        for k in range(max(0, node.smi_count())):
            s = node.smi_sample(k)
            if s.bdf in by_bdf:
                smi_to_id[k] = by_bdf[s.bdf]
        while not self._stop.is_set():
            for gi, ev in node.smi_wait_events(1000):
                dev = smi_to_id.get(gi)
                if dev is None:
                    continue
                if ev in (1, 3):   # VM fault, pre-reset
                    self._smi_quarantine[dev] = time.monotonic() + self.cfg.event_quarantine_s
                    self.state.set_health(dev, False, node.health_reason(node.UNHEALTHY_SMI_EVENT))

    def _watch_loop(self) -> None:
        while not self._stop.wait(self.cfg.watch_interval):
            sock_gone = _inode(self.cfg.socket_path) != self._socket_ino
            kubelet_new = (self.cfg.register and _inode(self.cfg.kubelet_socket) is not None
                           and _inode(self.cfg.kubelet_socket) != self._kubelet_ino)
            if not (sock_gone or kubelet_new):
                continue
            log.warning("kubelet restart detected (socket gone=%s, kubelet.sock new=%s); "
                        "re-serving and re-registering", sock_gone, kubelet_new)
            try:
                if self._server is not None:
                    self._server.stop(grace=0.2).wait()
                self.serve()
                if self.cfg.register:
                    self.register()
            except Exception:
                log.exception("re-registration failed; retrying")
                self._socket_ino = None


def _inode(path: str) -> Optional[int]:
    try:
        return os.stat(path).st_ino
    except OSError:
        return None


def run_forever(cfg: PluginConfig) -> None:
    plugin = AmdGpuDevicePlugin(cfg)
    while True:
        try:
            plugin.start()
            break
        except Exception as e:   # kubelet not up yet
            log.warning("start failed (%s); retrying in 5 s", e)
            plugin.stop()
            plugin = AmdGpuDevicePlugin(cfg)
            time.sleep(5)
    try:
        while True:
            time.sleep(3600)
    finally:
        plugin.stop()


def devices_summary(devs: Iterable) -> list[tuple[str, str]]:
    return [(d.ID, d.health) for d in devs]
