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
* health: the native N02 state machine (``native/libmxnode/monitor.cc``,
  ``node.HealthMonitor``) — KFD node / render node present, fault-injection
  file, amd-smi VM-fault / pre-reset events (quarantine ``event_quarantine_s``
  after the last one), uncorrectable ECC above the per-boot baseline (sticky
  until reboot, or ``ecc_quarantine_s``), thermal-throttle events counted and
  logged; every verdict change re-sends ListAndWatch and gates Allocate, and
  the verdicts are written to ``<state_dir>/health.json`` for the exporter;
* operand reconciliation (the GPU Operator's ClusterPolicy controller,
  README.md:269-271, in miniature): every ``reconcile_interval`` s the plugin
  re-enumerates the GPUs (re-advertising when the set or a render minor
  changed) and rewrites the CDI spec atomically when it no longer matches the
  live render nodes (a driver reload / GPU reset can renumber them);
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
import json
import logging
import os
import threading
import time
from typing import Callable, Iterable, Optional

import grpc

from . import api
from ..native import node
from ..partition import DRAIN_ACK_FILE, DRAIN_REASON, boot_id, read_drain
from ..validate import node as validate_node

log = logging.getLogger("mxk8s.deviceplugin")

RESOURCE_NAME = "amd.com/gpu"
CDI_KIND = "amd.com/gpu"
PARTITION_MODES = {2: "dpx", 4: "qpx", 8: "cpx"}   # partitions per device -> compute mode


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
    ecc_quarantine_s: float = 0.0            # <= 0: uncorrectable ECC is sticky until reboot
    state_dir: Optional[str] = None          # ECC baseline + health.json (hostPath /var/lib/mxk8s)
    cdi_spec_path: Optional[str] = None      # reconcile this CDI spec file (None: don't)
    reconcile_interval: float = 30.0
    # compute partitions (DPX/QPX/CPX): "single" advertises every partition as
    # <resource_name>; "mixed" advertises <resource_name>-<mode> (e.g.
    # amd.com/gpu-cpx), the GPU Operator's MIG "mixed strategy" counterpart
    partition_naming: str = "single"
    # node-validator markers (<state_dir>/validations/<step>-ready) that must
    # be valid for the current boot + driver instance before the plugin
    # serves, and while it advertises devices Healthy (operator-validator
    # gating: the NVIDIA plugin's init container waits on driver validation)
    require_validation: tuple = ()

    def effective_resource(self, gpus) -> str:
        if self.partition_naming != "mixed" or not gpus:
            return self.resource_name
        parts = {g.partitions for g in gpus}
        if len(parts) != 1 or parts == {1}:
            return self.resource_name     # SPX, or heterogeneous: plain name
        mode = PARTITION_MODES.get(parts.pop(), "xpx")
        base, dot, shared = self.resource_name.partition(".shared")
        return f"{base}-{mode}{dot}{shared}"

    def socket_for(self, resource: str) -> str:
        """Socket file of the plugin serving ``resource``: the configured name
        for the base resource, ``<stem>-<mode>.sock`` for a mixed-naming
        partition resource (a renamed resource never shares the old socket)."""
        if resource == self.resource_name:
            return self.socket_name
        stem, dot, ext = self.socket_name.rpartition(".")
        tail = resource.rpartition("/")[2]
        base = self.resource_name.rpartition("/")[2].split(".")[0]
        suffix = (tail[len(base):] if tail.startswith(base) else "-" + tail).replace(".", "-")
        return f"{stem}{suffix}.{ext}" if dot else f"{self.socket_name}{suffix}"

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
        self.epoch = 0                # bumped when the advertised resource changes
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

    def set_health_many(self, updates: dict) -> list:
        """{dev_id: (healthy, reason)} applied atomically: one ListAndWatch
        re-send carries every change of a health pass.  Returns the IDs whose
        health changed."""
        changed = []
        with self._cv:
            for dev_id, (healthy, reason) in updates.items():
                new = api.HEALTHY if healthy else api.UNHEALTHY
                if self.health.get(dev_id) == new:
                    continue
                self.health[dev_id] = new
                self.reasons[dev_id] = reason
                changed.append(dev_id)
            if changed:
                self.generation += 1
                self._cv.notify_all()
        return changed

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

    def snapshot(self, epoch: int):
        """(generation, devices) atomically, or None once the state is closed
        or the advertised resource changed since ``epoch``."""
        with self._cv:
            if self.closed or self.epoch != epoch:
                return None
            return self.generation, self.devices()

    def bump_epoch(self) -> None:
        with self._cv:
            self.epoch += 1
            self.generation += 1
            self._cv.notify_all()

    def replace_gpus(self, gpus: list[node.GpuInfo], gate: Optional[str] = None) -> None:
        """New GPU set (reconciliation): known IDs keep their health, new ones
        start healthy, vanished ones are withdrawn; ListAndWatch re-sends.
        ``gate`` (a partition drain or a pending validation): EVERY ID, new
        ones included, starts Unhealthy with that reason — a repartition
        during a drain must not advertise its new partitions before the next
        health pass."""
        with self._cv:
            self.gpus = {str(g.index): g for g in gpus}
            if gate:
                self.health = {i: api.UNHEALTHY for i in self.gpus}
                self.reasons = {i: gate for i in self.gpus}
            else:
                self.health = {i: self.health.get(i, api.HEALTHY) for i in self.gpus}
                self.reasons = {i: self.reasons.get(i, "healthy") for i in self.gpus}
            self.generation += 1
            self._cv.notify_all()

    def all_unhealthy(self) -> bool:
        with self._cv:
            return all(h == api.UNHEALTHY for h in self.health.values())


class AmdGpuDevicePlugin:
    """gRPC servicer + lifecycle (serve, register, health, kubelet-restart watch)."""

    def __init__(self, config: PluginConfig | None = None,
                 gpus: Optional[list[node.GpuInfo]] = None):
        self.cfg = config or PluginConfig()
        self.gpus = gpus if gpus is not None else node.enumerate_gpus(self.cfg.sysfs_root)
        self.resource_name = self.cfg.effective_resource(self.gpus)
        self.socket_name = self.cfg.socket_for(self.resource_name)
        self.state = DeviceState(self.gpus, self.cfg.replicas)
        self._server: Optional[grpc.Server] = None
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._mon_lock = threading.Lock()
        self._serve_lock = threading.RLock()   # serve / register / rename / kubelet-restart
        self.monitor = self._new_monitor()
        self.reconciles = {"gpus_changed": 0, "cdi_rewritten": 0}
        self.registrations = 0
        self._drain_acked: Optional[str] = None
        self._boot = boot_id()
        self._socket_ino: Optional[int] = None
        self._kubelet_ino: Optional[int] = None

    # ------------------------------------------------------------------ RPCs
    def GetDevicePluginOptions(self, request, context):
        return api.DevicePluginOptions(pre_start_required=False,
                                       get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        seen = -1
        epoch = self.state.epoch     # a resource rename ends the streams of the old one
        while not self._stop.is_set() and context.is_active():
            snap = self.state.snapshot(epoch)
            if snap is None:
                return
            gen, devices = snap
            if gen != seen:
                seen = gen
                yield api.ListAndWatchResponse(devices=devices)
            self.state.wait_change(seen, timeout=1.0)

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
                              f"time-sliced {self.resource_name}: request for "
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
        """Replica choice under time-slicing.  Keep ``must``; then decide which
        physical GPUs the request spans — one replica per GPU before any GPU
        gets a second (spread before stacking), drawn from the least-shared GPUs
        (most free replicas), and among those the xGMI-hive / NUMA-compact set
        the native policy picks for exclusive requests (``mx_preferred_allocation``);
        finally take replicas round-robin over that set."""
        free: dict[str, list[str]] = {}
        for did in avail:
            phys = self.state.physical(did)
            if phys is None:
                raise ValueError(f"unknown device id {did!r}")
            free.setdefault(phys, []).append(did)
        if len(must) > size or size > len(avail):
            raise ValueError(f"cannot pick {size} of {len(avail)} (must include {len(must)})")
        for p in free:
            free[p].sort(key=lambda x: int(x.partition("::")[2]))
        chosen, used = [], {}
        for did in must:
            phys = self.state.physical(did)
            if phys is None or did not in free.get(phys, []):
                raise ValueError(f"must-include id {did!r} is not available")
            free[phys].remove(did)
            chosen.append(did)
            used[phys] = used.get(phys, 0) + 1
        rest = size - len(chosen)
        if rest == 0:
            return chosen
        spare = [p for p in free if free[p] and p not in used]
        n_new = min(rest, len(spare))           # new GPUs this request spreads onto
        span = list(used)
        if n_new:
            # least-shared tier: every spare GPU with at least as many free
            # replicas as the n_new-th best one, then the topology policy
            counts = sorted((len(free[p]) for p in spare), reverse=True)
            tier = [p for p in spare if len(free[p]) >= counts[n_new - 1]]
            try:
                pick = node.preferred_allocation([int(p) for p in tier] + [int(p) for p in used],
                                                 [int(p) for p in used], len(used) + n_new,
                                                 self.cfg.sysfs_root)
                span += [str(i) for i in pick if str(i) not in used]
            except (ValueError, RuntimeError):
                span += sorted(tier, key=lambda p: (-len(free[p]), int(p)))[:n_new]
        while len(chosen) < size:
            cand = [p for p in span if free[p]] or [p for p in free if free[p]]
            phys = min(cand, key=lambda p: (used.get(p, 0), -len(free[p]), int(p)))
            chosen.append(free[phys].pop(0))
            used[phys] = used.get(phys, 0) + 1
        return chosen

    def container_response(self, ids: list[str]):
        c = api.ContainerAllocateResponse()
        gpus = [self.state.gpus[i] for i in sorted(ids, key=int)]
        c.envs["AMD_GPU_DEVICE_IDS"] = ",".join(str(g.index) for g in gpus)
        c.envs["AMD_GPU_BDFS"] = ",".join(g.bdf for g in gpus)
        c.envs["AMD_GPU_ARCH"] = gpus[0].arch if gpus else ""
        # the render nodes this container must see, and no others: the pod's
        # payload (mx-vector-add) checks /dev/dri against it (BASELINE.md:37)
        c.envs["AMD_GPU_RENDER_NODES"] = ",".join(dict.fromkeys(g.render_path for g in gpus))
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

    def _new_monitor(self) -> node.HealthMonitor:
        return node.HealthMonitor(root=self.cfg.sysfs_root or self.cfg.dev_root,
                                  fault_file=self.cfg.fault_file, state_dir=self.cfg.state_dir,
                                  event_quarantine_s=self.cfg.event_quarantine_s,
                                  ecc_quarantine_s=self.cfg.ecc_quarantine_s,
                                  use_smi=self.cfg.use_smi_events)

    @property
    def health_state_path(self) -> Optional[str]:
        return os.path.join(self.cfg.state_dir, "health.json") if self.cfg.state_dir else None

    def check_health_once(self, wait_ms: int = 0) -> None:
        """One N02 pass (waits up to ``wait_ms`` for amd-smi events), then map
        the verdicts onto the advertised devices (matched by PCI BDF)."""
        with self._mon_lock:
            mon = self.monitor
        mon.step(wait_ms)
        # the monitor enumerates the same root: its index i is GPU i (checked
        # against the BDF; partitions of one device share it)
        gpus = self.state.gpus

        def dev_of(index: int, bdf: str) -> Optional[str]:
            g = gpus.get(str(index))
            return str(index) if g is not None and g.bdf == bdf else None

        status = mon.status()
        bdf_of = {st.index: st.bdf for st in status}
        # a partition change in progress (mxk8s.partition drain handshake):
        # every device is withdrawn until the drain file goes away; so is
        # every device while a required validation is not valid for the
        # running driver instance (a driver reload voids the markers)
        gate = self._gate()
        drain = read_drain(self.cfg.state_dir, self._boot)
        for ev in mon.new_events():
            dev = dev_of(ev.index, bdf_of.get(ev.index, "")) if ev.index >= 0 else None
            level = logging.INFO if ev.kind in (node.EVT_GPU_POST_RESET,
                                                node.EVT_THERMAL_THROTTLE) else logging.WARNING
            log.log(level, "device %s: %s", dev, ev.message,
                    extra={"device": dev, "event": ev.name, "value": ev.value})
        updates, bdfs = {}, {}
        for st in status:
            dev = dev_of(st.index, st.bdf)
            if dev is None:
                continue
            updates[dev] = (False, gate) if gate else (st.healthy, st.reason)
            bdfs[dev] = st.bdf
        if gate:
            # devices the monitor did not match (index / BDF mismatch, a
            # partition the monitor does not enumerate) are withdrawn too
            for dev in list(gpus):
                if dev not in updates:
                    updates[dev] = (False, gate)
                    bdfs[dev] = gpus[dev].bdf
        for dev in self.state.set_health_many(updates):
            healthy, reason = updates[dev]
            log.warning("device %s -> %s (%s)", dev, "Healthy" if healthy else "Unhealthy",
                        reason, extra={"device": dev, "event": "health_change",
                                       "reason": reason, "bdf": bdfs[dev]})
        if drain and drain != self._drain_acked and self.state.all_unhealthy():
            # every advertised device is now Unhealthy in the state
            # ListAndWatch streams (checked, not assumed: only then may the
            # partition manager write the new modes)
            ack = os.path.join(self.cfg.state_dir, DRAIN_ACK_FILE)
            with open(ack + ".tmp", "w") as f:
                f.write(drain)
            os.replace(ack + ".tmp", ack)
            self._drain_acked = drain
            log.warning("partition drain %s: all devices withdrawn", drain,
                        extra={"event": "partition_drain"})
        elif not drain:
            self._drain_acked = None
        if self.health_state_path:
            os.makedirs(self.cfg.state_dir, exist_ok=True)
            mon.write_state(self.health_state_path)

    def reconcile_once(self) -> dict:
        """Re-check the operands this plugin owns: the GPU set it advertises
        and the CDI spec containerd resolves its device names with."""
        out = {"gpus_changed": False, "cdi_rewritten": False}
        gpus = node.enumerate_gpus(self.cfg.sysfs_root)
        ident = [(g.index, g.bdf, g.render_minor, g.card, g.uuid) for g in gpus]
        if ident != [(g.index, g.bdf, g.render_minor, g.card, g.uuid) for g in self.gpus]:
            log.warning("GPU set changed (%d -> %d GPUs or renumbered); re-advertising",
                        len(self.gpus), len(gpus), extra={"event": "gpus_changed"})
            self.gpus = gpus
            with self._mon_lock:
                old, self.monitor = self.monitor, self._new_monitor()
            old.close()
            name = self.cfg.effective_resource(gpus)
            renamed = name != self.resource_name
            if renamed:
                # held until the new resource is served: the kubelet-restart
                # watcher must not re-serve the retired socket in between
                self._serve_lock.acquire()
                self._retire_endpoint()      # before the new IDs exist in the state
            self.state.replace_gpus(gpus, gate=self._gate())
            out["gpus_changed"] = True
            self.reconciles["gpus_changed"] += 1
            if renamed:
                # a partition-mode change under "mixed" naming: a new resource.
                # The old resource's endpoint must go away, not keep streaming
                # the new device IDs: stopping its server ends every open
                # ListAndWatch (kubelet then zeroes the old resource), and the
                # new resource is served on a socket of its own.
                log.warning("resource %s -> %s after the partition change; re-serving and "
                            "re-registering", self.resource_name, name,
                            extra={"event": "resource_renamed", "resource": name})
                try:
                    self._rename(name)
                finally:
                    self._serve_lock.release()
                out["resource_renamed"] = name
        if self.cfg.cdi_spec_path:
            text = node.cdi_spec_text(self.cfg.sysfs_root, self.cfg.cdi_kind)
            try:
                with open(self.cfg.cdi_spec_path) as f:
                    have = json.load(f)
            except (OSError, ValueError):
                have = None
            if have != json.loads(text):
                d = os.path.dirname(self.cfg.cdi_spec_path) or "."
                os.makedirs(d, exist_ok=True)
                tmp = self.cfg.cdi_spec_path + ".tmp"
                with open(tmp, "w") as f:
                    f.write(text)
                os.replace(tmp, self.cfg.cdi_spec_path)
                log.warning("CDI spec %s %s; rewritten from the live render nodes",
                            self.cfg.cdi_spec_path, "missing/unreadable" if have is None else "stale",
                            extra={"event": "cdi_rewritten"})
                out["cdi_rewritten"] = True
                self.reconciles["cdi_rewritten"] += 1
        return out

    # ------------------------------------------------------------ lifecycle
    @property
    def socket_path(self) -> str:
        return os.path.join(self.cfg.plugin_dir, self.socket_name)

    def _retire_endpoint(self) -> None:
        """End every ListAndWatch stream of the resource being retired and stop
        its server (kubelet then drops the old resource's capacity)."""
        with self._serve_lock:
            self.state.bump_epoch()
            if self._server is not None:
                self._server.stop(grace=0.5).wait()
                self._server = None
            try:
                os.unlink(self.socket_path)
            except FileNotFoundError:
                pass

    def _rename(self, name: str) -> None:
        with self._serve_lock:
            if self._server is not None:
                self._retire_endpoint()
            self.resource_name = name
            self.socket_name = self.cfg.socket_for(name)
            self.serve()
            if self.cfg.register:
                self.register()

    def serve(self) -> None:
        os.makedirs(self.cfg.plugin_dir, exist_ok=True)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
        server = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=8))
        server.add_generic_rpc_handlers((api.generic_handler("DevicePlugin", self),))
        server.add_insecure_port("unix:" + self.socket_path)
        server.start()
        self._server = server
        self._socket_ino = _inode(self.socket_path)
        log.info("serving %s on %s (%d GPUs)", self.resource_name, self.socket_path,
                 len(self.gpus))

    def register(self, timeout: float = 10.0) -> None:
        with grpc.insecure_channel("unix:" + self.cfg.kubelet_socket) as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            stub = api.Stub(ch, "Registration")
            stub.Register(api.RegisterRequest(
                version=api.API_VERSION, endpoint=self.socket_name,
                resource_name=self.resource_name,
                options=api.DevicePluginOptions(pre_start_required=False,
                                                get_preferred_allocation_available=True)),
                timeout=timeout)
        self.registrations += 1
        self._kubelet_ino = _inode(self.cfg.kubelet_socket)
        log.info("registered %s with kubelet (%d)", self.resource_name, self.registrations)

    def _gate(self) -> Optional[str]:
        """Why every device must be withdrawn right now (None: nothing): a
        partition change in progress (mxk8s.partition drain handshake), or a
        required validation that is not valid for the running driver
        instance (a driver reload / repartition voids the markers)."""
        if read_drain(self.cfg.state_dir, self._boot):
            return DRAIN_REASON
        pending = self._validation_pending()
        return f"{pending} validation pending" if pending else None

    def _validation_pending(self) -> Optional[str]:
        """First required validation whose marker is not valid, or None."""
        if not self.cfg.require_validation or not self.cfg.state_dir:
            return None
        st = validate_node.status(self.cfg.state_dir, self.cfg.sysfs_root,
                                  self.cfg.require_validation)
        return next((k for k, ok in st.items() if not ok), None)

    def start(self) -> "AmdGpuDevicePlugin":
        if self.cfg.require_validation and self.cfg.state_dir:
            # serve nothing until the node validator vouched for this driver
            log.info("waiting for validation: %s", ",".join(self.cfg.require_validation))
            validate_node.wait_for(self.cfg.state_dir, self.cfg.require_validation,
                                   self.cfg.sysfs_root, poll=min(1.0, self.cfg.watch_interval),
                                   stop=self._stop.is_set)
            if self._stop.is_set():
                return self
        self.serve()
        if self.cfg.register:
            self.register()
        self._spawn(self._health_loop, "health")
        self._spawn(self._watch_loop, "kubelet-watch")
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
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass
        with self._mon_lock:
            self.monitor.close()

    def _spawn(self, fn: Callable[[], None], name: str) -> None:
        t = threading.Thread(target=fn, name=f"mxk8s-dp-{name}", daemon=True)
        t.start()
        self._threads.append(t)

    def _health_loop(self) -> None:
        last_reconcile = time.monotonic()
        while not self._stop.is_set():
            # with amd-smi the pass blocks on the event queue (an event wakes it
            # at once); without it, a plain interval
            smi = self.monitor.smi_active
            try:
                self.check_health_once(int(min(1.0, self.cfg.health_interval) * 1000) if smi else 0)
                if (self.cfg.reconcile_interval > 0 and
                        time.monotonic() - last_reconcile >= self.cfg.reconcile_interval):
                    last_reconcile = time.monotonic()
                    self.reconcile_once()
            except Exception:   # keep serving; a failed probe is logged, not fatal
                log.exception("health check failed")
            if not smi:
                self._stop.wait(self.cfg.health_interval)

    def _watch_loop(self) -> None:
        while not self._stop.wait(self.cfg.watch_interval):
            sock_gone = _inode(self.socket_path) != self._socket_ino
            kubelet_new = (self.cfg.register and _inode(self.cfg.kubelet_socket) is not None
                           and _inode(self.cfg.kubelet_socket) != self._kubelet_ino)
            if not (sock_gone or kubelet_new):
                continue
            log.warning("kubelet restart detected (socket gone=%s, kubelet.sock new=%s); "
                        "re-serving and re-registering", sock_gone, kubelet_new)
            try:
                with self._serve_lock:
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
