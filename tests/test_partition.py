"""Partition manager (MIG-manager counterpart) and partition-aware discovery
over fake sysfs trees: a scripted "driver" thread re-enumerates the KFD
topology when every device's ``current_compute_partition`` has been written,
the way amdgpu does after a partition change."""
import copy
import os
import shutil
import sys
import tempfile
import threading
import time

import pytest

from mxk8s import partition
from mxk8s.deviceplugin import api
from mxk8s.deviceplugin.fake_kubelet import FakeKubelet
from mxk8s.deviceplugin.plugin import AmdGpuDevicePlugin, PluginConfig
from mxk8s.native import node

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "fixtures"))
import make_sysfs  # noqa: E402


class FakeNodeClient:
    """The two KubeClient calls the manager makes, on an in-memory Node."""

    def __init__(self, name, labels=None):
        self.node = {"metadata": {"name": name, "labels": dict(labels or {}), "annotations": {}}}
        self.patches = []

    def get_node(self, name):
        return copy.deepcopy(self.node)

    def merge_patch(self, path, patch):
        self.patches.append(patch)
        md = patch.get("metadata", {})
        for k in ("labels", "annotations"):
            for key, v in md.get(k, {}).items():
                if v is None:
                    self.node["metadata"][k].pop(key, None)
                else:
                    self.node["metadata"][k][key] = v
        return self.node


def spx_root(tmp):
    root = os.path.join(tmp, "root")
    make_sysfs.tree_8gpu(root)
    for b in make_sysfs.MI355X_BDFS:
        make_sysfs.write_partition_files(root, b, "SPX", "NPS1")
    return root


class FakeDriver(threading.Thread):
    """Re-enumerates the topology once every device's compute mode is written."""

    def __init__(self, root):
        super().__init__(daemon=True)
        self.root, self.stop = root, threading.Event()
        self.switched = None

    def run(self):
        while not self.stop.wait(0.02):
            modes = partition.current_modes(self.root, make_sysfs.MI355X_BDFS)
            comp = {m["compute"] for m in modes.values()}
            mem = {m["memory"] for m in modes.values()}
            if len(comp) == 1 and len(mem) == 1 and comp != {self.switched or "SPX"}:
                target = comp.pop()
                tmp = self.root + ".new"
                shutil.rmtree(tmp, ignore_errors=True)
                if target == "SPX":
                    make_sysfs.tree_8gpu(tmp)
                    for b in make_sysfs.MI355X_BDFS:
                        make_sysfs.write_partition_files(tmp, b, "SPX", mem.pop() if mem else "NPS1")
                else:
                    make_sysfs.tree_partitioned(tmp, target, mem.pop())
                old = self.root + ".old"
                os.rename(self.root, old)
                os.rename(tmp, self.root)
                shutil.rmtree(old, ignore_errors=True)
                self.switched = target


def test_partitioned_enumeration_cpx_nps2(tmp_path):
    root = str(tmp_path / "cpx")
    make_sysfs.tree_partitioned(root, "CPX", "NPS2")
    gpus = node.enumerate_gpus(root)
    assert len(gpus) == 64
    g9 = gpus[9]
    assert (g9.bdf, g9.partition, g9.partitions, g9.num_xcc, g9.cu_count) == ("0000:15:00.0", 1, 8, 1, 32)
    assert g9.uuid.endswith("-p1") and len({g.uuid for g in gpus}) == 64
    assert g9.key == "0000:15:00.0#1" and gpus[8].key == "0000:15:00.0"
    assert abs(g9.vram_bytes / 2 ** 30 - 144) < 0.1            # NPS2: half the HBM
    assert (g9.render_minor, g9.card) == (137, 10)
    spec = node.cdi_spec(root)
    paths = [n["path"] for d in spec["devices"] if d["name"] == "9"
             for n in d["containerEdits"]["deviceNodes"]]
    assert paths == ["/dev/dri/renderD137", "/dev/dri/card10"]
    # allocation policy still keeps a request on one NUMA node
    pick = node.preferred_allocation(list(range(64)), [], 16, root)
    assert len({gpus[i].numa_node for i in pick}) == 1


def test_manager_applies_profile_and_reports(tmp_path):
    root = spx_root(str(tmp_path))
    client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "cpx-nps2"})
    drv = FakeDriver(root)
    drv.start()
    try:
        mgr = partition.PartitionManager(client, "n1", root, settle_timeout=10, poll=0.02)
        res = mgr.reconcile_once()
        assert res.state == "success" and res.applied, res
        assert len(node.enumerate_gpus(root)) == 64
        assert client.node["metadata"]["labels"][partition.STATE_LABEL] == "success"
        assert "64 GPU partitions" in client.node["metadata"]["annotations"][partition.MESSAGE_ANNOTATION]
        # idempotent: a second pass changes nothing and does not re-patch
        n_patches = len(client.patches)
        res = mgr.reconcile_once()
        assert res.state == "success" and not res.applied and len(client.patches) == n_patches
    finally:
        drv.stop.set()


def test_manager_waits_for_gpu_workloads(tmp_path):
    root = spx_root(str(tmp_path))
    client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "cpx-nps1"})
    users = ["ml/trainer-0/main"]
    mgr = partition.PartitionManager(client, "n1", root, busy=lambda: list(users),
                                     settle_timeout=1, poll=0.02)
    res = mgr.reconcile_once()
    assert res.state == "pending" and "trainer-0" in res.message
    assert partition.current_modes(root, [make_sysfs.MI355X_BDFS[0]])[make_sysfs.MI355X_BDFS[0]] == \
        {"compute": "SPX", "memory": "NPS1"}                     # nothing written
    assert client.node["metadata"]["labels"][partition.STATE_LABEL] == "pending"


@pytest.mark.parametrize("label,why", [("bogus", "unknown partition profile"),
                                       ("cpx-nps2", "not in")])
def test_manager_rejects_bad_profiles(tmp_path, label, why):
    root = spx_root(str(tmp_path))
    if label == "cpx-nps2":     # a device that cannot do NPS2
        with open(os.path.join(root, "sys/bus/pci/devices", make_sysfs.MI355X_BDFS[3],
                               "available_memory_partition"), "w") as f:
            f.write("NPS1\n")
    client = FakeNodeClient("n1", {partition.CONFIG_LABEL: label})
    res = partition.PartitionManager(client, "n1", root, settle_timeout=1).reconcile_once()
    assert res.state == "failed" and why in res.message
    assert client.node["metadata"]["labels"][partition.STATE_LABEL] == "failed"


def test_manager_pending_reboot_when_driver_does_not_reenumerate(tmp_path):
    """amdgpu takes the modes (sysfs reads them back) but
    does not re-enumerate in place (an NPS change needs a driver reload):
    pending-reboot, drain kept; after the "reboot" the next pass sees the
    layout, reports success and lifts the drain."""
    root = spx_root(str(tmp_path))
    state = str(tmp_path / "state")
    client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "dpx-nps1"})
    mgr = partition.PartitionManager(client, "n1", root, settle_timeout=0.2, poll=0.02,
                                     state_dir=state, boot="boot-a")
    res = mgr.reconcile_once()
    assert res.state == "pending-reboot" and "expected 16" in res.message and res.applied
    assert client.node["metadata"]["labels"][partition.STATE_LABEL] == "pending-reboot"
    assert partition.read_drain(state, "boot-a")          # devices stay withdrawn
    assert partition.read_drain(state, "boot-b") is None  # void after a reboot
    make_sysfs.tree_partitioned(root + ".dpx", "DPX", "NPS1")
    shutil.rmtree(root)
    os.rename(root + ".dpx", root)
    res = mgr.reconcile_once()
    assert res.state == "success" and not res.applied
    assert partition.read_drain(state, "boot-a") is None


def test_manager_fails_when_driver_rejects_mode(tmp_path):
    root = spx_root(str(tmp_path))
    client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "dpx-nps1"})

    class Rejecting(threading.Thread):      # amdgpu puts the old mode back
        def __init__(self):
            super().__init__(daemon=True)
            self.stop = threading.Event()

        def run(self):
            p = os.path.join(root, "sys/bus/pci/devices", make_sysfs.MI355X_BDFS[2],
                             "current_compute_partition")
            while not self.stop.wait(0.01):
                if open(p).read().strip() != "SPX":
                    open(p, "w").write("SPX\n")

    rej = Rejecting()
    rej.start()
    try:
        res = partition.PartitionManager(client, "n1", root, settle_timeout=0.3,
                                         poll=0.02).reconcile_once()
    finally:
        rej.stop.set()
    assert res.state == "failed" and make_sysfs.MI355X_BDFS[2] in res.message


def test_busy_probes_fail_closed(tmp_path):
    """an unavailable probe is never read as 'idle'."""
    root = spx_root(str(tmp_path))
    client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "cpx-nps1"})
    busy = partition.combined_busy(lambda: [], lambda: None)
    res = partition.PartitionManager(client, "n1", root, busy=busy, settle_timeout=1,
                                     poll=0.02).reconcile_once()
    assert res.state == "pending" and "cannot verify" in res.message
    assert partition.current_modes(root, [make_sysfs.MI355X_BDFS[0]])[make_sysfs.MI355X_BDFS[0]] == \
        {"compute": "SPX", "memory": "NPS1"}
    assert partition.pod_resources_users(str(tmp_path / "no-such.sock")) is None
    assert partition.combined_busy(lambda: ["a"], lambda: ["b"])() == ["a", "b"]


def test_drain_handshake_with_plugin_and_recheck(tmp_path):
    """The manager withdraws every device through the plugin (all Unhealthy,
    acknowledged) BEFORE writing sysfs, and re-checks busy() after the drain:
    a workload admitted in between keeps the layout unchanged."""
    root = spx_root(str(tmp_path))
    state = str(tmp_path / "state")
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    kube = FakeKubelet(d).start()
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=d, sysfs_root=root, health_interval=0.05,
                                             watch_interval=0.1, use_smi_events=False,
                                             reconcile_interval=0, state_dir=state)).start()
    try:
        reg = kube.wait_registration()
        watch = iter(kube.plugin_stub(reg.endpoint).ListAndWatch(api.Empty(), timeout=30))
        assert {x.health for x in next(watch).devices} == {api.HEALTHY}
        while not os.path.exists(os.path.join(state, "health.json")):
            time.sleep(0.02)
        calls = []

        def busy():     # idle at the first check, a pod sneaks in before the second
            calls.append(1)
            return [] if len(calls) == 1 else ["ml/late-pod/main"]

        client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "cpx-nps1"})
        mgr = partition.PartitionManager(client, "n1", root, busy=busy, settle_timeout=1,
                                         poll=0.02, state_dir=state, drain_timeout=5)
        res = mgr.reconcile_once()
        assert res.state == "pending" and "late-pod" in res.message and len(calls) == 2
        drained = False     # the plugin withdrew every device before the re-check
        for r in watch:
            if {x.health for x in r.devices} == {api.UNHEALTHY}:
                drained = True
                break
        assert drained
        assert plugin.state.reasons["0"] == partition.DRAIN_REASON
        assert partition.current_modes(root, make_sysfs.MI355X_BDFS[:1])[make_sysfs.MI355X_BDFS[0]] == \
            {"compute": "SPX", "memory": "NPS1"}
        assert not os.path.exists(os.path.join(state, partition.DRAIN_FILE))   # lifted
        end = time.monotonic() + 5
        while plugin.state.health["0"] != api.HEALTHY and time.monotonic() < end:
            time.sleep(0.02)
        assert plugin.state.health["0"] == api.HEALTHY
    finally:
        plugin.stop()
        kube.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_plugin_readvertises_partitions_with_mixed_naming(tmp_path):
    root = spx_root(str(tmp_path))
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    kube = FakeKubelet(d).start()
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=d, sysfs_root=root, health_interval=0.05,
                                             watch_interval=0.1, use_smi_events=False,
                                             reconcile_interval=0.1,
                                             partition_naming="mixed")).start()
    drv = FakeDriver(root)
    drv.start()
    try:
        reg = kube.wait_registration()
        assert reg.resource_name == "amd.com/gpu"
        old_stub = kube.plugin_stub(reg.endpoint)
        old_watch = iter(old_stub.ListAndWatch(api.Empty(), timeout=30))
        assert len(next(old_watch).devices) == 8
        client = FakeNodeClient("n1", {partition.CONFIG_LABEL: "cpx-nps2"})
        res = partition.PartitionManager(client, "n1", root, settle_timeout=10,
                                         poll=0.02).reconcile_once()
        assert res.state == "success"
        reg2 = kube.wait_registration(timeout=15)
        assert reg2.resource_name == "amd.com/gpu-cpx"
        # the old resource's stream ENDS (it must never advertise the
        # new partition IDs under the old name) and the new one has its own socket
        assert reg2.endpoint == "amd-gpu-cpx.sock" and reg.endpoint == "amd-gpu.sock"
        import grpc
        seen = []
        try:
            for resp in old_watch:
                seen.append(len(resp.devices))
        except grpc.RpcError:
            pass
        assert all(n == 8 for n in seen), seen
        assert not os.path.exists(os.path.join(d, "amd-gpu.sock"))
        stub = kube.plugin_stub(reg2.endpoint)
        devs = next(iter(stub.ListAndWatch(api.Empty(), timeout=10))).devices
        assert len(devs) == 64 and all(x.health == api.HEALTHY for x in devs)
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["9"])
        c = stub.Allocate(req, timeout=5).container_responses[0]
        assert [x.name for x in c.cdi_devices] == ["amd.com/gpu=9"]
        assert "/dev/dri/renderD137" in [x.host_path for x in c.devices]
        assert c.annotations["amd.com/gpu.devices"].endswith("-p1")
    finally:
        drv.stop.set()
        plugin.stop()
        kube.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_repartition_during_drain_keeps_new_partitions_withdrawn(tmp_path):
    """a repartition while the drain file is present must advertise
    the NEW partition IDs Unhealthy from the start (reconcile_once, before any
    health pass), and the drain ack is written only once every advertised ID
    is Unhealthy in the state ListAndWatch streams."""
    root = spx_root(str(tmp_path))
    state = str(tmp_path / "state")
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=str(tmp_path / "dp"), sysfs_root=root,
                                             use_smi_events=False, reconcile_interval=0,
                                             state_dir=state, register=False))
    assert set(plugin.state.health.values()) == {api.HEALTHY}
    mgr = partition.PartitionManager(FakeNodeClient("n1", {}), "n1", root, state_dir=state)
    mgr._set_drain("t1")
    ack = os.path.join(state, partition.DRAIN_ACK_FILE)
    # the driver re-enumerates as CPX x NPS2 while the drain is active
    tmp = root + ".new"
    make_sysfs.tree_partitioned(tmp, "CPX", "NPS2")
    shutil.rmtree(root)
    os.rename(tmp, root)
    out = plugin.reconcile_once()
    assert out["gpus_changed"] and len(plugin.state.gpus) == 64
    assert set(plugin.state.health.values()) == {api.UNHEALTHY}
    assert set(plugin.state.reasons.values()) == {partition.DRAIN_REASON}
    assert not os.path.exists(ack)              # no health pass yet, no ack
    plugin.check_health_once()
    assert set(plugin.state.health.values()) == {api.UNHEALTHY}
    assert open(ack).read() == "t1"
    # an ack is never written while some advertised ID is still Healthy
    os.unlink(ack)
    plugin._drain_acked = None
    real = plugin.state.set_health_many
    plugin.state.set_health_many = lambda updates: real(
        {k: v for k, v in updates.items() if k != "63"})
    plugin.state.health["63"] = api.HEALTHY
    plugin.check_health_once()
    assert not os.path.exists(ack)
    plugin.state.set_health_many = real
    plugin.check_health_once()
    assert os.path.exists(ack)
    # drain lifted: the partitions come back Healthy on the next pass
    mgr._set_drain(None)
    plugin.check_health_once()
    assert set(plugin.state.health.values()) == {api.HEALTHY}
    plugin.monitor.close()
