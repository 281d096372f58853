"""Contract tests: the real amd.com/gpu plugin against a fake kubelet over
unix-socket gRPC, on fake MI355X sysfs trees (SURVEY.md §4.2 'Contract')."""
import concurrent.futures
import os
import tempfile
import threading
import time

import grpc
import pytest

from mxk8s.deviceplugin import api
from mxk8s.deviceplugin.fake_kubelet import FakeKubelet
from mxk8s.deviceplugin.plugin import AmdGpuDevicePlugin, PluginConfig

FX = os.path.join(os.path.dirname(__file__), "fixtures", "sysfs")


@pytest.fixture
def plugin_dir():
    # unix socket paths must stay short (108 bytes)
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    yield d


def _start(plugin_dir, fixture="mi355x_8gpu", fault_file=None, **kw):
    kube = FakeKubelet(plugin_dir).start()
    cfg = PluginConfig(plugin_dir=plugin_dir, sysfs_root=os.path.join(FX, fixture),
                       fault_file=fault_file, health_interval=0.1, watch_interval=0.1,
                       use_smi_events=False, **kw)
    plugin = AmdGpuDevicePlugin(cfg).start()
    return kube, plugin


def test_register_and_list(plugin_dir):
    kube, plugin = _start(plugin_dir)
    try:
        reg = kube.wait_registration()
        assert reg.version == "v1beta1"
        assert reg.resource_name == "amd.com/gpu"
        assert reg.endpoint == "amd-gpu.sock"
        assert reg.options.get_preferred_allocation_available
        stub = kube.plugin_stub(reg.endpoint)
        opts = stub.GetDevicePluginOptions(api.Empty(), timeout=5)
        assert opts.get_preferred_allocation_available and not opts.pre_start_required
        first = next(iter(stub.ListAndWatch(api.Empty(), timeout=5)))
        assert [d.ID for d in first.devices] == [str(i) for i in range(8)]
        assert all(d.health == api.HEALTHY for d in first.devices)
        assert [d.topology.nodes[0].ID for d in first.devices] == [0, 0, 0, 0, 1, 1, 1, 1]
    finally:
        plugin.stop()
        kube.stop()


def test_allocate_cdi_and_devicespecs(plugin_dir):
    kube, plugin = _start(plugin_dir)
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["2", "0"])
        resp = stub.Allocate(req, timeout=5)
        c = resp.container_responses[0]
        assert [d.name for d in c.cdi_devices] == ["amd.com/gpu=0", "amd.com/gpu=2"]
        paths = [(d.container_path, d.host_path, d.permissions) for d in c.devices]
        assert paths[0] == ("/dev/kfd", "/dev/kfd", "rw")
        assert ("/dev/dri/renderD128", "/dev/dri/renderD128", "rw") in paths
        assert ("/dev/dri/renderD130", "/dev/dri/renderD130", "rw") in paths
        assert ("/dev/dri/card3", "/dev/dri/card3", "rw") in paths
        assert c.envs["AMD_GPU_DEVICE_IDS"] == "0,2"
        assert c.envs["AMD_GPU_ARCH"] == "gfx950"
        # the pod's payload compares /dev/dri with exactly these (BASELINE.md:37)
        assert c.envs["AMD_GPU_RENDER_NODES"] == "/dev/dri/renderD128,/dev/dri/renderD130"
        bad = api.AllocateRequest()
        bad.container_requests.add(devices_ids=["9"])
        with pytest.raises(grpc.RpcError) as e:
            stub.Allocate(bad, timeout=5)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    finally:
        plugin.stop()
        kube.stop()


def test_cdi_only_mode(plugin_dir):
    kube, plugin = _start(plugin_dir, use_device_specs=False)
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["5"])
        c = stub.Allocate(req, timeout=5).container_responses[0]
        assert [d.name for d in c.cdi_devices] == ["amd.com/gpu=5"] and len(c.devices) == 0
    finally:
        plugin.stop()
        kube.stop()


def test_preferred_allocation(plugin_dir):
    kube, plugin = _start(plugin_dir)
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)
        req = api.PreferredAllocationRequest()
        req.container_requests.add(available_deviceIDs=[str(i) for i in range(8)],
                                   must_include_deviceIDs=["5"], allocation_size=4)
        req.container_requests.add(available_deviceIDs=["0", "1", "4", "5", "6"],
                                   allocation_size=3)
        resp = stub.GetPreferredAllocation(req, timeout=5)
        assert list(resp.container_responses[0].deviceIDs) == ["4", "5", "6", "7"]
        assert list(resp.container_responses[1].deviceIDs) == ["4", "5", "6"]
    finally:
        plugin.stop()
        kube.stop()


def test_health_fault_injection_resends(plugin_dir, tmp_path):
    ff = tmp_path / "faults"
    ff.write_text("")
    kube, plugin = _start(plugin_dir, fault_file=str(ff))
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)
        stream = stub.ListAndWatch(api.Empty(), timeout=20)
        first = next(stream)
        assert all(d.health == api.HEALTHY for d in first.devices)
        ff.write_text("3\n")
        second = next(stream)
        health = {d.ID: d.health for d in second.devices}
        assert health["3"] == api.UNHEALTHY
        assert sum(h == api.HEALTHY for h in health.values()) == 7
        # an unhealthy device is refused by Allocate
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["3"])
        with pytest.raises(grpc.RpcError) as e:
            stub.Allocate(req, timeout=5)
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION
        ff.write_text("")
        third = next(stream)
        assert all(d.health == api.HEALTHY for d in third.devices)
        stream.cancel()
    finally:
        plugin.stop()
        kube.stop()


def test_missing_render_node_unhealthy(plugin_dir):
    kube, plugin = _start(plugin_dir, fixture="missing_render")
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)
        stream = stub.ListAndWatch(api.Empty(), timeout=10)
        deadline = time.time() + 5
        while time.time() < deadline:
            resp = next(stream)
            health = {d.ID: d.health for d in resp.devices}
            if health["3"] == api.UNHEALTHY:
                break
        assert health["3"] == api.UNHEALTHY and health["2"] == api.HEALTHY
        stream.cancel()
    finally:
        plugin.stop()
        kube.stop()


def test_kubelet_restart_reregisters(plugin_dir):
    kube, plugin = _start(plugin_dir)
    try:
        kube.wait_registration()
        kube.restart()   # wipes amd-gpu.sock, new kubelet.sock
        reg = kube.wait_registration(timeout=10)
        assert reg.resource_name == "amd.com/gpu"
        deadline = time.time() + 5
        while plugin.registrations < 2 and time.time() < deadline:
            time.sleep(0.05)
        assert plugin.registrations >= 2
        stub = kube.plugin_stub(reg.endpoint)
        first = next(iter(stub.ListAndWatch(api.Empty(), timeout=5)))
        assert len(first.devices) == 8
    finally:
        plugin.stop()
        kube.stop()


def test_concurrent_allocate_no_cross_talk(plugin_dir):
    """Allocate is stateless; concurrent calls must each get exactly their ids."""
    kube, plugin = _start(plugin_dir)
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)

        def one(i):
            req = api.AllocateRequest()
            req.container_requests.add(devices_ids=[str(i)])
            c = stub.Allocate(req, timeout=10).container_responses[0]
            return i, [d.name for d in c.cdi_devices]
        with concurrent.futures.ThreadPoolExecutor(8) as ex:
            for i, names in ex.map(one, [k % 8 for k in range(64)]):
                assert names == [f"amd.com/gpu={i}"]
    finally:
        plugin.stop()
        kube.stop()


def test_golden_wire_bytes():
    """Field numbers are pinned: a silent renumbering would break the kubelet."""
    r = api.RegisterRequest(version="v1beta1", endpoint="amd-gpu.sock",
                            resource_name="amd.com/gpu",
                            options=api.DevicePluginOptions(get_preferred_allocation_available=True))
    assert r.SerializeToString().hex() == (
        "0a0776316265746131120c616d642d6770752e736f636b1a0b616d642e636f6d2f67707522021001")
    d = api.Device(ID="3", health="Healthy")
    d.topology.nodes.add(ID=1)
    assert d.SerializeToString() == b"\x0a\x013\x12\x07Healthy\x1a\x04\x0a\x02\x08\x01"
    c = api.ContainerAllocateResponse()
    c.envs["K"] = "V"
    c.devices.add(container_path="/a", host_path="/b", permissions="rw")
    c.annotations["x"] = "y"
    c.cdi_devices.add(name="amd.com/gpu=0")
    assert c.SerializeToString() == (
        b"\x0a\x06\x0a\x01K\x12\x01V" + b"\x1a\x0c\x0a\x02/a\x12\x02/b\x1a\x02rw"
        + b"\x22\x06\x0a\x01x\x12\x01y" + b"\x2a\x0f\x0a\x0damd.com/gpu=0")
    p = api.ContainerPreferredAllocationRequest(available_deviceIDs=["1"],
                                                must_include_deviceIDs=["2"], allocation_size=3)
    assert p.SerializeToString() == b"\x0a\x011\x12\x012\x18\x03"
    assert api.method_path("DevicePlugin", "ListAndWatch") == "/v1beta1.DevicePlugin/ListAndWatch"


def test_time_slicing_replicas(plugin_dir):
    """GPU Operator time-slicing parity: <i>::<r> replicas, de-duplicated Allocate,
    spread-first preferred allocation, per-GPU health on every replica."""
    kube, plugin = _start(plugin_dir, replicas=3)
    try:
        reg = kube.wait_registration()
        assert reg.resource_name == "amd.com/gpu"
        stub = kube.plugin_stub(reg.endpoint)
        first = next(iter(stub.ListAndWatch(api.Empty(), timeout=5)))
        ids = [d.ID for d in first.devices]
        assert len(ids) == 24 and ids[:4] == ["0::0", "0::1", "0::2", "1::0"]
        assert [d.topology.nodes[0].ID for d in first.devices][12] == 1
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["2::1", "2::0", "0::2"])
        c = stub.Allocate(req, timeout=5).container_responses[0]
        assert [d.name for d in c.cdi_devices] == ["amd.com/gpu=0", "amd.com/gpu=2"]
        assert c.envs["AMD_GPU_DEVICE_IDS"] == "0,2"
        for bad_id in ("2", "2::3", "9::0", "x::y"):
            bad = api.AllocateRequest()
            bad.container_requests.add(devices_ids=[bad_id])
            with pytest.raises(grpc.RpcError) as e:
                stub.Allocate(bad, timeout=5)
            assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT, bad_id
        # preferred: GPU 0 already has one replica taken (0::0 missing) -> spread over
        # GPUs with the most free replicas first, one replica per GPU before stacking
        pref = api.PreferredAllocationRequest()
        avail = [f"{g}::{r}" for g in range(3) for r in range(3) if (g, r) != (0, 0)]
        pref.container_requests.add(available_deviceIDs=avail, allocation_size=3)
        pref.container_requests.add(available_deviceIDs=avail, must_include_deviceIDs=["0::2"],
                                    allocation_size=2)
        r = stub.GetPreferredAllocation(pref, timeout=5)
        assert list(r.container_responses[0].deviceIDs) == ["1::0", "2::0", "0::1"]
        assert list(r.container_responses[1].deviceIDs) == ["0::2", "1::0"]
    finally:
        plugin.stop()
        kube.stop()


def test_time_slicing_health_rename_and_limit(plugin_dir, tmp_path):
    ff = tmp_path / "faults"
    ff.write_text("")
    kube, plugin = _start(plugin_dir, fault_file=str(ff), replicas=2, rename_shared=True,
                          fail_requests_greater_than_one=True)
    try:
        reg = kube.wait_registration()
        assert reg.resource_name == "amd.com/gpu.shared"
        stub = kube.plugin_stub(reg.endpoint)
        stream = stub.ListAndWatch(api.Empty(), timeout=20)
        assert len(next(stream).devices) == 16
        ff.write_text("5\n")
        health = {d.ID: d.health for d in next(stream).devices}
        assert health["5::0"] == health["5::1"] == api.UNHEALTHY
        assert sum(h == api.HEALTHY for h in health.values()) == 14
        stream.cancel()
        two = api.AllocateRequest()
        two.container_requests.add(devices_ids=["1::0", "1::1"])
        with pytest.raises(grpc.RpcError) as e:
            stub.Allocate(two, timeout=5)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        one = api.AllocateRequest()
        one.container_requests.add(devices_ids=["1::1"])
        assert [d.name for d in stub.Allocate(one, timeout=5).container_responses[0].cdi_devices] \
            == ["amd.com/gpu=1"]
    finally:
        plugin.stop()
        kube.stop()
    with pytest.raises(ValueError):
        PluginConfig(replicas=0)


def test_time_slicing_preferred_allocation_is_numa_compact(plugin_dir):
    """Replica requests spanning several GPUs use the native hive/NUMA policy:
    with GPU 0 fully taken, 4 replicas land on NUMA node 1 (GPUs 4-7) instead
    of the lowest indices 1-4, which would cross NUMA nodes."""
    kube, plugin = _start(plugin_dir, replicas=2)
    try:
        stub = kube.plugin_stub(kube.wait_registration().endpoint)
        pref = api.PreferredAllocationRequest()
        avail = [f"{g}::{r}" for g in range(1, 8) for r in range(2)]
        pref.container_requests.add(available_deviceIDs=avail, allocation_size=4)
        r = stub.GetPreferredAllocation(pref, timeout=5)
        got = list(r.container_responses[0].deviceIDs)
        assert sorted(got) == ["4::0", "5::0", "6::0", "7::0"], got
        # more replicas than GPUs in the compact set: spread first, then stack
        pref = api.PreferredAllocationRequest()
        pref.container_requests.add(available_deviceIDs=avail, allocation_size=9)
        got = list(stub.GetPreferredAllocation(pref, timeout=5).container_responses[0].deviceIDs)
        phys = [g.partition("::")[0] for g in got]
        assert len(set(phys)) == 7 and len(got) == len(set(got)) == 9
    finally:
        plugin.stop()
        kube.stop()
