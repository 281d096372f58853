"""N02 health contract tests over the scriptable fake amd-smi library
(``native/libmxnode/tests/fake_amdsmi.cc``, loaded through MXK8S_AMDSMI_LIB so
the real smi.cc / monitor.cc code paths run): ECC increments, VM faults and
GPU resets each flip a device Unhealthy in ListAndWatch and make Allocate
refuse it, then recover after the quarantine; thermal throttles are counted
and logged, never fatal; the exporter reads the plugin's verdicts.
"""
import json
import logging
import os
import shutil
import subprocess
import tempfile
import time

import pytest

from mxk8s.deviceplugin import api
from mxk8s.deviceplugin.fake_kubelet import FakeKubelet
from mxk8s.deviceplugin.plugin import AmdGpuDevicePlugin, PluginConfig
from mxk8s.native import node

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FX = os.path.join(REPO, "tests", "fixtures", "sysfs")
FAKE_LIB = os.path.join(REPO, "build", "test", "libfake_amdsmi.so")
ROOT = os.path.join(FX, "mi355x_8gpu")


class FakeSmi:
    """Test handle on the fake amd-smi state directory."""

    def __init__(self, d, bdfs):
        self.d = d
        self.gpus = [{"bdf": b, "ecc_ue": 0, "ecc_ce": 0, "gfx": 5, "power": 300,
                      "xgmi_status": "1,1,1,1,1,1,1",
                      "xgmi_read_kb": ",".join(str(100 * (k + 1)) for k in range(7)),
                      "xgmi_write_kb": ",".join(str(50 * (k + 1)) for k in range(7))}
                     for b in bdfs]
        self.write()
        open(os.path.join(d, "events"), "w").close()
        open(os.path.join(d, "procs"), "w").close()

    def write(self):
        with open(os.path.join(self.d, "gpus.tmp"), "w") as f:
            for g in self.gpus:
                f.write(" ".join(f"{k}={v}" for k, v in g.items()) + "\n")
        os.replace(os.path.join(self.d, "gpus.tmp"), os.path.join(self.d, "gpus"))

    def set(self, i, **kv):
        self.gpus[i].update(kv)
        self.write()

    def event(self, gpu, code, msg="x"):
        with open(os.path.join(self.d, "events"), "a") as f:
            f.write(f"{gpu} {code} {msg}\n")

    def procs(self, lines):
        with open(os.path.join(self.d, "procs"), "w") as f:
            f.write("\n".join(lines) + "\n")


@pytest.fixture
def fake_smi(monkeypatch):
    if not os.path.exists(FAKE_LIB):
        subprocess.run(["make", "-C", REPO, "fake-amdsmi"], check=True, capture_output=True)
    d = tempfile.mkdtemp(prefix="mxsmi")
    node.smi_reset()
    monkeypatch.setenv("MXK8S_AMDSMI_LIB", FAKE_LIB)
    monkeypatch.setenv("MXK8S_FAKE_AMDSMI_DIR", d)
    fs = FakeSmi(d, [g.bdf for g in node.enumerate_gpus(ROOT)])
    yield fs
    node.smi_reset()
    shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def plugin_dir():
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _boot_file(tmp_path, boot="boot-a"):
    p = tmp_path / "boot_id"
    p.write_text(boot + "\n")
    return str(p)


def _wait(pred, timeout=5.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        v = pred()
        if v:
            return v
        time.sleep(0.02)
    return pred()


def _start(plugin_dir, state_dir, **kw):
    kube = FakeKubelet(plugin_dir).start()
    cfg = PluginConfig(plugin_dir=plugin_dir, sysfs_root=ROOT, health_interval=0.05,
                       watch_interval=0.1, use_smi_events=True, state_dir=state_dir,
                       reconcile_interval=0, **kw)
    plugin = AmdGpuDevicePlugin(cfg).start()
    return kube, plugin


def _watch(kube):
    stub = kube.plugin_stub(kube.wait_registration().endpoint)
    return stub, iter(stub.ListAndWatch(api.Empty(), timeout=30))


def _health(resp):
    return {d.ID: d.health for d in resp.devices}


def _allocate(stub, ids):
    import grpc
    req = api.AllocateRequest()
    req.container_requests.add(devices_ids=ids)
    try:
        stub.Allocate(req, timeout=5)
        return None
    except grpc.RpcError as e:
        return e


@pytest.mark.parametrize("code,name", [(node.EVT_VMFAULT, "vm fault"),
                                       (node.EVT_GPU_PRE_RESET, "pre-reset")])
def test_smi_event_quarantine_resend_refuse_recover(fake_smi, plugin_dir, tmp_path, code, name):
    kube, plugin = _start(plugin_dir, str(tmp_path / "state"), event_quarantine_s=0.6)
    try:
        assert plugin.monitor.smi_active
        stub, watch = _watch(kube)
        assert set(_health(next(watch)).values()) == {api.HEALTHY}
        fake_smi.event(3, code, name)
        h = _health(next(watch))                     # re-sent on the verdict change
        assert h["3"] == api.UNHEALTHY and sum(v == api.UNHEALTHY for v in h.values()) == 1
        err = _allocate(stub, ["3"])
        assert err is not None and "unhealthy" in err.details()
        assert _allocate(stub, ["2"]) is None        # the others keep serving
        h = _health(next(watch))                     # quarantine over -> healthy again
        assert h["3"] == api.HEALTHY
        assert _allocate(stub, ["3"]) is None
        st = plugin.monitor.status()[3]
        assert (st.vm_faults, st.resets) == ((1, 0) if code == node.EVT_VMFAULT else (0, 1))
    finally:
        plugin.stop()
        kube.stop()


def test_ecc_increment_quarantine_then_recover(fake_smi, plugin_dir, tmp_path):
    kube, plugin = _start(plugin_dir, str(tmp_path / "state"), ecc_quarantine_s=0.6)
    try:
        stub, watch = _watch(kube)
        next(watch)
        # errors already counted when the plugin starts are the baseline: wait for it
        assert _wait(lambda: plugin.monitor.status()[5].ecc_valid)
        fake_smi.set(5, ecc_ue=2)
        h = _health(next(watch))
        assert h["5"] == api.UNHEALTHY
        assert plugin.state.reasons["5"] == "uncorrectable ECC errors"
        assert _allocate(stub, ["5"]) is not None
        assert _health(next(watch))["5"] == api.HEALTHY
        assert plugin.monitor.status()[5].ecc_baseline == 2   # forgiven: new baseline
    finally:
        plugin.stop()
        kube.stop()


def test_ecc_sticky_per_boot_baseline(fake_smi, tmp_path):
    state = str(tmp_path / "state")
    boot = _boot_file(tmp_path, "boot-a")
    fake_smi.set(1, ecc_ue=4)      # errors from before the plugin started: the baseline
    m = node.HealthMonitor(root=ROOT, state_dir=state, boot_id_file=boot)
    m.step(0)
    assert all(s.healthy for s in m.status()) and m.status()[1].ecc_baseline == 4
    fake_smi.set(1, ecc_ue=5)
    m.step(0)
    assert m.status()[1].code == node.UNHEALTHY_ECC
    time.sleep(0.2)
    m.step(0)
    assert m.status()[1].code == node.UNHEALTHY_ECC          # sticky: no quarantine expiry
    ev = [e for e in m.new_events() if e.name == "ecc_uncorrectable"]
    assert len(ev) == 1 and ev[0].index == 1 and ev[0].value == 1
    m.close()
    # plugin restart, same boot: the baseline file keeps the GPU out
    m2 = node.HealthMonitor(root=ROOT, state_dir=state, boot_id_file=boot)
    m2.step(0)
    assert m2.status()[1].code == node.UNHEALTHY_ECC
    m2.close()
    # after a reboot (new boot id) the current count is the new baseline
    m3 = node.HealthMonitor(root=ROOT, state_dir=state, boot_id_file=_boot_file(tmp_path, "boot-b"))
    m3.step(0)
    assert m3.status()[1].healthy and m3.status()[1].ecc_baseline == 5
    m3.close()


def test_thermal_throttle_counted_and_logged_not_fatal(fake_smi, plugin_dir, tmp_path, caplog):
    caplog.set_level(logging.INFO, logger="mxk8s.deviceplugin")
    state = str(tmp_path / "state")
    kube, plugin = _start(plugin_dir, state)
    try:
        _watch(kube)
        fake_smi.event(6, node.EVT_THERMAL_THROTTLE, "hotspot 105C")
        fake_smi.event(6, node.EVT_THERMAL_THROTTLE, "hotspot 106C")
        assert _wait(lambda: plugin.monitor.status()[6].thermal_throttles == 2)
        assert plugin.state.health["6"] == api.HEALTHY
        recs = _wait(lambda: [r for r in caplog.records if getattr(r, "event", "") == "thermal_throttle"])
        assert len(recs) == 2 and recs[0].device == "6"
        doc = _wait(lambda: _read_json(os.path.join(state, "health.json")))
        assert _wait(lambda: _read_json(os.path.join(state, "health.json"))["gpus"][6]["thermal_throttles"] == 2)
        assert doc["smi"] is True and all(g["healthy"] for g in doc["gpus"])
    finally:
        plugin.stop()
        kube.stop()


def _read_json(p):
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def test_exporter_reads_plugin_health_state(fake_smi, plugin_dir, tmp_path):
    """amd_gpu_device_healthy comes from the plugin's verdicts, so the two can
    never disagree (an amd-smi quarantine is invisible to sysfs)."""
    from mxk8s.exporter import Exporter, ExporterConfig, SmiBackend

    state = str(tmp_path / "state")
    kube, plugin = _start(plugin_dir, state, event_quarantine_s=30)
    try:
        _watch(kube)
        fake_smi.event(2, node.EVT_VMFAULT, "fault")
        assert _wait(lambda: (_read_json(os.path.join(state, "health.json")) or {"gpus": [{}] * 8})
                     ["gpus"][2].get("healthy") is False)
        exp = Exporter(ExporterConfig(sysfs_root=ROOT, pod_resources=False,
                                      health_state_file=os.path.join(state, "health.json")),
                       backend=SmiBackend(ROOT))
        text = exp.sample_once()
        line = [l for l in text.splitlines() if l.startswith('amd_gpu_device_healthy{gpu="2"')]
        assert len(line) == 1 and line[0].endswith(" 0")
        assert 'source="device-plugin"' in line[0] and 'reason="amd-smi reset/fault event"' in line[0]
        other = [l for l in text.splitlines() if l.startswith('amd_gpu_device_healthy{gpu="1"')]
        assert other[0].endswith(" 1")
        assert [l for l in text.splitlines() if l.startswith('amd_gpu_vm_faults_total{gpu="2"')][0].endswith(" 1")
        # live xGMI state + traffic from amd-smi link metrics (fake: 7 links per GPU)
        up = [l for l in text.splitlines() if l.startswith('amd_gpu_xgmi_link_up{gpu="0"')]
        assert len(up) == 7 and all(l.endswith(" 1") for l in up)
        rd = [l for l in text.splitlines() if l.startswith('amd_gpu_xgmi_read_bytes_total{gpu="0"')]
        assert len(rd) == 7 and rd[0].endswith(f" {100 * 1024}") and 'peer_bdf="0000:15:00.0"' in rd[0]
        assert 'link="0"' not in rd[0]      # traffic is keyed by peer, state by link slot
        # a stale state file (plugin gone) falls back to the sysfs verdict
        doc = json.load(open(os.path.join(state, "health.json")))
        doc["unix_ms"] = 0
        stale = str(tmp_path / "stale.json")
        json.dump(doc, open(stale, "w"))
        exp2 = Exporter(ExporterConfig(sysfs_root=ROOT, pod_resources=False, health_state_file=stale),
                        backend=SmiBackend(ROOT))
        line = [l for l in exp2.sample_once().splitlines() if l.startswith('amd_gpu_device_healthy{gpu="2"')]
        assert 'source="sysfs"' in line[0] and line[0].endswith(" 1")
    finally:
        plugin.stop()
        kube.stop()


def test_reconcile_rewrites_stale_cdi_and_readvertises(plugin_dir, tmp_path):
    """A renumbered render node (driver reload) makes the CDI spec stale: the
    plugin rewrites it atomically and re-sends ListAndWatch."""
    root = str(tmp_path / "sysfs")
    shutil.copytree(ROOT, root, symlinks=True)
    cdi = str(tmp_path / "cdi" / "amd.com-gpu.json")
    kube = FakeKubelet(plugin_dir).start()
    cfg = PluginConfig(plugin_dir=plugin_dir, sysfs_root=root, health_interval=0.05,
                       watch_interval=0.1, use_smi_events=False, cdi_spec_path=cdi,
                       reconcile_interval=0.1)
    plugin = AmdGpuDevicePlugin(cfg).start()
    try:
        stub, watch = _watch(kube)
        next(watch)
        assert _wait(lambda: _read_json(cdi))                  # created when missing
        spec = _read_json(cdi)
        assert "/dev/dri/renderD135" in json.dumps(spec)
        # driver reload renumbers GPU 7's render node 135 -> 199
        props = _kfd_props_for_minor(root, 135)
        text = open(props).read().replace("drm_render_minor 135", "drm_render_minor 199")
        open(props, "w").write(text)
        os.rename(os.path.join(root, "dev", "dri", "renderD135"),
                  os.path.join(root, "dev", "dri", "renderD199"))
        resp = next(watch)                                     # re-advertised
        assert len(resp.devices) == 8
        assert _wait(lambda: "/dev/dri/renderD199" in json.dumps(_read_json(cdi) or {}))
        assert "/dev/dri/renderD135" not in json.dumps(_read_json(cdi))
        # the counters move just after the rename / resend the asserts above saw
        assert _wait(lambda: plugin.reconciles["cdi_rewritten"] >= 2)
        assert plugin.reconciles["gpus_changed"] == 1
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["7"])
        c = stub.Allocate(req, timeout=5).container_responses[0]
        assert "/dev/dri/renderD199" in [d.host_path for d in c.devices]
        # a hand-edited (stale) spec is put back
        with open(cdi, "w") as f:
            f.write("{}")
        assert _wait(lambda: (_read_json(cdi) or {}).get("kind") == "amd.com/gpu")
    finally:
        plugin.stop()
        kube.stop()


def _kfd_props_for_minor(root, minor):
    base = os.path.join(root, "sys", "class", "kfd", "kfd", "topology", "nodes")
    for n in os.listdir(base):
        p = os.path.join(base, n, "properties")
        if os.path.exists(p) and f"drm_render_minor {minor}\n" in open(p).read():
            return p
    raise AssertionError(f"no KFD node with render minor {minor}")


def test_json_log_format():
    import io

    from mxk8s.utils.logs import JsonFormatter
    rec = logging.LogRecord("mxk8s.deviceplugin", logging.WARNING, __file__, 1,
                            "device %s -> %s", ("3", "Unhealthy"), None)
    rec.device, rec.event, rec.reason, rec.other = "3", "health_change", "uncorrectable ECC errors", 7
    out = json.loads(JsonFormatter().format(rec))
    assert out["msg"] == "device 3 -> Unhealthy" and out["level"] == "WARNING"
    assert (out["device"], out["event"], out["reason"]) == ("3", "health_change", "uncorrectable ECC errors")
    assert out["extra"] == {"other": 7} and out["ts"].endswith("Z")
    del io


def test_exporter_process_vram_and_link_down(fake_smi, tmp_path):
    from mxk8s.exporter import Exporter, ExporterConfig, SmiBackend
    fake_smi.procs(["0 4242 python3 68719476736 trainer", "0 4243 rccl-proxy 1048576", "4 77 hip_vector_add 4096"])
    fake_smi.set(3, xgmi_status="1,1,0,1,1,2,1")
    exp = Exporter(ExporterConfig(sysfs_root=ROOT, pod_resources=False), backend=SmiBackend(ROOT))
    text = exp.sample_once()
    pm = [l for l in text.splitlines() if l.startswith("amd_gpu_process_memory_bytes{")]
    assert len(pm) == 3
    assert any('gpu="0"' in l and 'pid="4242"' in l and 'process="python3"' in l and l.endswith(" 68719476736")
               for l in pm)
    down = [l for l in text.splitlines() if l.startswith('amd_gpu_xgmi_link_up{gpu="3"') and l.endswith(" 0")]
    assert len(down) == 2 and any('status="disabled"' in l for l in down)


def test_exporter_energy_counter(fake_smi, tmp_path):
    """amdsmi_get_energy_count (accumulator x resolution, uJ) becomes
    amd_gpu_energy_joules_total; a GPU without the counter emits no series."""
    from mxk8s.exporter import Exporter, ExporterConfig, SmiBackend
    fake_smi.set(2, energy=1234567890)
    exp = Exporter(ExporterConfig(sysfs_root=ROOT, pod_resources=False), backend=SmiBackend(ROOT))
    text = exp.sample_once()
    en = [l for l in text.splitlines() if l.startswith("amd_gpu_energy_joules_total{")]
    assert len(en) == 1 and 'gpu="2"' in en[0]
    assert abs(float(en[0].rsplit(" ", 1)[1]) - 1234.568) < 0.05
    assert "# TYPE amd_gpu_energy_joules_total counter" in text


def test_refcounted_session_and_reinit_generation(fake_smi):
    ok, _ = node.smi_open()
    assert ok and node.smi_count() == 8
    g0 = node.smi_generation()
    ok2, _ = node.smi_open()                     # a second user shares the session
    assert ok2 and node.smi_generation() == g0
    node.smi_close()
    assert node.smi_count() == 8                 # still open for the first user
    # amd-smi enumerates at init: a grown GPU list is only seen after a re-init
    fake_smi.gpus += [dict(fake_smi.gpus[0], partition=1)]
    fake_smi.write()
    assert node.smi_count() == 8
    assert node.smi_reinit()[0] and node.smi_count() == 9
    assert node.smi_generation() != g0
    assert node.smi_sample(8).key == fake_smi.gpus[0]["bdf"] + "#1"
    node.smi_close()
    assert node.smi_count() == -1                # last reference gone


def test_spx_to_cpx_with_amd_smi_active(fake_smi, tmp_path):
    """SURVEY R26h / VERDICT r2 #1: a compute-partition change while amd-smi
    is live.  The plugin's new monitor re-initialises amd-smi (8 -> 64
    handles) and matches every partition by BDF + partition id, so ECC and
    VM-fault health cover all 64 partitions; ListAndWatch re-sends 64
    devices; an exporter backend opened before the change re-maps too."""
    import test_partition as tp
    from mxk8s import partition
    from mxk8s.exporter import Exporter, ExporterConfig, SmiBackend

    root = tp.spx_root(str(tmp_path))
    state = str(tmp_path / "state")
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    kube = FakeKubelet(d).start()
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=d, sysfs_root=root, health_interval=0.05,
                                             watch_interval=0.1, use_smi_events=True,
                                             state_dir=state, reconcile_interval=0.1,
                                             event_quarantine_s=30)).start()
    exp_backend = SmiBackend(root)
    drv = tp.FakeDriver(root)
    try:
        stub, watch = _watch(kube)
        assert len(next(watch).devices) == 8
        assert all(st.smi_index >= 0 for st in plugin.monitor.status())
        assert len(exp_backend.samples()) == 8
        # the node is repartitioned: KFD shows 64 GPUs, amd-smi (after init) 64
        fake_smi.gpus = [dict(fake_smi.gpus[k], partition=p) for k in range(8) for p in range(8)]
        fake_smi.write()
        drv.start()
        client = tp.FakeNodeClient("n1", {partition.CONFIG_LABEL: "cpx-nps2"})
        res = partition.PartitionManager(client, "n1", root, settle_timeout=10,
                                         poll=0.02).reconcile_once()
        assert res.state == "success", res
        devs = _wait(lambda: (lambda r: r.devices if len(r.devices) == 64 else None)(next(watch)),
                     timeout=10)
        assert devs and len(devs) == 64
        st = _wait(lambda: (lambda s: s if len(s) == 64 and all(x.smi_index >= 0 for x in s)
                            else None)(plugin.monitor.status()))
        assert st, [x.smi_index for x in plugin.monitor.status()]
        # amd-smi index k is the k-th line: device k // 8, partition k % 8 == KFD order
        assert [x.smi_index for x in st] == list(range(64))
        # health of a partition that did not exist before the change
        fake_smi.event(37, node.EVT_VMFAULT, "partition fault")
        h = _wait(lambda: (lambda r: r if _health(r).get("37") == api.UNHEALTHY else None)(next(watch)))
        assert h and sum(v == api.UNHEALTHY for v in _health(h).values()) == 1
        assert _wait(lambda: all(x.ecc_valid for x in plugin.monitor.status()))
        fake_smi.set(53, ecc_ue=1)
        assert _wait(lambda: plugin.state.health["53"] == api.UNHEALTHY)
        assert plugin.state.reasons["53"] == "uncorrectable ECC errors"
        # exporter: samples for every partition (re-mapped on the new generation)
        exp = Exporter(ExporterConfig(sysfs_root=root, pod_resources=False,
                                      health_state_file=os.path.join(state, "health.json")),
                       backend=exp_backend)
        text = exp.sample_once()
        pw = [l for l in text.splitlines() if l.startswith("amd_gpu_power_watts{")]
        assert len(pw) == 64 and any('bdf="0000:15:00.0"' in l and 'partition="1"' in l for l in pw)
        assert len(exp_backend.samples()) == 64
    finally:
        drv.stop.set()
        exp_backend.close()
        plugin.stop()
        kube.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_exporter_alone_reinits_after_partition_change(fake_smi, tmp_path):
    """The exporter runs in its own pod (its own amd-smi session): it notices
    the KFD / amd-smi count mismatch itself and re-initialises."""
    import test_partition as tp
    from mxk8s.exporter import SmiBackend

    root = str(tmp_path / "cpx")
    tp.make_sysfs.tree_partitioned(root, "CPX", "NPS2")
    be = SmiBackend(root)                          # session opened with 8 handles
    try:
        assert node.smi_count() == 8
        fake_smi.gpus = [dict(fake_smi.gpus[k], partition=p) for k in range(8) for p in range(8)]
        fake_smi.write()
        got = be.samples()
        assert len(got) == 64 and be.reinits == 1
        assert got["0000:15:00.0#1"].partition_id == 1
        assert len(be.samples()) == 64 and be.reinits == 1   # no re-init once they agree
    finally:
        be.close()
