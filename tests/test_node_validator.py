"""Node validator (operator-validator counterpart; the reference
waits for the operator's validator pods at /root/reference/README.md:283-286)
over fake sysfs trees and a fake kubelet: the marker chain, marker validity
per boot + driver instance, the device plugin holding until driver-ready
appears, withdrawal and re-validation after a simulated driver reload, and
the exporter / doctor views of the markers."""
import json
import os
import shutil
import tempfile
import threading
import time

import pytest

from mxk8s.deviceplugin import api
from mxk8s.deviceplugin.fake_kubelet import FakeKubelet
from mxk8s.deviceplugin.plugin import AmdGpuDevicePlugin, PluginConfig
from mxk8s.native import node
from mxk8s.validate import node as vnode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FX = os.path.join(REPO, "tests", "fixtures", "sysfs", "mi355x_8gpu")


def _root(tmp_path, boot="boot-a"):
    root = str(tmp_path / "root")
    shutil.copytree(FX, root, symlinks=True)
    os.makedirs(os.path.join(root, "sys/module/amdgpu"))
    _w(root, "sys/class/kfd/kfd/topology/generation_id", "1\n")
    _w(root, "proc/sys/kernel/random/boot_id", boot + "\n")
    return root


def _w(root, rel, text):
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(text)


def _wait(pred, timeout=5.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        v = pred()
        if v:
            return v
        time.sleep(0.02)
    return pred()


def test_driver_marker_valid_per_boot_and_driver_instance(tmp_path):
    root, state = _root(tmp_path), str(tmp_path / "state")
    v = vnode.NodeValidator(state, root, ["driver"], step_timeout=0.1, poll=0.01)
    assert v.run_chain()
    m = vnode.read_marker(state, "driver")
    assert m["ok"] and m["detail"]["gpus"] == 8 and m["detail"]["archs"] == ["gfx950"]
    assert vnode.marker_valid(state, "driver", root)
    # a driver reload re-creates the KFD topology: every marker is void at once
    _w(root, "sys/class/kfd/kfd/topology/generation_id", "2\n")
    assert not vnode.marker_valid(state, "driver", root)
    _w(root, "sys/class/kfd/kfd/topology/generation_id", "1\n")
    assert vnode.marker_valid(state, "driver", root)
    # a reboot voids it too
    _w(root, "proc/sys/kernel/random/boot_id", "boot-b\n")
    assert not vnode.marker_valid(state, "driver", root)


def test_driver_step_fails_without_module_or_render_node(tmp_path):
    root, state = _root(tmp_path), str(tmp_path / "state")
    os.rmdir(os.path.join(root, "sys/module/amdgpu"))
    ok, facts = vnode.check_driver(root)
    assert not ok and facts["amdgpu_module"] is False
    os.makedirs(os.path.join(root, "sys/module/amdgpu"))
    os.unlink(os.path.join(root, "dev/dri/renderD130"))
    ok, facts = vnode.check_driver(root)
    assert not ok and facts["missing_render_nodes"] == [2]
    v = vnode.NodeValidator(state, root, ["driver"], step_timeout=0.05, poll=0.01)
    assert not v.run_chain() and vnode.read_marker(state, "driver") is None


def test_cdi_step_waits_for_a_current_spec(tmp_path):
    root, state = _root(tmp_path), str(tmp_path / "state")
    spec = str(tmp_path / "cdi" / "amd.com-gpu.json")
    v = vnode.NodeValidator(state, root, ["driver", "cdi"], cdi_spec=spec, step_timeout=0.1,
                            poll=0.01)
    assert not v.run_chain()                        # spec missing
    assert vnode.status(state, root, ["driver", "cdi"]) == {"driver": True, "cdi": False}
    os.makedirs(os.path.dirname(spec))
    stale = node.cdi_spec(root)
    stale["devices"] = stale["devices"][:3]
    json.dump(stale, open(spec, "w"))
    assert not v.run_chain()                        # stale spec
    open(spec, "w").write(node.cdi_spec_text(root))
    assert v.run_chain() and vnode.status(state, root, ["driver", "cdi"]) == {"driver": True, "cdi": True}


def test_vectoradd_step_every_gpu(tmp_path):
    root, state = _root(tmp_path), str(tmp_path / "state")
    ran = []

    def run(i):
        ran.append(i)
        return (i != 5, "RESULT {}" if i != 5 else "mismatch")

    v = vnode.NodeValidator(state, root, ["vectoradd"], step_timeout=0.05, poll=0.01, vectoradd=run)
    assert not v.run_chain()
    assert sorted(set(ran)) == list(range(8))
    v2 = vnode.NodeValidator(state, root, ["vectoradd"], step_timeout=0.05, poll=0.01,
                             vectoradd=lambda i: (True, ""))
    assert v2.run_chain() and vnode.read_marker(state, "vectoradd")["detail"]["gpus"] == 8


def test_plugin_holds_until_driver_ready_then_revalidates_after_reload(tmp_path):
    """The plugin serves nothing before driver-ready; once serving, a driver
    reload (new KFD topology generation) withdraws every device until the
    validator re-validated the new driver instance."""
    root, state = _root(tmp_path), str(tmp_path / "state")
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    kube = FakeKubelet(d).start()
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=d, sysfs_root=root, health_interval=0.05,
                                             watch_interval=0.05, use_smi_events=False,
                                             reconcile_interval=0, state_dir=state,
                                             require_validation=("driver",)))
    t = threading.Thread(target=plugin.start, daemon=True)
    t.start()
    try:
        time.sleep(0.5)
        assert kube.registrations.empty() and not os.path.exists(os.path.join(d, "amd-gpu.sock"))
        v = vnode.NodeValidator(state, root, ["driver", "plugin"], plugin_dir=d, step_timeout=10,
                                poll=0.02)
        assert v.run_chain()                        # driver-ready, then the plugin answers
        reg = kube.wait_registration(timeout=5)
        assert reg.resource_name == "amd.com/gpu"
        pm = vnode.read_marker(state, "plugin")["detail"]
        assert pm["devices"] == 8 and pm["healthy"] == 8 and "/dev/kfd" in pm["allocate"]["devices"]
        watch = iter(kube.plugin_stub(reg.endpoint).ListAndWatch(api.Empty(), timeout=30))
        assert {x.health for x in next(watch).devices} == {api.HEALTHY}
        # driver reload: the old markers no longer match the driver instance
        _w(root, "sys/class/kfd/kfd/topology/generation_id", "7\n")
        r = next(watch)
        assert {x.health for x in r.devices} == {api.UNHEALTHY}
        assert plugin.state.reasons["0"] == "driver validation pending"
        # the validator's watch notices the new instance and re-validates
        fp = v.watch_once(None)
        v.steps = ["driver"]
        assert v.watch_once(fp) == fp and vnode.marker_valid(state, "driver", root)
        r = next(watch)
        assert {x.health for x in r.devices} == {api.HEALTHY}
    finally:
        plugin.stop()
        kube.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_watch_drops_markers_on_new_driver_instance(tmp_path):
    root, state = _root(tmp_path), str(tmp_path / "state")
    v = vnode.NodeValidator(state, root, ["driver", "vectoradd"], step_timeout=0.05, poll=0.01,
                            vectoradd=lambda i: (True, ""))
    fp = v.watch_once(None)
    assert all(vnode.status(state, root, v.steps).values()) and v.runs == 1
    assert v.watch_once(fp) == fp and v.runs == 1   # nothing to do
    _w(root, "sys/class/kfd/kfd/topology/generation_id", "9\n")
    fp2 = v.watch_once(fp)
    assert fp2 != fp and v.runs == 2 and all(vnode.status(state, root, v.steps).values())
    assert vnode.read_marker(state, "driver")["fingerprint"] == fp2


def test_wait_for_times_out_and_cli_wait(tmp_path):
    root, state = _root(tmp_path), str(tmp_path / "state")
    assert not vnode.wait_for(state, ["driver"], root, timeout=0.1, poll=0.02)
    assert vnode.main(["--state-dir", state, "--sysfs-root", root, "--steps", "driver",
                       "--log-format", "text"]) == 0
    assert vnode.main(["--state-dir", state, "--sysfs-root", root, "--wait", "driver",
                       "--timeout", "1", "--log-format", "text"]) == 0
    with pytest.raises(ValueError):
        vnode.NodeValidator(state, root, ["toolkit"])


def test_exporter_and_doctor_report_validations(tmp_path):
    from mxk8s import doctor
    from mxk8s.exporter import Exporter, ExporterConfig

    class Backend:
        ok, driver = True, "x"

        def gpus(self):
            return node.enumerate_gpus(root)

        def samples(self):
            return {}

        def health(self, i):
            return 0

    root = _root(tmp_path)
    state = os.path.join(root, "var/lib/mxk8s")
    vnode.NodeValidator(state, root, ["driver"], step_timeout=0.1, poll=0.01).run_chain()
    exp = Exporter(ExporterConfig(sysfs_root=root, pod_resources=False, state_dir=state),
                   backend=Backend())
    text = exp.sample_once()
    assert 'amd_gpu_stack_component_up{component="validation"} 0' in text   # cdi etc. missing
    assert 'amd_gpu_validation_ready{step="driver"} 1' in text
    assert 'amd_gpu_validation_ready{step="plugin"} 0' in text
    exp.cfg.validation_steps = ("driver",)
    assert 'amd_gpu_stack_component_up{component="validation"} 1' in exp.sample_once()
    checks = doctor.check_gpu(doctor.Host(root, kubectl=lambda *a: (127, "no kubectl")))
    c = next(c for c in checks if c.name == "node validation")
    assert c.status == "fail" and "driver=ready" in c.detail and "cdi-validation" in c.hint


def test_plugin_step_finds_the_mixed_naming_partition_socket(tmp_path):
    """with partitionNaming=mixed on a CPX node the plugin serves
    amd.com/gpu-cpx on amd-gpu-cpx.sock; the plugin validation must probe that
    socket (resolved as the plugin resolves it), not amd-gpu.sock — else the
    node-validator crash-loops on every partitioned node."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests", "fixtures"))
    import make_sysfs
    root = str(tmp_path / "root")
    make_sysfs.tree_partitioned(root, "CPX", "NPS2")
    state = str(tmp_path / "state")
    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    kube = FakeKubelet(d).start()
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=d, sysfs_root=root, health_interval=0.05,
                                             watch_interval=0.1, use_smi_events=False,
                                             reconcile_interval=0,
                                             partition_naming="mixed")).start()
    try:
        reg = kube.wait_registration()
        assert reg.resource_name == "amd.com/gpu-cpx" and reg.endpoint == "amd-gpu-cpx.sock"
        v = vnode.NodeValidator(state, root, ["plugin"], plugin_dir=d, step_timeout=5, poll=0.05,
                                partition_naming="mixed")
        assert v.plugin_socket_for(node.enumerate_gpus(root)) == "amd-gpu-cpx.sock"
        assert v.run_chain()
        pm = vnode.read_marker(state, "plugin")["detail"]
        assert pm["socket"].endswith("amd-gpu-cpx.sock") and pm["devices"] == 64
        # single naming on the same node: the base socket (what the plugin serves then)
        assert vnode.NodeValidator(state, root, ["plugin"], plugin_dir=d).plugin_socket_for(
            node.enumerate_gpus(root)) == "amd-gpu.sock"
    finally:
        plugin.stop()
        kube.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_chart_passes_the_plugin_naming_to_the_validator():
    from mxk8s.chart import render
    values = render.deep_merge(render.load_values(render.CHART_DIR),
                               {"devicePlugin": {"partitionNaming": "mixed"}})
    docs = render.manifests(render.render(values))
    ds = next(x for x in docs if x["kind"] == "DaemonSet"
              and x["metadata"]["name"].endswith("node-validator"))
    pod = ds["spec"]["template"]["spec"]
    for c in pod["initContainers"] + pod["containers"]:
        cmd = " ".join(c["command"])
        if "plugin" in cmd.split("--steps=", 1)[-1].split()[0]:
            assert "--partition-naming=mixed" in cmd and "--resource-name=amd.com/gpu" in cmd, cmd
