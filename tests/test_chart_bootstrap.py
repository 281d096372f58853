"""Offline helm rendering, generated deploy/ files, bootstrap dry runs,
containerd config editing and the doctor decision trees."""
import json
import os
import subprocess
import sys

import pytest
import yaml

from mxk8s.bootstrap import hostfiles as hf
from mxk8s.bootstrap import manifests, phases
from mxk8s.chart import gotpl, render
from mxk8s import doctor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FX = os.path.join(REPO, "tests", "fixtures", "sysfs")


# ------------------------------------------------------------------ gotpl
@pytest.mark.parametrize("src,vals,out", [
    ("a{{ .Values.x }}b", {"x": 1}, "a1b"),
    ("{{- if .Values.on }}yes{{ else }}no{{ end -}}", {"on": False}, "no"),
    ("{{ .Values.s | quote }}", {"s": "hi"}, '"hi"'),
    ("{{ .Values.missing | default \"d\" }}", {}, "d"),
    ("{{ range $i, $v := .Values.l }}{{ $i }}={{ $v }};{{ end }}", {"l": ["a", "b"]}, "0=a;1=b;"),
    ("{{ range $k, $v := .Values.m }}{{ $k }}:{{ $v }},{{ end }}", {"m": {"b": 2, "a": 1}}, "a:1,b:2,"),
    ("{{ with .Values.w }}{{ .n }}{{ end }}", {"w": {"n": 7}}, "7"),
    ("{{ if and .Values.a (not .Values.b) }}T{{ end }}", {"a": 1, "b": 0}, "T"),
    ("{{ if eq .Values.k \"x\" }}X{{ else if eq .Values.k \"y\" }}Y{{ end }}", {"k": "y"}, "Y"),
    ("{{ $n := int .Values.g }}{{ if gt $n 2 }}big{{ end }}", {"g": "5"}, "big"),
    ("{{ toYaml .Values.m | nindent 2 }}", {"m": {"a": 1}}, "\n  a: 1"),
    ("x\n  {{- /* comment */ -}}\ny", {}, "xy"),
    ("{{ printf \"%s-%d\" .Values.a 3 }}", {"a": "v"}, "v-3"),
    ("{{ join \",\" .Values.l }}", {"l": [1, 2]}, "1,2"),
])
def test_gotpl(src, vals, out):
    assert gotpl.render_string(src, vals) == out


def test_gotpl_define_include_fail():
    helpers = '{{- define "x.name" -}}{{ .Release.Name }}-x{{- end -}}'
    assert gotpl.render_string('{{ include "x.name" . }}', {}, {"Name": "r"}, helpers=helpers) == "r-x"
    with pytest.raises(gotpl.FailError):
        gotpl.render_string('{{ fail "nope" }}', {})
    with pytest.raises(gotpl.TemplateError):
        gotpl.render_string("{{ if .Values.a }}unterminated", {"a": 1})


# ------------------------------------------------------------------ chart
def _docs(values=None, **kw):
    return render.manifests(render.render(values, **kw))


def test_chart_default_render():
    docs = _docs()
    kinds = {(d["kind"], d["metadata"]["name"]) for d in docs}
    assert ("DaemonSet", "amd-gpu-stack-device-plugin") in kinds
    assert ("DaemonSet", "amd-gpu-stack-node-labeller") in kinds
    assert ("DaemonSet", "amd-gpu-stack-metrics-exporter") in kinds
    assert ("Service", "amd-gpu-stack-metrics") in kinds
    assert ("Job", "amd-gpu-stack-validator") in kinds
    for d in docs:
        if d["kind"] in ("DaemonSet", "Job"):
            spec = d["spec"]["template"]["spec"]
            keys = {t["key"] for t in spec["tolerations"]}
            assert "node-role.kubernetes.io/control-plane" in keys
            assert d["metadata"]["namespace"] == "amd-gpu"
    dp = next(d for d in docs if d["metadata"]["name"] == "amd-gpu-stack-device-plugin")
    assert dp["spec"]["template"]["metadata"]["labels"]["app"] == "amd-gpu-device-plugin"
    mounts = {v["name"]: v["hostPath"]["path"] for v in dp["spec"]["template"]["spec"]["volumes"]}
    assert mounts["device-plugins"] == "/var/lib/kubelet/device-plugins"
    assert mounts["cdi"] == "/etc/cdi"
    job = next(d for d in docs if d["kind"] == "Job")
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 1
    vol = job["spec"]["template"]["spec"]["volumes"][0]
    assert vol["emptyDir"]["medium"] == "Memory"
    ex = next(d for d in docs if d["metadata"]["name"] == "amd-gpu-stack-metrics")
    assert ex["spec"]["ports"][0]["port"] == 9400


def test_chart_driver_enabled_is_rejected():
    v = render.load_values(sets=["driver.enabled=true"])
    with pytest.raises(gotpl.FailError, match="driver.enabled=true is not supported"):
        render.render(v)


def test_chart_values_overrides():
    v = render.load_values(sets=["validator.gpus=8", "exporter.enabled=false",
                                 "validator.ddp.enabled=true", "devicePlugin.deviceSpecs=false"])
    docs = _docs(v)
    names = {d["metadata"]["name"] for d in docs}
    assert "amd-gpu-stack-metrics-exporter" not in names
    job = next(d for d in docs if d["kind"] == "Job")
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    assert "--ddp" in c["args"] and "--gpus=8" in c["args"]
    dp = next(d for d in docs if d["metadata"]["name"] == "amd-gpu-stack-device-plugin")
    assert "--device-specs=false" in dp["spec"]["template"]["spec"]["containers"][0]["args"]
    with pytest.raises(gotpl.FailError):
        render.render(render.load_values(sets=["validator.gpus=9"]))


def test_chart_rccl_env_matches_profiles():
    """rccl.profile / rccl.env render into the validator Job exactly as
    mxk8s/parallel/rccl_env.py resolves them (explicit env wins over the
    profile); unknown variables are rejected by the values schema."""
    from mxk8s.parallel import rccl_env

    def job_env(sets):
        docs = _docs(render.load_values(sets=sets))
        job = next(d for d in docs if d["kind"] == "Job")
        env = job["spec"]["template"]["spec"]["containers"][0]["env"]
        names = [e["name"] for e in env]
        assert len(names) == len(set(names))
        return {e["name"]: e["value"] for e in env if e["name"] != "HSA_ENABLE_IPC_MODE_LEGACY"}

    assert job_env([]) == rccl_env.resolve("xgmi-node")
    assert job_env(["rccl.profile=none"]) == {}
    got = job_env(["rccl.env.NCCL_MIN_NCHANNELS=32", "rccl.env.NCCL_IB_DISABLE=0"])
    assert got == rccl_env.resolve("xgmi-node", {"NCCL_MIN_NCHANNELS": "32", "NCCL_IB_DISABLE": "0"})
    assert got["NCCL_IB_DISABLE"] == "0"
    from mxk8s.config import validate_values
    assert validate_values(render.load_values(sets=["rccl.env.NCCL_PROTO=Simple"])) == []
    assert any("LD_PRELOAD" in e for e in
               validate_values(render.load_values(sets=["rccl.env.LD_PRELOAD=x"])))
    with pytest.raises(ValueError):
        rccl_env.resolve("xgmi-node", {"LD_PRELOAD": "x"})
    env = {"NCCL_IB_DISABLE": "0"}
    assert rccl_env.apply("xgmi-node", environ=env)["NCCL_IB_DISABLE"] == "0"   # set wins
    assert env["TORCH_NCCL_HIGH_PRIORITY"] == "1"
    ex = manifests.rccl_allreduce_8gpu()["spec"]["containers"][0]["env"]
    assert {e["name"] for e in ex} >= set(rccl_env.resolve("xgmi-node"))


def test_chart_service_monitor():
    """exporter.serviceMonitor (dcgm-exporter serviceMonitor counterpart):
    off by default; on, a ServiceMonitor selects the metrics Service's port."""
    assert not [d for d in _docs(render.load_values()) if d["kind"] == "ServiceMonitor"]
    v = render.load_values(sets=["exporter.serviceMonitor.enabled=true",
                                 "exporter.serviceMonitor.interval=30s"])
    v["exporter"]["serviceMonitor"]["additionalLabels"] = {"release": "kube-prometheus-stack"}
    docs = _docs(v)
    sm = next(d for d in docs if d["kind"] == "ServiceMonitor")
    svc = next(d for d in docs if d["kind"] == "Service")
    assert sm["apiVersion"] == "monitoring.coreos.com/v1"
    assert sm["metadata"]["labels"]["release"] == "kube-prometheus-stack"
    assert sm["spec"]["selector"]["matchLabels"].items() <= svc["metadata"]["labels"].items()
    ep = sm["spec"]["endpoints"][0]
    assert ep["port"] == svc["spec"]["ports"][0]["name"] == "metrics"
    assert ep["interval"] == "30s" and ep["honorLabels"] is False
    assert sm["spec"]["namespaceSelector"]["matchNames"] == [svc["metadata"]["namespace"]]
    # schema: a malformed interval is rejected
    from mxk8s import config
    errs = config.validate_values(render.load_values(sets=["exporter.serviceMonitor.interval=soon"]))
    assert any("serviceMonitor.interval" in e for e in errs), errs


def test_chart_time_slicing_args():
    v = render.load_values(sets=["devicePlugin.sharing.timeSlicing.replicas=4",
                                 "devicePlugin.sharing.timeSlicing.failRequestsGreaterThanOne=true"])
    dp = next(d for d in _docs(v) if d["metadata"]["name"] == "amd-gpu-stack-device-plugin")
    args = dp["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "--replicas=4" in args and "--fail-requests-greater-than-one=true" in args
    assert "--rename-shared=false" in args


def test_validator_follows_time_slicing():
    """The validator Job asks for the resource the plugin really advertises,
    and a request the plugin would refuse fails at render time."""
    v = render.load_values(sets=["devicePlugin.sharing.timeSlicing.replicas=2",
                                 "devicePlugin.sharing.timeSlicing.renameByDefault=true",
                                 "validator.gpus=2"])
    job = next(d for d in _docs(v) if d["kind"] == "Job")
    lim = job["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]
    assert lim["amd.com/gpu.shared"] == 2 and "amd.com/gpu" not in lim
    with pytest.raises(gotpl.FailError, match="failRequestsGreaterThanOne"):
        render.render(render.load_values(sets=[
            "devicePlugin.sharing.timeSlicing.replicas=2",
            "devicePlugin.sharing.timeSlicing.failRequestsGreaterThanOne=true", "validator.gpus=4"]))
    # replicas alone keep the plain resource name
    v = render.load_values(sets=["devicePlugin.sharing.timeSlicing.replicas=2"])
    job = next(d for d in _docs(v) if d["kind"] == "Job")
    assert "amd.com/gpu" in job["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"]


def test_validator_detects_stacked_replicas():
    from mxk8s.validate.__main__ import check_allocation
    assert check_allocation(2, {"AMD_GPU_DEVICE_IDS": "0,1"}) == (True, ["0", "1"])
    assert check_allocation(2, {"AMD_GPU_DEVICE_IDS": "3"}) == (False, ["3"])
    assert check_allocation(4, {}) == (True, [])


def test_chart_plugin_health_and_reconcile_args():
    dp = next(d for d in _docs(render.load_values()) if d["metadata"]["name"] == "amd-gpu-stack-device-plugin")
    c = dp["spec"]["template"]["spec"]["containers"][0]
    args = c["args"]
    assert "--ecc-quarantine=0" in args and "--state-dir=/var/lib/mxk8s" in args
    assert "--cdi-spec=/host/etc/cdi/amd.com-gpu.json" in args and "--log-format=json" in args
    mounts = {m["name"]: m["mountPath"] for m in c["volumeMounts"]}
    assert mounts["cdi"] == "/host/etc/cdi" and mounts["state"] == "/var/lib/mxk8s"
    ex = next(d for d in _docs(render.load_values()) if d["metadata"]["name"] == "amd-gpu-stack-metrics-exporter")
    ec = ex["spec"]["template"]["spec"]["containers"][0]
    assert "--health-state-file=/var/lib/mxk8s/health.json" in ec["args"]
    assert any(m["name"] == "state" and m.get("readOnly") for m in ec["volumeMounts"])


def test_chart_partition_manager():
    names = {d["metadata"]["name"] for d in _docs(render.load_values())}
    assert "amd-gpu-stack-partition-manager" not in names          # opt-in, like the MIG manager
    v = render.load_values(sets=["partitionManager.enabled=true", "devicePlugin.partitionNaming=mixed"])
    docs = _docs(v)
    pm = next(d for d in docs if d["metadata"]["name"] == "amd-gpu-stack-partition-manager")
    c = pm["spec"]["template"]["spec"]["containers"][0]
    assert c["command"] == ["python3", "-m", "mxk8s.partition"] and c["securityContext"]["privileged"]
    assert {m["name"] for m in c["volumeMounts"]} >= {"sys", "profiles", "pod-resources"}
    cm = next(d for d in docs if d["kind"] == "ConfigMap" and "partition" in d["metadata"]["name"])
    import json as _json
    assert _json.loads(cm["data"]["profiles.json"])["cpx-nps2"] == {"compute": "CPX", "memory": "NPS2"}
    dp = next(d for d in docs if d["metadata"]["name"] == "amd-gpu-stack-device-plugin")
    assert "--partition-naming=mixed" in dp["spec"]["template"]["spec"]["containers"][0]["args"]
    from mxk8s.config import validate_values
    assert validate_values(render.load_values(sets=["partitionManager.profiles.x.compute=XPX",
                                                    "partitionManager.profiles.x.memory=NPS1"]))


def test_deploy_files_are_up_to_date():
    """deploy/ must equal what the generators produce (single source of truth)."""
    with open(os.path.join(REPO, "deploy", "amd-gpu-stack.yaml")) as f:
        assert f.read().split("\n", 1)[1] == render.to_stream(render.render())
    for name, text in manifests.render_examples().items():
        with open(os.path.join(REPO, "deploy", "examples", name)) as f:
            assert f.read() == text, name
    with open(os.path.join(REPO, "deploy", "kubeadm-config.yaml")) as f:
        assert f.read() == manifests.HEADER + hf.kubeadm_config()


def test_example_manifests_semantics():
    ex = {n: fn() for n, fn in manifests.EXAMPLES.items()}
    hva = ex["hip-vector-add.yaml"]["spec"]
    assert hva["containers"][0]["resources"]["limits"]["amd.com/gpu"] == 1
    assert any(t["key"] == "node-role.kubernetes.io/control-plane" for t in hva["tolerations"])
    r8 = ex["rccl-allreduce-8gpu.yaml"]["spec"]
    assert r8["containers"][0]["resources"]["limits"]["amd.com/gpu"] == 8
    assert r8["volumes"][0]["emptyDir"]["medium"] == "Memory"
    assert "resources" not in ex["busybox-smoke.yaml"]["spec"]["containers"][0]


def test_flannel_manifest_pinned():
    with open(os.path.join(REPO, "deploy", "cni", "kube-flannel.yaml")) as f:
        docs = [d for d in yaml.safe_load_all(f) if d]
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    assert json.loads(cm["data"]["net-conf.json"])["Network"] == hf.POD_CIDR
    ds = next(d for d in docs if d["kind"] == "DaemonSet")
    images = [c["image"] for c in ds["spec"]["template"]["spec"]["containers"] +
              ds["spec"]["template"]["spec"]["initContainers"]]
    assert all(":" in i and not i.endswith(":latest") for i in images)


# ------------------------------------------------------------------ host files
def test_comment_swap():
    fstab = "UUID=1 / ext4 defaults 0 1\n/swap.img none swap sw 0 0\n# /old none swap sw 0 0\n"
    out = hf.comment_swap(fstab)
    assert "#/swap.img none swap sw 0 0" in out and out.startswith("UUID=1 / ext4")
    assert hf.comment_swap(out) == out   # idempotent


@pytest.mark.parametrize("ver", [2, 3])
def test_containerd_config(ver):
    base = hf.minimal_containerd_config(ver)
    out = hf.configure_containerd(base)
    assert "SystemdCgroup = true" in out and "SystemdCgroup = false" not in out
    assert "enable_cdi = true" in out
    assert 'cdi_spec_dirs = ["/etc/cdi", "/var/run/cdi"]' in out
    assert hf.configure_containerd(out) == out   # idempotent
    if ver == 3:
        assert 'io.containerd.cri.v1.runtime' in out


def test_kubeadm_config():
    docs = list(yaml.safe_load_all(hf.kubeadm_config("node1")))
    init, cluster, kubelet = docs
    assert init["nodeRegistration"]["taints"] == []
    assert cluster["networking"]["podSubnet"] == "10.244.0.0/16"
    assert cluster["kubernetesVersion"].startswith("v1.34")
    assert kubelet["cgroupDriver"] == "systemd"


# ------------------------------------------------------------------ bootstrap
def _fake_root(tmp_path):
    root = tmp_path / "root"
    import shutil
    shutil.copytree(os.path.join(FX, "mi355x_8gpu"), root)
    (root / "etc").mkdir(exist_ok=True)
    (root / "etc" / "fstab").write_text("UUID=1 / ext4 defaults 0 1\n/swap.img none swap sw 0 0\n")
    (root / "sys" / "module" / "amdgpu").mkdir(parents=True)
    (root / "proc").mkdir()
    (root / "proc" / "cmdline").write_text("BOOT_IMAGE=/vmlinuz root=/dev/sda1 iommu=pt\n")
    return str(root)


def test_bootstrap_dry_run_all_phases(tmp_path):
    root = _fake_root(tmp_path)
    ctx = phases.Context(root=root, dry_run=True, out=lambda s: None)
    ran = phases.run(ctx)
    assert ran == phases.PHASE_NAMES
    rd = lambda p: open(os.path.join(root, p.lstrip("/"))).read()  # noqa: E731
    assert rd("/etc/modules-load.d/k8s.conf").splitlines()[1:] == ["overlay", "br_netfilter"]
    assert "net.ipv4.ip_forward                 = 1" in rd("/etc/sysctl.d/k8s.conf")
    assert "kernel.numa_balancing = 0" in rd("/etc/sysctl.d/99-amd-gpu.conf")
    assert "#/swap.img" in rd("/etc/fstab")
    assert "enable_cdi = true" in rd("/etc/containerd/config.toml")
    spec = json.loads(rd(hf.CDI_SPEC_PATH))
    assert spec["kind"] == "amd.com/gpu" and len(spec["devices"]) == 17
    assert "podSubnet: 10.244.0.0/16" in rd("/etc/mxk8s/kubeadm-config.yaml")
    cmds = ctx.commands()
    assert "swapoff -a" in cmds and "sysctl --system" in cmds
    assert any(c.startswith("kubeadm init --config") for c in cmds)
    assert any("taint nodes --all node-role.kubernetes.io/control-plane-" in c for c in cmds)
    assert any("kube-flannel.yaml" in c for c in cmds)
    assert any("apt-mark hold kubelet kubeadm kubectl" == c for c in cmds)
    assert not any("nvidia" in c for c in cmds)
    # resumable: a second run skips every completed phase
    ctx2 = phases.Context(root=root, dry_run=True, out=lambda s: None)
    assert phases.run(ctx2) == []
    assert not [a for a in ctx2.actions if a[0] == "write" and a[1] != hf.PHASE_FILE]


def test_bootstrap_driver_gate_blocks(tmp_path):
    root = tmp_path / "bare"
    (root / "etc").mkdir(parents=True)
    ctx = phases.Context(root=str(root), dry_run=True, out=lambda s: None)
    with pytest.raises(phases.PhaseError, match="driver gate failed"):
        phases.run(ctx, until="driver-check")
    assert phases.completed(ctx) == ["preflight", "prep"]   # resumes at driver-check after the reboot


def test_cli_bootstrap_and_render(tmp_path):
    root = _fake_root(tmp_path)
    env = {**os.environ, "PYTHONPATH": REPO}
    r = subprocess.run([sys.executable, "-m", "mxk8s", "bootstrap", "--dry-run", "--root", root,
                        "--phase", "prep", "--phase", "cdi"], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    assert "modprobe br_netfilter" in r.stdout
    r = subprocess.run([sys.executable, "-m", "mxk8s", "render", "--set", "driver.enabled=true"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 1 and "not supported" in r.stderr


# ------------------------------------------------------------------ doctor
def _kubectl_fake(nodes, pods_by_label=None, pods_ns=None, pod=None):
    def k(*args):
        if args[:2] == ("get", "nodes"):
            return 0, json.dumps({"items": nodes})
        if args[:2] == ("get", "pods") and "-l" in args:
            return 0, json.dumps({"items": pods_by_label or []})
        if args[:2] == ("get", "pods") and "-n" in args:
            return 0, json.dumps({"items": (pods_ns or {}).get(args[args.index("-n") + 1], [])})
        if args[:2] == ("get", "pod"):
            return (0, json.dumps(pod)) if pod else (1, "NotFound")
        return 1, "unexpected"
    return k


def test_doctor_gpu_all_ok(tmp_path):
    root = _fake_root(tmp_path)
    ctx = phases.Context(root=root, dry_run=True, out=lambda s: None)
    phases.run(ctx, only=["runtime", "cdi"])
    os.makedirs(os.path.join(root, "var/lib/kubelet/device-plugins"))
    open(os.path.join(root, "var/lib/kubelet/device-plugins/amd-gpu.sock"), "w").close()
    nodes = [{"metadata": {"name": "n"}, "status": {"allocatable": {"amd.com/gpu": "8"}}}]
    pods = [{"status": {"phase": "Running"}}]
    h = doctor.Host(root, kubectl=_kubectl_fake(nodes, pods))
    checks = doctor.check_gpu(h)
    assert [c.name for c in checks if c.status == "fail"] == []
    lines = []
    assert doctor.run(checks, out=lines.append) == 0


def test_doctor_gpu_reports_first_failure(tmp_path):
    root = _fake_root(tmp_path)
    nodes = [{"metadata": {"name": "n"}, "status": {"allocatable": {"amd.com/gpu": "7"}}}]
    h = doctor.Host(root, kubectl=_kubectl_fake(nodes, [{"status": {"phase": "Running"}}]))
    checks = doctor.check_gpu(h)
    failed = [c.name for c in checks if c.status == "fail"]
    assert "CDI spec" in failed and "allocatable amd.com/gpu" in failed
    lines = []
    assert doctor.run(checks, out=lines.append) == 1
    assert "first failure: CDI spec" in lines[-1] and "fix:" in lines[-1]


def test_doctor_allocatable_with_time_slicing(tmp_path):
    root = _fake_root(tmp_path)
    ctx = phases.Context(root=root, dry_run=True, out=lambda s: None)
    phases.run(ctx, only=["runtime", "cdi"])
    os.makedirs(os.path.join(root, "var/lib/kubelet/device-plugins"))
    open(os.path.join(root, "var/lib/kubelet/device-plugins/amd-gpu.sock"), "w").close()
    pods = [{"status": {"phase": "Running"},
             "spec": {"containers": [{"args": ["--resource-name=amd.com/gpu", "--replicas=4",
                                               "--rename-shared=true"]}]}}]
    nodes = [{"metadata": {"name": "n"}, "status": {"allocatable": {"amd.com/gpu.shared": "32"}}}]
    checks = doctor.check_gpu(doctor.Host(root, kubectl=_kubectl_fake(nodes, pods)))
    c = next(c for c in checks if c.name.startswith("allocatable"))
    assert c.name == "allocatable amd.com/gpu.shared" and c.status == "ok", c
    nodes[0]["status"]["allocatable"] = {"amd.com/gpu": "8"}
    checks = doctor.check_gpu(doctor.Host(root, kubectl=_kubectl_fake(nodes, pods)))
    assert next(c for c in checks if c.name.startswith("allocatable")).status == "fail"


def test_doctor_pod_taint_diagnosis():
    pod = {"spec": {"containers": [{"resources": {"limits": {"amd.com/gpu": 1}}}]},
           "status": {"phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "False",
                      "message": "0/1 nodes are available: 1 node(s) had untolerated taint "
                                 "{node-role.kubernetes.io/control-plane: }"}]}}
    h = doctor.Host("/nonexistent", kubectl=_kubectl_fake([], pod=pod))
    checks = doctor.check_pod(h, "p")
    sched = next(c for c in checks if c.name == "scheduling")
    assert sched.status == "fail" and "toleration" in sched.hint


def test_doctor_node(tmp_path):
    root = tmp_path
    (root / "proc" / "sys" / "net" / "ipv4").mkdir(parents=True)
    (root / "proc" / "sys" / "net" / "bridge").mkdir(parents=True)
    (root / "proc" / "swaps").write_text("Filename Type Size Used Priority\n")
    (root / "proc" / "modules").write_text("overlay 1 0 - Live 0\nbr_netfilter 1 0 - Live 0\n")
    (root / "proc" / "sys" / "net" / "ipv4" / "ip_forward").write_text("1\n")
    (root / "proc" / "sys" / "net" / "bridge" / "bridge-nf-call-iptables").write_text("1\n")
    nodes = [{"metadata": {"name": "n"}, "spec": {"taints": []},
              "status": {"conditions": [{"type": "Ready", "status": "True", "message": "ok"}]}}]
    h = doctor.Host(str(root), kubectl=_kubectl_fake(nodes, pods_ns={"kube-system": [
        {"metadata": {"name": "coredns"}, "status": {"phase": "Running"}}]}))
    checks = doctor.check_node(h)
    assert all(c.status != "fail" for c in checks), [(c.name, c.detail) for c in checks]


def test_preflight_and_helm_phases_dry_run(tmp_path):
    root = tmp_path / "host"
    (root / "etc").mkdir(parents=True)
    (root / "etc/os-release").write_text('ID=ubuntu\nVERSION_ID="24.04"\n')
    (root / "proc").mkdir()
    (root / "proc/meminfo").write_text("MemTotal:       3170000000 kB\n")
    out = []
    ctx = phases.Context(root=str(root), dry_run=True, out=out.append)
    phases.phase_preflight(ctx)
    rep = json.loads(out[-1].split("preflight: ", 1)[1])
    assert rep["os_id"] == "ubuntu" and rep["os_version"] == "24.04" and rep["mem_gib"] > 3000
    assert not any("WARNING" in o for o in out)
    phases.phase_helm(ctx)
    cmds = ctx.commands()
    assert any("get.helm.sh/helm-v3" in c and c.startswith("curl") for c in cmds)
    assert any(c.endswith(".sha256sum") for c in cmds)       # checksum fetched, not trusted blindly
    assert any("/usr/local/bin/helm" in c for c in cmds)
    assert phases.PHASE_NAMES[0] == "preflight" and "helm" in phases.PHASE_NAMES
