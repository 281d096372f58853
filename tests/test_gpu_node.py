"""Node stack against the real MI355X box (SURVEY.md §4.2 "GPU unit" tier):
libmxnode's KFD enumeration, CDI spec, health check and amd-smi sampler on
live sysfs / amd-smi, and the native validator binaries (vectoradd, GEMM,
RCCL all-reduce at n = 1) the validator Job runs.  The CPU tier covers the
same code against fake sysfs trees (tests/test_node_native.py)."""
from __future__ import annotations

import json
import os
import subprocess

import pytest

from mxk8s.native import node

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "bin")


def _results(stdout: str) -> list[dict]:
    return [json.loads(line[7:]) for line in stdout.splitlines() if line.startswith("RESULT ")]


def _run(args, timeout=120):
    p = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (args, p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    return p.stdout


def test_live_enumeration_finds_gfx950_with_render_node():
    gpus = node.enumerate_gpus("")
    assert gpus, "no AMD GPU in the live KFD topology"
    mi = [g for g in gpus if g.arch == "gfx950"]
    assert mi, [g.arch for g in gpus]
    for g in mi:
        assert g.render_minor >= 128
        assert os.path.exists(f"/dev/dri/renderD{g.render_minor}")
        assert g.simd_count >= 1024          # 256 CUs x 4 SIMDs on MI355X
        assert node.health_check(g.index, "") == 0, node.health_reason(node.health_check(g.index, ""))


def test_live_cdi_spec_names_kfd_and_render_nodes():
    spec = node.cdi_spec("")
    assert spec["kind"] == "amd.com/gpu"
    top = [d["path"] for d in spec["containerEdits"]["deviceNodes"]]
    assert "/dev/kfd" in top
    names = {d["name"] for d in spec["devices"]}
    assert "all" in names and "0" in names
    dev0 = next(d for d in spec["devices"] if d["name"] == "0")
    paths = [n["path"] for n in dev0["containerEdits"]["deviceNodes"]]
    assert any(p.startswith("/dev/dri/renderD") for p in paths)


def test_live_smi_sample_is_sane():
    ok, err = node.smi_open()
    assert ok, f"amd-smi unavailable: {err}"
    assert node.smi_count() >= 1
    s = node.smi_sample(0)
    assert s.valid
    # 288 GB HBM3E per MI355X (the driver reports ~309e9 bytes)
    assert 250 * 2 ** 30 <= s.vram_total_bytes <= 300 * 2 ** 30, s.vram_total_bytes
    assert 0 <= s.vram_used_bytes <= s.vram_total_bytes
    assert 100 <= s.power_limit_w <= 3000, s.power_limit_w
    assert s.mclk_mhz > 0
    assert s.ecc_uncorrectable == 0


def test_live_energy_counter_tracks_power():
    """amd_gpu_energy_joules_total's source: the amd-smi accumulator advances
    by about socket power x elapsed time (probe on MI355X: 278.7 J over 1 s
    at 277 W)."""
    import time
    ok, err = node.smi_open()
    assert ok, err
    s1 = node.smi_sample(0)
    assert s1.energy_j is not None and s1.energy_j > 0
    t0 = time.perf_counter()
    time.sleep(1.0)
    s2 = node.smi_sample(0)
    dt = time.perf_counter() - t0
    de = s2.energy_j - s1.energy_j
    p = max(1, (s1.power_w + s2.power_w) / 2)
    assert 0.3 * p * dt <= de <= 3.0 * p * dt, (de, p, dt)


def test_vector_add_binary_passes():
    res = _results(_run([os.path.join(BIN, "mx-vector-add"), "--n", "50000"]))
    assert res and res[-1]["test"] == "vectoradd" and res[-1]["pass"], res


def test_vector_add_binary_checks_isolation():
    """Config 2's isolation criterion on the real device (BASELINE.md:37):
    the one-GPU box passes --expect-gpus 1 --expect-arch gfx950 with the
    Allocate environment of its own render node, and fails (exit 1,
    pass=false) when told to expect 8 GPUs, another arch or another node."""
    from mxk8s.validate import isolation
    exe = os.path.join(BIN, "mx-vector-add")
    ok = _results(_run([exe, "--n", "50000", "--bw-mib", "0", "--expect-gpus", "1",
                        "--expect-arch", "gfx950"]))
    r = ok[-1]
    assert r["pass"] and r["visible_gpus"] == 1 and r["arch"] == "gfx950", r
    assert all(r["isolation"].values()), r
    assert isolation.check_results(ok, gpus=1, arch="gfx950") == [], r
    env_ok = dict(os.environ, AMD_GPU_RENDER_NODES=",".join(r["render_nodes"]),
                  AMD_GPU_BDFS=",".join(r["bdfs"]), AMD_GPU_DEVICE_IDS="0", AMD_GPU_ARCH="gfx950")
    p = subprocess.run([exe, "--n", "50000", "--bw-mib", "0"], capture_output=True, text=True,
                       timeout=120, env=env_ok)
    assert p.returncode == 0, p.stdout[-2000:]
    for args, env in (
            (["--expect-gpus", "8"], None),
            (["--expect-arch", "gfx942"], None),
            ([], dict(env_ok, AMD_GPU_RENDER_NODES="/dev/dri/renderD250")),
            ([], dict(env_ok, AMD_GPU_BDFS="0000:ff:00.0"))):
        p = subprocess.run([exe, "--n", "50000", "--bw-mib", "0", *args], capture_output=True,
                           text=True, timeout=120, env=env or os.environ)
        bad = _results(p.stdout)
        assert p.returncode == 1 and bad and bad[-1]["pass"] is False, (args, p.stdout[-2000:])
        assert isolation.check_results(bad, gpus=1, arch="gfx950"), (args, bad)


def test_gemm_bench_binary_self_checks():
    out = _run([os.path.join(BIN, "mx-gemm-bench"), "--sizes", "4096", "--iters", "10",
                "--warmup-ms", "200"])
    res = _results(out)
    assert res, out[-2000:]
    r = res[-1]
    assert r["test"] == "gemm" and r["pass"], r
    assert r["tflops"] > 500, r
    assert 0 < r["max_abs_err"] <= r["spot_tolerance"] and r["rel_err_vs_rocblas"] is not None, r


def test_gemm_bench_binary_fails_when_kernel_skipped():
    """Fault injection: the checked launch is skipped, the poisoned output
    must fail both the fp32 spot check and the rocBLAS comparison."""
    env = dict(os.environ, MXK_GEMM_BENCH_SKIP_KERNEL="1")
    p = subprocess.run([os.path.join(BIN, "mx-gemm-bench"), "--sizes", "1024", "--iters", "3",
                        "--warmup-ms", "20"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0, p.stdout[-2000:]
    r = _results(p.stdout)[-1]
    assert r["pass"] is False and "error" in r, r


def test_allreduce_binary_single_gpu():
    out = _run([os.path.join(BIN, "mx-allreduce-perf"), "-b", "1M", "-e", "16M", "-f", "4",
                "-g", "1", "--iters", "5", "--warmup", "2"])
    pts = [r for r in _results(out) if r["test"] == "allreduce"]
    assert len(pts) >= 3, out[-2000:]
    assert all(r["pass"] and r["ngpus"] == 1 and r["algbw_GBps"] > 0 for r in pts), pts


def test_device_plugin_on_live_box_registers_and_allocates():
    """The real plugin (live sysfs, live amd-smi events) against the fake
    kubelet: amd.com/gpu registers, every visible GPU is healthy, and
    Allocate hands out the CDI name plus /dev/kfd and the render node."""
    import tempfile

    from mxk8s.deviceplugin import api
    from mxk8s.deviceplugin.fake_kubelet import FakeKubelet
    from mxk8s.deviceplugin.plugin import AmdGpuDevicePlugin, PluginConfig

    d = tempfile.mkdtemp(prefix="mxdp", dir="/tmp")
    kube = FakeKubelet(d).start()
    plugin = AmdGpuDevicePlugin(PluginConfig(plugin_dir=d, health_interval=0.2,
                                             watch_interval=0.2)).start()
    try:
        reg = kube.wait_registration()
        assert reg.resource_name == "amd.com/gpu"
        stub = kube.plugin_stub(reg.endpoint)
        first = next(iter(stub.ListAndWatch(api.Empty(), timeout=10)))
        n = len(node.enumerate_gpus(""))
        assert len(first.devices) == n >= 1
        assert all(dv.health == api.HEALTHY for dv in first.devices)
        req = api.AllocateRequest()
        req.container_requests.add(devices_ids=["0"])
        c = stub.Allocate(req, timeout=10).container_responses[0]
        assert [x.name for x in c.cdi_devices] == ["amd.com/gpu=0"]
        paths = [x.host_path for x in c.devices]
        assert "/dev/kfd" in paths and any(p.startswith("/dev/dri/renderD") for p in paths)
    finally:
        plugin.stop()
        kube.stop()


def test_exporter_on_live_box_serves_amd_smi_metrics():
    import urllib.request

    from mxk8s.exporter import Exporter, ExporterConfig, SmiBackend

    ex = Exporter(ExporterConfig(port=0, interval=0.2), backend=SmiBackend("")).start()
    try:
        body = urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/metrics", timeout=10).read().decode()
    finally:
        ex.stop()
    assert 'amd_gpu_stack_component_up{component="amd_smi"} 1' in body
    total = [float(line.rsplit(" ", 1)[1]) for line in body.splitlines()
             if line.startswith("amd_gpu_memory_total_bytes{")]
    assert total and all(250 * 2 ** 30 <= t <= 300 * 2 ** 30 for t in total), total
    assert any(line.startswith("amd_gpu_power_watts{") for line in body.splitlines())
    assert any(line.startswith("amd_gpu_device_healthy{") and line.endswith(" 1")
               for line in body.splitlines())


def test_live_xgmi_link_metrics_and_process_vram():
    """amd-smi's xGMI link state / traffic and the per-process VRAM list on the
    live MI355X, and the exporter series built from them.  A GPU process (this
    test's own torch context) must show up with non-zero VRAM."""
    import json as _json

    import torch

    from mxk8s.exporter import Exporter, ExporterConfig, SmiBackend

    ok, err = node.smi_open()
    assert ok, err
    x = torch.ones(64 << 20, device="cuda")       # 256 MiB held by this process
    torch.cuda.synchronize()
    be = SmiBackend("")
    text = Exporter(ExporterConfig(pod_resources=False), backend=be).sample_once()
    links = node.smi_xgmi_links(0)
    report = {"links": None if links is None else [l.__dict__ for l in links],
              "procs": [p.__dict__ for p in node.smi_processes(0)]}
    print("RESULT " + _json.dumps({"test": "live_xgmi_procs", **report}))
    if links is not None:                           # amd-smi supports the queries here
        assert links, "an MI355X has xGMI links"
        assert all(l.status in ("up", "down", "disabled", "unknown") for l in links)
        assert "amd_gpu_xgmi_link_up{" in text or "amd_gpu_xgmi_read_bytes_total{" in text
    # amd-smi reports host PIDs (the container's PID namespace differs), so
    # look for a process holding at least this test's 256 MiB
    procs = node.smi_processes(0)
    assert any(p.vram_bytes >= 256 << 20 for p in procs), report["procs"]
    assert "amd_gpu_process_memory_bytes{" in text
    del x


def test_health_monitor_on_live_box():
    """The N02 monitor with live amd-smi: every GPU matched to its amd-smi
    handle, the ECC baseline taken, healthy, and the state file written."""
    import json as _json
    import tempfile

    d = tempfile.mkdtemp()
    m = node.HealthMonitor(root="", state_dir=d, use_smi=True)
    try:
        assert m.smi_active
        m.step(100)
        st = m.status()
        assert st and all(s.smi_index >= 0 and s.ecc_valid and s.healthy for s in st), st
        assert m.write_state(os.path.join(d, "health.json"))
        doc = _json.load(open(os.path.join(d, "health.json")))
        assert doc["smi"] and all(g["healthy"] for g in doc["gpus"])
        assert open(os.path.join(d, "ecc-baseline")).read().startswith("boot ")
    finally:
        m.close()
