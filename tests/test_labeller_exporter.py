"""Node labeller (against a fake API server) and the Prometheus exporter
(fake amd-smi backend + fake kubelet PodResources socket)."""
import http.server
import json
import os
import tempfile
import threading
import urllib.request

import pytest

from mxk8s import labeller
from mxk8s.exporter import Exporter, ExporterConfig, render_metrics
from mxk8s.exporter import podresources as pr
from mxk8s.native import node
from mxk8s.utils.kube import KubeClient

FX = os.path.join(os.path.dirname(__file__), "fixtures", "sysfs")


def gpus8():
    return node.enumerate_gpus(os.path.join(FX, "mi355x_8gpu"))


def test_compute_labels_mi355x():
    L = labeller.compute_labels(gpus8(), driver_version="6.12.12", rocm="7.2.0")
    assert L["amd.com/gpu.present"] == "true"
    assert L["amd.com/gpu.count"] == "8"
    assert L["amd.com/gpu.arch"] == "gfx950"
    assert L["amd.com/gpu.family"] == "CDNA4"
    assert L["amd.com/gpu.product"] == "MI355X"
    assert L["amd.com/gpu.vram"] == "288G"
    assert L["amd.com/gpu.cu-count"] == "256"
    assert L["amd.com/gpu.xgmi"] == "true" and L["amd.com/gpu.xgmi-links"] == "7"
    assert L["amd.com/gpu.numa-nodes"] == "2"
    assert L["amd.com/gpu.xgmi-hive"] == "a20dcafe9b2f58bc"
    assert L["amd.com/gpu.rocm-version"] == "7.2.0"
    for v in L.values():
        assert len(v) <= 63 and labeller._LABEL_VALUE.match(v)


def test_partition_mode_labels(tmp_path):
    gpus = node.enumerate_gpus(os.path.join(FX, "mi355x_8gpu"))
    assert labeller.partition_modes(gpus, str(tmp_path)) == {}   # driver without the files
    for k, g in enumerate(gpus):
        d = tmp_path / "sys/bus/pci/devices" / g.bdf
        d.mkdir(parents=True)
        (d / "current_compute_partition").write_text("CPX\n" if k else "SPX\n")
        (d / "current_memory_partition").write_text("NPS1\n")
    modes = labeller.partition_modes(gpus, str(tmp_path))
    assert modes == {"compute": "mixed", "memory": "nps1"}
    labels = labeller.compute_labels(gpus, partitions=modes)
    assert labels["amd.com/gpu.compute-partitioning-mode"] == "mixed"
    assert labels["amd.com/gpu.memory-partitioning-mode"] == "nps1"
    assert "amd.com/gpu.compute-partitioning-mode" not in labeller.compute_labels(gpus)


def test_label_sanitize_and_patch():
    assert labeller.sanitize("Linux version 6.8 (gcc 12)!") == "Linux-version-6.8-gcc-12"
    assert len(labeller.sanitize("x" * 200)) == 63
    cur = {"amd.com/gpu.arch": "gfx942", "amd.com/gpu.old": "x", "other": "keep"}
    patch = labeller.label_patch(cur, {"amd.com/gpu.arch": "gfx950"})
    assert patch == {"amd.com/gpu.arch": "gfx950", "amd.com/gpu.old": None}
    assert labeller.compute_labels([]) == {"amd.com/gpu.present": "false", "amd.com/gpu.count": "0"}


class _FakeAPI(http.server.BaseHTTPRequestHandler):
    node = {"metadata": {"name": "n1", "labels": {"amd.com/gpu.stale": "1", "kubernetes.io/os": "linux"}}}
    patches = []

    def do_GET(self):
        assert self.headers["Authorization"] == "Bearer T0K"
        body = json.dumps(self.node).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.end_headers()
        self.wfile.write(body)

    def do_PATCH(self):
        assert self.headers["Content-Type"] == "application/merge-patch+json"
        n = int(self.headers["Content-Length"])
        self.patches.append(json.loads(self.rfile.read(n)))
        self.send_response(200)
        self.end_headers()
        self.wfile.write(b"{}")

    def log_message(self, *a):
        pass


def test_labeller_patches_node_and_writes_nfd_file(tmp_path):
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _FakeAPI)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        client = KubeClient(f"http://127.0.0.1:{srv.server_address[1]}", token="T0K")
        patch = labeller.run_once(client, "n1", gpus8(), "d1", "7.2.0", str(tmp_path))
    finally:
        srv.shutdown()
    sent = _FakeAPI.patches[-1]["metadata"]["labels"]
    assert sent["amd.com/gpu.arch"] == "gfx950"
    assert sent["amd.com/gpu.stale"] is None        # stale label removed
    assert "kubernetes.io/os" not in sent            # foreign labels untouched
    assert patch == sent
    nfd = (tmp_path / "amd-gpu").read_text()
    assert "amd-gpu.arch=gfx950" in nfd and "pci-1002.present=true" in nfd


class FakeBackend:
    ok = True
    driver = "6.12"

    def __init__(self, gpus):
        self._g = gpus

    def gpus(self):
        return self._g

    def samples(self):
        out = {}
        for g in self._g:
            out[g.bdf] = node.GpuSample(index=g.index, valid=True, gfx_activity_pct=50 + g.index,
                                        umc_activity_pct=10, vram_used_bytes=1 << 30,
                                        vram_total_bytes=g.vram_bytes, temp_edge_c=None,
                                        temp_hotspot_c=60.0, temp_mem_c=40.0, power_w=900,
                                        power_limit_w=1400, sclk_mhz=2100, mclk_mhz=2000,
                                        ecc_correctable=1, ecc_uncorrectable=0, num_processes=1,
                                        bdf=g.bdf)
        return out

    def health(self, i):
        return 0 if i != 3 else node.UNHEALTHY_NO_RENDER_NODE


def test_render_metrics_text_format():
    g = gpus8()
    text = render_metrics(g, FakeBackend(g).samples(), FakeBackend(g).health,
                          {"2": ("ml", "trainer-0", "main")}, "6.12", {"amd_smi": True}, 0.01)
    assert '# TYPE amd_gpu_utilization_percent gauge' in text
    assert 'amd_gpu_utilization_percent{gpu="5",bdf="0000:95:00.0",uuid="GPU-f4071d07e8ac5505"} 55' in text
    assert 'amd_gpu_temperature_celsius{gpu="0",bdf="0000:05:00.0",uuid="GPU-f4071d07e8ac5500",sensor="hotspot"} 60.0' in text
    assert 'sensor="edge"' not in text                    # unsupported sensor omitted
    assert 'namespace="ml",pod="trainer-0",container="main"' in text
    assert 'amd_gpu_device_healthy{gpu="3"' in text and \
        [l for l in text.splitlines() if l.startswith('amd_gpu_device_healthy{gpu="3"')][0].endswith(" 0")
    assert text.count("# TYPE amd_gpu_clock_mhz gauge") == 1
    assert 'amd_gpu_ecc_errors_total{gpu="0",bdf="0000:05:00.0",uuid="GPU-f4071d07e8ac5500",type="correctable"} 1' in text


def test_exporter_http_and_pod_resources():
    d = tempfile.mkdtemp(prefix="mxpr", dir="/tmp")
    sock = os.path.join(d, "kubelet.sock")
    resp = pr.ListPodResourcesResponse()
    p = resp.pod_resources.add(name="llama-0", namespace="train")
    c = p.containers.add(name="worker")
    c.devices.add(resource_name="amd.com/gpu", device_ids=["0", "1"])
    c.devices.add(resource_name="cpu-other", device_ids=["5"])
    srv = pr.serve_fake(sock, resp)
    try:
        assert pr.gpu_owners(sock) == {"0": [("train", "llama-0", "worker")],
                                       "1": [("train", "llama-0", "worker")]}
        g = gpus8()
        ex = Exporter(ExporterConfig(port=0, interval=0.05, pod_resources_socket=sock),
                      backend=FakeBackend(g)).start()
        try:
            body = urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/metrics", timeout=5).read().decode()
            assert 'pod="llama-0"' in body and "amd_gpu_power_watts" in body
            assert 'amd_gpu_stack_component_up{component="amd_smi"} 1' in body
            assert urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/healthz", timeout=5).read() == b"ok\n"
        finally:
            ex.stop()
    finally:
        srv.stop(0)


def test_link_metrics_from_kfd_topology():
    root = os.path.join(FX, "mi355x_8gpu")
    g = node.enumerate_gpus(root)
    text = render_metrics(g, {}, lambda i: 0, {}, "", {}, 0.0, node.links(root))
    up = [l for l in text.splitlines() if l.startswith("amd_gpu_topology_link{")]
    assert len([l for l in up if 'type="xgmi"' in l]) == 56          # 8 GPUs x 7 peers
    assert len([l for l in up if 'type="pcie"' in l]) == 8
    assert 'amd_gpu_topology_link{gpu="0",bdf="0000:05:00.0",uuid="GPU-f4071d07e8ac5500",peer="7",type="xgmi"} 1' in text
    # no live amd-smi link state: no amd_gpu_xgmi_link_up series is invented
    assert "amd_gpu_xgmi_link_up" not in text
    assert "# TYPE amd_gpu_link_max_bandwidth_bytes gauge" in text


def test_time_sliced_owner_attribution():
    """Replica IDs <i>::<r> under amd.com/gpu or its .shared rename map to GPU i;
    a GPU shared by two pods gets one amd_gpu_pod_info series per owner."""
    d = tempfile.mkdtemp(prefix="mxpr", dir="/tmp")
    sock = os.path.join(d, "kubelet.sock")
    resp = pr.ListPodResourcesResponse()
    for pod, ids, res in (("a-0", ["1::0"], "amd.com/gpu.shared"), ("b-0", ["1::1", "2::0"], "amd.com/gpu.shared"),
                          ("c-0", ["3"], "amd.com/gpu")):
        c = resp.pod_resources.add(name=pod, namespace="ml").containers.add(name="main")
        c.devices.add(resource_name=res, device_ids=ids)
    srv = pr.serve_fake(sock, resp)
    try:
        own = pr.gpu_owners(sock)
        assert own == {"1": [("ml", "a-0", "main"), ("ml", "b-0", "main")],
                       "2": [("ml", "b-0", "main")], "3": [("ml", "c-0", "main")]}
        g = gpus8()
        text = render_metrics(g, FakeBackend(g).samples(), FakeBackend(g).health, own, "", {}, 0.0)
        info = [l for l in text.splitlines() if l.startswith('amd_gpu_pod_info{gpu="1"')]
        assert len(info) == 2 and 'pod="a-0"' in info[0] and 'pod="b-0"' in info[1]
        assert [l for l in text.splitlines() if l.startswith('amd_gpu_pods{gpu="1"')][0].endswith(" 2")
        # shared GPU: no single pod label on its series; exclusive GPU: labelled
        util1 = [l for l in text.splitlines() if l.startswith('amd_gpu_utilization_percent{gpu="1"')][0]
        assert "pod=" not in util1
        util2 = [l for l in text.splitlines() if l.startswith('amd_gpu_utilization_percent{gpu="2"')][0]
        assert 'pod="b-0"' in util2
    finally:
        srv.stop(0)


def test_pod_uid_from_cgroup(tmp_path):
    from mxk8s.exporter import pod_uid_of
    (tmp_path / "42").mkdir()
    (tmp_path / "42" / "cgroup").write_text(
        "0::/kubepods.slice/kubepods-besteffort.slice/"
        "kubepods-besteffort-pod3f2c8a1e_5b7d_4c1a_9e0f_2a6b8c4d1e7f.slice/"
        "cri-containerd-0123abcd.scope\n")
    assert pod_uid_of(42, str(tmp_path)) == "3f2c8a1e-5b7d-4c1a-9e0f-2a6b8c4d1e7f"
    (tmp_path / "43").mkdir()
    (tmp_path / "43" / "cgroup").write_text(
        "12:memory:/kubepods/burstable/pod0b1c2d3e-aaaa-bbbb-cccc-0123456789ab/deadbeef\n")
    assert pod_uid_of(43, str(tmp_path)) == "0b1c2d3e-aaaa-bbbb-cccc-0123456789ab"
    assert pod_uid_of(44, str(tmp_path)) is None


def test_metrics_doc_names_exist():
    """Every exporter series named in docs/METRICS.md is one the exporter emits."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = open(os.path.join(root, "docs", "METRICS.md")).read()
    src = open(os.path.join(root, "mxk8s", "exporter", "__init__.py")).read()
    named = set(re.findall(r"\b(amd_gpu_[a-z_]+)", doc))
    assert named
    missing = sorted(n for n in named if f'"{n}"' not in src)
    assert not missing, missing
