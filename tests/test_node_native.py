"""libmxnode (C++) through its ctypes binding, over fake sysfs fixtures and the
sysfs tree captured on a real MI355X gpurun box."""
import json
import os
import subprocess
import tarfile

import pytest

from mxk8s.native import node

FX = os.path.join(os.path.dirname(__file__), "fixtures", "sysfs")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def root(name):
    return os.path.join(FX, name)


def test_enumerate_8gpu():
    gpus = node.enumerate_gpus(root("mi355x_8gpu"))
    assert len(gpus) == 8
    assert [g.index for g in gpus] == list(range(8))
    assert {g.arch for g in gpus} == {"gfx950"}
    assert {g.product for g in gpus} == {"MI355X"}
    assert [g.numa_node for g in gpus] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert all(g.cu_count == 256 and g.xgmi_links == 7 for g in gpus)
    assert gpus[0].render_path == "/dev/dri/renderD128"
    assert gpus[0].bdf == "0000:05:00.0"
    assert abs(gpus[0].vram_bytes / 2**30 - 288) < 0.1
    assert len({g.uuid for g in gpus}) == 8


def test_enumerate_filters_non_amd_and_errors():
    assert len(node.enumerate_gpus(root("mixed_nonamd"))) == 1
    with pytest.raises(RuntimeError, match="KFD"):
        node.enumerate_gpus(root("no_driver"))


def test_links_full_xgmi_mesh():
    ls = node.links(root("mi355x_8gpu"))
    x = [(l.from_index, l.to_index) for l in ls if l.is_xgmi]
    assert len(x) == 56
    assert set(x) == {(i, j) for i in range(8) for j in range(8) if i != j}


def test_cdi_spec_shape():
    spec = node.cdi_spec(root("mi355x_8gpu"))
    assert spec["cdiVersion"] == "0.6.0" and spec["kind"] == "amd.com/gpu"
    assert spec["containerEdits"]["deviceNodes"][0]["path"] == "/dev/kfd"
    names = [d["name"] for d in spec["devices"]]
    assert names[:2] == ["0", "GPU-f4071d07e8ac5500"]
    assert "all" in names and len(names) == 17
    dev3 = next(d for d in spec["devices"] if d["name"] == "3")
    paths = [n["path"] for n in dev3["containerEdits"]["deviceNodes"]]
    assert paths == ["/dev/dri/renderD131", "/dev/dri/card4"]
    alld = next(d for d in spec["devices"] if d["name"] == "all")
    assert len(alld["containerEdits"]["deviceNodes"]) == 16


def test_cdi_cli_matches_library(tmp_path):
    out = tmp_path / "amd.com-gpu.json"
    exe = os.path.join(REPO, "bin", "mx-cdi-gen")
    subprocess.run([exe, "--root", root("mi355x_8gpu"), "--output", str(out)], check=True)
    assert json.loads(out.read_text()) == node.cdi_spec(root("mi355x_8gpu"))
    assert subprocess.run([exe, "--root", root("mi355x_8gpu"), "--output", str(out),
                           "--check"]).returncode == 0
    assert subprocess.run([exe, "--root", root("mi355x_1gpu"), "--output", str(out),
                           "--check"], stderr=subprocess.DEVNULL).returncode == 1


def test_preferred_allocation_policy():
    r = root("mi355x_8gpu")
    assert node.preferred_allocation(range(8), [], 4, r) == [0, 1, 2, 3]
    assert node.preferred_allocation(range(8), [6], 2, r) == [4, 6]
    assert node.preferred_allocation([0, 4, 5, 6, 1], [], 3, r) == [4, 5, 6]
    assert node.preferred_allocation(range(8), [], 8, r) == list(range(8))
    with pytest.raises(ValueError):
        node.preferred_allocation(range(4), [], 5, r)
    with pytest.raises(ValueError):
        node.preferred_allocation(range(4), [7], 2, r)


def test_preferred_allocation_prefers_one_hive():
    # two hives of 4 on ONE numa node: a 4-GPU request must not straddle hives
    numa = [0] * 8
    hive = [1, 2, 1, 2, 1, 2, 1, 2]
    adj = [[int(i != j and hive[i] == hive[j]) for j in range(8)] for i in range(8)]
    assert node.preferred_allocation_topo(numa, hive, adj, range(8), [], 4) == [0, 2, 4, 6]
    assert node.preferred_allocation_topo(numa, hive, adj, range(8), [1], 2) == [1, 3]


def test_health(tmp_path):
    assert node.health_check(3, root("mi355x_8gpu")) == node.HEALTHY
    assert node.health_check(3, root("missing_render")) == node.UNHEALTHY_NO_RENDER_NODE
    assert node.health_check(9, root("mi355x_8gpu")) == node.UNHEALTHY_NO_KFD_NODE
    ff = tmp_path / "faults"
    ff.write_text("2\n")
    assert node.health_check(2, root("mi355x_8gpu"), str(ff)) == node.UNHEALTHY_FAULT_INJECTED
    assert node.health_reason(node.UNHEALTHY_FAULT_INJECTED) == "fault injected"


def test_captured_real_box_tree(tmp_path):
    """The KFD tree captured inside a 1-GPU container on the MI355X gpurun box."""
    tgz = os.path.join(os.path.dirname(__file__), "fixtures", "captured", "mi355x_gpurun_box.tar.gz")
    with tarfile.open(tgz) as t:
        t.extractall(tmp_path, filter="data")
    gpus = node.enumerate_gpus(str(tmp_path))
    assert len(gpus) == 1
    g = gpus[0]
    assert (g.arch, g.product, g.cu_count, g.gfx_target_version) == ("gfx950", "MI355X", 256, 90500)
    assert g.xgmi_links == 7 and g.max_sclk_mhz == 2400
    assert abs(g.vram_bytes / 2**30 - 288) < 0.1


def test_native_unit_tests_under_asan():
    """C++ host tests of libmxnode built with -fsanitize=address,undefined."""
    r = subprocess.run(["make", "-C", REPO, "-s", "test-native"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "libmxnode tests passed" in r.stdout


def test_native_thread_safety_under_tsan():
    """libmxnode entry points are re-entrant (ThreadSanitizer build, 8 threads)."""
    r = subprocess.run(["make", "-C", REPO, "-s", "test-native-tsan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "thread-safety test: ok" in r.stdout
