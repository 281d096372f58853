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


def test_vector_add_binary_passes():
    res = _results(_run([os.path.join(BIN, "mx-vector-add"), "--n", "50000"]))
    assert res and res[-1]["test"] == "vectoradd" and res[-1]["pass"], res


def test_gemm_bench_binary_self_checks():
    out = _run([os.path.join(BIN, "mx-gemm-bench"), "--sizes", "4096", "--iters", "10",
                "--warmup-ms", "200"])
    res = _results(out)
    assert res, out[-2000:]
    r = res[-1]
    assert r["test"] == "gemm" and r["pass"], r
    assert r["tflops"] > 500, r


def test_allreduce_binary_single_gpu():
    out = _run([os.path.join(BIN, "mx-allreduce-perf"), "-b", "1M", "-e", "16M", "-f", "4",
                "-g", "1", "--iters", "5", "--warmup", "2"])
    pts = [r for r in _results(out) if r["test"] == "allreduce"]
    assert len(pts) >= 3, out[-2000:]
    assert all(r["pass"] and r["ngpus"] == 1 and r["algbw_GBps"] > 0 for r in pts), pts
