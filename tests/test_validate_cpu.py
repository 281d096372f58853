"""CPU tests of the validator plumbing: rocprofv3 CSV summarising (derived
MFMA/LDS/clock/L2 ratios), roctx ranges, --debug environment, the collective
sweep's RESULT aggregation."""
import csv
import json
import os
import stat

import pytest

from mxk8s.utils import roctx
from mxk8s.validate import __main__ as V
from mxk8s.validate import profile


def _write_csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_profile_summary_derives_ratios(tmp_path):
    d = tmp_path / "pmc1"
    d.mkdir()
    k = "mxk_gemm_bf16_tn_w4b<0, false, 0>(...)"
    vals = {"SQ_VALU_MFMA_BUSY_CYCLES": 1.0e9, "GRBM_GUI_ACTIVE": 1.2e7 * 8 / 8,
            "SQ_WAVE_CYCLES": 4e8, "SQ_WAIT_ANY": 4e7, "SQ_LDS_BANK_CONFLICT": 0.0,
            "SQ_LDS_IDX_ACTIVE": 6e7, "TCC_HIT_sum": 80.0, "TCC_MISS_sum": 20.0}
    rows = [{"Dispatch_Id": str(i), "Kernel_Name": k, "Counter_Name": c, "Counter_Value": str(v)}
            for i in range(3) for c, v in vals.items()]
    rows.append({"Dispatch_Id": "9", "Kernel_Name": "other", "Counter_Name": "SQ_WAVE_CYCLES",
                 "Counter_Value": "1"})
    _write_csv(d / "run_counter_collection.csv", rows)
    _write_csv(d / "run_kernel_trace.csv", [
        {"Kernel_Name": k, "Start_Timestamp": "0", "End_Timestamp": str(int(0.7e6))}] * 3)
    s = profile.summarize([str(d)], "gemm")
    assert list(s) == [k]
    der = s[k]["derived"]
    assert der["median_us"] == pytest.approx(700.0)
    # GRBM_GUI_ACTIVE is summed over 8 XCDs: 1.2e7 / 8 / 0.7 ms = 2.14 GHz
    assert der["effective_clock_ghz"] == pytest.approx(1.2e7 / 8 / 0.7e-3 / 1e9)
    assert der["mfma_busy_frac"] == pytest.approx(1e9 / (1.2e7 / 8 * 1024))
    assert der["lds_bank_conflict_frac"] == 0.0
    assert der["l2_hit_rate"] == pytest.approx(0.8)
    assert der["sq_wait_any_frac"] == pytest.approx(0.1)
    assert "mfma_busy_frac" in profile.format_text(s)


def test_roctx_ranges_are_safe_everywhere(monkeypatch):
    with roctx.range("outer"):
        with roctx.range("inner"):
            roctx.mark("m")
    monkeypatch.setattr(roctx, "_tried", False)
    monkeypatch.setattr(roctx, "_lib", None)
    monkeypatch.setenv("MXK8S_ROCTX", "0")
    assert not roctx.available()
    with roctx.range("noop"):
        pass


def _fake_bin(tmp_path, name, body):
    p = tmp_path / name
    p.write_text("#!/bin/sh\n" + body)
    p.chmod(p.stat().st_mode | stat.S_IEXEC)


def test_debug_mode_serialises_kernels(tmp_path, monkeypatch, capsys):
    _fake_bin(tmp_path, "mx-vector-add",
              'echo "RESULT {\\"test\\":\\"vectoradd\\",\\"pass\\":true,'
              '\\"serialize\\":\\"$AMD_SERIALIZE_KERNEL\\",\\"blocking\\":\\"$HIP_LAUNCH_BLOCKING\\"}"\n')
    monkeypatch.setattr(V, "BIN", str(tmp_path))
    monkeypatch.setattr(V, "_extra_env", {})
    assert V.main(["--tests", "vectoradd", "--debug"]) == 0
    rs = [json.loads(l[7:]) for l in capsys.readouterr().out.splitlines() if l.startswith("RESULT ")]
    va = [r for r in rs if r["test"] == "vectoradd"][0]
    assert (va["serialize"], va["blocking"]) == ("3", "1")
    assert rs[-1]["test"] == "validator" and rs[-1]["pass"]


def test_rccl_summary_per_op(tmp_path, monkeypatch, capsys):
    lines = []
    for op, peak in (("allreduce", 310.5), ("allgather", 280.0)):
        lines.append(f'RESULT {{"test":"{op}","ngpus":1,"bytes":8,"pass":true}}')
        lines.append(f'RESULT {{"test":"{op}_summary","ngpus":1,"peak_busbw_GBps":{peak}}}')
    _fake_bin(tmp_path, "mx-allreduce-perf", "".join(f"echo '{l}'\n" for l in lines))
    monkeypatch.setattr(V, "BIN", str(tmp_path))
    assert V.main(["--tests", "rccl", "--rccl-ops", "allreduce,allgather"]) == 0
    rs = [json.loads(l[7:]) for l in capsys.readouterr().out.splitlines() if l.startswith("RESULT ")]
    summ = [r for r in rs if r["test"] == "rccl_summary"][0]
    assert summ["peak_busbw_GBps_by_ngpus"] == {"1": 310.5}
    assert summ["peak_busbw_GBps_by_op"]["allgather"] == {"1": 280.0}
