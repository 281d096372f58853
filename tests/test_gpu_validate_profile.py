"""BASELINE config 3 is the validator's bf16 MFMA GEMM "with rocprof counters".

The chart (``validator.profile: true``) and ``deploy/examples/gemm-validator.yaml``
pass ``--profile``; this runs that exact validator command on the GPU:
``mx-gemm-bench``, then three rocprofv3 counter passes of the GEMM
(``mxk8s.validate.profile``: one counter group per process, ``--kernel-trace``
only, the program directly after ``--``), and checks the RESULT lines the
Job log carries for the hand-written kernel."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_validator_gemm_profile_result_lines(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "mxk8s.validate", "--tests", "gemm", "--gemm-sizes", "8192",
           "--profile", "--profile-dir", str(tmp_path / "pmc")]
    env = {**os.environ, "PYTHONPATH": REPO, "TMPDIR": os.environ.get("TMPDIR", "/tmp")}
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=280, env=env)
    lines = [json.loads(l[7:]) for l in p.stdout.splitlines() if l.startswith("RESULT ")]
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    prof = [r for r in lines if r.get("test") == "gemm_profile"]
    mine = [r for r in prof if "mxk_gemm" in r.get("kernel", "")]
    assert mine, [r.get("kernel") for r in prof]
    for r in mine:
        assert r["pass"] is True
        assert 0.2 < r["mfma_busy_frac"] <= 1.0, r
        assert 0.0 < r["l2_hit_rate"] <= 1.0, r
        assert 1.0 < r["effective_clock_ghz"] < 3.0, r
        assert 0.0 <= r["lds_bank_conflict_frac"] < 0.5, r
    summary = [r for r in lines if r.get("test") == "validator"]
    assert summary and summary[-1]["results"].get("gemm_profile") is True
    with open(os.path.join(REPO, "deploy", "examples", "gemm-validator.yaml")) as f:
        assert "- --profile" in f.read()
