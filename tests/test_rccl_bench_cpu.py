"""mx-allreduce-perf's multi-process id handshake, exercised without a GPU:
the id file carries a per-job nonce, so a non-zero rank rejects a stale file
from an earlier run (and times out cleanly) instead of joining the wrong
communicator.  (The collective itself needs GPUs: tests/test_gpu_node.py.)"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "bin", "mx-allreduce-perf")


def _stale_id_file(path, nonce):
    with open(path, "wb") as f:
        f.write(b"MXKNCCL1" + len(nonce).to_bytes(4, "little") + nonce.encode() + b"\0" * 128)


@pytest.mark.skipif(not os.path.exists(BIN), reason="make tools first")
def test_rank1_rejects_stale_nonce(tmp_path):
    idf = str(tmp_path / "id")
    _stale_id_file(idf, "old-run:29500")
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MXK_RUN_NONCE="new-run:29501",
               MXK_ID_WAIT_S="1")
    p = subprocess.run([BIN, "--id-file", idf, "-b", "8", "-e", "64"], env=env, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 1
    assert "timed out waiting" in p.stderr and "new-run:29501" in p.stderr


@pytest.mark.skipif(not os.path.exists(BIN), reason="make tools first")
def test_multiproc_requires_nonce(tmp_path):
    env = {k: v for k, v in os.environ.items()
           if k not in ("MXK_RUN_NONCE", "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
    env.update(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    p = subprocess.run([BIN, "--id-file", str(tmp_path / "id")], env=env, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 1 and "no job nonce" in p.stderr


def test_sweep_plan_all_ops_host(tmp_path):
    """mx-allreduce-perf's size list, shapes, bus factors, iteration counts
    and whole-buffer mismatch chunking for all four ops at n = 1, 2, 4, 8
    (native/rccl_bench/sweep_plan.h, the logic the first 8-GPU run takes),
    compiled for the host under ASan + UBSan and run against collectives
    simulated from their definitions."""
    import shutil
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "test_sweep_plan")
    src = os.path.join(REPO, "native", "rccl_bench", "tests", "test_sweep_plan.cc")
    subprocess.run([cxx, "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-o", exe, src],
                   check=True, timeout=300)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "PASS sweep_plan" in p.stdout, p.stderr[-3000:]
