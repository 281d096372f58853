"""bench.py's contract on the CPU tier: the driver's JSON line, the --gpus N
self-relaunch under torch.distributed.run, max-over-ranks timing and the
all-reduce sweep (gloo stands in for RCCL; the GEMM is the PyTorch reference).
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*extra, timeout=240):
    env = dict(os.environ, MXK_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--size", "256", "--steps", "3",
           "--warmup", "1", "--warmup-s", "0", "--allreduce-sizes", "1,2", "--allreduce-mib", "2",
           "--ab-rounds", "2", "--ab-sizes", "128", *extra]
    p = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout   # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def _check_contract(out, n):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in out, key
    assert out["metric"] == "validator HIP GEMM TFLOPS + RCCL allreduce bus-bw at 1/2/4/8 amd.com/gpu"
    assert out["n_gpus"] == n and out["steps"] == 3 and out["warmup"] == 1
    assert out["config"]["parallelism"] == f"dp{n} (one GEMM per amd.com/gpu)"
    # value is the whole-job aggregate: n x per-step flops over the slowest rank's time
    flops = 2.0 * 256 ** 3
    expect = n * flops * 3 / (out["ms_per_step"] * 3e-3) / 1e12
    assert out["value"] == pytest.approx(expect, rel=0.02, abs=0.011)
    gc = out["gemm_check"]
    assert gc["elements"] == 256 * 256
    assert gc["max_abs_err_first"] <= gc["tolerance"] and gc["max_abs_err_after_timed"] <= gc["tolerance"]
    ar = out["allreduce"]
    assert ar["rccl_ranks"] == n and ar["op"] == "sum" and ar["dtypes"] == ["bf16", "fp32"]
    assert [(s["bytes"], s["dtype"]) for s in ar["sweep"]] == \
        [(1 << 20, "bf16"), (2 << 20, "bf16"), (1 << 20, "fp32"), (2 << 20, "fp32")]
    for s in ar["sweep"]:
        if n == 1:      # no meaningless "bandwidth" at n = 1
            assert s["algbw_GBps"] is None and s["busbw_GBps"] == 0.0
        else:
            assert s["busbw_GBps"] == pytest.approx(s["algbw_GBps"] * 2 * (n - 1) / n, rel=0.02,
                                                    abs=0.011)
    assert out["hipblaslt_ab"]["launches_each"] == 2 * 20
    assert [x["M"] for x in out["ab_other_sizes"]] == [128] and out["ab_other_sizes"][0]["check_ok"]


def test_bench_single_rank_contract():
    out = _run_bench()
    _check_contract(out, 1)
    assert out["allreduce"]["busbw_GBps"] == 0.0 and out["allreduce"]["algbw_GBps"] is None
    assert out["allreduce"]["busbw_peak_GBps"] is None


def test_protocol_allreduce_sizes():
    """Default sweep at n > 1: 8 B - 8 GiB in x2 steps (BASELINE.md protocol)."""
    sys.path.insert(0, REPO)
    import argparse

    import bench
    a = argparse.Namespace(allreduce_sizes="", allreduce_min_bytes=8, allreduce_max_bytes=8 << 30)
    sizes = bench.allreduce_sizes(a, 8)
    assert sizes[0] == 8 and sizes[-1] == 8 << 30 and len(sizes) == 31
    assert all(b == 2 * a_ for a_, b in zip(sizes, sizes[1:]))
    assert len(bench.allreduce_sizes(a, 1)) == 3


def test_bench_self_relaunch_four_ranks():
    out = _run_bench("--gpus", "4")
    _check_contract(out, 4)
    assert out["allreduce"]["backend"] == "gloo"
