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


def test_protocol_sweep_plan_is_bounded():
    """The driver's 8-GPU run does the whole 8 B - 8 GiB sweep for two dtypes:
    its call count and a pessimistic time model must stay bounded (VERDICT r4
    missing #4: this is the path the first 8-GPU node exercises)."""
    sys.path.insert(0, REPO)
    import argparse

    import bench
    a = argparse.Namespace(allreduce_sizes="", allreduce_min_bytes=8, allreduce_max_bytes=8 << 30)
    plan = bench.allreduce_plan(a, 8)
    assert [b for b, _ in plan] == bench.allreduce_sizes(a, 8)
    assert all(3 <= it <= 50 for _, it in plan)
    assert plan[0][1] == 50 and plan[-1] == (8 << 30, 3)
    calls = sum(it + bench.AR_WARM_CALLS for _, it in plan)
    assert calls <= 31 * 52
    # pessimistic: 100 us per call + 20 GB/s algbw (xGMI RCCL does >10x that)
    moved = sum((it + bench.AR_WARM_CALLS) * b for b, it in plan)
    est_s = 2 * (calls * 100e-6 + moved / 20e9)       # two dtypes
    assert est_s < 30, est_s


def test_bench_eight_ranks_protocol_sweep():
    """bench.py --gpus 8 on gloo: the default sweep schedule (every x2 size
    from 8 B, each with its planned call count) up to 64 KiB, both dtypes;
    bounded wall time; the zero fixed-point check passes."""
    import time as _t
    t0 = _t.time()
    env = dict(os.environ, MXK_BENCH_DEVICE="cpu", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--size", "128",
           "--steps", "2", "--warmup", "1", "--warmup-s", "0", "--no-reference",
           "--allreduce-max-bytes", str(64 << 10), "--allreduce-mib", "0"]
    p = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    wall = _t.time() - t0
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    ar = out["allreduce"]
    sys.path.insert(0, REPO)
    import bench
    sizes = [8 << i for i in range(14)]
    assert [(s["bytes"], s["dtype"]) for s in ar["sweep"]] == \
        [(b, d) for d in ("bf16", "fp32") for b in sizes]
    assert [s["iters"] for s in ar["sweep"]] == [bench.allreduce_iters(b) for b in sizes] * 2
    for s in ar["sweep"]:
        assert s["busbw_GBps"] == pytest.approx(s["algbw_GBps"] * 2 * 7 / 8, rel=0.02, abs=0.011)
    assert "zero" in ar["sweep_data"] and ar["rccl_ranks"] == 8
    assert wall < 240, wall
