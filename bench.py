#!/usr/bin/env python3
"""Headline benchmark: validator HIP GEMM TFLOPS + RCCL all-reduce bus-bw.

BASELINE.json names the metric "validator HIP GEMM TFLOPS + RCCL allreduce
bus-bw at 1/2/4/8 amd.com/gpu" (configs 3 and 4).  One process per GPU, and
``torch.distributed`` over RCCL at every N (a 1-rank communicator at N = 1,
so the all-reduce is a real ``ncclAllReduce`` there too).

Protocol (BASELINE.md "Measurement protocol"):

* a *step* is one 8192^3 bf16 GEMM on this rank's GPU through the hand-written
  CDNA4 MFMA kernel (``native/kernels/gemm_bf16.hip``), random uniform
  [-1, 1) operands (random data, never zeros: the chip clocks higher on zeros);
* correctness gate: the WHOLE output of the first launch and of the last timed
  launch is compared with an fp32 ``torch.matmul`` on the device, tolerance
  2^-7 * max|ref| (bf16 output rounding is 2^-8 relative);
* warm-up: ``--warmup`` launches, then more until ``--warmup-s`` (default 2 s)
  of back-to-back launches have run, whatever ``--warmup`` says (the GPU
  ramps its clock over ~1 s; a 5-launch warm-up times a cold chip);
* exactly K timed steps bracketed by a barrier and ``torch.cuda.synchronize()``
  on both sides; the slowest rank's wall time gives ``value`` = whole-job
  TFLOP/s = N x 2MNK x K / max-rank time.  The K launches run back to back
  between one hipEvent pair (``event_span_ms_per_step``); a second pass of K
  launches with an event between every two gives the per-launch median
  (event records between launches cost ~1 % at 8192^3, so they stay out of
  the timed region);
* hipBLASLt (``torch.mm``) on the same operands is timed A/B-interleaved with
  the hand-written kernel in blocks of back-to-back launches, one event pair
  per block (context, not the metric);
* RCCL all-reduce (sum, bf16): a correctness check, then a 1 MiB - 1 GiB size
  sweep with algbw = bytes/t and busbw = algbw * 2(n-1)/n (0 at n = 1 by
  definition); the slowest rank's time per size.

``--mode ddp`` runs the Llama-3-8B DDP training step (config 5) instead.

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
             bench.py --gpus N
On a host without a GPU (the CPU test tier) the same code runs over gloo with
the PyTorch reference GEMM, so the multi-rank plumbing is testable anywhere.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

METRIC = "validator HIP GEMM TFLOPS + RCCL allreduce bus-bw at 1/2/4/8 amd.com/gpu"


def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def _log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class _Timer:
    """Per-launch timing: hipEvents on a GPU, perf_counter on the CPU tier."""

    def __init__(self, dev):
        import torch
        self.cuda = dev.type == "cuda"
        self.torch = torch

    def marks(self, n):
        if self.cuda:
            return [self.torch.cuda.Event(enable_timing=True) for _ in range(n)]
        return [None] * n

    def record(self, marks, i):
        if self.cuda:
            marks[i].record()
        else:
            marks[i] = time.perf_counter()

    def elapsed_ms(self, marks):
        if self.cuda:
            self.torch.cuda.synchronize()
            return [marks[i].elapsed_time(marks[i + 1]) for i in range(len(marks) - 1)]
        return [(marks[i + 1] - marks[i]) * 1e3 for i in range(len(marks) - 1)]


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class _StdoutToStderr:
    """RCCL prints a version banner on stdout when a communicator is built;
    the driver reads rank 0's stdout for the ONE JSON line, so the banner goes
    to stderr (fd-level: it is written by the C library)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _init_group(backend, dev, world, rank):
    """Default process group at every N.  At N = 1 a 1-rank group on an
    in-process store: RCCL builds a real 1-rank communicator."""
    import torch.distributed as dist
    from mxk8s.parallel.dist import init_distributed

    with _StdoutToStderr():
        if world > 1:
            init_distributed(backend=backend, device=dev if backend == "nccl" else None)
        elif not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(backend=backend, store=dist.HashStore(), rank=0, world_size=1,
                                    **kw)
        _barrier(dev)     # the communicator exists (and has printed) by now
    return dist.group.WORLD


def _barrier(dev):
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        dist.barrier(device_ids=[dev.index])
    else:
        dist.barrier()


def _max_over_ranks(x, dev):
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64,
                     device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _full_check(A, Bt, C):
    """max |C - A.Bt^T| over the whole output against an fp32 GEMM on the same
    device; returns (max_abs_err, tolerance)."""
    import torch
    ref = torch.matmul(A.float(), Bt.float().t())
    err = (C.float() - ref).abs().max().item()
    tol = 2.0 ** -7 * ref.abs().max().item()
    del ref
    return err, tol


def allreduce_sizes(args, world) -> list[int]:
    """Message sizes (bytes) of the sweep: an explicit ``--allreduce-sizes``
    MiB list, else the protocol's 8 B - 8 GiB in x2 steps (BASELINE.md
    "Measurement protocol"; nccl-tests ``-b 8 -e 8G -f 2``) at n > 1, and three
    sizes at n = 1 (a 1-rank all-reduce moves no data: only the code path)."""
    if args.allreduce_sizes:
        return [int(s) << 20 for s in args.allreduce_sizes.split(",") if s]
    if world == 1:
        return [1 << 20, 64 << 20, 1 << 30]
    out, b = [], args.allreduce_min_bytes
    while b <= args.allreduce_max_bytes:
        out.append(b)
        b *= 2
    return out


def allreduce_iters(nbytes: int) -> int:
    """Timed calls per sweep size: ~4 GiB of data per size, 3..50 calls."""
    return max(3, min(50, (4 << 30) // max(nbytes, 1)))


AR_WARM_CALLS = 2   # untimed calls per size before its timed calls


def allreduce_plan(args, world) -> list[tuple[int, int]]:
    """(bytes, timed calls) per sweep size, in sweep order (per dtype)."""
    return [(b, allreduce_iters(b)) for b in allreduce_sizes(args, world)]


def run_allreduce(args, dev, world, rank) -> dict:
    """Real collective (RCCL at every N on GPUs): an exact-sum check per dtype,
    then the size sweep, each size timed with an event pair around its
    iterations (hipEvents on a GPU), slowest rank's time.

    The sweep buffer holds zeros, the fixed point of an in-place sum over
    ranks: every timed call reduces finite data (a buffer of ones would be
    multiplied by N at every call and reach inf after ~43 calls at N = 8),
    and the buffer is checked to be all zero after each dtype's sweep."""
    import torch
    import torch.distributed as dist

    dtypes = {"bf16": torch.bfloat16, "fp32": torch.float32}
    names = [d for d in args.allreduce_dtypes.split(",") if d]
    plan = allreduce_plan(args, world)
    timer = _Timer(dev)
    sweep = []
    for name in names:
        dt_ = dtypes[name]
        esz = torch.tensor([], dtype=dt_).element_size()
        # correctness: every rank contributes rank+1; the sum is exact in bf16 for n <= 8
        probe = torch.full(((1 << 20) // esz,), float(rank + 1), device=dev, dtype=dt_)
        dist.all_reduce(probe)
        _sync(dev)
        want = world * (world + 1) / 2
        bad = int((probe != want).sum().item())
        if bad:
            raise SystemExit(f"{name} all-reduce check failed on rank {rank}: {bad} elements != {want}")
        del probe
        buf = torch.zeros(max(b for b, _ in plan) // esz, device=dev, dtype=dt_)
        for nbytes, iters in plan:
            n = max(1, nbytes // esz)
            x = buf[:n]
            for _ in range(AR_WARM_CALLS):
                dist.all_reduce(x)
            _sync(dev)
            _barrier(dev)
            _sync(dev)
            mk = timer.marks(2)
            timer.record(mk, 0)
            for _ in range(iters):
                dist.all_reduce(x)
            timer.record(mk, 1)
            dt = timer.elapsed_ms(mk)[0] / iters / 1e3
            dt = _max_over_ranks(dt, dev)
            algbw = n * esz / dt / 1e9
            sweep.append({"bytes": n * esz, "dtype": name, "ms": round(dt * 1e3, 5), "iters": iters,
                          # a 1-rank all-reduce moves nothing: no bandwidth to report
                          "algbw_GBps": round(algbw, 2) if world > 1 else None,
                          "busbw_GBps": round(algbw * 2 * (world - 1) / world, 2)})
        _sync(dev)
        nonzero = int(torch.count_nonzero(buf).item())
        if nonzero:
            raise SystemExit(f"{name} all-reduce sweep buffer on rank {rank}: {nonzero} elements "
                             "left the zero fixed point")
        del buf
    head = next((s for s in sweep if s["bytes"] == args.allreduce_mib << 20 and s["dtype"] == names[0]),
                sweep[-1] if sweep else None)
    peak = {d: max((s["busbw_GBps"] for s in sweep if s["dtype"] == d), default=None) for d in names}
    return {
        "backend": dist.get_backend(),
        "rccl_ranks": dist.get_world_size(),
        "dtypes": names, "op": "sum", "check": "exact (sum of rank+1) per dtype",
        "sweep_data": "zeros, the in-place sum's fixed point (all zero after each sweep: checked)",
        "timing": "event pair around the iterations of each size (hipEvents on GPUs), slowest rank",
        "bytes": head["bytes"] if head else None,
        "ms": head["ms"] if head else None,
        "algbw_GBps": head["algbw_GBps"] if head else None,
        "busbw_GBps": head["busbw_GBps"] if head else None,
        "busbw_peak_GBps": peak if world > 1 else None,
        "sweep": sweep,
        "note": ("1-rank communicator: RCCL completes an in-place all-reduce without moving "
                 "data, so there is no algbw (null) and busbw is 0 by definition")
        if world == 1 else None,
    }


def ab_other_sizes(args, dev, timer) -> list:
    """The protocol's other square sizes (context for the headline shape):
    hand-written kernel vs hipBLASLt, A/B-interleaved blocks of back-to-back
    launches (median of 8 blocks per kernel) after a short warm-up on the
    warm chip, output checked against fp32."""
    import torch

    from mxk8s.ops import gemm_bf16_tn
    out = []
    for n in [int(x) for x in args.ab_sizes.split(",") if x]:
        if dev.type != "cuda" and n > 1024:
            continue
        g = torch.Generator(device=dev)
        g.manual_seed(n)
        A = (torch.rand((n, n), device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        Bt = (torch.rand((n, n), device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        C = torch.empty((n, n), device=dev, dtype=torch.bfloat16)
        C2 = torch.empty_like(C)
        gemm_bf16_tn(A, Bt, C)
        _sync(dev)
        err, tol = _full_check(A, Bt, C)
        fns = {"mxk": lambda: gemm_bf16_tn(A, Bt, C), "hipblaslt": lambda: torch.mm(A, Bt.t(), out=C2)}
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for f in fns.values():
                f()
            _sync(dev)
        # blocks of back-to-back launches bracketed by one event pair: at
        # 4096^3 a launch is ~0.1 ms, and an event record plus a Python call
        # per launch let the host fall behind the GPU (per-launch events put
        # both kernels ~4 % below their back-to-back rate, unevenly)
        ts = {k: [] for k in fns}
        reps = max(8, min(40, int(40 * (8192 / n) ** 3)))
        for r in range(8):
            for k in (("mxk", "hipblaslt") if r % 2 == 0 else ("hipblaslt", "mxk")):
                mk = timer.marks(2)
                timer.record(mk, 0)
                for _ in range(reps):
                    fns[k]()
                timer.record(mk, 1)
                ts[k].append(timer.elapsed_ms(mk)[0] / reps)
        med = {k: statistics.median(v) for k, v in ts.items()}
        fl = 2.0 * n ** 3
        out.append({"M": n, "N": n, "K": n, "check_ok": bool(err <= tol),
                    "mxk_tflops": round(fl / med["mxk"] / 1e9, 2),
                    "hipblaslt_tflops": round(fl / med["hipblaslt"] / 1e9, 2),
                    "mxk_over_hipblaslt": round(med["hipblaslt"] / med["mxk"], 4)})
        del A, Bt, C, C2
    return out


def run_validator(args) -> dict:
    import torch

    from mxk8s.ops import gemm_bf16_tn

    world, rank, local = _dist_env()
    cpu = os.environ.get("MXK_BENCH_DEVICE") == "cpu" or not torch.cuda.is_available()
    # MXK_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with fewer
    # GPUs than ranks (ranks share GPUs round-robin; RCCL refuses that).  The
    # measured configuration is always the default: RCCL, one rank per GPU.
    backend = "gloo" if cpu else os.environ.get("MXK_BENCH_BACKEND", "nccl")
    if cpu:
        dev = torch.device("cpu")
    else:
        if backend != "nccl":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    _init_group(backend, dev, world, rank)
    timer = _Timer(dev)

    M = N = K = args.size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    A = (torch.rand((M, K), device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand((N, K), device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    C_ref = torch.empty((M, N), device=dev, dtype=torch.bfloat16)

    def mxk():
        gemm_bf16_tn(A, Bt, C)

    def blas():
        torch.mm(A, Bt.t(), out=C_ref)

    # correctness gate before timing: the whole output vs fp32
    C.zero_()
    mxk()
    _sync(dev)
    err0, tol = _full_check(A, Bt, C)
    if not err0 <= tol:
        raise SystemExit(f"GEMM self-check failed: max|err| {err0} > {tol} (2^-7 max|ref|)")
    _log(rank, f"[bench] GEMM {M}x{N}x{K} bf16 full-output check ok "
               f"(max err {err0:.3g} <= {tol:.3g}); warmup >= {args.warmup} launches "
               f"and >= {args.warmup_s} s, steps {args.steps}")

    # time-floored warm-up; both kernels launched so neither is timed cold
    blas()
    t_w = time.perf_counter()
    n_warm = 0
    while True:
        for _ in range(10):
            mxk()
        n_warm += 10
        _sync(dev)
        if n_warm >= args.warmup and time.perf_counter() - t_w >= args.warmup_s:
            break
    warmup_s = time.perf_counter() - t_w

    # the timed region: exactly K back-to-back launches, barrier + sync on
    # both sides, one event pair around them (an event record between launches
    # is a queue packet of its own: per-launch events cost ~1 % of the wall
    # time at 8192^3, so they are taken in a second pass below)
    span = timer.marks(2)
    _sync(dev)
    _barrier(dev)
    _sync(dev)
    t0 = time.perf_counter()
    timer.record(span, 0)
    for i in range(args.steps):
        mxk()
    timer.record(span, 1)
    _sync(dev)
    dt = time.perf_counter() - t0   # the K launches, up to their completion
    _barrier(dev)
    _sync(dev)
    span_ms = timer.elapsed_ms(span)[0]
    dt_max = _max_over_ranks(dt, dev)

    # per-launch hipEvent times of another K launches (the median is reported
    # beside the wall-clock mean; not part of the headline)
    marks = timer.marks(args.steps + 1)
    for i in range(args.steps):
        timer.record(marks, i)
        mxk()
    timer.record(marks, args.steps)
    step_ms = timer.elapsed_ms(marks)
    flops = 2.0 * M * N * K
    per_gpu_tflops = flops * args.steps / dt / 1e12
    agg_tflops = world * flops * args.steps / dt_max / 1e12
    ev_med = statistics.median(step_ms)

    # the output of the last timed launch, whole, vs fp32
    err1, _ = _full_check(A, Bt, C)
    if not err1 <= tol:
        raise SystemExit(f"GEMM check after the timed loop failed: max|err| {err1} > {tol}")

    # A/B-interleaved hipBLASLt under the same event protocol
    ab = None
    if not args.no_reference:
        # blocks of n_ab back-to-back launches, one event pair per block (the
        # same protocol as the timed region), kernels alternating block by block
        n_ab = max(args.steps, 20)
        t_mxk, t_blas = [], []
        for r in range(args.ab_rounds):
            for fn, out in ((mxk, t_mxk), (blas, t_blas)) if r % 2 == 0 else ((blas, t_blas), (mxk, t_mxk)):
                mk = timer.marks(2)
                timer.record(mk, 0)
                for i in range(n_ab):
                    fn()
                timer.record(mk, 1)
                out.append(timer.elapsed_ms(mk)[0] / n_ab)
        m_mxk, m_blas = statistics.median(t_mxk), statistics.median(t_blas)
        ab = {"launches_each": n_ab * args.ab_rounds, "rounds": args.ab_rounds,
              "timing": "median over rounds of per-launch time in a block of back-to-back launches",
              "mxk_median_ms": round(m_mxk, 4), "hipblaslt_median_ms": round(m_blas, 4),
              "mxk_tflops": round(flops / m_mxk / 1e9, 2),
              "hipblaslt_tflops": round(flops / m_blas / 1e9, 2),
              "mxk_over_hipblaslt": round(m_blas / m_mxk, 4)}

    sizes_ab = [] if args.no_reference else ab_other_sizes(args, dev, timer)
    ar = None if args.no_allreduce else run_allreduce(args, dev, world, rank)

    return {
        "metric": METRIC,
        "value": round(agg_tflops, 2),
        "unit": "TFLOPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (uniform [-1,1) random bf16 operands)",
        "config": {"model": f"validator bf16 MFMA GEMM M=N=K={M} + RCCL allreduce",
                   "global_batch": world, "seq_len": None,
                   "parallelism": f"dp{world} (one GEMM per amd.com/gpu)"},
        "device": "cpu (reference GEMM, plumbing test)" if cpu else "cuda",
        "per_gpu_tflops": round(per_gpu_tflops, 2),
        "warmup_launches": n_warm,
        "warmup_s": round(warmup_s, 3),
        "event_span_ms_per_step": round(span_ms / args.steps, 4),
        "event_median_ms": round(ev_med, 4),
        "event_median_tflops": round(flops / ev_med / 1e9, 2),
        "gemm_check": {"max_abs_err_first": err0, "max_abs_err_after_timed": err1,
                       "tolerance": tol, "elements": M * N, "reference": "fp32 torch.matmul"},
        "hipblaslt_ab": ab,
        "hipblaslt_tflops_same_shape": None if ab is None else ab["hipblaslt_tflops"],
        "ab_other_sizes": sizes_ab,
        "launch": "eager",
        "allreduce": ar,
    }


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=None, help="number of GPUs (= WORLD_SIZE)")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--warmup-s", type=float, default=2.0,
                   help="validator mode: minimum seconds of warm-up launches")
    p.add_argument("--mode", choices=["validator", "ddp"], default="validator")
    p.add_argument("--size", type=int, default=8192, help="GEMM M=N=K (validator mode)")
    p.add_argument("--allreduce-mib", type=int, default=256, help="headline all-reduce size")
    p.add_argument("--allreduce-sizes", default="",
                   help="all-reduce sweep sizes in MiB (comma list); default: the protocol's "
                        "8 B - 8 GiB x2 sweep at n > 1")
    p.add_argument("--allreduce-min-bytes", type=int, default=8)
    p.add_argument("--allreduce-max-bytes", type=int, default=8 << 30)
    p.add_argument("--allreduce-dtypes", default="bf16,fp32")
    p.add_argument("--ab-rounds", type=int, default=12, help="A/B-interleaved hipBLASLt rounds")
    p.add_argument("--ab-sizes", default="4096,16384",
                   help="other square sizes A/B'd against hipBLASLt for context (not the metric)")
    p.add_argument("--no-reference", action="store_true")
    p.add_argument("--no-allreduce", action="store_true")
    p.add_argument("--seq-len", type=int, default=2048, help="ddp mode")
    p.add_argument("--micro-batch", type=int, default=8, help="ddp mode: sequences per GPU per step (8 x 2048 tokens: 197 GiB peak of 288 at 1 GPU)")
    p.add_argument("--layers", type=int, default=None, help="ddp mode: override (NOT headline)")
    p.add_argument("--bucket-mb", type=float, default=512.0, help="ddp mode: all-reduce bucket size")
    p.add_argument("--no-zero", action="store_true", help="ddp mode: replicated optimizer (no ZeRO-1)")
    p.add_argument("--no-tuned-gemms", action="store_true", help="ddp mode: default hipBLASLt picks")
    p.add_argument("--grad-reduce", choices=["bf16", "fp32"], default="bf16",
                   help="ddp mode: gradient wire format (fp32: one bf16 rounding instead of n-1)")
    p.add_argument("--rccl-profile", choices=["none", "xgmi-node"], default="xgmi-node",
                   help="RCCL environment preset for N > 1 (mxk8s/parallel/rccl_env.py); "
                        "variables already set win")
    args = p.parse_args(argv)

    world, rank, _ = _dist_env()
    if args.gpus is not None and args.gpus != world:
        if world == 1 and args.gpus > 1 and "TORCHELASTIC_RUN_ID" not in os.environ:
            # launched without torchrun: run ourselves under torch.distributed.run
            # as a child (never exec: nothing here has touched the GPU yet, but
            # a child keeps that true by construction)
            import socket
            import subprocess
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
                   f"--master-port={port}", os.path.abspath(__file__)] + \
                (list(argv) if argv is not None else sys.argv[1:])
            return subprocess.call(cmd)
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")

    rccl_vars = None
    if world > 1:
        # before anything initialises HIP / RCCL in this process
        from mxk8s.parallel import rccl_env
        rccl_vars = rccl_env.apply(args.rccl_profile)

    if args.mode == "validator":
        if args.steps is None:
            args.steps = 50
        if args.warmup is None:
            args.warmup = 10
        out = run_validator(args)
    else:
        if args.steps is None:
            args.steps = 10
        if args.warmup is None:
            args.warmup = 3
        from mxk8s.train.ddp_llama import run_ddp_bench
        out = run_ddp_bench(args)

    if rccl_vars is not None:
        out["rccl_env"] = {"profile": args.rccl_profile, "vars": rccl_vars}
    if rank == 0:
        print(json.dumps(out), flush=True)
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
    except Exception:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
