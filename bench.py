#!/usr/bin/env python3
"""Headline benchmark: validator HIP GEMM TFLOPS + RCCL all-reduce bus-bw.

BASELINE.json names the metric "validator HIP GEMM TFLOPS + RCCL allreduce
bus-bw at 1/2/4/8 amd.com/gpu" (configs 3 and 4).  One process per GPU
(``torch.distributed`` over RCCL when WORLD_SIZE > 1):

* a *step* is one 8192^3 bf16 GEMM on this rank's GPU through the hand-written
  CDNA4 MFMA kernel (``native/kernels/gemm_bf16.hip``), random uniform
  [-1, 1) operands (random data, never zeros: the chip clocks higher on zeros);
* W untimed warm-up steps, then exactly K timed steps bracketed by a barrier
  and ``torch.cuda.synchronize()``; the slowest rank's time is used;
* ``value`` = whole-job GEMM TFLOP/s = N x 2*M*N*K*K_steps / max-rank time;
* after the GEMM phase, an RCCL all-reduce (sum) of a 256 MiB bf16 buffer is
  timed across all ranks and reported as algbw / busbw = algbw * 2(n-1)/n;
* the same-shape hipBLASLt GEMM (``torch.matmul``) is timed for context.

``--mode ddp`` runs the Llama-3-8B DDP training step (config 5) instead.

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
             bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
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


def run_validator(args) -> dict:
    import torch
    import torch.distributed as dist

    from mxk8s.ops import gemm_bf16_tn
    from mxk8s.parallel.dist import init_distributed, max_over_ranks, barrier

    world, rank, local = _dist_env()
    # MXK_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with fewer
    # GPUs than ranks (ranks share GPUs round-robin; RCCL refuses that).  The
    # measured configuration is always the default: RCCL, one rank per GPU.
    backend = os.environ.get("MXK_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    init_distributed(backend=backend, device=dev)

    M = N = K = args.size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    A = (torch.rand((M, K), device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    Bt = (torch.rand((N, K), device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)

    # correctness gate on a sub-block before timing (fp32 reference)
    gemm_bf16_tn(A, Bt, C)
    torch.cuda.synchronize()
    ref = A[:256].float() @ Bt[:512].float().t()
    err = (C[:256, :512].float() - ref).abs().max().item()
    tol = 2e-2 * ref.abs().max().item() + 1e-2
    if not err <= tol:
        raise SystemExit(f"GEMM self-check failed: max|err| {err} > {tol}")

    _log(rank, f"[bench] GEMM {M}x{N}x{K} bf16 self-check ok (max err {err:.3g}); "
               f"warmup {args.warmup}, steps {args.steps}, "
               f"{'hipGraph replay' if args.graph else 'eager launches'}")
    # The K timed steps are K real GEMM launches.  With --graph they replay
    # from a hipGraph holding `chunk` back-to-back launches of the kernel (the
    # launcher is capture-safe: no sync, no allocation); steps not divisible by
    # the chunk run the remainder eagerly.  A 0.69 ms kernel already hides the
    # launch path, so eager is the default (graph replay measured equal).
    chunk = max(1, min(args.graph_chunk, args.steps))
    graph = None
    if args.graph:
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            gemm_bf16_tn(A, Bt, C)   # first launch outside capture (lazy init)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(chunk):
                gemm_bf16_tn(A, Bt, C)
        torch.cuda.synchronize()

    def run_steps(n):
        if graph is None:
            for _ in range(n):
                gemm_bf16_tn(A, Bt, C)
            return
        for _ in range(n // chunk):
            graph.replay()
        for _ in range(n % chunk):
            gemm_bf16_tn(A, Bt, C)

    run_steps(args.warmup)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, dev)
    flops = 2.0 * M * N * K
    per_gpu_tflops = flops * args.steps / dt / 1e12
    agg_tflops = world * flops * args.steps / dt_max / 1e12

    # hipBLASLt reference on the same data (context only; not the metric)
    ref_tflops = None
    if not args.no_reference:
        for _ in range(max(3, args.warmup // 4)):
            torch.matmul(A, Bt.t())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        nref = max(5, args.steps // 2)
        for _ in range(nref):
            torch.matmul(A, Bt.t())
        torch.cuda.synchronize()
        ref_tflops = flops * nref / (time.perf_counter() - t1) / 1e12

    # RCCL all-reduce over xGMI
    ar = None
    if not args.no_allreduce:
        nbytes = args.allreduce_mib << 20
        buf = torch.ones(nbytes // 2, device=dev, dtype=torch.bfloat16)
        iters = max(5, min(args.steps, 20))
        if world > 1:
            for _ in range(3):
                dist.all_reduce(buf)
            torch.cuda.synchronize()
            barrier()
            t2 = time.perf_counter()
            for _ in range(iters):
                dist.all_reduce(buf)
            torch.cuda.synchronize()
            barrier()
            ta = max_over_ranks((time.perf_counter() - t2) / iters, dev)
            algbw = nbytes / ta / 1e9
            busbw = algbw * 2 * (world - 1) / world
        else:
            # n = 1: no peer; busbw is 0 by definition — report the local
            # reduction-free copy rate as algbw (what RCCL does at n=1).
            tmp = torch.empty_like(buf)
            for _ in range(3):
                tmp.copy_(buf)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            for _ in range(iters):
                tmp.copy_(buf)
            torch.cuda.synchronize()
            ta = (time.perf_counter() - t2) / iters
            algbw = nbytes / ta / 1e9
            busbw = 0.0
        ar = {"bytes": nbytes, "dtype": "bf16", "op": "sum", "ms": ta * 1e3,
              "algbw_GBps": round(algbw, 2), "busbw_GBps": round(busbw, 2)}

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
        "per_gpu_tflops": round(per_gpu_tflops, 2),
        "hipblaslt_tflops_same_shape": None if ref_tflops is None else round(ref_tflops, 2),
        "gemm_self_check_max_abs_err": err,
        "launch": f"hipGraph x{chunk}" if graph is not None else "eager",
        "allreduce": ar,
    }


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=None, help="number of GPUs (= WORLD_SIZE)")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--mode", choices=["validator", "ddp"], default="validator")
    p.add_argument("--size", type=int, default=8192, help="GEMM M=N=K (validator mode)")
    p.add_argument("--allreduce-mib", type=int, default=256)
    p.add_argument("--no-reference", action="store_true")
    p.add_argument("--no-allreduce", action="store_true")
    p.add_argument("--graph", dest="graph", action="store_true", default=False,
                   help="validator mode: replay the timed GEMMs from a hipGraph "
                        "(measured equal to eager at 8192^3: profiles/r1_gemm_w4h/bench_graph_ab.log)")
    p.add_argument("--no-graph", dest="graph", action="store_false")
    p.add_argument("--graph-chunk", type=int, default=20, help="GEMM launches per captured graph")
    p.add_argument("--seq-len", type=int, default=2048, help="ddp mode")
    p.add_argument("--micro-batch", type=int, default=8, help="ddp mode: sequences per GPU per step (8 x 2048 tokens: 197 GiB peak of 288 at 1 GPU)")
    p.add_argument("--layers", type=int, default=None, help="ddp mode: override (NOT headline)")
    p.add_argument("--bucket-mb", type=float, default=512.0, help="ddp mode: all-reduce bucket size")
    p.add_argument("--no-zero", action="store_true", help="ddp mode: replicated optimizer (no ZeRO-1)")
    p.add_argument("--no-tuned-gemms", action="store_true", help="ddp mode: default hipBLASLt picks")
    args = p.parse_args(argv)

    world, rank, _ = _dist_env()
    if args.gpus is not None and args.gpus != world:
        if world == 1 and args.gpus > 1:
            # launched without torchrun: spawn ourselves under torch.distributed.run
            import subprocess
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
                   f"--master-port={29500 + os.getpid() % 1000}", os.path.abspath(__file__)] + \
                (argv if argv is not None else sys.argv[1:])
            return subprocess.call(cmd)
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")

    if args.mode == "validator":
        if args.steps is None:
            args.steps = 200
        if args.warmup is None:
            args.warmup = 100
        out = run_validator(args)
    else:
        if args.steps is None:
            args.steps = 10
        if args.warmup is None:
            args.warmup = 3
        from mxk8s.train.ddp_llama import run_ddp_bench
        out = run_ddp_bench(args)

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
