"""Llama-3 DDP training on synthetic tokens (BASELINE config 5).

One process per GPU (torchrun), RCCL over xGMI, flat bucketed all-reduce
overlapped with backward (``mxk8s.parallel.ddp.FlatDDP``), fused flat AdamW
(``mxk8s.parallel.optim.FlatAdamW``), bf16 compute.

    python -m torch.distributed.run --standalone --nproc-per-node 8 \\
        -m mxk8s.train.ddp_llama --steps 10 --seq-len 2048

``run_ddp_bench`` is what ``bench.py --mode ddp`` calls: W warm-up steps, K
timed steps bracketed by barrier + synchronize, slowest rank's time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

from ..models.llama import Llama, LlamaConfig
from ..parallel import dist as mxdist
from ..parallel.ddp import FlatDDP
from ..parallel.optim import FlatAdamW, ShardedFlatAdamW
from ..utils import roctx

MI355X_BF16_DENSE_PEAK = 2.5e15   # FLOP/s, dense (MI355X_MICROARCH.md)
TUNED_GEMMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning",
                           "tunableop_mi355x_llama3_8b.csv")


def library_gemms_in_step() -> bool:
    """True when an A/B switch routes some product of the step to torch's
    hipBLASLt / rocBLAS GEMMs (``MXK_WGRAD=0``, ``MXK_DGRAD=0``,
    ``MXK_FWD_LIB=1``); by default every product runs on the hand-written
    kernels and no library GEMM is called."""
    from ..ops import linear
    return not (linear._USE_MXK_WGRAD and linear._USE_MXK_DGRAD and not linear._FWD_LIB)


def use_tuned_gemms(path: str = TUNED_GEMMS) -> bool:
    """Load the PyTorch TunableOp table of the Llama-3-8B step's hipBLASLt /
    rocBLAS GEMMs (fastest solution per shape, found once with
    scripts/gpu/tune_gemms.sh on MI355X) read-only: no tuning at run time.
    Since round 3 every GEMM of the step runs on the hand-written kernels, so
    the table only matters for the A/B switches (MXK_WGRAD=0 / MXK_DGRAD=0)
    and shapes outside the kernels' tiling.
    TunableOp ignores the table if the torch / hipBLASLt / rocBLAS versions
    or the GPU arch recorded in it differ."""
    if not (torch.cuda.is_available() and os.path.exists(path)):
        return False
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.set_filename(path, insert_device_ordinal=False)
    return bool(tunable.read_file(path))


def build(cfg: LlamaConfig, device: torch.device, bucket_mb: float, lr: float = 3e-4,
          zero: bool = True, overlap: bool | None = None, reduce_dtype: str = "bf16",
          gather_overlap: bool = True):
    """Model + DDP + optimizer.  ``zero`` shards the AdamW state and step over
    the ranks (ZeRO-1, reduce-scatter + all-gather); it only applies with
    more than one rank.  ``overlap`` (``MXK_OPT_OVERLAP=1``) runs the
    unsharded AdamW on a side stream under the next forward
    (``FlatAdamW.enable_overlap``); bit-identical, but measured neutral on
    one MI355X (617-618 ms per step either way, profiles/r2_ddp/
    opt_overlap_ab.log: the forward GEMMs leave no CU slots for the update
    kernels), so off by default.  ``gather_overlap`` (ZeRO-1): each bucket's
    parameter all-gather is waited for by the forward pre-hook of the first
    module that reads it, so the all-gather of the whole model runs under the
    next forward instead of in front of it.  ``reduce_dtype`` "fp32" reduces
    gradients in fp32 on the wire (one bf16 rounding instead of world - 1)."""
    if overlap is None:
        overlap = os.environ.get("MXK_OPT_OVERLAP", "0") == "1"
    with torch.device(device):
        model = Llama(cfg)
    model = model.to(torch.bfloat16)
    ddp = FlatDDP(model, bucket_mb=bucket_mb, shard_optimizer=zero, reduce_dtype=reduce_dtype)
    if ddp.sharded:
        opt = ShardedFlatAdamW(ddp, lr=lr)
        if gather_overlap:
            opt.enable_overlap(overlap_stages(model))
    else:
        opt = FlatAdamW(ddp.space, lr=lr, grad_scale=ddp.grad_scale)
        if overlap and device.type == "cuda":
            opt.enable_overlap(overlap_stages(model))
    return model, ddp, opt


def overlap_stages(model: Llama):
    """AdamW stages in the order the forward reads parameters: the embedding
    with every 1-D weight (the fused norms read the next layer's weight one
    layer early), then each block's matrices, then the LM head."""
    one_d = [p for p in model.parameters() if p.requires_grad and p.dim() < 2]
    stages = [([model.embed.weight] + one_d, model.embed)]
    for layer in model.layers:
        stages.append(([p for p in layer.parameters() if p.dim() >= 2], layer))
    stages.append(([model.lm_head.weight], model.lm_head))
    return stages


def train_step(model, ddp, opt, tokens) -> torch.Tensor:
    # roctx ranges: host-side phases on rocprofv3 --marker-trace timelines
    with roctx.range("step.forward"):
        loss = model.loss(tokens)
    with roctx.range("step.backward+allreduce"):
        loss.backward()
        ddp.finish_grad_sync()
    with roctx.range("step.adamw"):
        opt.step()
        ddp.zero_grad()
    return loss.detach()


def run_ddp_bench(args) -> dict:
    world, rank, local = mxdist.world_info()
    if torch.cuda.is_available():
        # MXK_BENCH_BACKEND=gloo rehearses the multi-rank step (ZeRO-1
        # reduce-scatter / all-gather, side-stream events) with more ranks
        # than GPUs: ranks share GPUs round-robin, which RCCL refuses.  The
        # measured configuration is always RCCL with one rank per GPU.
        backend = os.environ.get("MXK_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
        backend = "gloo"
    mxdist.init_distributed(backend=backend, device=dev if backend == "nccl" else None)
    cfg = LlamaConfig.llama3_8b()
    model_name = "Llama-3-8B"
    if getattr(args, "layers", None):
        cfg.n_layers = args.layers
        model_name = f"Llama-3-8B-shape, {args.layers} layers (NOT the headline config)"
    if getattr(args, "tiny", False):
        cfg = LlamaConfig.tiny()
        model_name = "tiny-llama (test)"
    seq, mb = args.seq_len, args.micro_batch
    bucket_mb = getattr(args, "bucket_mb", 512.0)
    # the TunableOp table only matters when a library GEMM runs in the step
    lib_gemms = library_gemms_in_step()
    tuned = (use_tuned_gemms() if lib_gemms and not getattr(args, "no_tuned_gemms", False)
             else False)
    zero = not getattr(args, "no_zero", False)
    reduce_dtype = getattr(args, "grad_reduce", "bf16")
    model, ddp, opt = build(cfg, dev, bucket_mb, zero=zero, reduce_dtype=reduce_dtype)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    nbatches = 4
    batches = [torch.randint(0, cfg.vocab_size, (mb, seq + 1), device=dev, generator=g)
               for _ in range(nbatches)]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    start_step = 0
    if getattr(args, "resume", None):
        from . import checkpoint
        start_step = checkpoint.load(args.resume, ddp, opt)
    for i in range(args.warmup):
        train_step(model, ddp, opt, batches[i % nbatches])
    sync()
    mxdist.barrier()
    sync()
    t0 = time.perf_counter()
    losses = []
    # "bench.timed" bounds the steady-state steps on a rocprofv3 marker trace:
    # scripts/kernel_breakdown.py --trace keeps only the kernels inside it
    with roctx.range("bench.timed"):
        # continue the batch rotation after the warm-up: restarting at batch 0
        # re-fed the warm-up's batch, whose loss Adam's first (sign-sized)
        # update had just collapsed (0.87 at 2 layers: a memorised batch, not
        # a training signal)
        for i in range(args.steps):
            losses.append(train_step(model, ddp, opt, batches[(args.warmup + i) % nbatches]))
        sync()
    mxdist.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_max = mxdist.max_over_ranks(dt, dev)
    if getattr(args, "save_checkpoint", None):   # outside the timed region
        from . import checkpoint
        checkpoint.save(args.save_checkpoint, ddp, opt,
                        step=start_step + args.warmup + args.steps)
    tokens = world * mb * seq * args.steps
    tps = tokens / dt_max
    flops_tok = cfg.flops_per_token(seq)
    mfu = flops_tok * tps / (MI355X_BF16_DENSE_PEAK * world)
    peak_mem = torch.cuda.max_memory_allocated(dev) if dev.type == "cuda" else 0
    final_loss = float(torch.stack(losses).float().mean().item()) if losses else float("nan")
    return {
        "metric": "Llama-3-8B DDP training throughput (tokens/s, whole job)",
        "value": round(tps, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (uniform random token ids), random-init weights",
        "config": {"model": model_name, "global_batch": world * mb, "seq_len": seq,
                   "parallelism": f"dp{world}" + ("+zero1" if ddp.sharded else "")},
        "tokens_per_s_per_gpu": round(tps / world, 1),
        "mfu": round(mfu, 4),
        "params": cfg.num_params(),
        "peak_mem_gib": round(peak_mem / 2 ** 30, 2),
        "mean_loss": final_loss,
        "bucket_mb": bucket_mb,
        "backend": backend if world > 1 else None,
        "grad_reduce_dtype": reduce_dtype,
        "param_gather": ("overlapped with the next forward" if getattr(opt, "_module_buckets", None)
                         else "in step()") if ddp.sharded else None,
        "library_gemms": ({"tunableop_table": tuned} if lib_gemms else None),
        "grad_norm_last": float(opt.last_grad_norm.item()),
        "losses": [round(float(x), 6) for x in torch.stack(losses).float().tolist()] if losses else [],
    }


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--seq-len", type=int, default=2048)
    p.add_argument("--micro-batch", type=int, default=8)
    p.add_argument("--layers", type=int, default=None)
    p.add_argument("--bucket-mb", type=float, default=512.0)
    p.add_argument("--tiny", action="store_true")
    p.add_argument("--save-checkpoint", default=None, metavar="DIR",
                   help="write params + optimizer state after the run (mxk8s.train.checkpoint)")
    p.add_argument("--resume", default=None, metavar="DIR", help="restore a checkpoint first")
    p.add_argument("--no-tuned-gemms", action="store_true",
                   help="do not load the TunableOp GEMM table")
    p.add_argument("--no-zero", action="store_true",
                   help="replicate the optimizer (all-reduce) instead of ZeRO-1 sharding")
    p.add_argument("--grad-reduce", choices=["bf16", "fp32"], default="bf16",
                   help="gradient wire format of the reduce-scatter / all-reduce")
    a = p.parse_args(argv)
    out = run_ddp_bench(a)
    if mxdist.world_info()[1] == 0:
        print(json.dumps(out), flush=True)
    if mxdist.active():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
