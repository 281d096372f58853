"""The default multi-rank training path (ZeRO-1) rehearsed on one GPU.

BASELINE config 5 is DDP on ``amd.com/gpu=8``; with more than one rank
``mxk8s.train.ddp_llama.build`` shards AdamW (ZeRO-1): the grad hooks launch
``reduce_scatter_tensor`` per bucket (``mxk8s/parallel/ddp.py`` ``_launch``),
``ShardedFlatAdamW`` runs the HIP AdamW kernel on shard offsets and
all-gathers each bucket in place, and each module's forward pre-hook waits
for the all-gathers of its own buckets (``optim.py`` ``enable_overlap`` /
``_wait_buckets``).  On the CPU tier (tests/test_ddp_cpu.py) none of that runs
on HIP streams.  Here 2 and 4 gloo ranks share cuda:0 (RCCL needs one GPU
per rank), so the production code - unchanged, no shim - runs with the HIP
AdamW / clip kernels on the compute stream, the fp32 wire's casts on the
side stream and gloo's CUDA work waited for through stream waits.

Asserted after 3 steps of the tiny Llama through ``build(..., zero=True)``
with the bf16 and the fp32 wire, gather overlap on:

* parameters bit-identical across ranks (per run);
* each rank's shard of the fp32 master / second moment equals the
  replicated run's (``zero=False``) slice of the same state after step 1,
  to the wire's summation order (the clip norm is also summed per shard
  there, over the whole buffer here);
* after step 3 (the bf16 parameters feed back into the forward, so an
  element whose gradient is ~0 can take a different Adam step): every
  master element within 10 lr and at most 1 % beyond 1e-4;
* the gathered bf16 parameters are every rank's master shard rounded to
  bf16.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

LR = 1e-3
RUNS = {"zero_bf16": (True, "bf16"), "zero_fp32": (True, "fp32"),
        "plain_bf16": (False, "bf16"), "plain_fp32": (False, "fp32")}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, devtype="cuda"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.set_num_threads(2)
    import torch.distributed as dist
    from mxk8s.models.llama import LlamaConfig
    from mxk8s.train.ddp_llama import build, train_step
    dev = torch.device(devtype, 0) if devtype == "cuda" else torch.device("cpu")
    if devtype == "cuda":
        torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    g = torch.Generator(device=dev)
    g.manual_seed(100 + rank)
    batches = [torch.randint(0, cfg.vocab_size, (2, 129), device=dev, generator=g)
               for _ in range(3)]
    out = {}
    for name, (zero, wire) in RUNS.items():
        torch.manual_seed(0)
        model, ddp, opt = build(cfg, dev, bucket_mb=0.25, lr=LR, zero=zero,
                                reduce_dtype=wire, gather_overlap=True)
        assert ddp.sharded == zero and len(ddp.buckets) > 3
        rec = {}
        losses = []
        for step, b in enumerate(batches):
            losses.append(train_step(model, ddp, opt, b))
            if step in (0, len(batches) - 1):
                opt.synchronize()
                tag = "1" if step == 0 else "3"
                rec["master" + tag] = opt.master.to("cpu", copy=True)
                rec["m" + tag] = opt.exp_avg.to("cpu", copy=True)
                rec["v" + tag] = opt.exp_avg_sq.to("cpu", copy=True)
        if devtype == "cuda":
            torch.cuda.synchronize()
        rec.update(params=ddp.space.param_buf.to("cpu", copy=True), loss=torch.stack(losses).float().cpu(),
                   norm=opt.last_grad_norm.float().cpu())
        if zero:
            rec["ranges"] = torch.tensor([(*ddp.shard_range(b), b.shard_off) for b in ddp.buckets])
            rec["waits"] = len(opt.waits)
        out[name] = rec
        del model, ddp, opt
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_zero1_default_path_on_shared_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mxk8s.ops import _lib
    _lib.lib()   # the HIP library must load: the AdamW / clip kernels are what runs
    _check(world, "cuda")


def _check(world, devtype):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, devtype), nprocs=world, join=True)
        z = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(world)]
    for name in RUNS:
        for r in range(1, world):
            assert torch.equal(z[r][name]["params"], z[0][name]["params"]), (name, r)
        assert torch.isfinite(z[0][name]["loss"]).all(), name
    for wire in ("bf16", "fp32"):
        plain, zero = f"plain_{wire}", f"zero_{wire}"
        for r in range(world):
            P, Z = z[r][plain], z[r][zero]
            # the replicated state is the same on every rank
            assert torch.equal(P["master3"], z[0][plain]["master3"])
            assert Z["waits"] > 0                     # the forward pre-hooks waited
            assert torch.allclose(Z["loss"][0], P["loss"][0])   # same parameters, same batch
            sl = _shard_view(Z["ranges"].tolist())
            assert sum(hi - lo for lo, hi, _ in sl) * world == P["params"].numel()
            # step 1: identical parameters in, so the gradients agree up to
            # the wire's summation order, and Adam's first update is
            # lr * sign(g) nearly everywhere
            m1 = _gather(Z["master1"], sl)
            d1 = (m1 - _flat(P["master1"], sl)).abs()
            assert (d1 > 1e-6).float().mean().item() <= 1e-3, (wire, r)
            v1 = _gather(Z["v1"], sl)
            ref_v1 = _flat(P["v1"], sl)
            assert torch.allclose(v1, ref_v1, rtol=2e-2, atol=1e-3 * ref_v1.abs().max().item())
            # step 3: the bf16 parameters feed back into the forward, so an
            # element whose gradient is ~0 can take a different Adam step
            # (|step| <= a few lr); everything else agrees to fp32 noise
            d3 = (_gather(Z["master3"], sl) - _flat(P["master3"], sl)).abs()
            assert d3.max().item() <= 10 * LR, (wire, r, d3.max().item())
            assert (d3 > 1e-4).float().mean().item() <= 1e-2, (wire, r)
            assert torch.allclose(Z["norm"], P["norm"], rtol=1e-2)
            # the all-gather delivered every rank's AdamW output: rank 0's
            # parameters hold rank r's master chunks rounded to bf16
            assert torch.equal(_flat(z[0][zero]["params"], sl),
                               _gather(Z["master3"], sl).to(torch.bfloat16)), (wire, r)


def _shard_view(ranges):
    return [(lo, hi, so) for lo, hi, so in ranges]


def _gather(shard, sl):
    """The rank's shard, in bucket order (the shard-local layout)."""
    return torch.cat([shard[so:so + hi - lo] for lo, hi, so in sl])


def _flat(full, sl):
    """The same elements of a replicated (flat-layout) buffer."""
    return torch.cat([full[lo:hi] for lo, hi, _ in sl])
