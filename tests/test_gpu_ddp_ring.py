"""The fp32 gradient wire format's staging ring on real HIP streams.

On the CPU tier (tests/test_ddp_cpu.py) the ring runs without streams.  Here
two gloo ranks share cuda:0, so the casts into the fp32 slots, the
collectives issued from the side stream and the round-back to bf16 run on
their own HIP stream exactly as under RCCL, and the result must be
bit-identical to staging every bucket at once (stage_slots=0) and within one
bf16 rounding of the exact sum.  (RCCL itself needs one GPU per rank.)"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from mxk8s.models.llama import Llama, LlamaConfig
    from mxk8s.parallel.ddp import FlatDDP
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    g = torch.Generator(device=dev)
    g.manual_seed(100 + rank)
    tokens = torch.randint(0, cfg.vocab_size, (2, 65), device=dev, generator=g)
    out = {}
    for slots in (3, 0):
        torch.manual_seed(0)
        with torch.device(dev):
            model = Llama(cfg)
        model = model.to(torch.bfloat16)
        ddp = FlatDDP(model, bucket_mb=0.05, reduce_dtype="fp32", stage_slots=slots)
        assert (ddp._side is not None) and ddp.stage_slots == (3 if slots else len(ddp.buckets))
        with ddp.no_sync():
            model.loss(tokens).backward()
        local = ddp.space.grad_buf.clone()
        ddp.zero_grad()
        model.loss(tokens).backward()
        ddp.finish_grad_sync()
        torch.cuda.synchronize()
        out[slots] = (local.cpu(), ddp.space.grad_buf.cpu(), len(ddp.buckets))
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_fp32_wire_ring_on_hip_streams():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        z = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(world)]
    exact = sum(z[r][3][0].double() for r in range(world))
    big = exact.abs() > 1e-3 * exact.abs().max()
    for r in range(world):
        local, reduced, nb = z[r][3]
        assert nb > 3
        assert torch.equal(reduced, z[r][0][1])       # the 3-slot ring == every bucket at once
        assert torch.equal(reduced, z[0][3][1])       # both ranks agree
        rel = ((reduced.double() - exact).abs()[big] / exact.abs()[big]).max().item()
        assert rel <= 2.0 ** -8, rel
