"""Multi-process data-parallel logic on CPU (gloo, world_size 2): the flat
bucketed all-reduce must give every rank the SUM of all ranks' gradients,
identical to a single-process reference, and the flat AdamW must match
torch.optim.AdamW."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from mxk8s.models.llama import Llama, LlamaConfig
from mxk8s.parallel.ddp import FlatDDP, FlatParamSpace
from mxk8s.parallel.optim import FlatAdamW


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank, cfg):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randint(0, cfg.vocab_size, (2, 17), generator=g)


def _worker(rank, world, port, outdir, bucket_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    model = Llama(cfg)   # fp32 on CPU (the CPU reference path of every fused op)
    ddp = FlatDDP(model, bucket_mb=bucket_mb)
    assert (len(ddp.buckets) > 1) == (bucket_mb < 1)
    loss = model.loss(_batch(rank, cfg))
    loss.backward()
    ddp.finish_grad_sync()
    torch.save({"grad": ddp.space.grad_buf.clone(), "param": ddp.space.param_buf.clone()},
               os.path.join(outdir, f"r{rank}.pt"))
    # one optimizer step keeps replicas identical
    opt = FlatAdamW(ddp.space, lr=1e-3, grad_scale=ddp.grad_scale)
    opt.step()
    torch.save({"param_after": ddp.space.param_buf.clone()}, os.path.join(outdir, f"s{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [0.05, 512.0])
def test_flat_ddp_gloo_two_ranks(bucket_mb):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, bucket_mb), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(world)]
        s = [torch.load(os.path.join(d, f"s{i}.pt"), weights_only=True) for i in range(world)]
    assert torch.equal(r[0]["grad"], r[1]["grad"])
    assert torch.equal(s[0]["param_after"], s[1]["param_after"])
    # single-process reference: sum of per-rank gradients
    cfg = LlamaConfig.tiny()
    ref_sum = None
    for rank in range(world):
        torch.manual_seed(0)
        model = Llama(cfg)
        space = FlatParamSpace(model)
        model.loss(_batch(rank, cfg)).backward()
        ref_sum = space.grad_buf.clone() if ref_sum is None else ref_sum + space.grad_buf
    assert torch.allclose(r[0]["grad"], ref_sum, rtol=1e-5, atol=1e-6)


def test_flat_space_views_and_grad_accumulation():
    torch.manual_seed(0)
    model = Llama(LlamaConfig.tiny())
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    space = FlatParamSpace(model)
    for n, p in model.named_parameters():
        assert torch.equal(p.detach(), before[n])
        assert p.data_ptr() >= space.param_buf.data_ptr()
        assert p.grad is not None and p.grad.data_ptr() >= space.grad_buf.data_ptr()
    # 2-D (decay) params first, 1-D (norms) last
    dims = [p.dim() for p in space.params]
    assert dims == sorted(dims, reverse=True)
    assert all(o % 64 == 0 for o in space.offsets)
    tok = torch.randint(0, 1024, (2, 9))
    model.loss(tok).backward()
    g1 = space.grad_buf.clone()
    model.loss(tok).backward()   # accumulates in place into the flat buffer
    assert torch.allclose(space.grad_buf, 2 * g1, rtol=1e-5, atol=1e-7)
    space.zero_grad()
    # accumulated ranges (embedding, norms) are zeroed; direct-gradient
    # weights (mxk8s.ops.linear.Linear) are marked fresh instead of memset
    for a, b in space._accum_ranges:
        assert space.grad_buf[a:b].abs().sum() == 0
    assert all(p._mxk_grad_fresh for p in space.params)
    model.loss(tok).backward()   # fresh -> overwrite, not accumulate
    assert torch.allclose(space.grad_buf, g1, rtol=1e-5, atol=1e-7)


def test_flat_adamw_matches_torch_adamw():
    torch.manual_seed(1)
    lin = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.LayerNorm(32))
    ref = [p.detach().clone().requires_grad_() for p in lin.parameters()]
    space = FlatParamSpace(lin)
    opt = FlatAdamW(space, lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1,
                    max_grad_norm=0.0)
    decay = [r for r in ref if r.dim() >= 2]
    nodecay = [r for r in ref if r.dim() < 2]
    topt = torch.optim.AdamW([{"params": decay, "weight_decay": 0.1},
                              {"params": nodecay, "weight_decay": 0.0}],
                             lr=1e-2, betas=(0.9, 0.95), eps=1e-8)
    for step in range(3):
        x = torch.randn(4, 16)
        lin(x).pow(2).sum().backward()
        opt.step()
        space.zero_grad()
        # same grads for the reference params
        out = torch.nn.functional.layer_norm(
            torch.nn.functional.linear(x, ref[0], ref[1]), (32,), ref[2], ref[3])
        out.pow(2).sum().backward()
        topt.step()
        topt.zero_grad()
    for p, r in zip(lin.parameters(), ref):
        assert torch.allclose(p.detach(), r.detach(), rtol=1e-4, atol=1e-5)


def test_grad_clipping_reference():
    lin = torch.nn.Linear(8, 8, bias=False)
    space = FlatParamSpace(lin)
    opt = FlatAdamW(space, lr=0.0, weight_decay=0.0, max_grad_norm=1.0, grad_scale=0.5)
    space.grad_buf.fill_(1.0)
    opt.step()
    norm = float(opt.last_grad_norm)
    # the buffer holds the SUM over 2 ranks -> mean grad norm = 0.5 * ||1||
    assert abs(norm - 0.5 * (64 ** 0.5)) < 1e-4
    assert abs(float(opt._scale[0]) - 0.5 / (norm + 1e-6)) < 1e-6


def _zero_worker(rank, world, port, outdir, bucket_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from mxk8s.parallel.optim import ShardedFlatAdamW
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    out = {}
    for sharded in (False, True):
        torch.manual_seed(0)
        model = Llama(cfg)
        ddp = FlatDDP(model, bucket_mb=bucket_mb, shard_optimizer=sharded)
        if sharded:
            assert ddp.sharded and ddp.shard_numel * world == ddp.space.numel
            assert all((b.end - b.start) % (64 * world) == 0 for b in ddp.buckets)
            opt = ShardedFlatAdamW(ddp, lr=1e-3, max_grad_norm=0.5)
        else:
            opt = FlatAdamW(ddp.space, lr=1e-3, grad_scale=ddp.grad_scale, max_grad_norm=0.5)
        for step in range(3):
            model.loss(_batch(rank * 10 + step, cfg)).backward()
            ddp.finish_grad_sync()
            opt.step()
            ddp.zero_grad()
        out[sharded] = {n: p.detach().clone() for n, p in model.named_parameters()}
        out[f"norm{sharded}"] = opt.last_grad_norm.clone()
    torch.save({"plain": out[False], "zero": out[True], "n0": out["normFalse"],
                "n1": out["normTrue"]}, os.path.join(outdir, f"z{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [0.05, 512.0])
def test_zero1_sharded_optimizer_matches_replicated(bucket_mb):
    """ZeRO-1 (reduce-scatter + sharded AdamW + all-gather) must produce the
    same parameters as the replicated all-reduce + AdamW path, on every rank."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_zero_worker, args=(world, _free_port(), d, bucket_mb), nprocs=world, join=True)
        z = [torch.load(os.path.join(d, f"z{i}.pt"), weights_only=True) for i in range(world)]
    for r in range(world):
        assert torch.allclose(z[r]["n0"], z[r]["n1"], rtol=1e-3)
        for n, p in z[r]["plain"].items():
            # Adam normalises tiny gradients (unused embedding rows) to O(lr) steps,
            # so fp32 reduction-order noise shows up at ~1e-5 absolute
            assert torch.allclose(z[r]["zero"][n], p, rtol=1e-4, atol=1e-4), n
    for n in z[0]["zero"]:
        assert torch.equal(z[0]["zero"][n], z[1]["zero"][n]), n


def test_ddp_trainer_torchrun_two_ranks_cpu(tmp_path):
    """The trainer entry point under torch.distributed.run (gloo, 2 ranks, CPU):
    ZeRO-1 path end to end, one JSON result line from rank 0, a sharded
    checkpoint written after the timed steps."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ck = str(tmp_path / "ck")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "mxk8s.train.ddp_llama", "--tiny", "--steps", "2", "--warmup", "1",
           "--seq-len", "64", "--micro-batch", "1", "--bucket-mb", "0.5",
           "--save-checkpoint", ck]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": repo, "OMP_NUM_THREADS": "2"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2+zero1"
    assert d["value"] > 0 and d["steps"] == 2
    assert sorted(os.listdir(ck)) == ["meta.json", "step-000000003"]
    assert sorted(os.listdir(os.path.join(ck, "step-000000003"))) == [
        "optim-rank0.safetensors", "optim-rank1.safetensors", "params.safetensors"]
    meta = json.load(open(os.path.join(ck, "meta.json")))
    assert meta["step"] == 3 and meta["format"] == "mxk8s-flat-v2"


def _ckpt_worker(rank, world, port, outdir, sharded):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from mxk8s.parallel.optim import ShardedFlatAdamW
    from mxk8s.train import checkpoint
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()

    def build():
        torch.manual_seed(0)
        model = Llama(cfg)
        ddp = FlatDDP(model, bucket_mb=0.05, shard_optimizer=sharded)
        opt = ShardedFlatAdamW(ddp, lr=1e-3) if sharded else \
            FlatAdamW(ddp.space, lr=1e-3, grad_scale=ddp.grad_scale)
        return model, ddp, opt

    def steps(model, ddp, opt, lo, hi):
        for s in range(lo, hi):
            model.loss(_batch(rank * 100 + s, cfg)).backward()
            ddp.finish_grad_sync()
            opt.step()
            ddp.zero_grad()

    m1, d1, o1 = build()
    steps(m1, d1, o1, 0, 4)                       # uninterrupted run
    m2, d2, o2 = build()
    steps(m2, d2, o2, 0, 2)
    checkpoint.save(os.path.join(outdir, "ck"), d2, o2, step=2)
    m3, d3, o3 = build()                           # "restarted job"
    assert checkpoint.load(os.path.join(outdir, "ck"), d3, o3) == 2
    steps(m3, d3, o3, 2, 4)
    torch.save({"a": d1.space.param_buf.clone(), "b": d3.space.param_buf.clone(),
                "ma": o1.master.clone(), "mb": o3.master.clone()},
               os.path.join(outdir, f"c{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("sharded", [False, True])
def test_checkpoint_resume_matches_uninterrupted(sharded):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ckpt_worker, args=(world, _free_port(), d, sharded), nprocs=world, join=True)
        files = sorted(os.listdir(os.path.join(d, "ck")))
        assert "meta.json" in files
        sfiles = os.listdir(os.path.join(d, "ck", "step-000000002"))
        assert "params.safetensors" in sfiles
        assert ("optim-rank1.safetensors" in sfiles) == sharded
        for r in range(world):
            c = torch.load(os.path.join(d, f"c{r}.pt"), weights_only=True)
            assert torch.equal(c["a"], c["b"])
            assert torch.equal(c["ma"], c["mb"])


def test_checkpoint_rejects_layout_mismatch(tmp_path):
    from mxk8s.train import checkpoint
    torch.manual_seed(0)
    model = Llama(LlamaConfig.tiny())
    ddp = FlatDDP(model)
    opt = FlatAdamW(ddp.space)
    checkpoint.save(str(tmp_path / "ck"), ddp, opt, step=5)
    cfg2 = LlamaConfig.tiny()
    cfg2.n_layers = 1
    m2 = Llama(cfg2)
    d2 = FlatDDP(m2)
    with pytest.raises(ValueError, match="layout"):
        checkpoint.load(str(tmp_path / "ck"), d2, FlatAdamW(d2.space))


def test_checkpoint_interrupted_save_keeps_previous(tmp_path):
    """A save that dies before its commit record leaves the previous step
    directory and meta.json in charge: the job resumes from the last complete
    checkpoint; a shard overwritten under a committed step is refused."""
    import json
    from mxk8s.train import checkpoint
    torch.manual_seed(0)
    model = Llama(LlamaConfig.tiny())
    ddp = FlatDDP(model)
    opt = FlatAdamW(ddp.space)
    ck = str(tmp_path / "ck")
    checkpoint.save(ck, ddp, opt, step=5)
    saved = opt.master.clone()
    # a later save wrote its shards into step-8, then the job died (no meta.json)
    opt.step_count += 3
    with torch.no_grad():
        opt.master.add_(1.0)
    s8 = os.path.join(ck, checkpoint.step_dirname(8))
    os.makedirs(s8)
    checkpoint._atomic_save({"master": opt.master, "exp_avg": opt.exp_avg, "exp_avg_sq": opt.exp_avg_sq},
                            os.path.join(s8, "optim-rank0.safetensors"),
                            {"step_count": opt.step_count, "layout": checkpoint.layout_fingerprint(ddp.space),
                             "save_step": 8})
    assert checkpoint.load(ck, ddp, opt) == 5
    assert torch.equal(opt.master, saved) and opt.step_count == json.load(open(os.path.join(ck, "meta.json")))["optimizer_step"]
    # overwriting the committed step's shard in place is detected
    s5 = os.path.join(ck, checkpoint.step_dirname(5))
    checkpoint._atomic_save({"master": opt.master, "exp_avg": opt.exp_avg, "exp_avg_sq": opt.exp_avg_sq},
                            os.path.join(s5, "optim-rank0.safetensors"),
                            {"step_count": opt.step_count, "layout": checkpoint.layout_fingerprint(ddp.space),
                             "save_step": 8})
    with pytest.raises(ValueError, match="shard does not match meta.json"):
        checkpoint.load(ck, ddp, opt)


def test_checkpoint_retention_and_legacy_v1(tmp_path):
    """Only the `keep` newest step directories survive a save; a v1 directory
    (shards beside meta.json, shards without the save_step tag) still loads."""
    import json
    from safetensors.torch import save_file
    from mxk8s.train import checkpoint
    torch.manual_seed(0)
    model = Llama(LlamaConfig.tiny())
    ddp = FlatDDP(model)
    opt = FlatAdamW(ddp.space)
    ck = str(tmp_path / "ck")
    for st in (1, 2, 3, 4):
        checkpoint.save(ck, ddp, opt, step=st, keep=2)
    assert sorted(d for d in os.listdir(ck) if d.startswith("step-")) == \
        [checkpoint.step_dirname(3), checkpoint.step_dirname(4)]
    assert checkpoint.load(ck, ddp, opt) == 4
    assert json.load(open(os.path.join(ck, "meta.json")))["history"] == \
        [checkpoint.step_dirname(3), checkpoint.step_dirname(4)]
    # uncommitted directories never count toward `keep`.  A stale,
    # HIGHER-numbered step-900 (a run that died after writing its shards) and
    # an incomplete step-200 between the commits: resuming and saving 300
    # keeps the two newest COMMITTED steps (4, 300) and drops the leftovers.
    for stale in (900, 200):
        d = os.path.join(ck, checkpoint.step_dirname(stale))
        os.makedirs(d)
        open(os.path.join(d, "optim-rank0.safetensors"), "w").close()
    checkpoint.save(ck, ddp, opt, step=300, keep=2)
    assert sorted(d for d in os.listdir(ck) if d.startswith("step-")) == \
        [checkpoint.step_dirname(4), checkpoint.step_dirname(300)]
    assert checkpoint.load(ck, ddp, opt) == 300
    # legacy v1: written by an earlier version of save()
    v1 = str(tmp_path / "v1")
    os.makedirs(v1)
    fp = checkpoint.layout_fingerprint(ddp.space)
    save_file({"params": ddp.space.param_buf.detach().clone()}, os.path.join(v1, "params.safetensors"),
              metadata={"layout": fp})
    save_file({"master": opt.master.clone(), "exp_avg": opt.exp_avg.clone(),
               "exp_avg_sq": opt.exp_avg_sq.clone()}, os.path.join(v1, "optim-rank0.safetensors"),
              metadata={"layout": fp, "step_count": str(opt.step_count)})
    json.dump({"step": 7, "optimizer_step": opt.step_count, "world_size": 1, "sharded": False,
               "layout": fp, "numel": ddp.space.numel, "format": "mxk8s-flat-v1"},
              open(os.path.join(v1, "meta.json"), "w"))
    assert checkpoint.load(v1, ddp, opt) == 7


def test_overlap_stages_cover_every_parameter_once():
    """The AdamW overlap plan (forward-need order) names every trainable
    parameter exactly once, and each stage's ranges stay on one side of the
    weight-decay boundary; on the CPU the overlap stays off."""
    from mxk8s.train.ddp_llama import overlap_stages
    model = Llama(LlamaConfig.tiny())
    stages = overlap_stages(model)
    ids = [id(p) for params, _ in stages for p in params]
    assert len(ids) == len(set(ids)) == len([p for p in model.parameters() if p.requires_grad])
    assert stages[0][1] is model.embed and stages[-1][1] is model.lm_head
    assert [m for _, m in stages[1:-1]] == list(model.layers)
    space = FlatParamSpace(model)
    opt = FlatAdamW(space)
    assert opt.enable_overlap(stages) is False and opt._stages is None
    merged = opt._merge_ranges([(0, 10), (64, 100), (space.n_decay, space.n_decay + 4)])
    assert all((a < space.n_decay) == (b <= space.n_decay) for a, b in merged)


def _zero8_worker(rank, world, port, outdir):
    """8 gloo ranks, bf16 tiny Llama: ZeRO-1 with the bf16 and the fp32 wire
    format, and fp32 + the all-gather overlapped with the next forward."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from mxk8s.parallel.optim import ShardedFlatAdamW
    from mxk8s.train.ddp_llama import overlap_stages
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    out = {}
    for run, (rdt, overlap, slots) in {"bf16": ("bf16", False, 3), "fp32": ("fp32", False, 3),
                                       "fp32_overlap": ("fp32", True, 3),
                                       "fp32_full": ("fp32", False, 0)}.items():
        torch.manual_seed(0)
        model = Llama(cfg).to(torch.bfloat16)
        ddp = FlatDDP(model, bucket_mb=0.05, shard_optimizer=True, reduce_dtype=rdt,
                      stage_slots=slots)
        if rdt == "fp32":
            out[run + "_staging"] = (sum(t.numel() for t in ddp._slots),
                                     max(b.end - b.start for b in ddp.buckets), len(ddp.buckets))
        opt = ShardedFlatAdamW(ddp, lr=1e-3)
        seen = {}
        if overlap:
            stages = overlap_stages(model)
            opt.enable_overlap(stages)
            # runs AFTER the optimizer's wait hook: what the module reads
            for k, (params, module) in enumerate(stages):
                module.register_forward_pre_hook(
                    lambda m, a, k=k, params=params: seen.__setitem__(
                        k, [p.detach().clone() for p in params]))
        checks = []
        for step in range(3):
            loss = model.loss(_batch(rank * 10 + step, cfg))
            if overlap and step > 0:
                opt.synchronize()       # compare the forward's view with the final gather
                checks.append(all(torch.equal(a, p.detach()) for k, (params, _) in enumerate(stages)
                                  for a, p in zip(seen[k], params)))
            loss.backward()
            ddp.finish_grad_sync()
            if step == 0:
                out[run + "_local"] = ddp.space.grad_buf.clone()
                out[run + "_shard"] = ddp.grad_shard.clone()
                out[run + "_ranges"] = [ddp.shard_range(b) for b in ddp.buckets]
            opt.step()
            ddp.zero_grad()
        opt.synchronize()
        out[run + "_params"] = ddp.space.param_buf.clone()
        out[run + "_checks"] = checks
        out[run + "_waits"] = list(opt.waits)
        out[run + "_order"] = list(opt._order)
    torch.save(out, os.path.join(outdir, f"z8_{rank}.pt"))
    dist.destroy_process_group()


def test_zero1_eight_ranks_fp32_wire_and_gather_overlap():
    """at world 8 the bucketed reduce-scatter with the fp32 wire
    format equals the exact sum of the 8 local bf16 gradients to one bf16
    rounding (the bf16 wire format rounds at every hop); the all-gather
    overlapped with the next forward never lets a module read a bucket before
    its gather finished and changes no bit of the result."""
    world = 8
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_zero8_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        z = [torch.load(os.path.join(d, f"z8_{i}.pt"), weights_only=True) for i in range(world)]
    # same initial params -> same local gradients in every run
    for r in range(world):
        assert torch.equal(z[r]["bf16_local"], z[r]["fp32_local"])
    exact = sum(z[r]["fp32_local"].double() for r in range(world))
    errs = {}
    for run in ("bf16", "fp32"):
        worst = 0.0
        for r in range(world):
            shard = z[r][run + "_shard"].double()
            so = 0
            for lo, hi in z[r][run + "_ranges"]:
                ref = exact[lo:hi]
                got = shard[so:so + hi - lo]
                so += hi - lo
                big = ref.abs() > 1e-3 * exact.abs().max()
                if big.any():
                    worst = max(worst, ((got - ref).abs()[big] / ref.abs()[big]).max().item())
        errs[run] = worst
    assert errs["fp32"] <= 2.0 ** -8, errs                 # one bf16 rounding
    assert errs["bf16"] > errs["fp32"], errs               # 7 roundings at world 8
    for r in range(world):
        assert torch.equal(z[r]["fp32_overlap_params"], z[r]["fp32_params"])   # bit-identical
        assert z[r]["fp32_overlap_checks"] and all(z[r]["fp32_overlap_checks"])
        order = z[r]["fp32_overlap_order"]
        assert sorted(order) == list(range(len(order))) and order != sorted(order)
        assert set(z[r]["fp32_overlap_waits"]) == set(order)
    for r in range(1, world):
        assert torch.equal(z[r]["fp32_params"], z[0]["fp32_params"])
    # the fp32 staging is a ring of 3 bucket-sized slots, not a
    # copy of the whole gradient space, and gives bit-identical results to
    # staging every bucket at once
    for r in range(world):
        staged, biggest, nb = z[r]["fp32_staging"]
        assert nb > 3 and staged <= 3 * biggest, z[r]["fp32_staging"]
        assert z[r]["fp32_full_staging"][0] == nb * biggest
        assert torch.equal(z[r]["fp32_shard"], z[r]["fp32_full_shard"])
        assert torch.equal(z[r]["fp32_params"], z[r]["fp32_full_params"])


def _allreduce_fp32_worker(rank, world, port, outdir):
    """Replicated (all-reduce) fp32 wire format through the 3-slot ring vs
    every bucket staged at once, bf16 tiny Llama, 4 gloo ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    out = {}
    for slots in (3, 0):
        torch.manual_seed(0)
        model = Llama(cfg).to(torch.bfloat16)
        ddp = FlatDDP(model, bucket_mb=0.05, reduce_dtype="fp32", stage_slots=slots)
        with ddp.no_sync():          # the local gradients (the ring rounds results
            model.loss(_batch(rank * 10, cfg)).backward()    # back during backward)
        local = ddp.space.grad_buf.clone()
        ddp.zero_grad()
        model.loss(_batch(rank * 10, cfg)).backward()
        ddp.finish_grad_sync()
        out[slots] = (local, ddp.space.grad_buf.clone(), sum(t.numel() for t in ddp._slots),
                      max(b.end - b.start for b in ddp.buckets), len(ddp.buckets))
    torch.save(out, os.path.join(outdir, f"ar{rank}.pt"))
    dist.destroy_process_group()


def test_allreduce_fp32_wire_ring_staging():
    world = 4
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_allreduce_fp32_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        z = [torch.load(os.path.join(d, f"ar{i}.pt"), weights_only=True) for i in range(world)]
    exact = sum(z[r][3][0].double() for r in range(world))
    for r in range(world):
        local, reduced, staged, biggest, nb = z[r][3]
        assert nb > 3 and staged <= 3 * biggest
        assert torch.equal(reduced, z[r][0][1])                      # ring == all at once
        assert torch.equal(reduced, z[0][3][1])                      # every rank agrees
        big = exact.abs() > 1e-3 * exact.abs().max()
        rel = ((reduced.double() - exact).abs()[big] / exact.abs()[big]).max().item()
        assert rel <= 2.0 ** -8, rel                                 # one bf16 rounding


def _frozen_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = torch.nn.Linear(4, 4).to(torch.bfloat16)
    for p in m.parameters():
        p.requires_grad_(False)
    try:
        FlatDDP(m, reduce_dtype="fp32", stage_slots=3)
        msg = "constructed"
    except ValueError as e:                 # a clear error, not a max() of an empty list
        msg = str(e)
    torch.save({"msg": msg}, os.path.join(outdir, f"f{rank}.pt"))
    dist.destroy_process_group()


def test_fp32_wire_without_trainable_params():
    """no trainable parameters means no buckets; the fp32 staging
    ring must not be sized from the empty list (a clear ValueError instead)."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_frozen_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        z = [torch.load(os.path.join(d, f"f{i}.pt"), weights_only=True) for i in range(world)]
    assert all("no trainable parameters" in r["msg"] for r in z), z
