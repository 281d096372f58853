"""GPU numerics of the training path: fused flat AdamW + grad-norm kernels vs
the torch reference path, and a tiny Llama fwd/bwd through the HIP ops vs the
same model in fp32 on the CPU."""
import pytest
import torch

from mxk8s.models.llama import Llama, LlamaConfig
from mxk8s.parallel.ddp import FlatParamSpace
from mxk8s.parallel.optim import FlatAdamW

pytestmark = pytest.mark.gpu


def test_flat_adamw_kernel_vs_reference(cuda_device):
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(300, 520), torch.nn.LayerNorm(520),
                                torch.nn.Linear(520, 77)).to(torch.bfloat16)
    cpu_model = torch.nn.Sequential(torch.nn.Linear(300, 520), torch.nn.LayerNorm(520),
                                    torch.nn.Linear(520, 77)).to(torch.bfloat16)
    cpu_model.load_state_dict(model.state_dict())
    gpu_space = FlatParamSpace(model.to(cuda_device))
    cpu_space = FlatParamSpace(cpu_model)
    kw = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=0.5,
              grad_scale=0.25)
    go, co = FlatAdamW(gpu_space, **kw), FlatAdamW(cpu_space, **kw)
    g = torch.Generator().manual_seed(3)
    for step in range(4):
        grad = (torch.randn(cpu_space.numel, generator=g) * 0.3).to(torch.bfloat16)
        cpu_space.grad_buf.copy_(grad)
        gpu_space.grad_buf.copy_(grad.to(cuda_device))
        go.step()
        co.step()
        torch.cuda.synchronize()
        assert abs(float(go.last_grad_norm) - float(co.last_grad_norm)) <= 1e-3 * float(co.last_grad_norm)
        assert torch.allclose(go.master.cpu(), co.master, rtol=1e-5, atol=1e-6)
        assert torch.allclose(go.exp_avg_sq.cpu(), co.exp_avg_sq, rtol=1e-4, atol=1e-10)
        assert torch.equal(gpu_space.param_buf.cpu(), cpu_space.param_buf) or \
            (gpu_space.param_buf.cpu().float() - cpu_space.param_buf.float()).abs().max() <= 2 ** -7


def test_tiny_llama_gpu_matches_cpu_fp32(cuda_device):
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    ref = Llama(cfg)                      # fp32 CPU reference (pure torch ops)
    gpu = Llama(cfg)
    gpu.load_state_dict(ref.state_dict())
    gpu = gpu.to(cuda_device, torch.bfloat16)
    tok = torch.randint(0, cfg.vocab_size, (2, 129))   # S = 128: HIP attention path
    lr = ref.loss(tok)
    lg = gpu.loss(tok.to(cuda_device))
    assert abs(lr.item() - lg.item()) < 0.05, (lr.item(), lg.item())
    lr.backward()
    lg.backward()
    for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
        a, b = pr.grad.float(), pg.grad.float().cpu()
        rel = ((a - b).norm() / (a.norm() + 1e-12)).item()
        assert rel < 0.08, (n, rel)


def test_ddp_bench_tiny_single_gpu(cuda_device):
    import types
    from mxk8s.train.ddp_llama import run_ddp_bench
    a = types.SimpleNamespace(steps=3, warmup=1, seq_len=128, micro_batch=2, layers=None,
                              tiny=True, bucket_mb=1.0)
    out = run_ddp_bench(a)
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert out["mean_loss"] == out["mean_loss"]   # not NaN


def test_sharded_clip_kernels_vs_torch(cuda_device):
    """ZeRO-1 clip path: per-shard sum of squares + scale from the global sum."""
    from mxk8s.ops import _lib
    L = _lib.lib()
    g = torch.Generator(device=cuda_device).manual_seed(5)
    for n in (8, 1000, 3 * 2 ** 20 + 24):
        grad = (torch.randn(n, device=cuda_device, generator=g) * 0.7).bfloat16()
        parts = torch.zeros(L.mxk_sumsq_partials(n), device=cuda_device)
        sumsq = torch.zeros(1, device=cuda_device)
        _lib.check(L.mxk_grad_sumsq(grad.data_ptr(), n, parts.data_ptr(), sumsq.data_ptr(),
                                    _lib.stream_ptr(cuda_device)), "sumsq")
        ref = grad.float().pow(2).sum()
        assert torch.allclose(sumsq[0], ref, rtol=1e-4)
        out = torch.zeros(2, device=cuda_device)
        world, max_norm = 4, 1.0
        _lib.check(L.mxk_clip_scale_from_sumsq(sumsq.data_ptr(), 1.0 / world, max_norm,
                                               out.data_ptr(), _lib.stream_ptr(cuda_device)), "clip")
        norm = ref.sqrt().item() / world
        clip = max_norm / (norm + 1e-6) if norm > max_norm else 1.0
        assert abs(out[1].item() - norm) <= 1e-4 * norm
        assert abs(out[0].item() - clip / world) <= 1e-4 * clip / world


def test_overlapped_adamw_bit_identical(cuda_device):
    """FlatAdamW.enable_overlap (AdamW on a side stream, each block's forward
    waits for its own stage) gives bit-identical parameters, moments and
    losses to the serial step, and covers every parameter."""
    from mxk8s.train.ddp_llama import build, train_step
    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab_size, (2, 129), device=cuda_device,
                        generator=torch.Generator(device=cuda_device).manual_seed(1))
    runs = []
    for overlap in (False, True):
        torch.manual_seed(0)
        model, ddp, opt = build(cfg, cuda_device, bucket_mb=1.0, overlap=overlap)
        assert (opt._stages is not None) == overlap
        losses = [train_step(model, ddp, opt, tok) for _ in range(4)]
        opt_sync = getattr(opt, "synchronize", None)
        if opt_sync:
            opt_sync()
        torch.cuda.synchronize()
        runs.append((torch.stack(losses).cpu(), ddp.space.param_buf.clone(), opt.exp_avg.clone(),
                     opt.exp_avg_sq.clone(), opt.master.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
