"""Where does the variant-9 dQ kernel (attention_dq256.hip) differ from the
fp32 reference?  Calls mxk_attn_bwd_dq256 directly (any S % 64) and prints the
error by (head, 32-row tile, 32-dim block), plus the rowc pairs."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib, attention as A  # noqa: E402


def run(B, S, Hq, Hkv, causal):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    q, k, v = (torch.randn(B, S, h, 128, device=dev, generator=g).bfloat16() for h in (Hq, Hkv, Hkv))
    dout = torch.randn(B, S, Hq, 128, device=dev, generator=g).bfloat16()
    # o / lse from fp32 torch (the HIP forward needs S % 128)
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    sc = qf @ kf.transpose(-1, -2) / math.sqrt(128)
    if causal:
        sc = sc.masked_fill(torch.ones(S, S, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    lse = torch.logsumexp(sc, dim=-1).contiguous()
    o = A.attention_ref(q, k, v, causal=causal).contiguous()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    A.attention_ref(qr, kr, vr, causal=causal).backward(dout.float())
    dq = torch.full_like(q, float("nan"))
    rowc = torch.zeros(B, Hq, S, 2, device=dev)
    scale = 1 / math.sqrt(128)
    st = _lib.lib().mxk_attn_bwd_dq256(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                       dout.data_ptr(), lse.data_ptr(), dq.data_ptr(), rowc.data_ptr(),
                                       B, S, Hq, Hkv, q.stride(1), k.stride(1), v.stride(1), scale,
                                       int(causal), _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    print(f"== B{B} S{S} Hq{Hq} Hkv{Hkv} causal={causal} status={st}")
    want = qr.grad
    err = (dq.float() - want).abs()
    print("  max err", err.max().item(), "max |want|", want.abs().max().item(), "nan", torch.isnan(dq).sum().item())
    e = err.view(B, S // 32, 32, Hq, 4, 32).amax(dim=(0, 2, 5))   # [row tile, head, dim block]
    for rt in range(min(S // 32, 8)):
        print("  rows", rt * 32, " ".join(f"{x:.3f}" for x in e[rt].flatten().tolist()))
    # the error by row within a 32-row tile and by dim within a 32-dim block
    print("  by row%32", " ".join(f"{x:.2f}" for x in err.amax(dim=(0, 2, 3)).view(-1, 32).amax(0).tolist()))
    print("  by dim%32", " ".join(f"{x:.2f}" for x in err.amax(dim=(0, 1, 2)).view(4, 32).amax(0).tolist()))
    delta = (dout.float() * o.float()).sum(-1).transpose(1, 2)       # [B, Hq, S]
    print("  rowc lse err", (rowc[..., 0] + lse * math.sqrt(128)).abs().max().item(),
          "delta err", (rowc[..., 1] + delta).abs().max().item())
    # dq vs a ratio: is the wrong part a scaled copy?
    bad = err > 0.05 * max(1.0, want.abs().max().item())
    if bad.any():
        idx = bad.nonzero()[:5].tolist()
        for b_, s_, h_, d_ in idx:
            print("   ", (b_, s_, h_, d_), "got", dq[b_, s_, h_, d_].item(), "want", want[b_, s_, h_, d_].item())


def run_dbg(B, S, Hq, Hkv):
    """Non-causal: dS^T := 1 / S / dP -> dQ = scale * X @ K per head."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(6)
    q, k, v = (torch.randn(B, S, h, 128, device=dev, generator=g).bfloat16() for h in (Hq, Hkv, Hkv))
    dout = torch.randn(B, S, Hq, 128, device=dev, generator=g).bfloat16()
    o = torch.zeros_like(dout)
    lse = torch.full((B, Hq, S), 30.0, device=dev)     # P = exp(s - 30) > 0, tiny
    scale = 1 / math.sqrt(128)
    kf = k.float().repeat_interleave(Hq // Hkv, dim=2)             # [B, S, Hq, D]
    vf = v.float().repeat_interleave(Hq // Hkv, dim=2)
    sc = torch.einsum("bqhd,bkhd->bhqk", q.float(), kf)
    dp = torch.einsum("bqhd,bkhd->bhqk", dout.float(), vf)
    for mode, X in ((1, torch.ones_like(sc)), (2, sc), (3, dp)):
        Xb = X.bfloat16().float()
        want = scale * torch.einsum("bhqk,bkhd->bqhd", Xb, kf)
        dq = torch.full_like(q, float("nan"))
        rowc = torch.zeros(B, Hq, S, 2, device=dev)
        st = _lib.lib().mxk_attn_bwd_dq256_dbg(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                               dout.data_ptr(), lse.data_ptr(), dq.data_ptr(),
                                               rowc.data_ptr(), B, S, Hq, Hkv, q.stride(1), k.stride(1),
                                               v.stride(1), scale, mode, _lib.stream_ptr(dev))
        torch.cuda.synchronize()
        err = (dq.float() - want).abs()
        print(f"== dbg {mode} B{B} S{S} Hq{Hq} Hkv{Hkv} st={st} max err {err.max().item():.4f} "
              f"max|want| {want.abs().max().item():.3f} nan {torch.isnan(dq).sum().item()}")
        e = err.view(B, S // 32, 32, Hq, 4, 32).amax(dim=(0, 2, 5))
        for rt in range(min(S // 32, 8)):
            print("  rows", rt * 32, " ".join(f"{x:.3f}" for x in e[rt].flatten().tolist()))
        print("  by row%32", " ".join(f"{x:.2f}" for x in err.amax(dim=(0, 2, 3)).view(-1, 32).amax(0).tolist()))
        print("  by dim%32", " ".join(f"{x:.2f}" for x in err.amax(dim=(0, 1, 2)).view(4, 32).amax(0).tolist()))


for args in [(1, 64, 4, 1), (1, 256, 4, 1)]:
    run_dbg(*args)

for args in [(1, 64, 4, 1, False), (1, 128, 4, 1, False), (1, 256, 4, 1, False), (1, 128, 4, 1, True),
             (1, 256, 8, 2, True)]:
    run(*args)
