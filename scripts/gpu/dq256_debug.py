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
    o, lse = A.attn_fwd(q, k, v, causal=causal)
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


for args in [(1, 64, 4, 1, False), (1, 128, 4, 1, False), (1, 256, 4, 1, False), (1, 128, 4, 1, True),
             (1, 256, 8, 2, True)]:
    run(*args)
