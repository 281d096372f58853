"""Forward variant 10 debug: where do wrong / NaN rows appear (small shapes)."""
import torch
from mxk8s.ops import attention as A

dev = torch.device("cuda")
for causal in (False, True):
    for S in (256, 512):
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(1, S, 1, 128, device=dev, generator=g).bfloat16()
        k = torch.randn(1, S, 1, 128, device=dev, generator=g).bfloat16()
        v = torch.randn(1, S, 1, 128, device=dev, generator=g).bfloat16()
        o, lse = A.attn_fwd(q, k, v, causal=causal, variant=10)
        o4, lse4 = A.attn_fwd(q, k, v, causal=causal, variant=4)
        torch.cuda.synchronize()
        bad = (o.float() - o4.float()).abs().amax(dim=-1)[0, :, 0]
        nan_rows = torch.isnan(o.float()).any(-1)[0, :, 0].nonzero().flatten().tolist()
        lse_d = (lse - lse4).abs()[0, 0]
        print(f"causal={causal} S={S} max|o-o4|={bad.nan_to_num(1e9).max().item():.4g} "
              f"nan rows={nan_rows[:8]}{'...' if len(nan_rows) > 8 else ''} n_nan={len(nan_rows)} "
              f"max|lse-lse4|={lse_d.nan_to_num(1e9).max().item():.4g}")
        rows = (bad.nan_to_num(1e9) > 1e-2).nonzero().flatten().tolist()
        print("   bad rows:", rows[:16], "count", len(rows))
        print("   lse[0:4]", lse[0, 0, :4].tolist(), "ref", lse4[0, 0, :4].tolist())

# detail: causal S = 256, rows 64.. (wave 1, group 0)
g = torch.Generator(device=dev).manual_seed(0)
S = 256
q = torch.randn(1, S, 1, 128, device=dev, generator=g).bfloat16()
k = torch.randn(1, S, 1, 128, device=dev, generator=g).bfloat16()
v = torch.randn(1, S, 1, 128, device=dev, generator=g).bfloat16()
o, lse = A.attn_fwd(q, k, v, causal=True, variant=10)
o4, lse4 = A.attn_fwd(q, k, v, causal=True, variant=4)
for r in (31, 32, 63, 64, 65, 95, 96, 128, 200, 255):
    print(r, "lse", round(lse[0, 0, r].item(), 4), round(lse4[0, 0, r].item(), 4),
          "o", [round(x, 3) for x in o[0, r, 0, :4].float().tolist()],
          [round(x, 3) for x in o4[0, r, 0, :4].float().tolist()])
