"""Forward v10, causal, uniform attention (q = 0): O[row][0] = mean of the
keys the kernel let in, O[row][1] = sum of weights (should be 1)."""
import torch
from mxk8s.ops import attention as A

dev = torch.device("cuda")
S = 256
q = torch.zeros(1, S, 1, 128, device=dev).bfloat16()
k = torch.randn(1, S, 1, 128, device=dev).bfloat16()
v = torch.zeros(1, S, 1, 128, device=dev)
v[0, :, 0, 0] = torch.arange(S, device=dev).float() / 64.0     # exact in bf16 up to 256/64
v[0, :, 0, 1] = 1.0
v[0, :, 0, 2:34] = (torch.arange(S, device=dev).float()[:, None] // 32 == torch.arange(32, device=dev)[None, :] % 8).float()
v = v.bfloat16()
o, lse = A.attn_fwd(q, k, v, causal=True, variant=10)
o4, _ = A.attn_fwd(q, k, v, causal=True, variant=4)
torch.cuda.synchronize()
for r in (0, 31, 32, 63, 64, 80, 95, 96, 127, 128, 160, 191, 192, 224, 255):
    print(r, "mean key", round(o[0, r, 0, 0].item() * 64, 2), "ref", round(o4[0, r, 0, 0].item() * 64, 2),
          "wsum", round(o[0, r, 0, 1].item(), 3),
          "per-32-key-block weight", [round(x, 2) for x in o[0, r, 0, 2:10].float().tolist()],
          "ref", [round(x, 2) for x in o4[0, r, 0, 2:10].float().tolist()])
