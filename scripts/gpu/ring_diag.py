"""Diagnose a wrong GEMM variant on one 256x256 tile: where the bad outputs
are (16x16 block, lane row/col) and whether the error matches a missing or
repeated k-step (32-deep) contribution."""
import sys

import torch

from mxk8s.ops import _lib

L = _lib.lib()
dev = torch.device("cuda", 0)
v = int(sys.argv[1])
for K in (32, 64, 96, 128):
    M = N = 256
    g = torch.Generator(device=dev)
    g.manual_seed(7 + K)
    A = (torch.rand((M, K), device=dev, generator=g) * 2 - 1).bfloat16()
    B = (torch.rand((N, K), device=dev, generator=g) * 2 - 1).bfloat16()
    ref = A.float() @ B.float().t()
    C = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    st = L.mxk_gemm_bf16_tn_variant(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, K, N, v,
                                    _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    err = C.float() - ref
    bad = err.abs() > 0.05 + 2 ** -7 * ref.abs().max().item()
    nb = int(bad.sum())
    print(f"K={K} status {st} bad {nb}", flush=True)
    if not nb:
        continue
    blk = bad.view(16, 16, 16, 16).sum(dim=(1, 3))      # [row block][col block]
    nzb = blk.nonzero().tolist()
    print("  bad 16x16 blocks (rb, cb, count):", [(r, c, int(blk[r, c])) for r, c in nzb[:24]],
          "n blocks", len(nzb))
    rr = bad.view(16, 16, 256).sum(dim=(0, 2)).tolist()
    cc = bad.view(256, 16, 16).sum(dim=(0, 1)).tolist()
    print("  by row%16:", [int(x) for x in rr])
    print("  by col%16:", [int(x) for x in cc])
    steps = [A[:, 32 * s:32 * s + 32].float() @ B[:, 32 * s:32 * s + 32].float().t()
             for s in range(K // 32)]
    e = err[bad]
    for s, cs in enumerate(steps):
        for sign in (-1, 1):
            d = (e - sign * cs[bad]).abs().max().item()
            print(f"  err vs {'+' if sign > 0 else '-'}step{s}: max |err - ({sign})*C_s| = {d:.3g}")
    print("  C nan:", int(torch.isnan(C.float()).sum()), flush=True)
