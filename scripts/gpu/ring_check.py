"""Correctness sweep of the GEMM schedule variants over K (catches prologue /
tail bugs that one large K hides): max |C - fp32| per (variant, M, N, K)."""
import sys

import torch

from mxk8s.ops import _lib

L = _lib.lib()
dev = torch.device("cuda", 0)
variants = [int(v) for v in sys.argv[1].split(",")]
shapes = [(256, 256, k) for k in (64, 128, 192, 256, 320, 384, 448, 512)] + \
         [(4096, 4096, 4096), (4608, 4608, 2048), (16384, 6144, 4096), (8192, 8192, 8192)]
ok_all = True
for M, N, K in shapes:
    g = torch.Generator(device=dev)
    g.manual_seed(M + N + K)
    A = (torch.rand((M, K), device=dev, generator=g) * 2 - 1).bfloat16()
    B = (torch.rand((N, K), device=dev, generator=g) * 2 - 1).bfloat16()
    ref = A.float() @ B.float().t()
    tol = 2 ** -7 * ref.abs().max().item() + 1e-3
    for v in variants:
        C = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        st = L.mxk_gemm_bf16_tn_variant(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, K, N,
                                        v, _lib.stream_ptr(dev))
        torch.cuda.synchronize()
        err = (C.float() - ref).abs()
        e = err.max().item()
        bad = int((err > tol).sum().item())
        ok = st == 0 and e <= tol
        ok_all &= ok
        where = ""
        if not ok and bad:
            nz = (err > tol).nonzero()
            idx = nz[:4].tolist()
            r, c = nz[:, 0], nz[:, 1]
            where = (f" first bad (row,col) {idx} rows [{int(r.min())}, {int(r.max())}]"
                     f" cols [{int(c.min())}, {int(c.max())}] distinct tiles "
                     f"{sorted(set((int(a) // 256, int(b) // 256) for a, b in nz[::97].tolist()))[:8]}"
                     f" rows%128 {sorted(set((r % 128).tolist()))[:40]}")
        print(f"v{v} {M}x{N}x{K}: status {st} max_err {e:.4g} tol {tol:.3g} bad {bad}{where}",
              flush=True)
print("ALL OK" if ok_all else "FAILURES", flush=True)
sys.exit(0 if ok_all else 1)
