"""Time the fused SwiGLU-backward down-projection dgrad on the Llama-3-8B
shape (16k tokens, F 14336, d 4096), checked against fp32 on 512 rows.

    python scripts/gpu/swiglu_dgrad_time.py
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from mxk8s.ops import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M, F, K = 16384, 14336, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    dy = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
    w2 = ((torch.rand(K, F, device=dev, generator=g) * 2 - 1) * 0.02).bfloat16()
    gu = (torch.rand(M, 2 * F, device=dev, generator=g) * 4 - 2).bfloat16()
    dgu = torch.empty_like(gu)
    L = _lib.lib()

    def run():
        st = L.mxk_gemm_bf16_dgrad_swiglu(dy.data_ptr(), w2.data_ptr(), gu.data_ptr(), dgu.data_ptr(),
                                          M, F, K, dy.stride(0), w2.stride(0), _lib.stream_ptr(dev))
        _lib.check(st, "dgrad_swiglu")

    run()
    torch.cuda.synchronize()
    rows = slice(0, 512)
    d = dy[rows].float() @ w2.float()
    gg, uu = gu[rows, :F].float(), gu[rows, F:].float()
    s = torch.sigmoid(gg)
    ref = torch.cat([d * uu * s * (1 + gg * (1 - s)), d * gg * s], 1)
    err = (dgu[rows].float() - ref).abs().max().item()
    assert err <= 2 ** -6 * ref.abs().max().item() + 1e-3, err
    plain = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    from mxk8s.ops.gemm import gemm_bf16_ex
    fns = {"fused": run, "plain_dgrad": lambda: gemm_bf16_ex(dy, w2, True, False, plain)}
    for _ in range(5):
        for f in fns.values():
            f()
    torch.cuda.synchronize()
    ts = {k: [] for k in fns}
    for r in range(8):
        for k, f in fns.items():
            s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(10):
                f()
            e0.record()
            e0.synchronize()
            ts[k].append(s0.elapsed_time(e0) / 10)
    for k, v in ts.items():
        med = statistics.median(v)
        print(f"RESULT {k} median_ms={med:.4f} tflops={2.0 * M * F * K / med / 1e9:.1f}", flush=True)
    print(f"RESULT fused max_err={err:.3g}")


if __name__ == "__main__":
    main()
