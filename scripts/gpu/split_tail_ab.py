"""A/B of the layout GEMM's split tail on the Llama-3-8B weight-gradient
shapes whose tile count leaves the last round half empty (16k tokens):
split tail on / off (same process, interleaved blocks of back-to-back
launches, median over blocks) and hipBLASLt on the same operands.

    python scripts/gpu/split_tail_ab.py
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from mxk8s.ops import gemm  # noqa: E402

SHAPES = [  # (name, M, N, K): dW [M][N] = dy^T [M][K] . x [K][N]
    ("wqkv_wgrad", 6144, 4096, 16384),
    ("w2_wgrad", 4096, 14336, 16384),
    ("wo_wgrad", 4096, 4096, 16384),      # 256 tiles: no tail (control)
]


def block(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K in SHAPES:
        a = (torch.rand(K, M, device=dev, generator=g) * 2 - 1).bfloat16()
        b = (torch.rand(K, N, device=dev, generator=g) * 2 - 1).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = a.float().t() @ b.float()

        def run(split):
            def f():
                gemm._USE_SPLIT_TAIL = split
                assert gemm.gemm_bf16_ex(a, b, False, False, out)
            return f
        fns = {"split": run(True), "nosplit": run(False),
               "hipblaslt": lambda: torch.matmul(a.t(), b, out=out)}
        for k, f in fns.items():
            out.zero_()
            f()
            torch.cuda.synchronize()
            err = (out.float() - ref).abs().max().item()
            assert err <= 2 ** -7 * ref.abs().max().item() + 1e-3, (name, k, err)
        del ref
        for _ in range(3):
            for f in fns.values():
                block(f, 5)
        ts = {k: [] for k in fns}
        for r in range(8):
            order = list(fns) if r % 2 == 0 else list(reversed(list(fns)))
            for k in order:
                ts[k].append(block(fns[k], 10))
        fl = 2.0 * M * N * K
        med = {k: statistics.median(v) for k, v in ts.items()}
        print(f"RESULT {name} M={M} N={N} K={K} tiles={(M // 256) * (N // 256)} " +
              " ".join(f"{k}={med[k] * 1e3:.1f}us/{fl / med[k] / 1e9:.0f}TF" for k in fns), flush=True)
        gemm._USE_SPLIT_TAIL = True


if __name__ == "__main__":
    main()
