"""Same-box A/B of the Llama-3-8B DDP step (bench.py --mode ddp) against
variants that exist only here, as monkeypatches (the package itself has one
path per op):

  current        the package as shipped
  hipblaslt_fwd  forward GEMMs through torch.matmul (hipBLASLt), as in round 2
  unfused_w13    the MLP up-projection as GEMM + separate SwiGLU kernel

usage: python scripts/gpu/ddp_ab.py VARIANT [bench.py ddp args...]
Run each variant in its own process (the 8B model + AdamW state is ~197 GiB).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import bench  # noqa: E402
from mxk8s.ops import linear  # noqa: E402


def _torch_fwd(x, weight):
    return torch.matmul(x, weight.t())


def main() -> int:
    variant = sys.argv[1]
    if variant == "hipblaslt_fwd":
        linear._fwd = _torch_fwd
        linear._USE_FUSED_W13 = False
    elif variant == "unfused_w13":
        linear._USE_FUSED_W13 = False
    elif variant != "current":
        raise SystemExit(f"unknown variant {variant}")
    print(f"ddp_ab variant={variant}", flush=True)
    return bench.main(["--mode", "ddp"] + sys.argv[2:])


if __name__ == "__main__":
    sys.exit(main())
