"""bf16 MFMA GEMM op (``native/kernels/gemm_bf16.hip``).

``gemm_bf16_tn(a, bt)`` computes ``a @ bt.T`` with ``a`` [M, K] and ``bt``
[N, K] (the nn.Linear weight layout), fp32 accumulation, bf16 output.
GPU tensors always run the hand-written CDNA4 kernel (256x256 MFMA tile when
M, N are multiples of 256 and K of 64, a bounds-checked 64x64 MFMA kernel
otherwise); CPU tensors use an fp32 PyTorch reference.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

# Split tail (mxk_gemm_bf16_ex_ws): an output whose 256^2 tiles leave the
# last round of the CUs at most half full (the Llama-3-8B wqkv / w2 weight
# gradients: 384 / 896 tiles on 256 CUs; the wo forward at micro-batch 1:
# 128 tiles) runs its tail tiles as two K halves each, for every operand
# layout including the forward's TN; MXK_SPLIT_TAIL=0 turns it off (A/B).
_USE_SPLIT_TAIL = os.environ.get("MXK_SPLIT_TAIL", "1") != "0"
_split_ws: dict = {}


def _split_workspace(device: torch.device) -> torch.Tensor:
    """fp32 partial-tile workspace of the split tail, one per (device,
    stream): GEMMs on one stream run in order, so they can share it; two
    streams must not (their GEMMs may overlap)."""
    key = (device, _lib.stream_ptr(device))
    ws = _split_ws.get(key)
    if ws is None:
        n = int(_lib.lib().mxk_gemm_bf16_split_workspace())
        ws = _split_ws[key] = torch.empty(n, dtype=torch.uint8, device=device)
    return ws


def _check_operand(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name} must be bfloat16, got {t.dtype}")
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(t.shape)}")
    if t.stride(1) != 1:
        raise ValueError(f"{name} must be K-contiguous (stride(1) == 1)")


def gemm_bf16_tn(a: torch.Tensor, bt: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _check_operand(a, "a")
    _check_operand(bt, "bt")
    M, K = a.shape
    N, K2 = bt.shape
    if K != K2:
        raise ValueError(f"K mismatch: a is {tuple(a.shape)}, bt is {tuple(bt.shape)}")
    if a.device.type == "cpu":
        ref = (a.float() @ bt.float().t()).to(torch.bfloat16)
        if out is not None:
            out.copy_(ref)
            return out
        return ref
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out")
        if tuple(out.shape) != (M, N):
            raise ValueError(f"out must be [{M}, {N}]")
    L = _lib.lib()
    st = L.mxk_gemm_bf16_tn(a.data_ptr(), bt.data_ptr(), out.data_ptr(), M, N, K,
                            a.stride(0), bt.stride(0), out.stride(0),
                            _lib.stream_ptr(a.device))
    _lib.check(st, "mxk_gemm_bf16_tn")
    return out


def is_fast_shape(M: int, N: int, K: int) -> bool:
    return M % 256 == 0 and N % 256 == 0 and K % 64 == 0


def gemm_flops(M: int, N: int, K: int) -> float:
    return 2.0 * M * N * K


def gemm_bf16_ex(a: torch.Tensor, b: torch.Tensor, a_kmajor: bool, b_kmajor: bool,
                 out: torch.Tensor, variant: int = 1) -> bool:
    """``out[M][N] = A . B`` on the layout-generic MFMA kernel
    (``native/kernels/gemm_bf16_layouts.hip``).

    ``a`` is [M, K] if ``a_kmajor`` else [K, M]; ``b`` is [N, K] if
    ``b_kmajor`` else [K, N]; all row-major with unit inner stride, bf16.
    Returns False (nothing launched) when the shape does not tile exactly
    (M, N multiples of 256, K of 64) so the caller can use the library GEMM.
    ``variant`` 1 (default) picks per layout: both K-major -> the validator's
    TN kernel, both N/M-major (weight gradients) -> the x2 schedule at
    hipBLASLt's instruction positions, mixed (dgrad) -> x2; 2 / 3 / 0 force
    x2-hipBLASLt-positions / x2 / the one-barrier x kernel (A/B)."""
    if a.dim() != 2 or b.dim() != 2 or a.stride(1) != 1 or b.stride(1) != 1 or \
            out.stride(1) != 1 or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return False
    M, K = (a.shape if a_kmajor else (a.shape[1], a.shape[0]))
    N, K2 = (b.shape if b_kmajor else (b.shape[1], b.shape[0]))
    if K != K2 or tuple(out.shape) != (M, N) or not is_fast_shape(M, N, K):
        return False
    if variant == 1 and _USE_SPLIT_TAIL:
        ws = _split_workspace(a.device)
        split = ctypes.c_int(0)
        st = _lib.lib().mxk_gemm_bf16_ex_ws(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K,
                                            a.stride(0), b.stride(0), out.stride(0),
                                            int(a_kmajor), int(b_kmajor), ws.data_ptr(), ws.numel(),
                                            ctypes.byref(split), _lib.stream_ptr(a.device))
    else:
        st = _lib.lib().mxk_gemm_bf16_ex_variant(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N,
                                                 K, a.stride(0), b.stride(0), out.stride(0),
                                                 int(a_kmajor), int(b_kmajor), int(variant),
                                                 _lib.stream_ptr(a.device))
    if st == 1:   # hipErrorInvalidValue: layout/stride limits -> library GEMM
        return False
    _lib.check(st, "mxk_gemm_bf16_ex")
    return True


# ---- planning for CUs taken by collectives ----------------
# RCCL's kernels hold some CUs for as long as a collective runs (the ZeRO-1
# reduce-scatter under the backward, the parameter all-gather under the
# forward).  The GEMM launchers size their rounds and the split tail for the
# CUs that are left once told how many are taken (mxk_gemm_set_reserved_cus;
# env MXK_GEMM_RESERVED_CUS).  scripts/contention_bench.py measures both.
XBK = 64


def split_plan(nwg: int, K: int, cus: int) -> tuple[int, int]:
    """(whole tiles, tail tiles run as K halves) for ``nwg`` 256^2 output
    tiles on ``cus`` CUs: the tail of a last round at most half full is split
    so it occupies the CUs a whole round would, instead of leaving the rest
    idle.  Mirrors ``mxk_gemm_split_plan`` (gemm_bf16_layouts.hip)."""
    tail = nwg % cus if nwg > 0 and cus > 0 else 0
    want = tail > 0 and 2 * tail <= cus and K % (2 * XBK) == 0 and K >= 16 * XBK
    return (nwg - tail, tail) if want else (nwg, 0)


def rounds(nwg: int, K: int, cus: int) -> float:
    """Chip rounds the plan takes, in whole-tile times: a split tail is one
    more round of half-depth workgroups (2 x tail <= cus of them)."""
    whole, tail = split_plan(nwg, K, cus)
    return whole // cus + 0.5 if tail else float(-(-nwg // cus))


def set_reserved_cus(n: int) -> None:
    """Tell the GEMM planner that ``n`` CUs are taken by other kernels."""
    _lib.lib().mxk_gemm_set_reserved_cus(int(n))


def available_cus() -> int:
    return int(_lib.lib().mxk_gemm_available_cus())


def set_exclusive(on: bool) -> None:
    """GEMM launches claim the whole LDS of their CU (no other kernel's
    workgroup can share a CU with a GEMM tile; mx_common.h mxk_excl_lds)."""
    _lib.lib().mxk_gemm_set_exclusive(int(bool(on)))


def exclusive() -> bool:
    return bool(_lib.lib().mxk_gemm_exclusive())


# ---- staggered rounds (gemm_bf16.hip schedule 54) --------------------------
def stagger_plan(T: int, K: int, cus: int) -> int:
    """Split tiles per XCD of the staggered-round schedule, 0 when it does not
    apply.  Mirrors ``mxk_gemm_stagger_plan`` (gemm_bf16.hip)."""
    if T <= 0 or T % 8 or cus < 16 or K % (2 * XBK) or K < 4 * XBK:
        return 0
    tx, cx = T // 8, cus // 8
    sx = cx // 2
    return sx if sx > 0 and tx >= 2 * cx else 0


def stagger_part(b: int, T: int, sx: int) -> tuple[int, int, int]:
    """(virtual tile, part, slot) of workgroup ``b``: part 0 a whole tile, 1
    the first K half of a split tile (its fp32 partial goes to ``slot``), 2
    the second half (waits for ``slot``).  Mirrors ``stagger_part``
    (gemm_tn_core.h)."""
    x, i = b & 7, b >> 3
    tx = T >> 3
    f = tx - sx
    if i < 2 * sx and i & 1:
        return x + 8 * (f + (i >> 1)), 1, x * sx + (i >> 1)
    if i < 2 * sx:
        return x + 8 * (i >> 1), 0, -1
    if i < tx:
        return x + 8 * (i - sx), 0, -1
    return x + 8 * (f + i - tx), 2, x * sx + (i - tx)


def stagger_part_xcd(b: int, T: int, cx: int) -> tuple[int, int, int]:
    """(virtual tile, part, slot) of workgroup ``b`` in the XCD-group stagger
    (schedule 57): XCDs 0-3 whole tiles, XCDs 4-7 start with cx first K halves
    and end with their second halves; part -1: an idle workgroup.  Mirrors
    ``stagger_part_xcd`` (gemm_tn_core.h)."""
    x, i = b & 7, b >> 3
    tx = T >> 3
    if x < 4:
        return (x + 8 * i, 0, -1) if i < tx else (x, -1, -1)
    if i < cx:
        return x + 8 * i, 1, (x - 4) * cx + i
    if i < tx:
        return x + 8 * i, 0, -1
    return x + 8 * (i - tx), 2, (x - 4) * cx + (i - tx)
