"""ctypes binding to the in-tree HIP kernel library ``mxk8s/_lib/libmxkernels.so``.

The kernels are plain C-ABI launchers (``native/kernels/*.hip``) that take raw
device pointers and a ``hipStream_t``.  Binding them with ctypes instead of a
torch C++ extension keeps the build to one ``hipcc`` link (seconds, no torch
headers) and lets the same ``.so`` serve the standalone validator binaries.

There is deliberately NO silent fallback for GPU tensors: if the library is
missing or a launch fails, the op raises.  CPU tensors take the PyTorch
reference path (that is what the CPU test tier exercises).
"""
from __future__ import annotations

import ctypes
import os
import threading

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")
# MXK_KERNELS_LIB points at an alternative build (A/B runs of a kernel change).
KERNEL_LIB_PATH = os.environ.get("MXK_KERNELS_LIB") or os.path.join(_LIB_DIR, "libmxkernels.so")

_lock = threading.Lock()
_lib = None

_vp = ctypes.c_void_p
_i = ctypes.c_int
_l = ctypes.c_long
_f = ctypes.c_float
_fp = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes)
_SIGNATURES = {
    "mxk_gemm_set_reserved_cus": (None, [_i]),
    "mxk_gemm_set_exclusive": (None, [_i]),
    "mxk_gemm_w13_set_sched": (None, [_i]),
    "mxk_gemm_swiglu_set_epi": (None, [_i]),
    "mxk_gemm_x2_set_order": (None, [_i]),
    "mxk_gemm_exclusive": (_i, []),
    "mxk_gemm_reserved_cus": (_i, []),
    "mxk_gemm_available_cus": (_i, []),
    "mxk_gemm_split_plan": (_i, [_l, _i, _i, ctypes.POINTER(ctypes.c_long)]),
    "mxk_gemm_stagger_plan": (_i, [_l, _i, _i]),
    "mxk_gemm_stagger_part": (None, [_i, _i, _i, ctypes.POINTER(ctypes.c_int)]),
    "mxk_gemm_stagger_part_xcd": (None, [_i, _i, _i, ctypes.POINTER(ctypes.c_int)]),
    "mxk_stream_create_cu_masked": (_i, [_i, _i, _i, ctypes.POINTER(ctypes.c_void_p)]),
    "mxk_stream_create_cu_masked_groups": (_i, [_i, _i, _i, ctypes.POINTER(ctypes.c_void_p)]),
    "mxk_stream_destroy": (_i, [_vp]),
    "mxk_hbm_stream": (_i, [_vp, _vp, _l, _i, _i, _vp]),
    "mxk_hbm_stream_paced": (_i, [_vp, _vp, _l, _i, _i, _i, _vp]),
    "mxk_cu_probe": (_i, [_vp, _i, _i, _vp]),
    "mxk_stream_create_cu_masked_bits": (_i, [ctypes.POINTER(ctypes.c_int), _i, ctypes.POINTER(ctypes.c_void_p)]),
    "mxk_gemm_bf16_tn": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp]),
    "mxk_gemm_bf16_tn_is_fast": (_i, [_i, _i, _i]),
    "mxk_gemm_bf16_ex": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "mxk_gemm_bf16_ex_variant": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "mxk_gemm_bf16_ex_ws": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _l,
                                 ctypes.POINTER(ctypes.c_int), _vp]),
    "mxk_gemm_bf16_split_workspace": (_l, []),
    "mxk_gemm_bf16_dgrad_swiglu": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "mxk_gemm_bf16_w13_swiglu": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "mxk_gemm_bf16_tn_variant": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "mxk_gemm_bf16_tn_num_variants": (_i, []),
    "mxk_gemm_bf16_tn_is_ablation": (_i, [_i]),
    "mxk_gemm_bf16_tn_variant_built": (_i, [_i]),
    "mxk_attn_fwd_variant_built": (_i, [_i]),
    "mxk_gemm_bf16_ex_variant_built": (_i, [_i]),
    "mxk_gemm_bf16_tn_variant_name": (ctypes.c_char_p, [_i]),
    "mxk_vector_add_f32": (_i, [_vp, _vp, _vp, _l, _vp]),
    "mxk_vector_add_bf16": (_i, [_vp, _vp, _vp, _l, _vp]),
    "mxk_error_string": (ctypes.c_char_p, [_i]),
    "mxk_rmsnorm_fwd": (_i, [_vp, _vp, _vp, _vp, _i, _i, _f, _vp]),
    "mxk_rmsnorm_bwd_workspace": (_l, [_i, _i]),
    "mxk_add_rmsnorm_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _f, _vp]),
    "mxk_rmsnorm_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    "mxk_swiglu_fwd": (_i, [_vp, _vp, _l, _i, _vp]),
    "mxk_swiglu_bwd": (_i, [_vp, _vp, _vp, _l, _i, _vp]),
    "mxk_rope": (_i, [_vp, _vp, _vp, _vp, _l, _i, _i, _i, _f, _vp]),
    "mxk_rope_strided": (_i, [_vp, _vp, _vp, _vp, _l, _i, _i, _i, _f, _l, _l, _vp]),
    "mxk_sumsq_partials": (_i, [_l]),
    "mxk_grad_clip_scale": (_i, [_vp, _l, _vp, _f, _f, _vp, _vp]),
    "mxk_grad_sumsq": (_i, [_vp, _l, _vp, _vp, _vp]),
    "mxk_clip_scale_from_sumsq": (_i, [_vp, _f, _f, _vp, _vp]),
    "mxk_attn_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _l, _l, _l, _f, _i, _vp]),
    "mxk_attn_fwd_variant": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _l, _l, _l, _f, _i, _i,
                                  _vp]),
    "mxk_attn_bwd_workspace": (_l, [_i, _i, _i]),
    "mxk_attn_bwd_workspace_variant": (_l, [_i, _i, _i, _i]),
    "mxk_attn_bwd_dq256": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _l, _l, _l,
                                _f, _i, _vp]),
    "mxk_attn_bwd_dq256_dbg": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _l, _l,
                                    _l, _f, _i, _vp]),
    "mxk_attn_bwd_dq256_stamps": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _l, _l,
                                       _l, _f, _vp, _vp]),
    "mxk_attn_bwd_variant": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i,
                                  _i, _l, _l, _l, _l, _l, _f, _i, _i, _vp]),
    "mxk_gemm_bf16_rope": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp]),
    "mxk_attn_bwd_rope": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i,
                               _l, _l, _l, _l, _l, _l, _vp, _vp, _f, _i, _vp]),
    "mxk_attn_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i,
                          _l, _l, _l, _l, _l, _f, _i, _vp]),
    "mxk_xent_fwd": (_i, [_vp, _vp, _vp, _vp, _l, _i, _l, _vp]),
    "mxk_xent_bwd": (_i, [_vp, _vp, _vp, _vp, _l, _i, _l, _vp]),
    "mxk_adamw_bf16": (_i, [_vp, _vp, _vp, _vp, _vp, _l, _f, _f, _f, _f, _f, _i, _vp, _vp]),
}


class KernelLibraryMissing(RuntimeError):
    pass


def kernels_available() -> bool:
    return os.path.exists(KERNEL_LIB_PATH)


def lib() -> ctypes.CDLL:
    """Load (once) and return the kernel library; raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(KERNEL_LIB_PATH):
            raise KernelLibraryMissing(
                f"{KERNEL_LIB_PATH} not built: run `make kernels` (or "
                "`python -c 'import __graft_entry__ as g; g.build()'`)")
        # torch must be loaded first so libamdhip64.so.7 is already resident and
        # our NEEDED entry binds to the same HIP runtime instance as torch.
        import torch  # noqa: F401
        handle = ctypes.CDLL(KERNEL_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().mxk_error_string(status)
        raise RuntimeError(f"{what} failed: hip error {status} ({msg.decode() if msg else '?'})")


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
