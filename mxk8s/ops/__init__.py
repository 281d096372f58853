"""Hand-written CDNA4 (gfx950) HIP kernels exposed as torch ops.

* :func:`gemm_bf16_tn`  — bf16 MFMA GEMM (validator config 3)
* :func:`vector_add`    — smoke-test payload (config 2)
* :func:`rmsnorm`, :func:`swiglu`, :func:`rope` — fused training ops (config 5)
"""
from .gemm import gemm_bf16_tn, gemm_flops, is_fast_shape
from .vector_add import vector_add
from .fused import rmsnorm, swiglu, rope, rope_tables
from ._lib import kernels_available, KERNEL_LIB_PATH

__all__ = ["gemm_bf16_tn", "gemm_flops", "is_fast_shape", "vector_add", "rmsnorm", "swiglu",
           "rope", "rope_tables", "kernels_available", "KERNEL_LIB_PATH"]
