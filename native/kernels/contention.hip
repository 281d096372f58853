// CU-masked streams and an HBM-streaming kernel: the 1-GPU rehearsal of
// compute / collective co-residency (BASELINE config 5 at
// amd.com/gpu=8).
//
// At n > 1 the ZeRO-1 reduce-scatter runs under the backward and the
// parameter all-gather under the next forward; RCCL's kernels then hold a
// set of CUs for as long as each collective lasts.  On one GPU the same
// pressure is produced by a copy kernel confined to k CUs with
// hipExtStreamCreateWithCUMask: its waves are resident on those CUs for the
// whole backward, so no GEMM workgroup (4 waves x 512 registers, all of a
// SIMD's register file) can be placed there, exactly as beside an RCCL
// kernel.  scripts/contention_bench.py times the training step beside it,
// with and without the GEMM planner knowing about the k CUs
// (mxk_gemm_set_reserved_cus, gemm_bf16_layouts.hip).
#include <vector>

#include "mx_common.h"

namespace {

int hw_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return 256;
  return n;
}

// 16-B copy, grid-stride, `iters` passes; every lane keeps 4 loads in flight
__global__ void __launch_bounds__(256)
mxk_hbm_stream_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst, long n16,
                      int iters) {
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (int it = 0; it < iters; ++it) {
    for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += 4 * stride) {
      u32x4_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * stride < n16) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * stride < n16) __builtin_nontemporal_store(v[u], dst + i + u * stride);
    }
  }
}

}  // namespace

// A stream whose kernels may only use CUs [first, first + n) (invert = 0) or
// every CU but those (invert = 1).  *out receives the hipStream_t.
MXK_API int mxk_stream_create_cu_masked(int first, int n, int invert, void** out) {
  const int cus = hw_cus();
  if (!out || first < 0 || n < 0 || first + n > cus) return static_cast<int>(hipErrorInvalidValue);
  std::vector<uint32_t> mask((cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) {
    const bool in = c >= first && c < first + n;
    if (in != (invert != 0)) mask[c / 32] |= 1u << (c % 32);
  }
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data());
  *out = s;
  return static_cast<int>(e);
}

// A stream on the CUs c with c % group < per_group (invert = 0) or on every
// other CU (invert = 1).  group = CUs per XCD spreads the set evenly over the
// XCDs when the mask's bit order is XCD-major (the `xcd` placement of
// scripts/contention_bench.py checks that it is: an unbalanced set makes the
// GEMMs' XCD finish last).
MXK_API int mxk_stream_create_cu_masked_groups(int per_group, int group, int invert, void** out) {
  const int cus = hw_cus();
  if (!out || group <= 0 || per_group < 0 || per_group > group || cus % group)
    return static_cast<int>(hipErrorInvalidValue);
  std::vector<uint32_t> mask((cus + 31) / 32, 0u);
  for (int c = 0; c < cus; ++c) {
    const bool in = c % group < per_group;
    if (in != (invert != 0)) mask[c / 32] |= 1u << (c % 32);
  }
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data());
  *out = s;
  return static_cast<int>(e);
}

MXK_API int mxk_stream_destroy(void* s) {
  return static_cast<int>(hipStreamDestroy(static_cast<hipStream_t>(s)));
}

// Stream `bytes` (multiple of 16) from src to dst `iters` times with nwg
// 256-thread workgroups on `stream`.
MXK_API int mxk_hbm_stream(const void* src, void* dst, long bytes, int iters, int nwg,
                           hipStream_t stream) {
  if (bytes <= 0 || bytes % 16 || iters <= 0 || nwg <= 0 ||
      reinterpret_cast<uintptr_t>(src) % 16 || reinterpret_cast<uintptr_t>(dst) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_hbm_stream_kernel, dim3(nwg), dim3(256), 0, stream,
                     static_cast<const u32x4_t*>(src), static_cast<u32x4_t*>(dst), bytes / 16, iters);
  MXK_RETURN_LAUNCH_STATUS();
}
