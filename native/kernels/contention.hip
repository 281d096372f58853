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

// 16-B copy, grid-stride, `iters` passes; every lane keeps 4 loads in flight.
// pace > 0: s_sleep 8 (512 clocks) `pace` times after every 4 x 16 B per lane,
// so a few workgroups can be held to an RCCL-like HBM rate instead of
// saturating HBM (an 8-rank ring reduce-scatter moves ~0.3-0.4 TB/s per GPU).
__global__ void __launch_bounds__(256)
mxk_hbm_stream_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst, long n16,
                      int iters, int pace) {
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
      for (int p = 0; p < pace; ++p) __builtin_amdgcn_s_sleep(8);
    }
  }
}

// Where each workgroup runs: out[2 b] = HW_ID (wave / SIMD / CU / SH / SE
// fields), out[2 b + 1] = XCC_ID.  One wave per workgroup; the wave spins
// ~spin_clocks so the workgroups of one launch are resident together.
__global__ void __launch_bounds__(64) mxk_cu_probe_kernel(int* out, int spin_clocks) {
  const int hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID, 32 bits
  const int xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
  const long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < spin_clocks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

}  // namespace

// Placement probe: nwg one-wave workgroups on `stream` (e.g. a CU-masked
// one) record their HW_ID / XCC_ID into out[2 * nwg] (scripts/cu_mask_map.py
// decodes which XCD / SE / CU each mask bit names).
MXK_API int mxk_cu_probe(void* out, int nwg, int spin_clocks, hipStream_t stream) {
  if (!out || nwg <= 0 || spin_clocks < 0) return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_cu_probe_kernel, dim3(nwg), dim3(64), 0, stream, static_cast<int*>(out),
                     spin_clocks);
  MXK_RETURN_LAUNCH_STATUS();
}

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

// A stream on exactly the CUs whose mask bits are listed in bits[0..n).
MXK_API int mxk_stream_create_cu_masked_bits(const int* bits, int n, void** out) {
  const int cus = hw_cus();
  if (!out || !bits || n <= 0) return static_cast<int>(hipErrorInvalidValue);
  std::vector<uint32_t> mask((cus + 31) / 32, 0u);
  for (int i = 0; i < n; ++i) {
    if (bits[i] < 0 || bits[i] >= cus) return static_cast<int>(hipErrorInvalidValue);
    mask[bits[i] / 32] |= 1u << (bits[i] % 32);
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
// 256-thread workgroups on `stream`, `pace` sleeps of 512 clocks per 64 B
// moved by each lane (0: as fast as the workgroups go).
MXK_API int mxk_hbm_stream_paced(const void* src, void* dst, long bytes, int iters, int nwg,
                                 int pace, hipStream_t stream) {
  if (bytes <= 0 || bytes % 16 || iters <= 0 || nwg <= 0 || pace < 0 ||
      reinterpret_cast<uintptr_t>(src) % 16 || reinterpret_cast<uintptr_t>(dst) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_hbm_stream_kernel, dim3(nwg), dim3(256), 0, stream,
                     static_cast<const u32x4_t*>(src), static_cast<u32x4_t*>(dst), bytes / 16, iters,
                     pace);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_hbm_stream(const void* src, void* dst, long bytes, int iters, int nwg,
                           hipStream_t stream) {
  return mxk_hbm_stream_paced(src, dst, bytes, iters, nwg, 0, stream);
}
