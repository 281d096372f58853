// Shared helpers for the mxk8s CDNA4 (gfx950) kernels.
//
// Everything here is written for MI355X only: 64-lane wavefronts, MFMA
// matrix cores, 160 KiB LDS per CU, 8 XCDs with private L2s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MXK_API extern "C" __attribute__((visibility("default")))

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

namespace mxk {
using u32x4 = u32x4_t;

constexpr int kWave = 64;   // CDNA wavefront width
constexpr int kXcds = 8;    // MI355X: 8 accelerator complex dies

// bf16 <-> f32 by bit manipulation (round-to-nearest-even, NaN stays NaN).
__device__ __forceinline__ float bf2f(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  // A plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 and keeps NaNs.
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
}

// Bijective XCD-aware remap of a 1-D block id: blocks b and b+8 share an
// XCD (round-robin dispatch), so give each XCD a contiguous run of logical
// work ids.  Speed-only: correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % kXcds;
  const int q = nwg / kXcds, r = nwg % kXcds;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / kXcds;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// LDS-DMA piece (16 B per lane, `buffer_load_dwordx4 ... offen lds`) issued
// through inline asm: the compiler then sees no pending LDS write, so it does
// not put an `s_waitcnt vmcnt(0)` in front of every ds_read_b64_tr_b16 (it
// cannot prove the transposed reads do not alias the DMA and serialises
// them, 2-4x slower in the layout GEMM).  Ordering is the caller's: counted
// `s_waitcnt vmcnt` + s_barrier (the compiler does not track these loads, so
// a __syncthreads() alone does NOT wait for them).  M0 is compiler-owned:
// saved and restored around the load.
__device__ __forceinline__ u32x4 make_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  u32x4 r;
  r[0] = static_cast<unsigned>(a);
  r[1] = static_cast<unsigned>(a >> 32);   // stride 0
  r[2] = bytes;                            // num_records
  r[3] = 0x00020000u;
  return r;
}
__device__ __forceinline__ void dma16(const u32x4& rsrc, const char* lds, uint32_t voff,
                                      uint32_t soff) {
  const uint32_t m = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds)));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(m), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

}  // namespace mxk

// Host-side error plumbing: every launcher returns hipError_t as int so the
// Python (ctypes) side can raise with the HIP error string.
#define MXK_RETURN_LAUNCH_STATUS() return static_cast<int>(hipGetLastError())
