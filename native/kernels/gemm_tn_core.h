// Shared core of the bf16 TN MFMA GEMM (gemm_bf16.hip): tile constants, the
// LDS-DMA panel descriptor, the table-driven three-barrier K-tile at
// hipBLASLt's gfx950 instruction positions (mx_common.h SchedHB) and the
// production kernel built on it.  The experiments-only schedules
// (experiments/gemm_tn_exp.hip) include this header too.
#pragma once
#include <type_traits>

#include "mx_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int W4_THREADS = 256;
constexpr int W4B_OP_BYTES = 256 * 128;            // 32 KiB per operand per stage
constexpr int W4B_STAGE_BYTES = 2 * W4B_OP_BYTES;  // 64 KiB (A + B), two stages

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ bf16x8_t lds_read_b128(const char* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// The accumulators live in AGPRs for the whole kernel (256 of them per lane);
// left to the builtin, the compiler's allocation shuffles them through VGPRs.
// A chain of MFMAs accumulating into the same registers needs no wait states;
// mxk::mfma_drain() must separate the last MFMA from any read of the result.
__device__ __forceinline__ void mfma_16x16x32_agpr(f32x4_t& acc, bf16x8_t a, bf16x8_t b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N == 0 || N == 13 || N == 14 || N == 15 || N == 16 || N == 22 || N == 30,
                "vm_wait: add the count");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  else if constexpr (N == 22) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
  else if constexpr (N == 30) asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
}

using mxk::w4b_tile;
}  // namespace

struct DmaK {
  __amdgpu_buffer_rsrc_t rsrc;   // 256-row panel, whole K
  uint32_t voff[8];              // piece p: row-in-piece * ld * 2 + swizzled chunk + (4p + wave) * 8 rows
  __device__ __forceinline__ void issue(char* lds_op, int p, int k_bytes, int wave_s) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_op + (p * 4 + wave_s) * 1024),
                                             16, voff[p], k_bytes, 0, 0);
  }
};

__device__ __forceinline__ DmaK make_dmak(const uint16_t* src, int ld, int row0, int lane,
                                          int wave, int swm = 7) {
  DmaK d;
  const uint16_t* base = src + static_cast<size_t>(row0) * ld;
  d.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, 256 * ld * 2,
                                             0x00020000);
  const int r = lane >> 3;
  // swm 7: the full XOR swizzle; 4: only the 64-B halves swap (each 4-lane
  // group keeps an ascending 64-B source run); 0: linear (A/B variants 37/38)
  const int c = (lane & 7) ^ ((4 * (wave & 1) + (r >> 1)) & swm);
  const uint32_t lane_off = static_cast<uint32_t>(r * ld * 2 + c * 16);
#pragma unroll
  for (int p = 0; p < 8; ++p)
    d.voff[p] = lane_off + static_cast<uint32_t>((p * 4 + wave) * 8 * ld * 2);
  return d;
}

// PAR 0/1: the K-tile reads stage buffer PAR (compile-time LDS bases);
// PAR 2: runtime parity `par` (the once-per-tile tail: one instantiation per
// MODE keeps the register assignment of the unrolled loop intact — a
// runtime-parity branch between two static tails spilled ~1300 VGPRs).

using mxk::SchedHB;
using mxk::SchedTwoBarrier;

// Table-driven K-tile: S gives, per MFMA index m, the fragment reads, DMA
// pieces, waits and barriers that follow MFMA m (see w4i_ktile for MODE).
// SPLITA: A fragments 0-3 at a_base, 4-7 at a_hi (the w13 SwiGLU kernel
// rotates one wave's row blocks by 4); otherwise a_hi is unused.
// HOOK(m) runs after MFMA m (the trickle-store kernel's one C store per
// K-tile); m is a constant once the loops are unrolled.
using mxk::NoHook;

template <class S, int PAR, int MODE, int ORDER = 0, int PRIO = 0, bool SPLITA = false,
          class HOOK = NoHook>
__device__ __forceinline__ void w4j_ktile(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                          bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                          bf16x8_t (&f1b)[8], char* smem, int a_base, int b_base,
                                          int off_k0, int off_k1, const DmaK& dma_a,
                                          const DmaK& dma_b, int kb2, int wave_s, int par = 0,
                                          int a_hi = 0, const HOOK& hook = HOOK{}) {
  constexpr int SUB = 2048;
  auto aoff = [&](int r) { return SPLITA && r >= 4 ? a_hi + (r - 4) * SUB : a_base + r * SUB; };
  const int px = PAR == 2 ? par : PAR;
  char* X = smem + px * W4B_STAGE_BYTES;
  char* Y = smem + (px ^ 1) * W4B_STAGE_BYTES;
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int o = 0; o < 8; ++o) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int m = h * 64 + o * 8 + q;
        // ORDER 0: A fragment outer (consecutive MFMAs share srcB); 1: B outer
        const int i = ORDER ? q : o, j = ORDER ? o : q;
        if (h == 0) mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
        else mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
        hook(m);
        if (S::a1(m) >= 0) f1a[S::a1(m)] = lds_read_b128(X + aoff(S::a1(m)) + off_k1);
        if (MODE == 1 && m == S::W1) {
          hook.at(0);
          __builtin_amdgcn_s_waitcnt(0xC07F);
        }
        if (MODE == 1 && m == S::B1) {
          __builtin_amdgcn_s_barrier();
          hook.at(1);
        }
        if (MODE == 1 && S::adma(m) >= 0) dma_a.issue(X, S::adma(m), kb2, wave_s);
        if (S::b1(m) >= 0) f1b[S::b1(m)] = lds_read_b128(X + b_base + S::b1(m) * SUB + off_k1);
        if (MODE == 1 && m == S::W2) {
          hook.at(2);
          __builtin_amdgcn_s_waitcnt(0xC07F);
        }
        if (MODE == 1 && m == S::B2) {
          __builtin_amdgcn_s_barrier();
          hook.at(3);
        }
        if (MODE == 1 && S::bdma(m) >= 0)
          dma_b.issue(X + W4B_OP_BYTES, S::bdma(m), kb2, wave_s);
        if (MODE != 3 && m == S::W3) {
          if (MODE == 1) hook.at(4);
          if constexpr (MODE == 1) vm_wait<S::VM3>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (MODE != 3 && m == S::B3) {
          __builtin_amdgcn_s_barrier();
          if (MODE == 1) hook.at(5);
        }
        if (MODE != 3 && S::k0(m) >= 0) {
          const int r = S::k0(m);
          if (r < 8) f0b[r] = lds_read_b128(Y + b_base + r * SUB + off_k0);
          else f0a[r - 8] = lds_read_b128(Y + aoff(r - 8) + off_k0);
        }
      }
    }
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
}

using mxk::store_block_wide;
using mxk::store_block_narrow;

// K-tile of schedule SCHED (0: w4i knobs LATE/R1, 1: hipBLASLt positions,

// ---------------------------------------------------------------------------
// The production kernel: 256x256 tile, 4 waves, the three-barrier K-tile at
// hipBLASLt's positions (SchedHB), XCD super-block tile map (MAP 1).  EPI:
// 4 = C staged through LDS and stored as whole lines (default, schedule 26),
// 2 = non-temporal widened stores (schedule 6), 0 = 8-byte stores (schedule 1:
// C not 16-B aligned or ldc % 8 != 0).
template <int MAP, int EPI>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4j(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, M / BM, N / BN, &m0, &n0);
  const DmaK dma_a = make_dmak(A, lda, m0, lane, wave_s);
  const DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ ((frow >> 1) & 7);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = K / BK;
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_a.issue(smem, p, 0, wave_s);
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_OP_BYTES, p, 0, wave_s);
  if (ns > 1) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem + W4B_STAGE_BYTES, p, BK * 2, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p)
      dma_b.issue(smem + W4B_STAGE_BYTES + W4B_OP_BYTES, p, BK * 2, wave_s);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
  __builtin_amdgcn_s_waitcnt(0xC07F);

  // K-tiles 0 .. ns-3 carry the DMA of stage s+2 (k offset kb = (s+2)*128 B)
  int s = 0;
  int kb = 2 * BK * 2;
  for (; s + 2 <= ns - 2; s += 2) {
    w4j_ktile<SchedHB, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, kb, wave_s);
    w4j_ktile<SchedHB, 1, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, kb + BK * 2, wave_s);
    kb += 2 * BK * 2;
  }
  if (s < ns - 2) {   // s even
    w4j_ktile<SchedHB, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, kb, wave_s);
    ++s;
  }
  // the last two K-tiles (or the only one): no DMA
  if (ns >= 2) {
    w4j_ktile<SchedHB, 2, 2>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, 0, wave_s, s & 1);
    ++s;
  }
  w4j_ktile<SchedHB, 2, 3>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                        dma_b, 0, wave_s, s & 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mxk::mfma_drain(acc);

  if constexpr (EPI == 4) {
    // whole-line stores through LDS; every wave's last fragment reads retired first
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    mxk::store_block_lds<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane,
                               smem + wave_s * mxk::kStoreLdsWave);
  } else if constexpr (EPI == 1) store_block_wide<false>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
  else if constexpr (EPI == 2) store_block_wide<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
  else store_block_narrow(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
}

