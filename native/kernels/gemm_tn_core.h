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
using mxk::StaggerPart;
using mxk::stagger_part_xcd;

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

using mxk::SchedHB;
using mxk::SchedTwoBarrier;

// Table-driven K-tile: S gives, per MFMA index m, the fragment reads, DMA
// pieces, waits and barriers that follow MFMA m.  MODE 1: DMA of stage s+2,
// counted vmcnt at the stage wait; MODE 2: no DMA, vmcnt(0) (stage s+1 is
// the last one issued); MODE 3: no DMA, no stage wait, no next-k0 reads (the
// last K-tile).  PAR 0/1: the K-tile reads stage buffer PAR (compile-time LDS
// bases); PAR 2: runtime parity `par` (the once-per-tile tail: one
// instantiation per MODE keeps the register assignment of the unrolled loop
// intact — a runtime-parity branch between two static tails spilled ~1300
// VGPRs).
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

// ---------------------------------------------------------------------------
// The production kernel: 256x256 tile, 4 waves, the three-barrier K-tile at
// hipBLASLt's positions (SchedHB), XCD super-block tile map (MAP 1).  EPI:
// 4 = C staged through LDS and stored as whole lines (default, schedule 26),
// 2 = non-temporal widened stores (schedule 6), 0 = 8-byte stores (schedule 1:
// C not 16-B aligned or ldc % 8 != 0).
// The K loop of one 256x256 tile over ns K-tiles (A / Bt at the first k of
// the range, rows m0 / n0): prologue DMA of stages 0 and 1, the unrolled
// three-barrier K-tiles, the two DMA-free tail K-tiles and the MFMA drain.
// INIT: the accumulators start from init[(i * 8 + j) * 64] (this lane's fp32
// partial of acc[i][j], the staggered schedule's first K half) instead of 0.
// ---- L2 prefetch (schedule 56) ---------------------------------------------
// With the operands HBM-cold (a training step: every GEMM reads activations
// another kernel just wrote and weights nothing has touched since the last
// step) the three-barrier K-tile's last B piece has ~0.75 K-tile (~0.9 us)
// before its wait, about one HBM miss under load: 16384x4096x4096 runs 3.4 %
// and 16384x6144x4096 4.7 % slower cold than cache-warm, hipBLASLt 1.4-1.8 %
// (profiles/r4_gemm/cold_vs_warm.log).  Each K-tile therefore also pulls
// stage s+4 into L2 with one dword per 128-B line (buffer_load_dword ... lds
// into a 1 KiB LDS sink nobody reads: no VGPR is written, so no register
// hazard), issued after stage s+2's last piece: it is older than stage s+3,
// so K-tile s+2's stage wait covers it (~1.75 K-tiles of lead) and stage
// s+4's real DMA in K-tile s+2 hits L2.  The 32 workgroups of an XCD's
// 8 x 4 sub-block share 8 A and 4 B panels: waves 0-1 take a quarter of the
// workgroup's A panel (by its sub-block column), waves 2-3 an eighth of its B
// panel (by its row), so each line is pulled about once per XCD.
constexpr int kPfSink = 2 * W4B_STAGE_BYTES;      // LDS byte offset of the sink
constexpr int kPfLds = kPfSink + 4 * 256;         // LDS bytes of a prefetching kernel

struct SchedHBPf : SchedHB {
  static constexpr int PF = 125;                 // after stage s+2's last piece (m 124)
  static constexpr int VM3 = SchedHB::VM3 + 1;   // the previous K-tile's prefetch is younger
};

struct L2Prefetch : NoHook {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff;
  char* sink;
  int kb;
  __device__ __forceinline__ void operator()(int m) const {
    if (m == SchedHBPf::PF)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)sink, 4, voff, kb, 0, 0);
  }
};

__device__ __forceinline__ L2Prefetch make_l2pf(const DmaK& dma_a, const DmaK& dma_b, int lda,
                                                int ldb, char* smem, int lane, int wave_s) {
  const int pos = (blockIdx.x >> 3) & 31;         // MAP 1 sub-block position
  L2Prefetch h;
  if (wave_s < 2) {   // A rows [64 (pos >> 3) + 32 wave, +32): lanes 32..63 repeat 0..31
    h.rsrc = dma_a.rsrc;
    h.voff = static_cast<uint32_t>((64 * (pos >> 3) + 32 * wave_s + (lane & 31)) * lda * 2);
  } else {            // B rows [32 (pos & 7) + 16 (wave - 2), +16)
    h.rsrc = dma_b.rsrc;
    h.voff = static_cast<uint32_t>((32 * (pos & 7) + 16 * (wave_s - 2) + (lane & 15)) * ldb * 2);
  }
  h.sink = smem + kPfSink + wave_s * 256;
  h.kb = 0;
  return h;
}

template <bool INIT = false, bool PF = false>
__device__ __forceinline__ void w4j_mainloop(f32x4_t (&acc)[8][8], char* smem,
                                             const uint16_t* __restrict__ A,
                                             const uint16_t* __restrict__ Bt, int lda, int ldb,
                                             int m0, int n0, int ns, int lane, int wave_s,
                                             const f32x4_t* init = nullptr) {
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  const DmaK dma_a = make_dmak(A, lda, m0, lane, wave_s);
  const DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ ((frow >> 1) & 7);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (INIT) acc[i][j] = init[(i * 8 + j) * 64];
      else acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  if constexpr (INIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // before the counted DMA waits

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
  if constexpr (PF) {
    // stage s+4's lines into L2; past the last stage the last one again (an
    // L2 hit), so every K-tile issues the same number of vector-memory ops
    L2Prefetch pf = make_l2pf(dma_a, dma_b, lda, ldb, smem, lane, wave_s);
    const int kb_last = (ns - 1) * BK * 2;
    for (; s + 2 <= ns - 2; s += 2) {
      pf.kb = min(kb + 2 * BK * 2, kb_last);
      w4j_ktile<SchedHBPf, 0, 1, 0, 0, false, L2Prefetch>(acc, f0a, f0b, f1a, f1b, smem, a_base,
                                                          b_base, off_k0, off_k1, dma_a, dma_b, kb,
                                                          wave_s, 0, 0, pf);
      pf.kb = min(kb + 3 * BK * 2, kb_last);
      w4j_ktile<SchedHBPf, 1, 1, 0, 0, false, L2Prefetch>(acc, f0a, f0b, f1a, f1b, smem, a_base,
                                                          b_base, off_k0, off_k1, dma_a, dma_b,
                                                          kb + BK * 2, wave_s, 0, 0, pf);
      kb += 2 * BK * 2;
    }
    if (s < ns - 2) {   // s even
      pf.kb = min(kb + 2 * BK * 2, kb_last);
      w4j_ktile<SchedHBPf, 0, 1, 0, 0, false, L2Prefetch>(acc, f0a, f0b, f1a, f1b, smem, a_base,
                                                          b_base, off_k0, off_k1, dma_a, dma_b, kb,
                                                          wave_s, 0, 0, pf);
      ++s;
    }
  } else {
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
}

template <int EPI>
__device__ __forceinline__ void w4j_epilogue(f32x4_t (&acc)[8][8], char* smem,
                                             uint16_t* __restrict__ C, int ldc, int m0, int n0,
                                             int lane, int wave_s) {
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
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

template <int MAP, int EPI, bool PF = false>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4j(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[PF ? kPfLds : 2 * W4B_STAGE_BYTES];
  const int lane = threadIdx.x & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, M / BM, N / BN, &m0, &n0);
  f32x4_t acc[8][8];
  w4j_mainloop<false, PF>(acc, smem, A, Bt, lda, ldb, m0, n0, K / BK, lane, wave_s);
  w4j_epilogue<EPI>(acc, smem, C, ldc, m0, n0, lane, wave_s);
}

// ---------------------------------------------------------------------------
// Staggered rounds (schedule 54).  With T tiles over the CUs in whole rounds,
// every CU finishes its tile at the same moment and all of them store their
// C tiles at once: a 32 MB burst per round at 8192^3 (three times that for
// the SwiGLU epilogues) that HBM drains while the matrix cores idle.  Here
// half the CUs of every XCD start with HALF a tile: tiles are split into K
// halves for sx tiles per XCD; the first halves run in the first wave of
// workgroups (alternating with whole tiles), so those CUs run half a tile
// out of phase for the whole kernel, and the second halves run last, where
// the first-half CUs free up half a tile early.  A first half leaves its
// fp32 partial in ws (uncached memory) and raises flags[slot]; the matching
// second half (dispatched later on the same XCD, so the wait cannot
// deadlock) waits for the flag, adds the partial and stores the tile.
// Workgroup b runs on XCD b % 8; its local index i = b / 8 on that XCD:
//   i < 2 sx, even   whole tile i / 2
//   i < 2 sx, odd    first K half of split tile i / 2 (slot x sx + i / 2)
//   2 sx <= i < tx   whole tile i - sx
//   tx <= i          second K half of split tile i - tx
// (tx = T / 8 tiles per XCD; the split tiles are the XCD's last sx tiles of
// the map).  Virtual tile v = x + 8 * (local tile) keeps the map's XCD.
__host__ __device__ inline StaggerPart stagger_part(int b, int T, int sx) {
  const int x = b & 7, i = b >> 3;
  const int tx = T >> 3, f = tx - sx;
  StaggerPart r;
  if (i < 2 * sx && (i & 1)) {
    r.part = 1; r.slot = x * sx + (i >> 1); r.vtile = x + 8 * (f + (i >> 1));
  } else if (i < 2 * sx) {
    r.part = 0; r.slot = -1; r.vtile = x + 8 * (i >> 1);
  } else if (i < tx) {
    r.part = 0; r.slot = -1; r.vtile = x + 8 * (i - sx);
  } else {
    r.part = 2; r.slot = x * sx + (i - tx); r.vtile = x + 8 * (f + i - tx);
  }
  return r;
}

// fp32 partial of one tile in accumulator order: wave w's acc[i][j] of lane l
// at float4 index ((w * 64 + i * 8 + j) * 64 + l) of the slot (256 KiB)
__device__ __forceinline__ void partial_store(const f32x4_t (&acc)[8][8], float* ws, int slot,
                                              int wave_s, int lane) {
  f32x4_t* p = reinterpret_cast<f32x4_t*>(ws) + (static_cast<size_t>(slot) * 4 + wave_s) * 4096 + lane;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) p[(i * 8 + j) * 64] = acc[i][j];
}

// STYLE 0: stagger_part (per CU, sx split tiles per XCD); 1: stagger_part_xcd
// (sx = CUs per XCD).
template <int MAP, int EPI, int STYLE = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4j_stag(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                          uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc,
                          float* __restrict__ ws, int* __restrict__ flags, int sx) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int lane = threadIdx.x & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int T = (M / BM) * (N / BN);
  const StaggerPart sp = STYLE ? stagger_part_xcd(blockIdx.x, T, sx) : stagger_part(blockIdx.x, T, sx);
  if (sp.part < 0) return;
  int m0, n0;
  w4b_tile<MAP>(sp.vtile, T, M / BM, N / BN, &m0, &n0);
  const int ns = sp.part ? (K / BK) >> 1 : K / BK;
  f32x4_t acc[8][8];
  if (sp.part == 2) {
    // second K half: start from the first half's partial (written half a
    // tile after the kernel began, by a workgroup dispatched earlier on this
    // XCD), then run the upper K range and store the tile as usual
    if (threadIdx.x == 0)
      while (__hip_atomic_load(flags + sp.slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        __builtin_amdgcn_s_sleep(4);
    __syncthreads();
    const f32x4_t* init =
        reinterpret_cast<const f32x4_t*>(ws) + (static_cast<size_t>(sp.slot) * 4 + wave_s) * 4096 + lane;
    w4j_mainloop<true>(acc, smem, A + ns * BK, Bt + ns * BK, lda, ldb, m0, n0, ns, lane, wave_s, init);
    if (threadIdx.x == 0)
      __hip_atomic_store(flags + sp.slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    w4j_mainloop(acc, smem, A, Bt, lda, ldb, m0, n0, ns, lane, wave_s);
    if (sp.part == 1) {
      partial_store(acc, ws, sp.slot, wave_s, lane);
      __builtin_amdgcn_s_waitcnt(0);             // this wave's partial reached memory
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_store(flags + sp.slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
  w4j_epilogue<EPI>(acc, smem, C, ldc, m0, n0, lane, wave_s);
}


// ---------------------------------------------------------------------------
// w4k: ONE barrier per K-tile (A/B record 47; candidate default).
//
// Stamps of the three-barrier K-tile (scripts/gpu/gemm_stamps.py, schedule
// 45) put ~64 + 64 + 46 cycles per K-tile into its three waits: the MFMA pipe
// of a wave that waits at a barrier idles (one wave per SIMD).  Two of the
// three barriers exist only to let the DMA refill a stage in place ("every
// wave finished reading X.A / X.B").  Here A has THREE 32 KiB slots and B two
// (3 x 32 + 2 x 32 KiB = the whole 160 KiB LDS): stage s+2's A goes into the
// slot stage s-1 used, which every wave left before the previous K-tile's
// barrier, so it is issued early in K-tile s with no barrier at all; stage
// s+2's B goes into B slot s%2 right after the K-tile's single barrier, by
// which every wave has read its k-half-1 B fragments of stage s.  Per K-tile
// (m = MFMA index 0..127):
//   m  0..14 even  A k-half-1 fragments (A slot s%3)
//   m 16..30 even  B k-half-1 fragments (B slot s%2)
//   m 33..61 /4    DMA of stage s+2, A pieces -> A slot (s+2)%3
//   m  92          lgkmcnt(0) + vmcnt(8) (stage s+1 landed; the 8 A pieces
//                  of s+2 stay in flight) + the barrier
//   m 93..123      next K-tile's k-half-0 fragments (stage s+1), SchedHB order
//   m 94..115      DMA of stage s+2, B pieces -> B slot s%2
// The stage slots repeat every 6 K-tiles; the loop is unrolled by 6 so every
// LDS address is a compile-time offset.
struct SchedA3 {
  static constexpr int WB = 92;
  __host__ __device__ static constexpr int a1(int m) { return m < 16 && (m & 1) == 0 ? m >> 1 : -1; }
  __host__ __device__ static constexpr int b1(int m) {
    return m >= 16 && m < 32 && (m & 1) == 0 ? (m - 16) >> 1 : -1;
  }
  __host__ __device__ static constexpr int adma(int m) {
    return m >= 33 && m <= 61 && (m - 33) % 4 == 0 ? (m - 33) / 4 : -1;
  }
  __host__ __device__ static constexpr int bdma(int m) {
    return m == 94 ? 0 : m == 96 ? 1 : m == 99 ? 2 : m == 101 ? 3 : m == 104 ? 4 : m == 107 ? 5
         : m == 110 ? 6 : m == 115 ? 7 : -1;
  }
  __host__ __device__ static constexpr int k0(int m) { return SchedHB::k0(m); }
};

constexpr int A3_SLOT = W4B_OP_BYTES;          // 32 KiB
constexpr int A3_B0 = 3 * A3_SLOT;             // B slots after the three A slots
constexpr int A3_LDS = 5 * A3_SLOT;            // 160 KiB

// K-tile of stage s with A in slot AS = s % 3 and B in slot BS = s % 2
// (compile-time; AS/BS = -1: runtime `as`/`bs`, for the two tail K-tiles).
// ABL (timing ablations only, wrong outputs; experiments variants 48-51):
// bit 0 skips the DMA pieces, bit 1 the fragment reads, bit 2 the waits and
// the barrier, bit 3 the C store (the epilogue's price).
// ORDER 1: the B fragment is the outer MFMA loop (srcA held for 8 MFMAs,
// srcB changing - hipBLASLt's operand order) instead of the A fragment.
// SPLITA: A fragments 0-3 at a_base, 4-7 at a_hi (the w13 SwiGLU kernel).
template <int AS, int BS, int MODE, class HOOK = NoHook, int ABL = 0, int ORDER = 0,
          bool SPLITA = false>
__device__ __forceinline__ void w4k_ktile(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                          bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                          bf16x8_t (&f1b)[8], char* smem, int a_base, int b_base,
                                          int off_k0, int off_k1, const DmaK& dma_a,
                                          const DmaK& dma_b, int kb2, int wave_s, int as = 0,
                                          int bs = 0, const HOOK& hook = HOOK{}, int a_hi = 0) {
  using S = SchedA3;
  constexpr int SUB = 2048;
  auto aoff = [&](int r) { return SPLITA && r >= 4 ? a_hi + (r - 4) * SUB : a_base + r * SUB; };
  const int a_cur = AS >= 0 ? AS : as, b_cur = BS >= 0 ? BS : bs;
  const int a_nxt = a_cur == 2 ? 0 : a_cur + 1;
  const int a_ref = a_cur == 0 ? 2 : a_cur - 1;
  char* XA = smem + a_cur * A3_SLOT;
  char* XB = smem + A3_B0 + b_cur * A3_SLOT;
  char* YA = smem + a_nxt * A3_SLOT;
  char* YB = smem + A3_B0 + (b_cur ^ 1) * A3_SLOT;
  char* RA = smem + a_ref * A3_SLOT;   // refill slot of A (stage s+2)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int o = 0; o < 8; ++o) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int m = h * 64 + o * 8 + q;
        const int i = ORDER ? q : o, j = ORDER ? o : q;
        if (h == 0) mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
        else mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
        hook(m);
        if (!(ABL & 2) && S::a1(m) >= 0)
          f1a[S::a1(m)] = lds_read_b128(XA + aoff(S::a1(m)) + off_k1);
        if (!(ABL & 2) && S::b1(m) >= 0)
          f1b[S::b1(m)] = lds_read_b128(XB + b_base + S::b1(m) * SUB + off_k1);
        if (!(ABL & 1) && MODE == 1 && S::adma(m) >= 0) dma_a.issue(RA, S::adma(m), kb2, wave_s);
        if (!(ABL & 4) && MODE != 3 && m == S::WB) {
          hook.at(4);
          __builtin_amdgcn_s_waitcnt(0xC07F);          // this wave's B k1 reads retired
          if constexpr (MODE == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          hook.at(5);
        }
        if (!(ABL & 1) && MODE == 1 && S::bdma(m) >= 0) dma_b.issue(XB, S::bdma(m), kb2, wave_s);
        if (!(ABL & 2) && MODE != 3 && S::k0(m) >= 0) {
          const int r = S::k0(m);
          if (r < 8) f0b[r] = lds_read_b128(YB + b_base + r * SUB + off_k0);
          else f0a[r - 8] = lds_read_b128(YA + aoff(r - 8) + off_k0);
        }
      }
    }
  }
}

// The one-barrier K loop over ns K-tiles into acc (zeroed here): prologue DMA
// of stages 0 and 1, the K-tiles unrolled by the 6-K-tile slot cycle, the two
// DMA-free tail K-tiles, the MFMA drain.  smem: A3_LDS bytes; b_base relative
// to a B slot.
// pre (the persistent kernel's second and later tiles): stage 0 was issued
// before the previous tile's epilogue, whose 32 C stores per wave are still
// counted in vmcnt; stage 1 goes out after a barrier (its slots held the
// epilogue's LDS slices).
// PRE_VM: the vmcnt that, in a pre call, leaves stage 1's 16 DMA pieces and
// the previous epilogue's stores in flight but waits for stage 0 (32 plain
// C stores: 48; at most 63)
template <int ABL = 0, int ORDER = 0, bool SPLITA = false, int PRE_VM = 48>
__device__ __forceinline__ void w4k_mainloop(f32x4_t (&acc)[8][8], char* smem, const DmaK& dma_a,
                                             const DmaK& dma_b, int a_base, int a_hi, int b_base,
                                             int ns, int lane, int wave_s, bool pre = false) {
  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ ((frow >> 1) & 7);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  auto aoff = [&](int r) { return SPLITA && r >= 4 ? a_hi + (r - 4) * SUB : a_base + r * SUB; };

  // an opaque zero: a constant zero is hoisted out of the persistent tile
  // loop, held in VGPRs across the K loop and spilled (its reload carried a
  // vmcnt(0) that drained the next tile's prefetched stage)
  float z = 0.f;
  asm volatile("" : "+v"(z));
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{z, z, z, z};

  // stages 0 and 1: A slots 0, 1 and B slots 0, 1
  if (!pre) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem, p, 0, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_b.issue(smem + A3_B0, p, 0, wave_s);
  } else {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
  }
  if (ns > 1) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem + A3_SLOT, p, BK * 2, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_b.issue(smem + A3_B0 + A3_SLOT, p, BK * 2, wave_s);
    if (pre) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PRE_VM) : "memory");   // + the stores
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + A3_B0 + b_base + j * SUB + off_k0);
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + aoff(i) + off_k0);
  __builtin_amdgcn_s_waitcnt(0xC07F);

  // K-tiles 0 .. ns-3 carry the DMA of stage s+2 (k offset (s+2)*128 B)
  int s = 0;
  int kb = 2 * BK * 2;
#define MXK_W4K(as_, bs_)                                                                       \
  w4k_ktile<as_, bs_, 1, NoHook, ABL, ORDER, SPLITA>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, \
                                                     off_k0, off_k1, dma_a, dma_b, kb, wave_s, 0, 0, \
                                                     NoHook{}, a_hi);                            \
  kb += BK * 2;
  for (; s + 6 <= ns - 2; s += 6) {
    MXK_W4K(0, 0) MXK_W4K(1, 1) MXK_W4K(2, 0) MXK_W4K(0, 1) MXK_W4K(1, 0) MXK_W4K(2, 1)
  }
  // s % 6 == 0 here: the remaining DMA-carrying K-tiles have compile-time slots
  const int r = ns - 2 - s;
  if (r > 0) { MXK_W4K(0, 0) }
  if (r > 1) { MXK_W4K(1, 1) }
  if (r > 2) { MXK_W4K(2, 0) }
  if (r > 3) { MXK_W4K(0, 1) }
  if (r > 4) { MXK_W4K(1, 0) }
#undef MXK_W4K
  s += r > 0 ? r : 0;
  // the last two K-tiles (or the only one): no DMA, runtime slots
  if (ns >= 2) {
    w4k_ktile<-1, -1, 2, NoHook, 0, ORDER, SPLITA>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base,
                                                   off_k0, off_k1, dma_a, dma_b, 0, wave_s, s % 3,
                                                   s & 1, NoHook{}, a_hi);
    ++s;
  }
  w4k_ktile<-1, -1, 3, NoHook, 0, ORDER, SPLITA>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base,
                                                 off_k0, off_k1, dma_a, dma_b, 0, wave_s, s % 3,
                                                 s & 1, NoHook{}, a_hi);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mxk::mfma_drain(acc);
}

template <int MAP, int EPI, int ABL = 0, int ORDER = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4k(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc,
                     const float* __restrict__ rcos = nullptr,
                     const float* __restrict__ rsin = nullptr, int rope_S = 0,
                     int rope_cols = 0) {
  __shared__ __attribute__((aligned(16))) char smem[A3_LDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, M / BM, N / BN, &m0, &n0);
  const DmaK dma_a = make_dmak(A, lda, m0, lane, wave_s);
  const DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);
  constexpr int SUB = 2048;
  f32x4_t acc[8][8];
  w4k_mainloop<ABL, ORDER>(acc, smem, dma_a, dma_b, wm * 8 * SUB, 0, wn * 8 * SUB, K / BK, lane,
                           wave_s);

  if constexpr (ABL & 8) {
    return;
  } else if constexpr (EPI == 4) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    mxk::store_block_lds<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane,
                               smem + wave_s * mxk::kStoreLdsWave);
  } else if constexpr (EPI == 5) {
    // EPI 4 with the rotary embedding of the columns below rope_cols (the
    // q / k heads of a fused QKV projection; each wave's 128 columns are one
    // head)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    // an opaque lane id: the epilogue's lane-derived addresses are formed
    // here, not hoisted above the K loop (where they spilled)
    int lane_e = lane;
    asm volatile("" : "+v"(lane_e));
    mxk::store_block_lds_rope<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane_e,
                                    smem + wave_s * mxk::kStoreLdsWave, rcos, rsin, rope_S,
                                    n0 + wn * 128 < rope_cols);
  } else if constexpr (EPI == 2) store_block_wide<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
  else store_block_narrow(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
}

// Persistent form of the default schedule (52): one workgroup per CU walks
// tiles t = blockIdx.x, + gridDim.x, ... of the same MAP (with 256
// workgroups a workgroup keeps its XCD and super-block position, the rounds
// advance as in the one-shot launch).  After a tile's K loop the next tile's
// stage 0 (A slot 0, B slot 0) is issued BEFORE the epilogue, so its fetch
// latency hides behind the C stores instead of opening the next K loop; the
// epilogue's LDS slices move to A slots 1-2 (waves 0-2) and B slot 1 (wave
// 3), which stage 1 refills only after a barrier.
template <int MAP, int ORDER = 1>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4p(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  static_assert(3 * mxk::kStoreLdsWave <= 2 * A3_SLOT && mxk::kStoreLdsWave <= A3_SLOT,
                "epilogue slices in A slots 1-2 and B slot 1");
  __shared__ __attribute__((aligned(16))) char smem[A3_LDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  const int ntiles = (M / BM) * (N / BN);
  constexpr int SUB = 2048;
  char* slice = wave_s < 3 ? smem + A3_SLOT + wave_s * mxk::kStoreLdsWave : smem + A3_B0 + A3_SLOT;
  int t = blockIdx.x;
  int m0, n0;
  w4b_tile<MAP>(t, ntiles, M / BM, N / BN, &m0, &n0);
  bool pre = false;
  for (;;) {
    f32x4_t acc[8][8];
    int lane_k = lane;   // opaque per tile (see lane_e below)
    asm volatile("" : "+v"(lane_k));
    // the DMA descriptors are rebuilt per tile (only m0 / n0 cross the
    // loop): carried, their 16 offset VGPRs pushed the K loop into spills
    const DmaK dma_a = make_dmak(A, lda, m0, lane_k, wave_s);
    const DmaK dma_b = make_dmak(Bt, ldb, n0, lane_k, wave_s);
    w4k_mainloop<0, ORDER>(acc, smem, dma_a, dma_b, wm * 8 * SUB, 0, wn * 8 * SUB, K / BK, lane_k,
                           wave_s, pre);
    // every wave's last fragment reads retired: all slots free
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    const int tn = t + static_cast<int>(gridDim.x);
    int m1 = 0, n1 = 0;
    if (tn < ntiles) {
      // opaque tile counts: the map's divisions by them are redone here,
      // not hoisted out of the loop as VGPR reciprocals that then spill
      int tiles_m = M / BM, tiles_n = N / BN;
      asm volatile("" : "+s"(tiles_m), "+s"(tiles_n));
      w4b_tile<MAP>(tn, ntiles, tiles_m, tiles_n, &m1, &n1);
      const DmaK na = make_dmak(A, lda, m1, lane_k, wave_s);
      const DmaK nb = make_dmak(Bt, ldb, n1, lane_k, wave_s);
#pragma unroll
      for (int p = 0; p < 8; ++p) na.issue(smem, p, 0, wave_s);
#pragma unroll
      for (int p = 0; p < 8; ++p) nb.issue(smem + A3_B0, p, 0, wave_s);
    }
    // an opaque lane id: the epilogue's lane-derived addresses are formed
    // here, not hoisted out of the tile loop (live across the K loop they
    // made the allocator spill)
    int lane_e = lane;
    asm volatile("" : "+v"(lane_e));
    mxk::store_block_lds<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane_e, slice);
    if (tn >= ntiles) break;
    t = tn;
    m0 = m1;
    n0 = n1;
    pre = true;
  }
}
