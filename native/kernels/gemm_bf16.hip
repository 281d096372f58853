// CDNA4 bf16 MFMA GEMM — the validator's compute payload (BASELINE config 3).
//
//   C[M][N] (bf16) = A[M][K] (bf16, row-major) · Bt[N][K]^T (bf16, row-major)
//   fp32 accumulation in the MFMA accumulators.
//
// "Bt" is the nn.Linear weight layout ([out][in]); both operands are read
// K-contiguous, which is what the MFMA A/B lane maps want, so neither tile
// needs a transpose on the way into LDS.
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §5):
//  * 256x256 macro tile, BK = 64, 256 threads = 4 waves (one per SIMD), each
//    owning a 128x128 block = 8x8 v_mfma_f32_16x16x32_bf16 tiles with the
//    fp32 accumulators pinned to AGPRs.  16x16x32 holds a higher clock than
//    32x32x16 on random data (MI355X_MICROARCH 'DVFS give-back' 7).
//  * Operands swapped in the MFMA (D' = Bt·A^T): a lane holds 4 consecutive
//    N-columns of one C row; v_permlane16_swap pairs two 16x16 tiles so the
//    store tail is 32 dwordx4 (non-temporal) per lane.
//  * Global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into two 64 KiB
//    stages; lane-linear image, XOR swizzle applied to the source address
//    (rule 21): chunk c of row r at c ^ ((r >> 1) & 7), conflict-free
//    ds_read_b128 (tests/test_gemm_swizzle.py).
//  * Three barriers per K-tile (hipBLASLt's gfx950 structure, read off its
//    disassembly): the stage just consumed is refilled in place with stage
//    s+2 once each operand's last fragment read retired, so the DMA pieces
//    spread over ~64 MFMAs and have ~130-200 MFMAs to land; counted vmcnt,
//    raw s_barrier.
//  * K loop unrolled by two (compile-time LDS bases), k step as the DMA's
//    soffset: no address arithmetic ahead of the MFMA stream; the last two
//    K-tiles carry no DMA.
//  * XCD-aware super-block tile map (mx_common.h w4b_tile<1>): the 256
//    resident tiles form one 16x16 block, 8x4 per XCD (L2 reuse) and 32
//    panels chip-wide (Infinity Cache reuse).
//
// Schedules (mxk_gemm_bf16_tn_variant, A/B-timed by python -m
// mxk8s.validate.gemm --variants all).  The production library builds 1, 6,
// 9, 26 (mxk_gemm_bf16_tn_w4j) and 47 / 52 (mxk_gemm_bf16_tn_w4k, both in
// gemm_tn_core.h); every other schedule is
// an A/B record in experiments/gemm_tn_exp.hip, compiled only into `make
// gemm-exp`'s libmxkernels_exp.so (-DMXK_GEMM_EXPERIMENTS):
//   0 w4i   super-block map, non-temporal widened stores, late barrier #3
//   1 w4j   26's K-tile with 8-byte stores (C not 16-B aligned or
//           ldc % 8 != 0; the w4i K-tile until round 4)
//   2 w4i   widened plain stores, barrier #3 after m 91
//   3 w4i   widened plain stores, barrier #3 after m 96
//   4 w4i   variant 3 with A k1 reads at even m and barrier #1 after m 21
//   5 w4ip  persistent w4i (one workgroup per CU)
//   6 w4j   w4i with every read/DMA/wait at hipBLASLt's MFMA positions
//           (+0.5-2 % over 0 on squares and the Llama-3-8B shapes)
//   7 w4j   two barriers per K-tile (SchedTwoBarrier)
//   8 w4j   variant 6 with plain (temporal) widened stores
//   9 x2    the layout kernel of gemm_bf16_layouts.hip (same schedule as 6,
//           inline-asm LDS-DMA with the LDS address bound to M0)
//  10 DIAG  variant 6 without the C store tail (timing ablation only)
//  11 w4ip  persistent, schedule 6, plain (temporal) widened stores
//  12 w4ip  persistent, schedule 6, non-temporal widened stores
//  13 w4j   schedule 6 with every B piece before the stage wait (vmcnt 16)
//  14 w4j   schedule 6 with the next-k0 reads spread over odd m 93..123
//  15 w4j   schedule 6, B fragment as the outer MFMA loop
//  16 w4j   schedule 6 under s_setprio 1
//  17 w4j   schedule 6, K loop rotated per XCD (different K-slices per XCD)
//  18 w4j   schedule 6, K loop rotated per workgroup
//  19 pp8   8 waves, two per SIMD, compute / load ping-pong (mxk_gemm_bf16_tn_pp8)
//  20 pp8   19 with the second group at s_setprio 1
//  21-24 w4j schedule 6 with a staggered first round (four CU groups start
//           1/2/4/8 x ~1024 clocks apart, so C store bursts do not coincide)
//  25 w4j   variant 23 with plain (temporal) widened stores
//  26 w4j   round-2/3 default: schedule 6 with the C tile stored through LDS, read
//           back row-major so every store covers whole lines (4 rows x 256 B
//           per wave-instruction instead of 16 x 64 B): +1.3 / +3.0 / +0.4 %
//           over 6 at 8192^3 / 4096^3 / 16384^3 (profiles/r2_gemm_ab/)
//  27 w4j   26 with ONE barrier per K-tile (SchedOneBarrier), 28 the same
//           with the DMA spread: -5 / -1 % at 8192^3, -6 / -10 % at 16384^3
//           (profiles/r3_gemm/)
//  33-36    26 with its K loop moved against the 64-B instruction-fetch
//           blocks by s_nop padding in front of it: loop head at 16 / 0 /
//           28 / 4 mod 64 B (26 itself: 48)
//  37-38    26 without the operand XOR swizzle (37: linear LDS image, the
//           DMA reads each row's 128 B in lane order; 38: only the 64-B
//           halves swapped) - prices the permuted DMA source against the
//           LDS bank conflicts it removes; 39 / 40: XOR masks 6 / 5
//  41-43    26 with the XCD sub-block of the super-block tile map 4 x 8 /
//           2 x 16 / 16 x 2 tiles instead of 8 x 4 (L2-miss A/B); 44: 26 with
//           the K loop rotated per XCD (17's rotation on the LDS-staged store)
//  45 DIAG  26 with s_memtime stamps around its waits (mxk_gemm_stamps_read)
//  46       26 built from the full-flag experiments template (the same K loop
//           in other registers: A/B of the production kernel's own template)
//  47 w4k   ONE barrier per K-tile: A triple-buffered (3 + 2 x 32 KiB = all of
//           LDS), stage s+2's A refilled early into the slot stage s-1 used,
//           B right after the barrier (gemm_tn_core.h mxk_gemm_bf16_tn_w4k)
//  48-51 DIAG 47 without its DMA pieces / fragment reads / waits and barrier /
//           all three (timing ablations, wrong outputs)
//  52 w4k   DEFAULT (round 4): 47 with the B fragment as the outer MFMA loop
//           (srcA held for 8 MFMAs, hipBLASLt's operand order); against 26
//           on two boxes: +1.8 / +0.5 % at 8192^3, 0 % at 4096^3, +0.2 % at
//           16384^3, -0.2 / +2.5 % at 4096x4096x16384 (profiles/r4_gemm/)
//  53 DIAG  47 without the C store (prices the epilogue: ~2 % at 8192^3)
//  54-55    26 with staggered rounds (mxk_gemm_bf16_tn_w4j_stag): half of
//           each XCD's CUs start with a K-half tile so the C-store bursts fall
//           half a tile apart; 54 exchanges the fp32 partials through
//           uncached memory (-8 % at 8192^3, profiles/r4_gemm/), 55 through
//           plain memory (same-XCD L2; A/B of the uncached traffic)
//  57 w4j   staggered by XCD group (stagger_part_xcd): XCDs 4-7 half a tile
//           out of phase with XCDs 0-3, every CU of an XCD in phase
//  56 w4j   26 with an L2 prefetch of stage s+4 per K-tile (gemm_tn_core.h
//           L2Prefetch; for HBM-cold operands): -1.5..-3 % warm, -1.7 % cold
//           (profiles/r4_gemm/cold_vs_warm_prefetch56.txt)
//  29-30    gemm_bf16_ring.hip: a ring of 4 / 5 32-deep k slots, one
//           barrier per k-step, refills 4-5 steps ahead: -9 % at 8192^3,
//           -23 % at 16384^3 (a k32 slot row is half a 128-B line, so each
//           line is fetched twice; profiles/r3_gemm/)
// The earlier schedules (one-barrier w4b, 8-wave, 4-deep ring, w4h, ...)
// were retired when an ISA audit (tests/test_isa_hazards.py) found their
// loop-exit accumulator copies racing the inline-asm MFMAs; their A/B logs
// stay in profiles/r1_gemm_*/ (numbered by the old ids: old 34 = 0,
// 31 = 1, 29 = 2, 30 = 3, 32 = 4, 35 = 5, 36 = 6).
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "gemm_tn_core.h"

// ---------------------------------------------------------------------------
// MLP up-projection with the SwiGLU activation in its epilogue:
//   gu[M][2F] = x[M][K] . W13[2F][K]^T   (W13 = [gate | up] rows, as stored)
//   h[M][F]   = silu(gu[:, :F]) * gu[:, F:]   (from the fp32 accumulators)
// The separate element-wise pass (read gu, write h: 1.4 GB per Llama-3-8B
// layer at micro-batch 8) disappears; gu is still written (the backward's
// fused dgrad-SwiGLU epilogue reads it).  A 256-column tile is 128 gate
// columns [g0, g0+128) and the MATCHING 128 up columns [F+g0, F+g0+128): the
// B panel's pieces 4..7 (tile rows 128-255) read W13 rows F-128 further down,
// so waves wn = 0 hold g and waves wn = 1 hold u of the same (row, column)
// in the same lane/register positions.  Epilogue: both store their half of
// gu (LDS-staged, whole lines); then each pair exchanges half its rows
// through LDS (the gate wave keeps rows 0-63 and takes u of them, the up wave
// takes g of rows 64-127) and each computes and stores h of 64 rows.
// Same K loop as the default schedule (hipBLASLt's instruction positions).
template <int PAR, int MODE>
__device__ __forceinline__ void w13_ktile(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                          bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                          bf16x8_t (&f1b)[8], char* smem, int a_lo, int a_hi,
                                          int b_base, int off_k0, int off_k1, const DmaK& dma_a,
                                          const DmaK& dma_b, int kb2, int wave_s, int par = 0) {
  w4j_ktile<SchedHB, PAR, MODE, 0, 0, true>(acc, f0a, f0b, f1a, f1b, smem, a_lo, b_base, off_k0,
                                            off_k1, dma_a, dma_b, kb2, wave_s, par, a_hi);
}

// ONEBAR: the K loop of the default TN schedule 52 (gemm_tn_core.h
// w4k_mainloop: one barrier per K-tile, A in three LDS slots) instead of the
// three-barrier w4j loop; MXK_W13_SCHED=1 selects it (A/B in the step).
// GUNT: gu (read again only by the backward, a step later) stored
// non-temporally so it does not displace the A/B panels; MXK_W13_SCHED=2.
template <bool ONEBAR, bool GUNT = false>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_w13_swiglu_k(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W13,
                           uint16_t* __restrict__ GU, uint16_t* __restrict__ H, int M, int F, int K,
                           int ldx, int ldw, int ldgu, int ldh) {
  __shared__ __attribute__((aligned(16))) char smem[ONEBAR ? A3_LDS : 2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;               // 0: gate columns, 1: up columns
  int m0, n0v;
  w4b_tile<1>(blockIdx.x, gridDim.x, M / BM, F / 128, &m0, &n0v);
  const int g0 = n0v >> 1;                 // first gate column of the tile
  const DmaK dma_a = make_dmak(X, ldx, m0, lane, wave_s);
  DmaK dma_b = make_dmak(W13, ldw, g0, lane, wave_s);
  // tile rows 128..255 of the B panel are the up rows F + g0 ..: pieces 4..7
  dma_b.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(W13 + static_cast<size_t>(g0) * ldw),
                                                 0, (F + 128) * ldw * 2, 0x00020000);
#pragma unroll
  for (int p = 4; p < 8; ++p) dma_b.voff[p] += static_cast<uint32_t>((F - 128) * ldw * 2);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  // the up waves accumulate their row blocks rotated by 4 (acc[i] = rows
  // 16 ((i + 4) & 7)): then every wave hands acc[4..7] to its partner and
  // keeps acc[0..3], one code path for both roles
  const int a_lo = (wm * 8 + (wn ? 4 : 0)) * SUB;
  const int a_hi = (wm * 8 + (wn ? 0 : 4)) * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;

  f32x4_t acc[8][8];
  const int ns = K / BK;
  if constexpr (ONEBAR) {
    w4k_mainloop<0, 1, true>(acc, smem, dma_a, dma_b, a_lo, a_hi, wn * 8 * SUB, ns, lane, wave_s);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem, p, 0, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_OP_BYTES, p, 0, wave_s);
    if (ns > 1) {
#pragma unroll
      for (int p = 0; p < 8; ++p) dma_a.issue(smem + W4B_STAGE_BYTES, p, BK * 2, wave_s);
#pragma unroll
      for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_STAGE_BYTES + W4B_OP_BYTES, p, BK * 2, wave_s);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();

    bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      f0a[i] = lds_read_b128(smem + (i < 4 ? a_lo + i * SUB : a_hi + (i - 4) * SUB) + off_k0);
    __builtin_amdgcn_s_waitcnt(0xC07F);

    int s = 0;
    int kb = 2 * BK * 2;
    for (; s + 2 <= ns - 2; s += 2) {
      w13_ktile<0, 1>(acc, f0a, f0b, f1a, f1b, smem, a_lo, a_hi, b_base, off_k0, off_k1, dma_a, dma_b,
                      kb, wave_s);
      w13_ktile<1, 1>(acc, f0a, f0b, f1a, f1b, smem, a_lo, a_hi, b_base, off_k0, off_k1, dma_a, dma_b,
                      kb + BK * 2, wave_s);
      kb += 2 * BK * 2;
    }
    if (s < ns - 2) {
      w13_ktile<0, 1>(acc, f0a, f0b, f1a, f1b, smem, a_lo, a_hi, b_base, off_k0, off_k1, dma_a, dma_b,
                      kb, wave_s);
      ++s;
    }
    if (ns >= 2) {
      w13_ktile<2, 2>(acc, f0a, f0b, f1a, f1b, smem, a_lo, a_hi, b_base, off_k0, off_k1, dma_a, dma_b,
                      0, wave_s, s & 1);
      ++s;
    }
    w13_ktile<2, 3>(acc, f0a, f0b, f1a, f1b, smem, a_lo, a_hi, b_base, off_k0, off_k1, dma_a, dma_b, 0,
                    wave_s, s & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mxk::mfma_drain(acc);
  }


  // 1. gu: each wave its half (gate -> columns g0.., up -> F + g0..), its two
  //    64-row passes swapped back for the rotated up waves
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  mxk::store_block_lds<GUNT>(acc, GU, ldgu, m0 + wm * 128, (wn ? F : 0) + g0, lane,
                              smem + wave_s * mxk::kStoreLdsWave, wn);
  __builtin_amdgcn_s_barrier();            // every staging slice is free again
  // 2. hand acc[4..7] to the partner (gate: g of rows 64-127, up: u of rows
  //    0-63) through region (wm, wn); take the partner's from (wm, wn ^ 1)
  char* mine_out = smem + (wm * 2 + wn) * 32768 + lane * 16;
  const char* theirs = smem + (wm * 2 + (wn ^ 1)) * 32768 + lane * 16;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      *reinterpret_cast<f32x4_t*>(mine_out + (i * 8 + j) * 1024) = acc[4 + i][j];
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  const bool up = wn != 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4_t o = *reinterpret_cast<const f32x4_t*>(theirs + (i * 8 + j) * 1024);
      f32x4_t hv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = up ? o[e] : acc[i][j][e], u = up ? acc[i][j][e] : o[e];
        hv[e] = g * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(g * -1.44269504f)) * u;
      }
      acc[i][j] = hv;
    }
  // 3. h of the kept 64 rows (gate wave: rows 0-63 of its block, up: 64-127)
  mxk::store_block_wide<false, 4, 8>(reinterpret_cast<const f32x4_t(&)[4][8]>(acc[0]), H, ldh,
                                     m0 + wm * 128 + (wn ? 64 : 0), g0, lane);
}

#ifdef MXK_GEMM_EXPERIMENTS
// Persistent form of the fused up-projection (A/B record, MXK_W13_SCHED=3):
// one workgroup per CU walks tiles t = blockIdx.x, + gridDim.x, ... with the
// one-barrier K loop (TN schedule 52's, A fragments split gate / up).  After
// a tile's K loop the NEXT tile's stage 0 (A slot 0, B slot 0) is issued
// before this tile's epilogue, so the gu / h stores drain while the next K
// loop starts instead of ahead of a fresh workgroup's prologue.  The
// epilogue works in the LDS that stage 0 leaves free: gu staged through A
// slots 1-2 (waves 0-2) and B slot 1 (wave 3), then the gate / up hand-off
// in two rounds of 16 KiB per wave through A slots 1-2 (the one-shot kernel
// hands over 32 KiB per wave in one round, 128 KiB, more than is free).
__device__ __forceinline__ DmaK make_dmak_w13(const uint16_t* W13, int ldw, int g0, int F, int lane,
                                              int wave_s) {
  DmaK d = make_dmak(W13, ldw, g0, lane, wave_s);
  // tile rows 128..255 of the B panel are the up rows F + g0 ..: pieces 4..7
  d.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(W13 + static_cast<size_t>(g0) * ldw), 0,
                                             (F + 128) * ldw * 2, 0x00020000);
#pragma unroll
  for (int p = 4; p < 8; ++p) d.voff[p] += static_cast<uint32_t>((F - 128) * ldw * 2);
  return d;
}

__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_w13_swiglu_p(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W13,
                           uint16_t* __restrict__ GU, uint16_t* __restrict__ H, int M, int F, int K,
                           int ldx, int ldw, int ldgu, int ldh) {
  static_assert(3 * mxk::kStoreLdsWave <= 2 * A3_SLOT && mxk::kStoreLdsWave <= A3_SLOT,
                "gu slices in A slots 1-2 and B slot 1");
  __shared__ __attribute__((aligned(16))) char smem[A3_LDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;               // 0: gate columns, 1: up columns
  const int ntiles = (M / BM) * (F / 128);
  constexpr int SUB = 2048;
  const int a_lo = (wm * 8 + (wn ? 4 : 0)) * SUB;
  const int a_hi = (wm * 8 + (wn ? 0 : 4)) * SUB;
  char* slice = wave_s < 3 ? smem + A3_SLOT + wave_s * mxk::kStoreLdsWave : smem + A3_B0 + A3_SLOT;
  int t = blockIdx.x;
  int m0, n0v;
  w4b_tile<1>(t, ntiles, M / BM, F / 128, &m0, &n0v);
  bool pre = false;
  for (;;) {
    f32x4_t acc[8][8];
    int lane_k = lane;   // opaque per tile (gemm_tn_core.h w4p)
    asm volatile("" : "+v"(lane_k));
    const int g0 = n0v >> 1;
    const DmaK dma_a = make_dmak(X, ldx, m0, lane_k, wave_s);
    const DmaK dma_b = make_dmak_w13(W13, ldw, g0, F, lane_k, wave_s);
    // stage 0 issued before the previous epilogue's 32 gu + 16 h stores:
    // vmcnt 63 (stage 1's 16 pieces + 47 of the stores) waits for it
    w4k_mainloop<0, 1, true, 63>(acc, smem, dma_a, dma_b, a_lo, a_hi, wn * 8 * SUB, K / BK, lane_k,
                                 wave_s, pre);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    const int tn = t + static_cast<int>(gridDim.x);
    int m1 = 0, n1v = 0;
    if (tn < ntiles) {
      int tiles_m = M / BM, tiles_n = F / 128;
      asm volatile("" : "+s"(tiles_m), "+s"(tiles_n));
      w4b_tile<1>(tn, ntiles, tiles_m, tiles_n, &m1, &n1v);
      const DmaK na = make_dmak(X, ldx, m1, lane_k, wave_s);
      const DmaK nb = make_dmak_w13(W13, ldw, n1v >> 1, F, lane_k, wave_s);
#pragma unroll
      for (int p = 0; p < 8; ++p) na.issue(smem, p, 0, wave_s);
#pragma unroll
      for (int p = 0; p < 8; ++p) nb.issue(smem + A3_B0, p, 0, wave_s);
    }
    int lane_e = lane;
    asm volatile("" : "+v"(lane_e));
    // 1. gu: each wave its half, the two 64-row passes swapped back for the
    //    rotated up waves
    mxk::store_block_lds<false>(acc, GU, ldgu, m0 + wm * 128, (wn ? F : 0) + g0, lane_e, slice, wn);
    const bool up = wn != 0;
    // 2. the gate / up hand-off of acc[4..7] in two rounds of two row blocks
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();         // slices (round 0) / round 0's reads (round 1) done
      char* mine_out = smem + A3_SLOT + (wm * 2 + wn) * 16384 + lane_e * 16;
      const char* theirs = smem + A3_SLOT + (wm * 2 + (wn ^ 1)) * 16384 + lane_e * 16;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          *reinterpret_cast<f32x4_t*>(mine_out + (ii * 8 + j) * 1024) = acc[4 + 2 * r + ii][j];
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4_t o = *reinterpret_cast<const f32x4_t*>(theirs + (ii * 8 + j) * 1024);
          f32x4_t hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float g = up ? o[e] : acc[2 * r + ii][j][e], u = up ? acc[2 * r + ii][j][e] : o[e];
            hv[e] = g * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(g * -1.44269504f)) * u;
          }
          acc[2 * r + ii][j] = hv;
        }
    }
    // 3. h of the kept 64 rows
    mxk::store_block_wide<false, 4, 8>(reinterpret_cast<const f32x4_t(&)[4][8]>(acc[0]), H, ldh,
                                       m0 + wm * 128 + (wn ? 64 : 0), g0, lane_e);
    if (tn >= ntiles) break;
    t = tn;
    m0 = m1;
    n0v = n1v;
    pre = true;
  }
}
#endif

// ---------------------------------------------------------------------------
// Generic bounds-checked MFMA GEMM (any M, N, K; K-contiguous operands).
// 64x64 tile, 256 threads (2x2 waves of 32x32), register-staged through LDS.
// Used for shapes the 256x256 kernel does not tile exactly.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
mxk_gemm_bf16_tn_generic(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                         uint16_t* __restrict__ C, int M, int N, int K,
                         int lda, int ldb, int ldc) {
  constexpr int T = 64, TK = 32;
  __shared__ __attribute__((aligned(16))) uint16_t sA[T][TK + 8];
  __shared__ __attribute__((aligned(16))) uint16_t sB[T][TK + 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += TK) {
    // 64 rows x 32 k per operand = 2048 elements; 256 threads x 8 elements.
    {
      const int r = tid >> 2, c = (tid & 3) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int gm = m0 + r, gk = k0 + c + e;
        sA[r][c + e] = (gm < M && gk < K) ? A[static_cast<size_t>(gm) * lda + gk] : 0;
        const int gn = n0 + r;
        sB[r][c + e] = (gn < N && gk < K) ? Bt[static_cast<size_t>(gn) * ldb + gk] : 0;
      }
    }
    __syncthreads();
    const int fr = lane & 15, fk = (lane >> 4) * 8;
    bf16x8_t a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[i][e] = static_cast<short>(sA[wm * 32 + i * 16 + fr][fk + e]);
        b[i][e] = static_cast<short>(sB[wn * 32 + i * 16 + fr][fk + e]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  const int crow = lane & 15, ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + wm * 32 + i * 16 + crow;
      if (m >= M) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + j * 16 + ccol + r;
        if (n < N) C[static_cast<size_t>(m) * ldc + n] = mxk::f2bf(acc[i][j][r]);
      }
    }
}

// ---------------------------------------------------------------------------
// Host launchers (C ABI, stream-ordered, capture-safe: no sync, no malloc).
// ---------------------------------------------------------------------------
MXK_API int mxk_gemm_bf16_ex_variant(const void* A, const void* B, void* C, int M, int N, int K,
                                     int lda, int ldb, int ldc, int a_kmajor, int b_kmajor,
                                     int variant, hipStream_t stream);

MXK_API int mxk_gemm_available_cus(void);   // gemm_bf16_layouts.hip

// Staggered-round plan (schedule 54, mxk_gemm_bf16_tn_w4j_stag): split tiles
// per XCD (half the XCD's CUs), or 0 when it does not apply - T % 8, fewer
// than two whole rounds, or K halves shorter than two K-tiles / not whole
// K-tiles.  Pure host arithmetic (tests/test_gemm_plan.py).
MXK_API int mxk_gemm_stagger_plan(long T, int K, int cus) {
  if (T <= 0 || T % 8 || cus < 16 || K % (2 * BK) || K < 4 * BK) return 0;
  const long tx = T / 8;
  const int cx = cus / 8;
  const int sx = cx / 2;
  if (sx <= 0 || tx < 2 * cx) return 0;
  return sx;
}

// stagger_part() of workgroup b on the host: out = {virtual tile, part, slot}
MXK_API void mxk_gemm_stagger_part(int b, int T, int sx, int* out) {
  const StaggerPart p = stagger_part(b, T, sx);
  out[0] = p.vtile;
  out[1] = p.part;
  out[2] = p.slot;
}

MXK_API void mxk_gemm_stagger_part_xcd(int b, int T, int cx, int* out) {
  const StaggerPart p = stagger_part_xcd(b, T, cx);
  out[0] = p.vtile;
  out[1] = p.part;
  out[2] = p.slot;
}

namespace {
constexpr int kNumVariants = 59;
constexpr int kDefaultVariant = 52;
constexpr int kNarrowCVariant = 1;
constexpr const char* kVariantNames[kNumVariants] = {
    "w4i", "w4i_narrow", "w4i_b3_91", "w4i_b3_96", "w4i_r1", "w4ip", "w4j_hb", "w4j_2bar",
    "w4j_hb_st", "x2_hb", "diag_nostore", "w4ip_hb_st", "w4ip_hb_nt", "w4j_earlyb",
    "w4j_spreadk0", "w4j_hb_bouter", "w4j_hb_prio", "w4j_rot_xcd", "w4j_rot_wg", "pp8",
    "pp8_prio", "w4j_stag1", "w4j_stag2", "w4j_stag4", "w4j_stag8", "w4j_stag4_st", "w4j_hb_ldsst", "w4j_1bar_ldsst", "w4j_1bar_spread_ldsst", "ring4_ldsst", "ring5_ldsst", "w4t_trickle", "w4t_trickle_lds", "w4j_ldsst_aln64", "w4j_ldsst_aln64p4",
    "w4j_ldsst_aln64p8", "w4j_ldsst_aln64p12", "w4j_ldsst_linear", "w4j_ldsst_swz_half",
    "w4j_ldsst_swz6", "w4j_ldsst_swz5", "w4j_ldsst_map4x8", "w4j_ldsst_map2x16",
    "w4j_ldsst_map16x2", "w4j_ldsst_rot_xcd", "diag_stamps", "w4i_ldsst_full_template",
    "w4k_1bar_a3_ldsst", "diag_w4k_nodma", "diag_w4k_noreads", "diag_w4k_nowait",
    "diag_w4k_mfma_only", "w4k_border", "diag_w4k_nostore", "w4j_stagger", "w4j_stagger_cached", "w4j_l2pf", "w4j_stagger_xcd",
    "w4p_persistent"};

}  // namespace
#ifdef MXK_GEMM_EXPERIMENTS
int mxk_gemm_tn_exp_launch(int v, int nwg, hipStream_t stream, const void* A, const void* Bt,
                           void* C, int M, int N, int K, int lda, int ldb, int ldc);
#endif
namespace {

template <int EPI>
void launch_w4j(int nwg, hipStream_t stream, const void* a, const void* b, void* c, int M, int N,
                int K, int lda, int ldb, int ldc) {
  MXK_LAUNCH_GEMM((mxk_gemm_bf16_tn_w4j<1, EPI>), dim3(nwg), dim3(W4_THREADS), stream,
                     static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b),
                     static_cast<uint16_t*>(c), M, N, K, lda, ldb, ldc);
}

void launch_256(int v, int nwg, hipStream_t stream, const void* A, const void* Bt, void* C, int M,
                int N, int K, int lda, int ldb, int ldc) {
  switch (v) {
    case 47:
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_tn_w4k<1, 4>), dim3(nwg), dim3(W4_THREADS), stream,
                         static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(Bt),
                         static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc);
      break;
    case 52:
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_tn_w4k<1, 4, 0, 1>), dim3(nwg), dim3(W4_THREADS), stream,
                         static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(Bt),
                         static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc);
      break;
#ifdef MXK_GEMM_EXPERIMENTS
    case 58: {
      // persistent: one workgroup per available CU (at most one per tile);
      // an A/B record (profiles/r5_gemm/persistent_58_ab.txt: equal to 52
      // within noise at 8192^3 and the step shapes)
      const int cus = mxk_gemm_available_cus();
      const int grid = cus > 0 && cus < nwg ? cus : nwg;
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_tn_w4p<1, 1>), dim3(grid), dim3(W4_THREADS), stream,
                         static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(Bt),
                         static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc);
      break;
    }
#endif
    case 1: launch_w4j<0>(nwg, stream, A, Bt, C, M, N, K, lda, ldb, ldc); break;
    case 6: launch_w4j<2>(nwg, stream, A, Bt, C, M, N, K, lda, ldb, ldc); break;
    case 9:
      // the layout kernel (gemm_bf16_layouts.hip) on K-major operands
      mxk_gemm_bf16_ex_variant(A, Bt, C, M, N, K, lda, ldb, ldc, 1, 1, 2, stream);
      break;
    case 26: launch_w4j<4>(nwg, stream, A, Bt, C, M, N, K, lda, ldb, ldc); break;
    default:
#ifdef MXK_GEMM_EXPERIMENTS
      mxk_gemm_tn_exp_launch(v, nwg, stream, A, Bt, C, M, N, K, lda, ldb, ldc);
#endif
      break;
  }
}

// Production builds carry the default (52), its ORDER-0 twin (47), the
// round-3 default (26) and its non-LDS-store base (6), the 8-byte-store
// fallback (1, 26's K-tile) and the layout kernel (9); every
// other schedule is an A/B record in experiments/gemm_tn_exp.hip, built only
// with -DMXK_GEMM_EXPERIMENTS (`make gemm-exp` -> libmxkernels_exp.so).
bool variant_built(int v) {
#ifdef MXK_GEMM_EXPERIMENTS
  return v >= 0 && v < kNumVariants;
#else
  return v == 1 || v == 6 || v == 9 || v == 26 || v == 47 || v == 52;
#endif
}

// MXK_TN_VARIANT=v: another built schedule as the default (same-box A/B of
// the training step; the validator times schedules directly)
int default_variant() {
  static const int v = [] {
    const char* e = std::getenv("MXK_TN_VARIANT");
    const int x = e ? std::atoi(e) : kDefaultVariant;
    return variant_built(x) && x != kNarrowCVariant ? x : kDefaultVariant;
  }();
  return v;
}

// every schedule but 1 stores 16 B per lane: C 16-B aligned, ldc % 8 == 0
bool wide_c_ok(const void* C, int ldc) {
  return (ldc % 8 == 0) && (reinterpret_cast<uintptr_t>(C) % 16 == 0);
}
}  // namespace

// Benchmark hook: run schedule `variant` of the 256x256 kernel (fast shapes only).
MXK_API int mxk_gemm_bf16_tn_variant(const void* A, const void* Bt, void* C, int M, int N, int K,
                                     int lda, int ldb, int ldc, int variant, hipStream_t stream) {
  if (M % BM || N % BN || K % BK || variant < 0 || variant >= kNumVariants ||
      (variant != kNarrowCVariant && !wide_c_ok(C, ldc)))
    return static_cast<int>(hipErrorInvalidValue);
  if (!variant_built(variant)) return static_cast<int>(hipErrorNotSupported);
  launch_256(variant, (M / BM) * (N / BN), stream, A, Bt, C, M, N, K, lda, ldb, ldc);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_gemm_bf16_tn_num_variants(void) { return kNumVariants; }
MXK_API const char* mxk_gemm_bf16_tn_variant_name(int variant) {
  return variant >= 0 && variant < kNumVariants ? kVariantNames[variant] : nullptr;
}
MXK_API int mxk_gemm_bf16_tn_variant_built(int variant) { return variant_built(variant); }
// Variant 10 is a timing ablation (no C store): never correctness-checked or used.
MXK_API int mxk_gemm_bf16_tn_is_ablation(int variant) {
  return variant == 10 || variant == 45 || (variant >= 48 && variant <= 51) || variant == 53;
}

MXK_API int mxk_gemm_bf16_tn(const void* A, const void* Bt, void* C, int M, int N, int K,
                             int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return static_cast<int>(hipErrorInvalidValue);
  const bool fast = (M % BM == 0) && (N % BN == 0) && (K % BK == 0) && (lda % 8 == 0) &&
                    (ldb % 8 == 0) && (ldc % 4 == 0) &&
                    (reinterpret_cast<uintptr_t>(A) % 16 == 0) &&
                    (reinterpret_cast<uintptr_t>(Bt) % 16 == 0) &&
                    (reinterpret_cast<uintptr_t>(C) % 8 == 0);
  if (fast) {
    launch_256(wide_c_ok(C, ldc) ? default_variant() : kNarrowCVariant, (M / BM) * (N / BN), stream,
               A, Bt, C, M, N, K, lda, ldb, ldc);
  } else {
    dim3 grid((N + 63) / 64, (M + 63) / 64);
    hipLaunchKernelGGL(mxk_gemm_bf16_tn_generic, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(Bt),
                       static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc);
  }
  MXK_RETURN_LAUNCH_STATUS();
}

// gu = x . W13^T and h = silu(gu[:, :F]) * gu[:, F:] in one launch (see the
// kernel).  M % 256, F % 128, K % 64, 16-B aligned operands, ld* % 8.
namespace {
std::atomic<int> g_w13_sched{-1};
int w13_sched() {
  int v = g_w13_sched.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("MXK_W13_SCHED");
    v = e ? std::atoi(e) : 0;
    g_w13_sched.store(v, std::memory_order_relaxed);
  }
  return v;
}
}  // namespace

// K loop of the fused up-projection: 0 three-barrier w4j (default), 1 the
// one-barrier loop of TN schedule 52, 2 = 0 with non-temporal gu stores,
// 3 the persistent form (experiments library; env MXK_W13_SCHED)
MXK_API void mxk_gemm_w13_set_sched(int v) { g_w13_sched.store(v >= 1 && v <= 3 ? v : 0); }

MXK_API int mxk_gemm_bf16_w13_swiglu(const void* x, const void* w13, void* gu, void* h, int M,
                                     int F, int K, int ldx, int ldw, int ldgu, int ldh,
                                     hipStream_t stream) {
  auto al = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (M <= 0 || F <= 0 || K <= 0 || M % BM || F % 128 || K % BK || ldx % 8 || ldw % 8 ||
      ldgu % 8 || ldh % 8 || !al(x) || !al(w13) || !al(gu) || !al(h) ||
      static_cast<long>(F + 128) * ldw * 2 >= (1L << 31))
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = (M / BM) * (F / 128);
#ifdef MXK_GEMM_EXPERIMENTS
  // A/B records (experiments library): 1 = one-barrier K loop, 2 = non-temporal
  // gu stores; both step-neutral (profiles/r4_step/)
  if (w13_sched() == 3) {
    const int cus = mxk_gemm_available_cus();
    const int grid = cus > 0 && cus < nwg ? cus : nwg;
    MXK_LAUNCH_GEMM(mxk_gemm_bf16_w13_swiglu_p, dim3(grid), dim3(W4_THREADS), stream,
                    static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w13),
                    static_cast<uint16_t*>(gu), static_cast<uint16_t*>(h), M, F, K, ldx, ldw, ldgu, ldh);
  } else if (w13_sched() == 2)
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_w13_swiglu_k<false, true>), dim3(nwg), dim3(W4_THREADS), stream,
                    static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w13),
                    static_cast<uint16_t*>(gu), static_cast<uint16_t*>(h), M, F, K, ldx, ldw, ldgu, ldh);
  else if (w13_sched() == 1)
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_w13_swiglu_k<true>), dim3(nwg), dim3(W4_THREADS), stream,
                    static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w13),
                    static_cast<uint16_t*>(gu), static_cast<uint16_t*>(h), M, F, K, ldx, ldw, ldgu, ldh);
  else
#endif
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_w13_swiglu_k<false>), dim3(nwg), dim3(W4_THREADS), stream,
                    static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w13),
                    static_cast<uint16_t*>(gu), static_cast<uint16_t*>(h), M, F, K, ldx, ldw, ldgu, ldh);
  MXK_RETURN_LAUNCH_STATUS();
}

// C = A . Bt^T with the rotary embedding applied to output columns
// [0, rope_cols) in the epilogue (the q / k heads of a fused QKV
// projection, head_dim 128; row t at position t % S; rcos / rsin [S][64]
// fp32): the default schedule's K loop (52) with EPI 5, so q / k leave
// rotated and the stand-alone RoPE pass over them disappears.  Bit for bit
// the GEMM followed by that pass.  Tiled shapes only (M, N % 256, K % 64,
// S % 256, M % S, rope_cols % 128); hipErrorInvalidValue otherwise.
MXK_API int mxk_gemm_bf16_rope(const void* A, const void* Bt, void* C, int M, int N, int K,
                               int lda, int ldb, int ldc, const float* rcos, const float* rsin,
                               int S, int rope_cols, hipStream_t stream) {
  auto al = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK || lda % 8 || ldb % 8 ||
      ldc % 8 || S <= 0 || S % 256 || M % S || rope_cols < 0 || rope_cols % 128 ||
      rope_cols > N || !al(A) || !al(Bt) || !al(C) || !rcos || !rsin || !al(rcos) || !al(rsin))
    return static_cast<int>(hipErrorInvalidValue);
  MXK_LAUNCH_GEMM((mxk_gemm_bf16_tn_w4k<1, 5, 0, 1>), dim3((M / BM) * (N / BN)), dim3(W4_THREADS),
                  stream, static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(Bt),
                  static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc, rcos, rsin, S, rope_cols);
  MXK_RETURN_LAUNCH_STATUS();
}

// 1 if (M, N, K) takes the tiled MFMA fast path.
MXK_API int mxk_gemm_bf16_tn_is_fast(int M, int N, int K) {
  return (M % BM == 0) && (N % BN == 0) && (K % BK == 0);
}
