// bf16 TN GEMM schedule A/B records, built only into the experiments library
// (`make gemm-exp` -> libmxkernels_exp.so; -DMXK_GEMM_EXPERIMENTS), reached
// through mxk_gemm_bf16_tn_variant (gemm_bf16.hip) -> mxk_gemm_tn_exp_launch.
// The schedule list and what each measured is in gemm_bf16.hip's header.
#include <map>
#include <mutex>
#include <tuple>
#include "gemm_tn_core.h"

// ---------------------------------------------------------------------------
// w4i: the three-barrier K-tile.  Per K-tile (stage s in buffer X, stage
// s+1 in Y), m = MFMA index 0..127 (k-half 0: m < 64):
//   m  1..15 odd   A k-half-1 fragments from X (8 ds_read_b128)
//   m  19          lgkmcnt(0) + barrier #1: X.A consumed by every wave
//   m 21..49 /4    B k-half-1 fragments from X
//   m 23..51 /4    DMA of stage s+2, A pieces, into X.A (refill in place)
//   m  55          lgkmcnt(0) + barrier #2: X.B consumed
//   m 57..  /BSP   DMA of stage s+2, B pieces, into X.B
//   m  B3          vmcnt(8 + NB3) + barrier #3: stage s+1 landed everywhere
//   m  B3+1..  odd next K-tile's k-half-0 fragments from Y (B, then A: the
//                  order its MFMAs consume them)
// (LATE: B3 = 96, BSP = 6 — the last B piece goes out after barrier #3;
// otherwise B3 = 91, BSP = 4.)  A first version of this schedule computed
// the stage-dependent addresses per K-tile; hipcc hoisted that arithmetic
// (~20 SALU) ahead of the first MFMA while the matrix pipe drained, so:
//  * the loop is unrolled by two, so X/Y (and every M0 value) are
//    compile-time per parity;
//  * the k step is the DMA's SGPR soffset on a fixed panel descriptor
//    (one s_add per K-tile) instead of a new descriptor base per stage;
//  * the last two K-tiles run without DMA (no clamped re-reads of the last
//    stage), the last one without the next-k0 reads or barrier #3.
// MODE 1: DMA of stage s+2, vmcnt(8 + NB3) at barrier #3; MODE 2: no DMA,
// vmcnt(0) at barrier #3 (stage s+1 is the last one issued); MODE 3: no
// DMA, no barrier #3, no next-k0 reads (last K-tile).
template <int PAR, int MODE, int LATE, int R1 = 0>
__device__ __forceinline__ void w4i_ktile(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                          bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                          bf16x8_t (&f1b)[8], char* smem, int a_base, int b_base,
                                          int off_k0, int off_k1, const DmaK& dma_a,
                                          const DmaK& dma_b, int kb2, int wave_s, int par = 0) {
  constexpr int SUB = 2048;
  constexpr int B3 = LATE ? 96 : 91;
  constexpr int BSP = LATE ? 6 : 4;
  constexpr int NB3 = (B3 - 57) / BSP + 1 < 8 ? (B3 - 57) / BSP + 1 : 8;
  const int px = PAR == 2 ? par : PAR;
  char* X = smem + px * W4B_STAGE_BYTES;
  char* Y = smem + (px ^ 1) * W4B_STAGE_BYTES;
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = h * 64 + i * 8 + j;
        if (h == 0) mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
        else mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
        // R1 1: A k-half-1 reads at even m 0..14 and barrier #1 after m 21
        // (7 MFMAs between the last read and its lgkmcnt(0), as hipBLASLt)
        if (m < 16 && (m & 1) == (R1 ? 0 : 1))
          f1a[m >> 1] = lds_read_b128(X + a_base + (m >> 1) * SUB + off_k1);
        if (MODE == 1 && m == (R1 ? 21 : 19)) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
        }
        if (m >= 20 && m < 52 && (m & 3) == 1)
          f1b[(m - 21) >> 2] = lds_read_b128(X + b_base + ((m - 21) >> 2) * SUB + off_k1);
        if (MODE == 1 && m >= 20 && m < 52 && (m & 3) == 3)
          dma_a.issue(X, (m - 23) >> 2, kb2, wave_s);
        if (MODE == 1 && m == 55) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
        }
        if (MODE == 1 && m >= 57 && (m - 57) % BSP == 0 && (m - 57) / BSP < 8)
          dma_b.issue(X + W4B_OP_BYTES, (m - 57) / BSP, kb2, wave_s);
        if (MODE != 3 && m == B3) {
          if constexpr (MODE == 1) vm_wait<8 + NB3>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        if (MODE != 3 && m > B3 && m < B3 + 32 && ((m - B3) & 1)) {
          const int r = (m - B3 - 1) >> 1;
          if (r < 8) f0b[r] = lds_read_b128(Y + b_base + r * SUB + off_k0);
          else f0a[r - 8] = lds_read_b128(Y + a_base + (r - 8) * SUB + off_k0);
        }
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

// SCHED 1 ("HB"): every LDS read, DMA piece, wait and barrier at the MFMA
// position hipBLASLt's gfx950 MT256x256x64 loop puts it (its disassembly,
// instruction after MFMA m): A k1 reads at even m 0..14, lgkmcnt(0) after 20
// + barrier after 21; B k1 reads 24..42; A pieces 22..34 (5) + 52..58 (3);
// lgkmcnt(0) after 50 + barrier after 51; B pieces 61, 64, 85, 87, 89, 96,
// 100, 124; vmcnt(13) after 91 + barrier after 92 (three pieces still to
// go); next-k0 reads 93..123 (front-loaded).

// 2: two barriers)
template <int SCHED, int PAR, int MODE, int LATE, int R1>
__device__ __forceinline__ void ktile_sched(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                            bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                            bf16x8_t (&f1b)[8], char* smem, int a_base, int b_base,
                                            int off_k0, int off_k1, const DmaK& dma_a,
                                            const DmaK& dma_b, int kb2, int wave_s, int par = 0) {
  if constexpr (SCHED == 1)
    w4j_ktile<SchedHB, PAR, MODE>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                  dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 3)
    w4j_ktile<mxk::SchedEarlyB, PAR, MODE>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                           off_k1, dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 4)
    w4j_ktile<mxk::SchedSpreadK0, PAR, MODE>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                             off_k1, dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 5)   // SchedHB, B fragment outer
    w4j_ktile<SchedHB, PAR, MODE, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                     dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 6)   // SchedHB with raised wave priority
    w4j_ktile<SchedHB, PAR, MODE, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                        off_k1, dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 7)
    w4j_ktile<mxk::SchedOneBarrier, PAR, MODE>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                               off_k1, dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 8)
    w4j_ktile<mxk::SchedOneBarrierSpread, PAR, MODE>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base,
                                                     off_k0, off_k1, dma_a, dma_b, kb2, wave_s, par);
  else if constexpr (SCHED == 2)
    w4j_ktile<SchedTwoBarrier, PAR, MODE>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                          off_k1, dma_a, dma_b, kb2, wave_s, par);
  else
    w4i_ktile<PAR, MODE, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                   dma_a, dma_b, kb2, wave_s, par);
}

template <int MAP, int EPI, int LATE = 0, int R1 = 0, int SCHED = 0, int ROT = 0, int STAG = 0,
          int ALN = 0, int SWM = 7>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4i(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  if constexpr (STAG > 0) {
    // STAG: staggered first round.  The first 256 workgroups (one per CU)
    // start in four groups STAG x ~1024 clocks apart (group = CU slot within
    // the XCD mod 4), so the workgroups of a round finish, and burst their C
    // tiles to HBM, at four moments instead of one; later workgroups inherit
    // the offset from the CU they land on.
    if (blockIdx.x < 256) {
      const int g = __builtin_amdgcn_readfirstlane((blockIdx.x >> 3) & 3);
      for (int i = 0; i < g * STAG; ++i) __builtin_amdgcn_s_sleep(16);
    }
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, M / BM, N / BN, &m0, &n0);
  const DmaK dma_a = make_dmak(A, lda, m0, lane, wave_s, SWM);
  const DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wave_s, SWM);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ ((frow >> 1) & SWM);
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
  // ROT 1: the K loop starts at K-tile (xcd * ns / 8) and wraps, so the eight
  // XCDs stream different K-slices at any moment (spreads the HBM / MALL
  // channels a lockstep K sweep piles onto); ROT 2: a per-workgroup start.
  // The DMA stage offset is wrapped modulo the K extent in bytes.
  const int kbytes = K * 2;
  int rot = 0;
  if constexpr (ROT == 1) rot = ((blockIdx.x & 7) * ns / 8) * BK * 2;
  else if constexpr (ROT == 2) rot = ((blockIdx.x * 37) % ns) * BK * 2;
  rot = __builtin_amdgcn_readfirstlane(rot);
  auto wrap = [&](int kb) {
    if constexpr (ROT == 0) return kb;
    const int r = kb + rot;
    return r >= kbytes ? r - kbytes : r;
  };
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_a.issue(smem, p, wrap(0), wave_s);
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_OP_BYTES, p, wrap(0), wave_s);
  if (ns > 1) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem + W4B_STAGE_BYTES, p, wrap(BK * 2), wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p)
      dma_b.issue(smem + W4B_STAGE_BYTES + W4B_OP_BYTES, p, wrap(BK * 2), wave_s);
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
  // ALN (A/B of code placement): pad with s_nop to a 64-B boundary here,
  // then ALN - 1 more 4-B s_nops, so the K loop's first instruction moves
  // against the instruction-fetch blocks (MI355X_MICROARCH 'code-placement
  // sensitivity')
  if constexpr (ALN >= 1) {
    asm volatile(".p2alignl 6, 0xbf800000" ::: "memory");
#pragma unroll
    for (int i = 1; i < ALN; ++i) asm volatile("s_nop 0" ::: "memory");
  }
  for (; s + 2 <= ns - 2; s += 2) {
    ktile_sched<SCHED, 0, 1, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, wrap(kb), wave_s);
    ktile_sched<SCHED, 1, 1, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, wrap(kb + BK * 2), wave_s);
    kb += 2 * BK * 2;
  }
  if (s < ns - 2) {   // s even
    ktile_sched<SCHED, 0, 1, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, wrap(kb), wave_s);
    ++s;
  }
  // the last two K-tiles (or the only one): no DMA
  if (ns >= 2) {
    ktile_sched<SCHED, 2, 2, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, 0, wave_s, s & 1);
    ++s;
  }
  ktile_sched<SCHED, 2, 3, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
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
  else if constexpr (EPI == 3) {
    // DIAGNOSTIC ONLY (ablation variant 10): one lane per wave stores one value,
    // so the timing shows what the C store tail costs; the output is NOT C
    if (lane == 0) C[static_cast<size_t>(m0 + wm * 128) * ldc + n0 + wn * 128] = mxk::f2bf(acc[0][0][0]);
  } else store_block_narrow(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
}

// ---------------------------------------------------------------------------
// w4s (schedule 45, DIAGNOSTIC): schedule 26 with s_memtime stamps around the
// three waits of every DMA-carrying K-tile (cdna_hip_programming.md §7
// "In-kernel stamps").  Per wave it sums, in shader cycles: [0] wait #1 +
// barrier #1 (A k-half-1 reads retired), [1] wait #2 + barrier #2, [2] the
// stage wait vmcnt + barrier #3, [3] the K-tile period (barrier #3 to
// barrier #3), [4] the number of K-tiles summed, [5] the whole main loop.
// The stamps cost cycles themselves (each s_memtime is an SMEM round trip),
// so the numbers rank the waits; they are not the production kernel's times.
__device__ unsigned long long g_mxk_gemm_stamps[4096 * 4 * 8];

struct StampHook : mxk::NoHook {
  unsigned long long* t;      // [0..5] stamps of the current K-tile
  unsigned long long* sum;    // [0..4] running sums
  __device__ __forceinline__ void at(int p) const {
    t[p] = __builtin_amdgcn_s_memtime();
    if (p == 5) {
      sum[0] += t[1] - t[0];
      sum[1] += t[3] - t[2];
      sum[2] += t[5] - t[4];
      if (t[6]) sum[3] += t[4] - t[6];
      t[6] = t[4];
      sum[4] += 1;
    }
  }
};

template <int PAR>
__device__ __forceinline__ void w4s_ktile(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                          bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                          bf16x8_t (&f1b)[8], char* smem, int a_base, int b_base,
                                          int off_k0, int off_k1, const DmaK& dma_a,
                                          const DmaK& dma_b, int kb2, int wave_s,
                                          const StampHook& h) {
  w4j_ktile<SchedHB, PAR, 1, 0, 0, false, StampHook>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base,
                                                     off_k0, off_k1, dma_a, dma_b, kb2, wave_s, 0,
                                                     0, h);
}

__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4s(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  int m0, n0;
  w4b_tile<1>(blockIdx.x, gridDim.x, M / BM, N / BN, &m0, &n0);
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
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_a.issue(smem + W4B_STAGE_BYTES, p, BK * 2, wave_s);
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_STAGE_BYTES + W4B_OP_BYTES, p, BK * 2, wave_s);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  unsigned long long t[7] = {0, 0, 0, 0, 0, 0, 0}, sum[5] = {0, 0, 0, 0, 0};
  const StampHook h{{}, t, sum};
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  int s = 0;
  int kb = 2 * BK * 2;
  for (; s + 2 <= ns - 2; s += 2) {
    w4s_ktile<0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a, dma_b, kb,
                 wave_s, h);
    w4s_ktile<1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a, dma_b,
                 kb + BK * 2, wave_s, h);
    kb += 2 * BK * 2;
  }
  if (s < ns - 2) {
    w4s_ktile<0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a, dma_b, kb,
                 wave_s, h);
    ++s;
  }
  ktile_sched<1, 2, 2, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                             dma_b, 0, wave_s, s & 1);
  ++s;
  ktile_sched<1, 2, 3, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                             dma_b, 0, wave_s, s & 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mxk::mfma_drain(acc);
  const unsigned long long t_end = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  mxk::store_block_lds<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane,
                             smem + wave_s * mxk::kStoreLdsWave);
  const int slot = static_cast<int>(blockIdx.x) * 4 + wave_s;
  if (lane == 0 && slot < 4096 * 4) {
    unsigned long long* o = g_mxk_gemm_stamps + slot * 8;
    o[0] = sum[0];
    o[1] = sum[1];
    o[2] = sum[2];
    o[3] = sum[3];
    o[4] = sum[4];
    o[5] = t_end - t_start;
    o[6] = t_start;
    o[7] = t_end;
  }
}

// copy the stamps of the last schedule-45 launch: n values (8 per wave)
MXK_API int mxk_gemm_stamps_read(void* dst, int n) {
  const int cap = 4096 * 4 * 8;
  return static_cast<int>(hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_mxk_gemm_stamps),
                                              sizeof(unsigned long long) * (n < cap ? n : cap)));
}

// ---------------------------------------------------------------------------
// w4ip (schedule 5): w4i made persistent (grid <= one workgroup per CU,
// tiles t = blockIdx.x + r * grid).  Between tiles the LDS is free once every
// wave passed the last K-tile (barrier), so the next tile's two prologue
// stages are issued BEFORE the finished tile's store tail and land under it.
// vmcnt at the top of a later tile: 32 DMA pieces then 32 stores per wave
// are outstanding, vmcnt(48) retires exactly stage 0 (16 pieces + 32 stores
// -> vmcnt(32) when K has a single stage).  Every wave runs the same trip
// count, so all reach every barrier and leave the loop together.
template <int MAP, int EPI, int SCHED = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4ip(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                      uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  static_assert(EPI == 1 || EPI == 2, "w4ip counts 32 store instructions per wave");
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int ntiles = tiles_m * tiles_n;
  const int ns = K / BK;

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;

  int t = blockIdx.x;
  int m0, n0;
  w4b_tile<MAP>(t, ntiles, tiles_m, tiles_n, &m0, &n0);
  DmaK dma_a = make_dmak(A, lda, m0, lane, wave_s);
  DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);
  auto prologue = [&]() {
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
    }
  };
  prologue();
  bool first = true;
  while (true) {
    if (first) {
      if (ns > 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ns > 1) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();

    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
#pragma unroll
    for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
    __builtin_amdgcn_s_waitcnt(0xC07F);

    int s = 0;
    int kb = 2 * BK * 2;
    for (; s + 2 <= ns - 2; s += 2) {
      ktile_sched<SCHED, 0, 1, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                     dma_a, dma_b, kb, wave_s);
      ktile_sched<SCHED, 1, 1, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                     dma_a, dma_b, kb + BK * 2, wave_s);
      kb += 2 * BK * 2;
    }
    if (s < ns - 2) {
      ktile_sched<SCHED, 0, 1, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                     dma_a, dma_b, kb, wave_s);
      ++s;
    }
    if (ns >= 2) {
      ktile_sched<SCHED, 2, 2, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                     dma_a, dma_b, 0, wave_s, s & 1);
      ++s;
    }
    ktile_sched<SCHED, 2, 3, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                   dma_a, dma_b, 0, wave_s, s & 1);
    // every wave's LDS reads retired (and no DMA is in flight): LDS is free
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    mxk::mfma_drain(acc);

    const int cm0 = m0, cn0 = n0;
    const int tn = t + static_cast<int>(gridDim.x);
    if (tn < ntiles) {
      w4b_tile<MAP>(tn, ntiles, tiles_m, tiles_n, &m0, &n0);
      dma_a = make_dmak(A, lda, m0, lane, wave_s);
      dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);
      prologue();
    }
    store_block_wide<EPI == 2>(acc, C, ldc, cm0 + wm * 128, cn0 + wn * 128, lane);
    if (tn >= ntiles) break;
    t = tn;
    first = false;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ---------------------------------------------------------------------------
// w4t (schedule 31): persistent schedule 26 whose C store tail is trickled
// into the next tile's main loop instead of burst at the end of each tile.
//
// The store tail costs ~3.4 % at 8192^3 (no-store ablation, variant 10):
// every CU finishes its tile at the same moment and 256 x 128 KiB = 32 MiB
// go to HBM at once, while the next tiles' first DMA waits sit behind those
// stores (vmcnt counts loads and stores together, in issue order).  Here a
// tile's C leaves in two halves through the same LDS staging as schedule 26
// (whole-line stores): rows 64..127 of each wave block as a 16 MiB burst
// issued AFTER the next tile's two prologue stages (so the first stage wait
// does not include them), rows 0..63 kept in 64 VGPRs (16 x 16 B per lane)
// and stored one whole-line instruction per K-tile during the next tile's
// first 16 K-tiles (MFMA 3, ahead of that K-tile's DMA pieces).  Waits: the
// first K-tile's stage wait lets the 16 burst stores and its trickle store
// stay in flight (vmcnt 30), the other trickle K-tiles their one store (14).
// Needs K >= 18 * 64 (16 trickle K-tiles + the two DMA-less tails); the
// launcher runs schedule 26 below that.
struct SchedHBTrk0 : mxk::SchedHB { static constexpr int VM3 = 30; };
struct SchedHBTrk0L : mxk::SchedHB { static constexpr int VM3 = 22; };
struct SchedHBTrk : mxk::SchedHB { static constexpr int VM3 = 14; };

// Trickle K-tiles Q, Q + 1 (of NQ): Q < 16 stores VGPR vector buf[Q] (C row
// 4 Q + lane/16 of the previous tile's wave block), 16 <= Q < 24 the LDS
// vector Q - 16 of rows 64..95 (lane-linear, 1 KiB per vector per wave).
template <int Q, int NQ, class S0>
__device__ __forceinline__ void trickle_ktiles(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                               bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                               bf16x8_t (&f1b)[8], char* smem, int a_base,
                                               int b_base, int off_k0, int off_k1,
                                               const DmaK& dma_a, const DmaK& dma_b, int& kb,
                                               int wave_s, const u32x4_t (&buf)[16], uint16_t* tp,
                                               size_t tstride, const char* lsrc) {
  auto one = [&](auto qc, auto parc, int kbx) {
    constexpr int q = decltype(qc)::value;
    constexpr int par = decltype(parc)::value;
    using SS = std::conditional_t<q == 0, S0, SchedHBTrk>;
    if constexpr (q < 16) {
      const mxk::TrickleStore h{{}, buf[q], tp + q * tstride};
      w4j_ktile<SS, par, 1, 0, 0, false, mxk::TrickleStore>(acc, f0a, f0b, f1a, f1b, smem, a_base,
                                                       b_base, off_k0, off_k1, dma_a, dma_b, kbx,
                                                       wave_s, 0, 0, h);
    } else {
      u32x4_t v;
      const mxk::TrickleLds h{{}, lsrc + (q - 16) * 1024, tp + q * tstride, v};
      w4j_ktile<SS, par, 1, 0, 0, false, mxk::TrickleLds>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base,
                                                     off_k0, off_k1, dma_a, dma_b, kbx, wave_s, 0,
                                                     0, h);
    }
  };
  one(std::integral_constant<int, Q>{}, std::integral_constant<int, 0>{}, kb);
  one(std::integral_constant<int, Q + 1>{}, std::integral_constant<int, 1>{}, kb + BK * 2);
  kb += 2 * BK * 2;
  if constexpr (Q + 2 < NQ)
    trickle_ktiles<Q + 2, NQ, S0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                  dma_a, dma_b, kb, wave_s, buf, tp, tstride, lsrc);
}

// LQ (schedule 32): the LDS grows to the full 160 KiB and its last 32 KiB
// hold rows 64..95 of each wave block (8 KiB per wave), trickled in K-tiles
// 16..23, so only rows 96..127 (8 MiB chip-wide) leave as a burst.
template <int MAP, bool LQ>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4t(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  constexpr int XTRA = LQ ? 32768 : 0;
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES + XTRA];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int ntiles = tiles_m * tiles_n;
  const int ns = K / BK;                       // >= 18 (launcher)

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;
  const int rr = lane >> 4, cc = (lane & 15) * 8;
  const size_t tstride = static_cast<size_t>(4) * ldc;   // trickle vector it -> it + 1

  int t = blockIdx.x;
  int m0, n0;
  w4b_tile<MAP>(t, ntiles, tiles_m, tiles_n, &m0, &n0);
  DmaK dma_a = make_dmak(A, lda, m0, lane, wave_s);
  DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);
  auto prologue = [&]() {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem, p, 0, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_OP_BYTES, p, 0, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem + W4B_STAGE_BYTES, p, BK * 2, wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_b.issue(smem + W4B_STAGE_BYTES + W4B_OP_BYTES, p, BK * 2, wave_s);
  };
  prologue();
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // stage 0
  __builtin_amdgcn_s_barrier();

  u32x4_t buf[16];                                    // previous tile's rows 0..63
  uint16_t* tp = C;
  bool trickle = false;
  while (true) {
    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
#pragma unroll
    for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
    __builtin_amdgcn_s_waitcnt(0xC07F);

    int s = 0;
    int kb = 2 * BK * 2;
    char* xq = smem + 2 * W4B_STAGE_BYTES + wave_s * 8192 + lane * 16;   // LQ vectors
    if (trickle) {
      if constexpr (LQ) {
        trickle_ktiles<0, 24, SchedHBTrk0L>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                            off_k1, dma_a, dma_b, kb, wave_s, buf, tp, tstride, xq);
        s = 24;
      } else {
        trickle_ktiles<0, 16, SchedHBTrk0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0,
                                           off_k1, dma_a, dma_b, kb, wave_s, buf, tp, tstride, xq);
        s = 16;
      }
    }
    for (; s + 2 <= ns - 2; s += 2) {
      ktile_sched<1, 0, 1, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                 dma_a, dma_b, kb, wave_s);
      ktile_sched<1, 1, 1, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                 dma_a, dma_b, kb + BK * 2, wave_s);
      kb += 2 * BK * 2;
    }
    if (s < ns - 2) {
      ktile_sched<1, 0, 1, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                                 dma_a, dma_b, kb, wave_s);
      ++s;
    }
    ktile_sched<1, 2, 2, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                               dma_a, dma_b, 0, wave_s, s & 1);
    ++s;
    ktile_sched<1, 2, 3, 1, 0>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1,
                               dma_a, dma_b, 0, wave_s, s & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mxk::mfma_drain(acc);
    // every wave's last fragment reads retired: the stages are free for staging
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();

    char* lds = smem + wave_s * mxk::kStoreLdsWave;
    uint16_t* row0 = C + static_cast<size_t>(m0 + wm * 128 + rr) * ldc + n0 + wn * 128 + cc;
    const int tn = t + static_cast<int>(gridDim.x);
    if (tn >= ntiles) {
      u32x4_t hi[16];
      mxk::stage_half(acc, 0, lane, lds, buf);
      mxk::stage_half(acc, 1, lane, lds, hi);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        __builtin_nontemporal_store(buf[it], reinterpret_cast<u32x4_t*>(row0 + it * tstride));
        __builtin_nontemporal_store(hi[it], reinterpret_cast<u32x4_t*>(row0 + (16 + it) * tstride));
      }
      break;
    }
    u32x4_t hi[16];
    mxk::stage_half(acc, 0, lane, lds, buf);
    mxk::stage_half(acc, 1, lane, lds, hi);
    if constexpr (LQ) {
#pragma unroll
      for (int it = 0; it < 8; ++it) *reinterpret_cast<u32x4_t*>(xq + it * 1024) = hi[it];
    }
    tp = row0;
    __builtin_amdgcn_s_barrier();                     // every wave read its slice back
    t = tn;
    w4b_tile<MAP>(t, ntiles, tiles_m, tiles_n, &m0, &n0);
    dma_a = make_dmak(A, lda, m0, lane, wave_s);
    dma_b = make_dmak(Bt, ldb, n0, lane, wave_s);
    prologue();
#pragma unroll
    for (int it = LQ ? 8 : 0; it < 16; ++it)
      __builtin_nontemporal_store(hi[it], reinterpret_cast<u32x4_t*>(tp + (16 + it) * tstride));
    // stage 0 landed (stage 1 and the 16 / 8 burst stores still in flight)
    if constexpr (LQ) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    trickle = true;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// pp8 (schedule 19): 8 waves, two per SIMD, in a compute / load ping-pong.
// The 4-wave kernel above runs one wave per SIMD, so every barrier, LDS
// latency and DMA wait of that wave leaves the SIMD's matrix pipe idle (PMC:
// MFMA busy 83.5 %).  Here a 512-thread workgroup keeps the 256x256 tile but
// splits it over two groups of four waves (group g = waves 4g..4g+3, one wave
// of each group per SIMD); each wave owns 128 x 64 of C (32 16x16x32 tiles,
// 128 AGPR accumulators) and ONE K-tile of fragments (96 VGPRs).  Every wave
// runs the same straight-line sequence per K-tile t
//     L_t: read K-tile t's fragments from LDS  | barrier
//     C_t: its 64 MFMAs                        | barrier
// and group 1 runs it one phase behind group 0 (one extra barrier first), so
// in every phase one wave per SIMD issues MFMAs while its partner reads LDS.
// Group 0 also moves the data: in L_t it issues the LDS-DMA of stage t+1 into
// the buffer both groups finished reading in the two phases before, and waits
// for it at the end of C_t.  No branch touches fragments or accumulators, so
// the register allocation is the single-K-tile one.  Same LDS image, swizzle,
// DMA piece map (group 0 plays the 4 waves of make_dmak) and store tail as the
// 4-wave kernel.  Measured (profiles/r2_gemm_ab/pp8_pingpong_ab.log): correct
// (bit-identical to schedule 6) but 6 % slower at 8192^3 and 11 % at 16384^3:
// with two 64 KiB stages the DMA of stage t+1 can only start when both groups
// have left buffer t-1, so it gets ~1 phase (~1000 cycles) to land against
// ~100-200 MFMAs (1500-3000 cycles) in schedule 6, and every K-tile pays two
// workgroup barriers.  Kept as an A/B variant, not the default.
constexpr int PP_THREADS = 512;

__device__ __forceinline__ void pp_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int PAR>
__device__ __forceinline__ void pp_load(bf16x8_t (&fa)[2][8], bf16x8_t (&fb)[2][4],
                                        const char* smem, int a_base, int b_base, int off_k0,
                                        int off_k1) {
  constexpr int SUB = 2048;
  const char* X = smem + PAR * W4B_STAGE_BYTES;
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[0][j] = lds_read_b128(X + b_base + j * SUB + off_k0);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[0][i] = lds_read_b128(X + a_base + i * SUB + off_k0);
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[1][j] = lds_read_b128(X + b_base + j * SUB + off_k1);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[1][i] = lds_read_b128(X + a_base + i * SUB + off_k1);
}

__device__ __forceinline__ void pp_compute(f32x4_t (&acc)[8][4], const bf16x8_t (&fa)[2][8],
                                           const bf16x8_t (&fb)[2][4]) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mfma_16x16x32_agpr(acc[i][j], fb[h][j], fa[h][i]);
}

template <int PAR>
__device__ __forceinline__ void pp_dma(char* smem, const DmaK& dma_a, const DmaK& dma_b, int kb,
                                       int wl) {
  char* X = smem + PAR * W4B_STAGE_BYTES;
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_a.issue(X, p, kb, wl);
#pragma unroll
  for (int p = 0; p < 8; ++p) dma_b.issue(X + W4B_OP_BYTES, p, kb, wl);
}

// K-tile t with buffer parity PAR = t & 1: L_t | barrier | C_t | barrier
template <int PAR>
__device__ __forceinline__ void pp_ktile(f32x4_t (&acc)[8][4], bf16x8_t (&fa)[2][8],
                                         bf16x8_t (&fb)[2][4], char* smem, int a_base, int b_base,
                                         int off_k0, int off_k1, const DmaK& dma_a,
                                         const DmaK& dma_b, int g, int wl, int t, int ns) {
  pp_load<PAR>(fa, fb, smem, a_base, b_base, off_k0, off_k1);
  // stage t+1 into the other buffer (read by group 0 in L_{t-1}, group 1 in
  // L_{t-1} one phase later: both done); stage 1 came with the prologue
  if (g == 0 && t >= 1 && t + 1 < ns) pp_dma<PAR ^ 1>(smem, dma_a, dma_b, (t + 1) * BK * 2, wl);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  pp_fence();
  __builtin_amdgcn_s_barrier();
  pp_fence();
  pp_compute(acc, fa, fb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // group 0: stage t+1 landed
  pp_fence();
  __builtin_amdgcn_s_barrier();
  pp_fence();
}

template <int MAP, int PRIO>
__global__ void __launch_bounds__(PP_THREADS, 1)
mxk_gemm_bf16_tn_pp8(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2;          // group
  const int wl = wave & 3;          // wave within the group (DMA piece map)
  const int wm = wl & 1;            // 128-row half of the tile
  const int wn = (wl >> 1) + 2 * g; // 64-column quarter
  if constexpr (PRIO) {
    if (g == 1) __builtin_amdgcn_s_setprio(1);   // the younger half loses arbitration otherwise
  }
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, M / BM, N / BN, &m0, &n0);
  const DmaK dma_a = make_dmak(A, lda, m0, lane, wl);
  const DmaK dma_b = make_dmak(Bt, ldb, n0, lane, wl);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 4 * SUB;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t fa[2][8], fb[2][4];

  const int ns = K / BK;
  // prologue: group 0 moves stage 0, group 1 stage 1 (each as the 4-wave map)
  if (g == 0) pp_dma<0>(smem, dma_a, dma_b, 0, wl);
  else if (ns > 1) pp_dma<1>(smem, dma_a, dma_b, BK * 2, wl);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (g == 1) __builtin_amdgcn_s_barrier();      // group 1 runs one phase behind
  pp_fence();
  int t = 0;
  for (; t + 2 <= ns; t += 2) {
    pp_ktile<0>(acc, fa, fb, smem, a_base, b_base, off_k0, off_k1, dma_a, dma_b, g, wl, t, ns);
    pp_ktile<1>(acc, fa, fb, smem, a_base, b_base, off_k0, off_k1, dma_a, dma_b, g, wl, t + 1, ns);
  }
  if (t < ns)
    pp_ktile<0>(acc, fa, fb, smem, a_base, b_base, off_k0, off_k1, dma_a, dma_b, g, wl, t, ns);
  mxk::mfma_drain(acc);
  store_block_wide<true, 8, 4>(acc, C, ldc, m0 + wm * 128, n0 + wn * 64, lane);
  if (g == 0) __builtin_amdgcn_s_barrier();      // same barrier count as group 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


int mxk_gemm_bf16_tn_ring_launch(int slots, const void* A, const void* Bt, void* C, int M, int N,
                                 int K, int lda, int ldb, int ldc, hipStream_t stream);

namespace {
// compute units of the current device (persistent grids: one workgroup per CU)
int num_cus() {
  static thread_local int dev_cached = -1, cus = 256;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && dev != dev_cached) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
    dev_cached = dev;
  }
  return cus;
}

template <int MAP, int EPI, int LATE, int R1 = 0, int SCHED = 0, int ROT = 0, int STAG = 0, int ALN = 0,
          int SWM = 7>
void launch_w4i(int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b, uint16_t* c,
                int M, int N, int K, int lda, int ldb, int ldc) {
  hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4i<MAP, EPI, LATE, R1, SCHED, ROT, STAG, ALN, SWM>), dim3(nwg),
                     dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc);
}
}  // namespace

// Launch A/B record `v` (any schedule the production build does not carry);
// ---- staggered rounds (schedules 54 / 55, mxk_gemm_bf16_tn_w4j_stag in
// gemm_tn_core.h): per-(device, stream) workspace of fp32 partial tiles and
// their flags, zeroed once and reset by every consumer.  54: uncached memory
// (the two halves meet through memory, whatever XCD each runs on); 55: plain
// device memory (the halves meet in their XCD's L2 - correct only while
// workgroup b runs on XCD b % 8, an A/B of the uncached traffic's price).
MXK_API int mxk_gemm_stagger_plan(long T, int K, int cus);
MXK_API int mxk_gemm_available_cus(void);

namespace {
struct StagWs {
  float* ws = nullptr;
  int* flags = nullptr;
  int slots = 0;
};
std::mutex g_stag_mu;
std::map<std::tuple<int, hipStream_t, bool>, StagWs> g_stag;

const StagWs* stag_ws(hipStream_t stream, int slots, bool uncached) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_stag_mu);
  StagWs& w = g_stag[{dev, stream, uncached}];
  if (w.slots >= slots) return &w;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
    return nullptr;                     // no allocation inside a capture: plain schedule
  if (w.ws) (void)hipFree(w.ws);
  if (w.flags) (void)hipFree(w.flags);
  w = StagWs{};
  const unsigned fl_kind = uncached ? hipDeviceMallocUncached : hipDeviceMallocDefault;
  void *ws = nullptr, *fl = nullptr;
  if (hipExtMallocWithFlags(&ws, static_cast<size_t>(slots) * BM * BN * 4, fl_kind) != hipSuccess ||
      hipExtMallocWithFlags(&fl, static_cast<size_t>(slots) * 4, fl_kind) != hipSuccess ||
      hipMemsetAsync(fl, 0, static_cast<size_t>(slots) * 4, stream) != hipSuccess) {
    if (ws) (void)hipFree(ws);
    if (fl) (void)hipFree(fl);
    return nullptr;
  }
  w.ws = static_cast<float*>(ws);
  w.flags = static_cast<int*>(fl);
  w.slots = slots;
  return &w;
}

void launch_stag_xcd(int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b, uint16_t* c,
                     int M, int N, int K, int lda, int ldb, int ldc) {
  const int cx = mxk_gemm_available_cus() / 8;
  const long tx = nwg / 8;
  const bool ok = nwg % 8 == 0 && cx > 0 && tx >= 2 * cx && K % (2 * BK) == 0 && K >= 4 * BK;
  const StagWs* w = ok ? stag_ws(stream, 4 * cx, true) : nullptr;
  if (!w) {
    hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4j<1, 4>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc);
    return;
  }
  hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4j_stag<1, 4, 1>), dim3(nwg + 8 * cx), dim3(W4_THREADS), 0,
                     stream, a, b, c, M, N, K, lda, ldb, ldc, w->ws, w->flags, cx);
}

void launch_stag(bool uncached, int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b,
                 uint16_t* c, int M, int N, int K, int lda, int ldb, int ldc) {
  const int sx = mxk_gemm_stagger_plan(nwg, K, mxk_gemm_available_cus());
  const StagWs* w = sx > 0 ? stag_ws(stream, 8 * sx, uncached) : nullptr;
  if (!w) {
    hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4j<1, 4>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc);
    return;
  }
  hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4j_stag<1, 4>), dim3(nwg + 8 * sx), dim3(W4_THREADS), 0,
                     stream, a, b, c, M, N, K, lda, ldb, ldc, w->ws, w->flags, sx);
}
}  // namespace

// returns 0, or -1 when v is not an experiments schedule.
int mxk_gemm_tn_exp_launch(int v, int nwg, hipStream_t stream, const void* A, const void* Bt,
                           void* C, int M, int N, int K, int lda, int ldb, int ldc) {
  auto* a = static_cast<const uint16_t*>(A);
  auto* b = static_cast<const uint16_t*>(Bt);
  auto* c = static_cast<uint16_t*>(C);
  switch (v) {
    case 0: launch_w4i<1, 2, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    // 26 as the full-flag template instantiated it before the production
    // kernel got its own (mxk_gemm_bf16_tn_w4j): same loop, other registers
    case 46: launch_w4i<1, 4, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 48:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4k<1, 4, 1>), dim3(nwg), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    case 49:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4k<1, 4, 2>), dim3(nwg), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    case 50:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4k<1, 4, 4>), dim3(nwg), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    case 56:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4j<1, 4, true>), dim3(nwg), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    case 57: launch_stag_xcd(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 54:
    case 55: launch_stag(v == 54, nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 53:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4k<1, 4, 8>), dim3(nwg), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    case 51:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4k<1, 4, 7>), dim3(nwg), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    case 31:
    case 32: {
      if (K < (v == 31 ? 18 : 26) * BK) {   // fewer K-tiles than the trickle phase needs
        launch_w4i<1, 4, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc);
        break;
      }
      const int grid = nwg < num_cus() ? nwg : num_cus();
      if (v == 31)
        hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4t<1, false>), dim3(grid), dim3(W4_THREADS), 0, stream,
                           a, b, c, M, N, K, lda, ldb, ldc);
      else
        hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4t<1, true>), dim3(grid), dim3(W4_THREADS), 0, stream,
                           a, b, c, M, N, K, lda, ldb, ldc);
      break;
    }
    case 2: launch_w4i<1, 1, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 3: launch_w4i<1, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 4: launch_w4i<1, 1, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 5: {
      const int grid = nwg < num_cus() ? nwg : num_cus();
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4ip<1, 2>), dim3(grid), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    }
    case 7: launch_w4i<1, 2, 1, 0, 2>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 8: launch_w4i<1, 1, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 10: launch_w4i<1, 3, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 13: launch_w4i<1, 2, 1, 0, 3>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 14: launch_w4i<1, 2, 1, 0, 4>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 15: launch_w4i<1, 2, 1, 0, 5>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 16: launch_w4i<1, 2, 1, 0, 6>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 17: launch_w4i<1, 2, 1, 0, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 18: launch_w4i<1, 2, 1, 0, 1, 2>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 21: launch_w4i<1, 2, 1, 0, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 22: launch_w4i<1, 2, 1, 0, 1, 0, 2>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 23: launch_w4i<1, 2, 1, 0, 1, 0, 4>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 24: launch_w4i<1, 2, 1, 0, 1, 0, 8>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 25: launch_w4i<1, 1, 1, 0, 1, 0, 4>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 27: launch_w4i<1, 4, 1, 0, 7>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 28: launch_w4i<1, 4, 1, 0, 8>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 33: launch_w4i<1, 4, 1, 0, 1, 0, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 34: launch_w4i<1, 4, 1, 0, 1, 0, 0, 23>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 35: launch_w4i<1, 4, 1, 0, 1, 0, 0, 14>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 36: launch_w4i<1, 4, 1, 0, 1, 0, 0, 24>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 37: launch_w4i<1, 4, 1, 0, 1, 0, 0, 0, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 38: launch_w4i<1, 4, 1, 0, 1, 0, 0, 0, 4>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 39: launch_w4i<1, 4, 1, 0, 1, 0, 0, 0, 6>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 40: launch_w4i<1, 4, 1, 0, 1, 0, 0, 0, 5>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 41: launch_w4i<2, 4, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 42: launch_w4i<3, 4, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 43: launch_w4i<4, 4, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 44: launch_w4i<1, 4, 1, 0, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 45:
      hipLaunchKernelGGL(mxk_gemm_bf16_tn_w4s, dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N,
                         K, lda, ldb, ldc);
      break;
    case 29: mxk_gemm_bf16_tn_ring_launch(4, A, Bt, C, M, N, K, lda, ldb, ldc, stream); break;
    case 30: mxk_gemm_bf16_tn_ring_launch(5, A, Bt, C, M, N, K, lda, ldb, ldc, stream); break;
    case 19:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_pp8<1, 0>), dim3(nwg), dim3(PP_THREADS), 0, stream, a, b,
                         c, M, N, K, lda, ldb, ldc);
      break;
    case 20:
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_pp8<1, 1>), dim3(nwg), dim3(PP_THREADS), 0, stream, a, b,
                         c, M, N, K, lda, ldb, ldc);
      break;
    case 11:
    case 12: {
      const int grid = nwg < num_cus() ? nwg : num_cus();
      if (v == 11)
        hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4ip<1, 1, 1>), dim3(grid), dim3(W4_THREADS), 0, stream,
                           a, b, c, M, N, K, lda, ldb, ldc);
      else
        hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4ip<1, 2, 1>), dim3(grid), dim3(W4_THREADS), 0, stream,
                           a, b, c, M, N, K, lda, ldb, ldc);
      break;
    }
    default:
      return -1;
  }
  return 0;
}
