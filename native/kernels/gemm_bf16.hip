// CDNA4 bf16 MFMA GEMM — the validator's compute payload (BASELINE config 3).
//
//   C[M][N] (bf16) = A[M][K] (bf16, row-major) · Bt[N][K]^T (bf16, row-major)
//   fp32 accumulation in the MFMA accumulators.
//
// "Bt" is the nn.Linear weight layout ([out][in]); both operands are read
// K-contiguous, which is what the MFMA A/B lane maps want, so neither tile
// needs a transpose on the way into LDS.
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §5).
// The default schedule is w4i (variant 34, below); the older schedules stay
// as A/B variants (mxk_gemm_bf16_tn_variant, python -m mxk8s.validate.gemm):
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
//  * Three barriers per K-tile (hipBLASLt's gfx950 structure): the stage just
//    consumed is refilled in place with stage s+2 once each operand's last
//    fragment read retired, so DMA pieces spread over ~64 MFMAs and have
//    ~130-200 MFMAs to land; counted vmcnt, raw s_barrier.
//  * K loop unrolled by two (compile-time LDS bases), k step as the DMA's
//    soffset: no address arithmetic ahead of the MFMA stream.
//  * XCD-aware super-block tile map: 256 resident tiles = one 16x16 block,
//    8x4 per XCD (L2 reuse) and 32 panels chip-wide (Infinity Cache reuse).
#include "mx_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int TILE_BYTES = BM * BK * 2;          // 32 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;      // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;       // double buffered: 128 KiB
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) void lds_void;

// One quarter of an operand tile (64 rows x 64 k = 8 KiB) per call:
// 512 lanes x 16 B.  Lane t of the block writes LDS bytes [q*8192 + t*16, +16)
// (lane-linear per wave: wave base + lane*16), i.e. row q*64 + t/8, physical
// chunk t%8, which must hold logical chunk (t%8) ^ ((row>>1)&7).
__device__ __forceinline__ void stage_quarter(const uint16_t* __restrict__ src, int ld,
                                              int row0, int k0, char* lds_tile,
                                              int q, int tid) {
  const int row = q * 64 + (tid >> 3);
  const int pc = tid & 7;
  const int c = pc ^ ((row >> 1) & 7);
  const uint16_t* g = src + static_cast<size_t>(row0 + row) * ld + k0 + c * 8;
  char* dst = lds_tile + q * 8192 + (tid >> 6) * 1024;   // wave-uniform base
  __builtin_amdgcn_global_load_lds(g, (lds_void*)dst, 16, 0, 0);
}

__device__ __forceinline__ bf16x8_t lds_read_b128(const char* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

}  // namespace

// Main-loop schedules (selected at compile time; A/B-benchmarked in one process
// through mxk_gemm_bf16_tn_variant):
//   0: per phase {4 B + 4 A ds_reads, 1/4 of the next tile's DMA, 16 MFMA}
//   1: whole next-tile DMA issued right after the barrier; all 24 fragment
//      reads of the tile issued up front, then 64 MFMAs (compiler places the
//      counted lgkmcnt waits)
//   2: whole next-tile DMA up front; per k-step {12 reads, 32 MFMA}
template <int V>
__global__ void __launch_bounds__(NTHREADS, 2)
mxk_gemm_bf16_tn_256x256(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                         uint16_t* __restrict__ C, int M, int N, int K,
                         int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2;   // 0..1 -> 128 rows each
  const int wn = wave & 3;    // 0..3 -> 64 cols each

  // ---- block -> output tile (XCD remap, then GROUP_M swizzle) ----
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  const int tm = first_m + in_group % gsize;
  const int tn = in_group / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- fragment read offsets (bytes, within a 16-row block of a tile) ----
  // lane l reads row (l & 15), logical chunk ks*4 + (l >> 4), stored at
  // physical chunk (ks*4 + (l>>4)) ^ ((l & 15) >> 1).
  const int frow = lane & 15;
  const int fch0 = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch0 * 16;
  const int off_k1 = frow * 128 + (fch0 ^ 4) * 16;
  const int a_wave = wm * 128 * 128;   // byte offset of this wave's first A row
  const int b_wave = wn * 64 * 128;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nt = K / BK;

  // prologue: stage K tile 0 into buffer 0
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    stage_quarter(A, lda, m0, 0, smem, q, tid);
    stage_quarter(Bt, ldb, n0, 0, smem + TILE_BYTES, q, tid);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int t = 0; t < nt; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    char* nxt = smem + ((t + 1) & 1) * STAGE_BYTES;
    const bool more = (t + 1) < nt;
    const int kn = (t + 1) * BK;
    const char* As = cur + a_wave;
    const char* Bs = cur + TILE_BYTES + b_wave;

    if constexpr (V == 0) {
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int ks = ph >> 1;
        const int mh = ph & 1;
        const int koff = ks ? off_k1 : off_k0;
        bf16x8_t a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = lds_read_b128(Bs + j * 2048 + koff);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = lds_read_b128(As + (mh * 4 + i) * 2048 + koff);
        if (more) {
          stage_quarter(A, lda, m0, kn, nxt, ph, tid);
          stage_quarter(Bt, ldb, n0, kn, nxt + TILE_BYTES, ph, tid);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[mh * 4 + i][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[mh * 4 + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
      // The next tile's buffer was released by the barrier that ended tile
      // t-1, so its whole DMA can start now and has the full tile to land.
      if (more) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          stage_quarter(A, lda, m0, kn, nxt, q, tid);
          stage_quarter(Bt, ldb, n0, kn, nxt + TILE_BYTES, q, tid);
        }
      }
      if constexpr (V == 1) {
        bf16x8_t a[2][8], b[2][4];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int koff = ks ? off_k1 : off_k0;
#pragma unroll
          for (int j = 0; j < 4; ++j) b[ks][j] = lds_read_b128(Bs + j * 2048 + koff);
#pragma unroll
          for (int i = 0; i < 8; ++i) a[ks][i] = lds_read_b128(As + i * 2048 + koff);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ks][j], a[ks][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int koff = ks ? off_k1 : off_k0;
          bf16x8_t a[8], b[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = lds_read_b128(Bs + j * 2048 + koff);
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = lds_read_b128(As + i * 2048 + koff);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
      }
    }
    // Retire the next tile's DMA (issued by this wave), then a barrier so every
    // wave's DMA has landed and every wave is done reading `cur` before it is
    // overwritten by the tile after next.
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: lane holds C[m][n..n+3] for each 16x16 tile ----
  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + crow;
    uint16_t* crow_ptr = C + static_cast<size_t>(m) * ldc + n0 + wn * 64 + ccol;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4_t v = acc[i][j];
      uint2 pk;
      pk.x = mxk::pack2bf(v[0], v[1]);
      pk.y = mxk::pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(crow_ptr + j * 16) = pk;
    }
  }
}

// ---------------------------------------------------------------------------
// Schedule 3/4: 4 waves (one per SIMD), each owning a 128x128 output block
// (8x8 tiles of 16x16 -> 256 fp32 accumulators, kept in the AGPR half of the
// unified 512-entry register file), BK = 32 K-stages in an NS-deep LDS ring.
//
// Per 32-deep stage a wave issues 16 ds_read_b128 for 64 MFMAs (half the LDS
// bytes per FLOP of the 8-wave 128x64 layout); the LDS-DMA for stage s+NS-1
// is issued NS-2 stages ahead of its use, and the fragments of stage s+1 are
// read into a second register set while stage s's MFMAs run, so the matrix
// pipe is fed from registers right after every barrier.
//
// Stage s lives in LDS buffer s % NS:   [A 256 rows x 64 B | B 256 rows x 64 B]
// Row r's 16-B chunk c sits at chunk c ^ h((r >> 2) & 3), h = {0,2,3,1}: every
// 16-lane ds_read_b128 group then hits 16 distinct 16-B bank slots
// (tests/test_gemm_swizzle.py).
// ---------------------------------------------------------------------------
namespace {
constexpr int W4_BK = 32;
constexpr int W4_THREADS = 256;
constexpr int W4_OP_BYTES = 256 * W4_BK * 2;        // 16 KiB per operand per stage
constexpr int W4_STAGE_BYTES = 2 * W4_OP_BYTES;     // 32 KiB

__device__ __forceinline__ int w4_h(int q) { return (((q ^ (q >> 1)) & 1) << 1) | (q >> 1); }

// MFMA with the accumulator pinned to AGPRs ("+a"): with 256 accumulators per
// wave the compiler's own allocation shuffles them through VGPRs every trip.
// A chain of MFMAs accumulating into the same registers needs no wait states;
// the caller pads before the accumulators are read by non-MFMA code.
__device__ __forceinline__ void mfma_16x16x32_agpr(f32x4_t& acc, bf16x8_t a, bf16x8_t b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// LDS-DMA stream of one operand as `buffer_load_dwordx4 ... offen lds`: the
// operand panel (row0 .. row0+255) is a buffer resource in SGPRs, each lane's
// row/chunk offset is ONE VGPR computed once, and the piece / k offset is a
// scalar soffset — so a piece costs one VMEM instruction plus one `s_add m0`
// (no per-piece 64-bit VALU address math, no v_readfirstlane for M0; the
// hipBLASLt MT256x256x64 kernel issues its pieces the same way).
struct DmaStream {
  __amdgpu_buffer_rsrc_t rsrc;   // uniform: panel base, 256 rows * ld * 2 bytes
  uint32_t lane_off;             // per lane: (row-in-piece * ld + swizzled chunk * 8) * 2
  uint32_t piece_stride;         // uniform: rows-per-piece * ld * 2
  __device__ __forceinline__ void issue(char* lds_op, int piece, int piece_bytes, int k_bytes,
                                        int wave_s) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsrc, (lds_void*)(lds_op + piece * piece_bytes + wave_s * 1024), 16, lane_off,
        k_bytes + piece * piece_stride, 0, 0);
  }
};

// rows_per_piece = threads / 4 (64 B rows, 4 lanes per row)
__device__ __forceinline__ DmaStream make_dma(const uint16_t* src, int ld, int row0, int tid,
                                              int rows_per_piece) {
  DmaStream d;
  const uint16_t* base = src + static_cast<size_t>(row0) * ld;
  d.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, 256 * ld * 2,
                                             0x00020000);
  const int row = tid >> 2;                        // row within a piece
  const int c = (tid & 3) ^ w4_h((row >> 2) & 3);  // (row>>2)&3 is piece-invariant
  d.lane_off = static_cast<uint32_t>((row * ld + c * 8) * 2);
  d.piece_stride = static_cast<uint32_t>(rows_per_piece * ld * 2);
  return d;
}

// One quarter (64 rows x 32 k) of an operand stage = 1 glds per thread.
__device__ __forceinline__ void w4_stage_quarter(const uint16_t* __restrict__ src, int ld, int row0,
                                                 int k0, char* lds_op, int q, int tid) {
  const int row = q * 64 + (tid >> 2);
  const int c = (tid & 3) ^ w4_h((row >> 2) & 3);
  const uint16_t* g = src + static_cast<size_t>(row0 + row) * ld + k0 + c * 8;
  __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_op + q * 4096 + (tid >> 6) * 1024), 16, 0, 0);
}

// One operand stage (256 rows x 32 k) = 4 glds per thread (1 KiB per wave
// instruction = 16 rows of 64 B).
__device__ __forceinline__ void w4_stage_operand(const uint16_t* __restrict__ src, int ld, int row0,
                                                 int k0, char* lds_op, int tid) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = q * 64 + (tid >> 2);
    const int pc = tid & 3;
    const int c = pc ^ w4_h((row >> 2) & 3);
    const uint16_t* g = src + static_cast<size_t>(row0 + row) * ld + k0 + c * 8;
    char* dst = lds_op + q * 4096 + (tid >> 6) * 1024;
    __builtin_amdgcn_global_load_lds(g, (lds_void*)dst, 16, 0, 0);
  }
}
}  // namespace

// ABL (ablation, timing-only builds; outputs are wrong): 1 = skip the
// steady-state LDS-DMA, 2 = skip the fragment prefetch reads.
template <int NS, int ABL = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                    uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[NS * W4_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1;   // 0..1 -> 128 rows
  const int wn = wave & 1;    // 0..1 -> 128 cols

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const int frow = lane & 15;
  const int foff = frow * 64 + (((lane >> 4) ^ w4_h((frow >> 2) & 3)) * 16);
  const int a_off = wm * 128 * 64 + foff;               // + i*1024 for subtile i
  const int b_off = W4_OP_BYTES + wn * 128 * 64 + foff;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const DmaStream dma_a = make_dma(A, lda, m0, tid, 64);
  const DmaStream dma_b = make_dma(Bt, ldb, n0, tid, 64);

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = K / W4_BK;
  // prologue: stages 0 .. NS-2 in flight (clamped past the end)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    const int kk = (s < ns ? s : ns - 1) * W4_BK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      dma_a.issue(smem + s * W4_STAGE_BYTES, q, 4096, kk * 2, wave_s);
      dma_b.issue(smem + s * W4_STAGE_BYTES + W4_OP_BYTES, q, 4096, kk * 2, wave_s);
    }
  }
  // stage 0 landed (8 glds per later stage may stay in flight)
  if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  bf16x8_t fa[2][8], fb[2][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[0][i] = lds_read_b128(smem + a_off + i * 1024);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb[0][j] = lds_read_b128(smem + b_off + j * 1024);

  // Uniform steady state (ns is even: K % 64 == 0 on this path).  Past the
  // end the DMA re-fetches the last stage into the free buffer and the
  // fragment reads hit stale LDS: both harmless, and every trip keeps the
  // same vmcnt bookkeeping (no tail branches inside the loop).
  for (int s = 0; s < ns; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int st = s + u;
      // (1) own part of stage st+1 landed; the barrier publishes every wave's
      //     part and certifies all waves finished reading stage st-1.
      if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // (2)-(4) 64 MFMAs on stage st straight from registers.  Slotted between
      // them (so the matrix pipe never waits on issue): the 16 fragment reads
      // of stage st+1 into the other register set (one ds_read_b128 per 4
      // MFMAs) and the 8 LDS-DMA pieces of stage st+NS-1 into the buffer stage
      // st-1 used (one glds per 8 MFMAs).
      {
        const char* nb = smem + ((st + 1) % NS) * W4_STAGE_BYTES;
        const int sn = st + NS - 1;
        const int kk = (sn < ns ? sn : ns - 1) * W4_BK;
        char* buf = smem + (sn % NS) * W4_STAGE_BYTES;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            mfma_16x16x32_agpr(acc[i][j], fb[u][j], fa[u][i]);
            if ((j & 3) == 3 && ABL != 2) {
              const int r = i * 2 + (j >> 2);   // 0..15
              if (r < 8) fb[u ^ 1][r] = lds_read_b128(nb + b_off + r * 1024);
              else fa[u ^ 1][r - 8] = lds_read_b128(nb + a_off + (r - 8) * 1024);
            }
            if (j == 7 && ABL != 1) {
              if (i < 4) dma_a.issue(buf, i, 4096, kk * 2, wave_s);
              else dma_b.issue(buf + W4_OP_BYTES, i - 4, 4096, kk * 2, wave_s);
            }
          }
        }
        __builtin_amdgcn_s_setprio(0);
      }
      // Retire the prefetch reads here (they had the whole MFMA block to
      // land).  lgkmcnt only counts to 15, so if they were still pending at
      // the next stage's first MFMA the compiler would have to wait
      // lgkmcnt(0) on the NEW prefetch as well.  0xC07F = lgkmcnt(0) only.
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
  }
  // MFMA results -> VALU/accvgpr reads: 16x16x32 is an 8-pass op, pad >= 10
  // wait states before the epilogue reads the accumulators.
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + crow;
    uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4_t v = acc[i][j];
      uint2 pk;
      pk.x = mxk::pack2bf(v[0], v[1]);
      pk.y = mxk::pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(cp + j * 16) = pk;
    }
  }
}

// ---------------------------------------------------------------------------
// Schedule 4: 8 waves (two per SIMD), each owning a 128x64 output block
// (8x4 tiles of 16x16 -> 128 fp32 accumulators pinned to AGPRs), on the same
// BK = 32, 4-deep LDS ring as schedule 3.  Two waves per SIMD let one wave's
// LDS-DMA issue (~60 cycles per piece among MFMAs, MI355X_MICROARCH.md
// cycle constants) hide under its partner's MFMAs, which a single wave per
// SIMD cannot do.  Per 32-deep stage a wave issues 32 MFMAs, 12 fragment
// reads for the next stage and 4 LDS-DMA pieces (2 per operand).
// ---------------------------------------------------------------------------
namespace {
constexpr int W8_THREADS = 512;

// One half (128 rows x 32 k) of an operand stage = 1 glds per thread.
__device__ __forceinline__ void w8_stage_half(const uint16_t* __restrict__ src, int ld, int row0,
                                              int k0, char* lds_op, int q, int tid) {
  const int row = q * 128 + (tid >> 2);
  const int c = (tid & 3) ^ w4_h((row >> 2) & 3);
  const uint16_t* g = src + static_cast<size_t>(row0 + row) * ld + k0 + c * 8;
  __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_op + q * 8192 + (tid >> 6) * 1024), 16, 0, 0);
}
}  // namespace

template <int NS>
__global__ void __launch_bounds__(W8_THREADS, 2)
mxk_gemm_bf16_tn_w8(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                    uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[NS * W4_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2;   // 0..1 -> 128 rows
  const int wn = wave & 3;    // 0..3 -> 64 cols

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const int frow = lane & 15;
  const int foff = frow * 64 + (((lane >> 4) ^ w4_h((frow >> 2) & 3)) * 16);
  const int a_off = wm * 128 * 64 + foff;               // + i*1024 for subtile i
  const int b_off = W4_OP_BYTES + wn * 64 * 64 + foff;  // + j*1024
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const DmaStream dma_a = make_dma(A, lda, m0, tid, 128);
  const DmaStream dma_b = make_dma(Bt, ldb, n0, tid, 128);

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = K / W4_BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) {
    const int kk = (s < ns ? s : ns - 1) * W4_BK;
    char* buf = smem + s * W4_STAGE_BYTES;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      dma_a.issue(buf, q, 8192, kk * 2, wave_s);
      dma_b.issue(buf + W4_OP_BYTES, q, 8192, kk * 2, wave_s);
    }
  }
  // stage 0 landed: 4 glds per later stage may stay in flight
  if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  bf16x8_t fa[2][8], fb[2][4];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[0][i] = lds_read_b128(smem + a_off + i * 1024);
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[0][j] = lds_read_b128(smem + b_off + j * 1024);

  for (int s = 0; s < ns; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int st = s + u;
      __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's prefetch reads done
      if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      {
        const char* nb = smem + ((st + 1) % NS) * W4_STAGE_BYTES;
        const int sn = st + NS - 1;
        const int kk = (sn < ns ? sn : ns - 1) * W4_BK;
        char* buf = smem + (sn % NS) * W4_STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            mfma_16x16x32_agpr(acc[i][j], fb[u][j], fa[u][i]);
            const int t = i * 4 + j;          // MFMA index 0..31
            if ((t & 1) == 1 && t < 24) {      // 12 reads, one per 2 MFMAs
              const int r = t >> 1;
              if (r < 4) fb[u ^ 1][r] = lds_read_b128(nb + b_off + r * 1024);
              else fa[u ^ 1][r - 4] = lds_read_b128(nb + a_off + (r - 4) * 1024);
            }
            if ((t & 7) == 4) {               // 4 DMA pieces, one per 8 MFMAs
              const int q = t >> 3;
              if (q < 2) dma_a.issue(buf, q, 8192, kk * 2, wave_s);
              else dma_b.issue(buf + W4_OP_BYTES, q - 2, 8192, kk * 2, wave_s);
            }
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + crow;
    uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 64 + ccol;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4_t v = acc[i][j];
      uint2 pk;
      pk.x = mxk::pack2bf(v[0], v[1]);
      pk.y = mxk::pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(cp + j * 16) = pk;
    }
  }
}

// ---------------------------------------------------------------------------
// Schedules 5/6: 4 waves (one per SIMD), 128x128 AGPR accumulators per wave,
// BK = 64 stages in a 2-stage LDS ring (128 KiB), two 32-deep k-steps of 64
// MFMAs per stage.  Register set 0 holds the fragments of k-step s.0, set 1
// those of s.1; each k-step prefetches the other set while its MFMAs run.
//
// DMA pieces are 8 rows x 128 B (whole cache lines).  k-step s.1 issues all
// 16 pieces of stage s+2 into buffer s; ONE barrier per stage (between s.0
// and s.1).  Swizzle: chunk c of row r at c ^ ((r>>1)&7).  Schedule 5
// addresses the DMA with one lane VGPR + a per-piece SGPR offset, 6 and 13
// with a VGPR offset per piece (hipBLASLt-style, +2.8%); 13 (the default)
// also has exact LDS waits (ORD 4 below).
// (Half-line pieces, 16 rows x 64 B, spread the DMA evenly over both
// k-steps but double the cache-line requests: slower here and in w4q.)
// (A 64-B pad per 1-KiB piece, hipBLASLt-style, measured within noise of the
// dense layout: the DMA landing banks are not the limiter.)
// Layouts are conflict-free for the 16x16x32 fragment reads and the DMA
// source swizzle inverts the read one (tests/test_gemm_swizzle.py).
// ---------------------------------------------------------------------------
namespace {
constexpr int W4B_OP_BYTES = 256 * 128;            // 32 KiB per operand per stage
constexpr int W4B_STAGE_BYTES = 2 * W4B_OP_BYTES;  // 64 KiB

__device__ __forceinline__ int w4b_h(int q) { return (((q ^ (q >> 1)) & 1) << 1) | (q >> 1); }

// CP: cache-policy bits of the LDS-DMA loads (aux operand: 1 = sc0, 2 = nt,
// 16 = sc1).  hipBLASLt's MT256x256x64 kernels issue theirs with sc1.
template <int CP = 0>
struct DmaStream64 {
  // CP & 32 ("VOFF" addressing, hipBLASLt-style): one precomputed VGPR offset
  // per piece, soffset 0 and the k step folded into a per-stage descriptor
  // base; otherwise one lane VGPR + a per-piece SGPR soffset.
  static constexpr bool VOFF = (CP & 32) != 0;
  static constexpr int AUX = CP & 31;
  __amdgpu_buffer_rsrc_t rsrc;   // uniform: 256-row panel
  uint32_t lane_off;             // per lane: row-in-piece * ld * 2 + swizzled chunk * 16
  uint32_t piece_stride;         // uniform: rows per piece * ld * 2
  const char* base;              // VOFF: panel base
  uint32_t bytes;                // VOFF: panel bytes
  uint32_t voff[8];              // VOFF: lane_off + (p*4 + wave) * piece_stride
  // piece g = p*4 + wave (rows 8g .. 8g+7) -> LDS [g*1024, +1024)
  __device__ __forceinline__ void issue(char* lds_op, int p, int k_bytes, int wave_s) const {
    const int g = p * 4 + wave_s;
    const int dst = g * 1024;
    if constexpr (VOFF) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char*>(base + k_bytes), 0, static_cast<int>(bytes), 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(lds_op + dst), 16, voff[p], 0, 0,
                                               AUX);
    } else {
      const int soff = k_bytes + g * piece_stride;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_op + dst), 16, lane_off, soff,
                                               0, AUX);
    }
  }
};

template <int CP = 0>
__device__ __forceinline__ DmaStream64<CP> make_dma64(const uint16_t* src, int ld, int row0,
                                                        int lane, int wave) {
  DmaStream64<CP> d;
  const uint16_t* base = src + static_cast<size_t>(row0) * ld;
  d.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, 256 * ld * 2,
                                             0x00020000);
  const int r = lane >> 3;                      // row within the 8-row piece
  // row = 8g + r with g = 4p + wave: (row >> 1) & 7 = (4 (wave & 1) + (r >> 1)) & 7
  const int c = (lane & 7) ^ ((4 * (wave & 1) + (r >> 1)) & 7);
  d.lane_off = static_cast<uint32_t>(r * ld * 2 + c * 16);
  d.piece_stride = static_cast<uint32_t>(8 * ld * 2);
  d.base = reinterpret_cast<const char*>(base);
  d.bytes = static_cast<uint32_t>(256 * ld * 2);
#pragma unroll
  for (int p = 0; p < 8; ++p) d.voff[p] = d.lane_off + (p * 4 + wave) * d.piece_stride;
  return d;
}
}  // namespace

// ABL (timing ablations, wrong results): 1 = no DMA, 2 = no fragment reads,
// 3 = no vmcnt before the barrier.  ORD (whole-line mode) places k-step s.1's
// 16 DMA pieces and 16 prefetch reads: 0 = interleaved (one of each per 4
// MFMAs), 1 = DMA over the first 32 MFMAs then reads over the last 32,
// 2 = reads first, then DMA, 3 = a mid-k-step barrier (lockstep waves).
// ORD >= 4 drops the lgkmcnt(0) at the top of k-step s.0: the scalar loads
// are drained before the loop so the compiler's per-operand LDS waits are
// exact counts, and the MFMAs start while the last prefetch reads of s.1 are
// still in flight.  ORD 4 also spreads s.0's reads one per 3 MFMAs, so the
// barrier's lgkmcnt(0) finds them long retired; ORD 5 keeps s.0's placement.
// Diagnostic build only (ABL == 5): s_memtime stamps split every k-iteration
// into k-step 0 / wait + barrier / k-step 1; per-segment cycle sums of all
// waves land in g_w4b_stamps (read by mxk_gemm_bf16_stamps).  The stamps'
// fences forbid overlaps the real kernel has: read the SHARES, not the time.
__device__ unsigned long long g_w4b_stamps[4];

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

using mxk::w4b_tile;

// EPI 1: widened store tail (guide T21 with v_permlane16_swap): the bf16
// quads of 16x16 tiles j and j+1 are exchanged between lane rows so every
// lane holds 8 consecutive columns -> 32 global_store_dwordx4 per lane
// instead of 64 dwordx2 (the tail is store-issue bound).  Needs ldc % 8 == 0
// and a 16-B aligned C.
template <int ABL = 0, int ORD = 0, int CP = 0, int MAP = 0, int EPI = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4b(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 1;
  const int wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, tiles_m, tiles_n, &m0, &n0);

  const DmaStream64<CP> dma_a = make_dma64<CP>(A, lda, m0, lane, wave_s);
  const DmaStream64<CP> dma_b = make_dma64<CP>(Bt, ldb, n0, lane, wave_s);

  // fragment offsets: lane reads row x = (l & 15) of a 16-row subtile,
  // logical chunk ks*4 + (l >> 4)
  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;                      // bytes per 16-row subtile
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = K / BK;   // 64-deep stages
  auto kbytes = [&](int st) { return (st < ns ? st : ns - 1) * BK * 2; };
  // prologue: stages 0 and 1
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    char* buf = smem + s * W4B_STAGE_BYTES;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      dma_a.issue(buf, p, kbytes(s), wave_s);
      dma_b.issue(buf + W4B_OP_BYTES, p, kbytes(s), wave_s);
    }
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // stage 0 (own pieces) landed
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);

  unsigned long long seg0 = 0, seg1 = 0, seg2 = 0, t0 = 0;
  // ORD 4: drain everything (incl. kernel-argument scalar loads) here, so the
  // compiler's per-register LDS waits inside the loop are exact counts
  if constexpr (ORD >= 4) __builtin_amdgcn_s_waitcnt(0xC07F);
  for (int s = 0; s < ns; ++s) {
    char* cur = smem + (s & 1) * W4B_STAGE_BYTES;
    char* nxt = smem + ((s + 1) & 1) * W4B_STAGE_BYTES;
    // ---- k-step s.0: MFMAs on set 0, prefetch set 1 (s.1) from `cur`
    if constexpr (ORD < 4) __builtin_amdgcn_s_waitcnt(0xC07F);
    if constexpr (ABL == 5) t0 = stamp();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
        if (ORD == 3 && i == 3 && j == 7) __builtin_amdgcn_s_barrier();   // lockstep waves
        if (ORD == 4) {
          // one read per 3 MFMAs: the last lands 17 MFMAs before the
          // barrier's lgkmcnt(0) instead of right at it
          const int m = i * 8 + j;
          if (m % 3 == 1 && m / 3 < 16 && ABL != 2) {
            const int r = m / 3;
            if (r < 8) f1b[r] = lds_read_b128(cur + b_base + r * SUB + off_k1);
            else f1a[r - 8] = lds_read_b128(cur + a_base + (r - 8) * SUB + off_k1);
          }
        } else if ((j & 3) == 3 && ABL != 2) {
          const int r = i * 2 + (j >> 2);
          if (r < 8) f1b[r] = lds_read_b128(cur + b_base + r * SUB + off_k1);
          else f1a[r - 8] = lds_read_b128(cur + a_base + (r - 8) * SUB + off_k1);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    unsigned long long t1 = 0;
    if constexpr (ABL == 5) t1 = stamp();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    // own pieces of stage s+1 landed
    if (ABL != 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    unsigned long long t2 = 0;
    if constexpr (ABL == 5) {
      t2 = stamp();
      seg0 += t1 - t0;
      seg1 += t2 - t1;
    }
    // ---- k-step s.1: MFMAs on set 1, prefetch set 0 ((s+1).0) from `nxt`,
    //      DMA of stage s+2 into `cur`, fully consumed:
    //      certified by the barrier
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
        if (ORD == 3 && i == 3 && j == 7) __builtin_amdgcn_s_barrier();
        if (ORD == 1 || ORD == 2) {
          // halves of the k-step: slot t = (i & 3) * 4 + (j >> 1) on odd j
          const bool first = i < 4;
          if ((j & 1) == 1) {
            const int t = (i & 3) * 4 + (j >> 1);
            if (first == (ORD == 2)) {
              if (ABL != 2) {
                if (t < 8) f0b[t] = lds_read_b128(nxt + b_base + t * SUB + off_k0);
                else f0a[t - 8] = lds_read_b128(nxt + a_base + (t - 8) * SUB + off_k0);
              }
            } else if (ABL != 1) {
              if (t < 8) dma_a.issue(cur, t, kbytes(s + 2), wave_s);
              else dma_b.issue(cur + W4B_OP_BYTES, t - 8, kbytes(s + 2), wave_s);
            }
          }
          continue;
        }
        if ((j & 3) == 1 && ABL != 2) {
          const int r = i * 2 + (j >> 2);
          if (r < 8) f0b[r] = lds_read_b128(nxt + b_base + r * SUB + off_k0);
          else f0a[r - 8] = lds_read_b128(nxt + a_base + (r - 8) * SUB + off_k0);
        }
        if (ABL != 1 && (j & 3) == 3) {
          const int p = i * 2 + (j >> 2);   // 0..15
          if (p < 8) dma_a.issue(cur, p, kbytes(s + 2), wave_s);
          else dma_b.issue(cur + W4B_OP_BYTES, p - 8, kbytes(s + 2), wave_s);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (ABL == 5) seg2 += stamp() - t2;
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  if constexpr (ABL == 5) {
    if (lane == 0) {
      atomicAdd(&g_w4b_stamps[0], seg0);
      atomicAdd(&g_w4b_stamps[1], seg1);
      atomicAdd(&g_w4b_stamps[2], seg2);
      atomicAdd(&g_w4b_stamps[3], 1ull);
    }
  } else {
    (void)seg0; (void)seg1; (void)seg2; (void)t0;
  }

  const int crow = lane & 15;
  if constexpr (EPI == 1) {
    // v_permlane16_swap(x, y): odd lane rows of x <-> even lane rows of y.
    // Row q then holds tile j + (q & 1), columns (q >> 1) * 8 .. + 7.
    const int q = lane >> 4;
    const int ccol = (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + crow;
      uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const uint32_t x0 = mxk::pack2bf(acc[i][j][0], acc[i][j][1]);
        const uint32_t x1 = mxk::pack2bf(acc[i][j][2], acc[i][j][3]);
        const uint32_t y0 = mxk::pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]);
        const uint32_t y1 = mxk::pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        uint4 v;
        v.x = s0[0];
        v.y = s1[0];
        v.z = s0[1];
        v.w = s1[1];
        *reinterpret_cast<uint4*>(cp + j * 16) = v;
      }
    }
  } else {
    const int ccol = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + crow;
      uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4_t v = acc[i][j];
        uint2 pk;
        pk.x = mxk::pack2bf(v[0], v[1]);
        pk.y = mxk::pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(cp + j * 16) = pk;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Schedule 22+ ("w4h"): the w4b tile, LDS image and DMA addressing on a
// three-barrier K-tile — the structure of hipBLASLt's gfx950 MT256x256x64
// kernel, read off its disassembly: the buffer X being consumed is refilled
// IN PLACE with stage s+2 as soon as each operand's last fragment read of X
// has retired, so the 16 DMA pieces spread over ~64 MFMAs and get ~130-200
// MFMAs (instead of 64-128) to land.  Per K-tile, m = MFMA index 0..127:
//   m  1..15  : A fragments of k-half 1 from X (8 reads)
//   m  19     : lgkmcnt(0) + barrier #1   (X.A consumed by every wave)
//   m 21..49  : B fragments of k-half 1 from X, one per 4 MFMAs
//   m 23..51  : DMA of stage s+2, A pieces, into X.A
//   m  55     : lgkmcnt(0) + barrier #2   (X.B consumed)
//   m 57..85  : DMA of stage s+2, B pieces, into X.B
//   m  91     : vmcnt(16) + barrier #3    (stage s+1 in Y landed everywhere)
//   m 93..123 : k-half-0 fragments of stage s+1 from Y (B first, then A:
//               the order the next K-tile's MFMAs consume them)
// ---------------------------------------------------------------------------
// Knobs (A/B variants): MO 1 = MFMA order j-outer (srcA fixed for 8 MFMAs,
// as hipBLASLt's stream; next-k0 reads then A first).  LATE 1 = B pieces
// every 6 MFMAs from m 57, barrier #3 after m 96 with vmcnt(15): the last
// piece goes out after it (hipBLASLt waits vmcnt(13) with 3 pieces after).
// PRIO 0 = no s_setprio around the MFMA stream.
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N == 15 || N == 16, "vm_wait: add the count");
  if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
}

template <int MAP, int EPI, int MO = 0, int LATE = 0, int PRIO = 1>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4h(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  const int tiles_m = M / BM, tiles_n = N / BN;
  int m0, n0;
  w4b_tile<MAP>(blockIdx.x, gridDim.x, tiles_m, tiles_n, &m0, &n0);
  const DmaStream64<32> dma_a = make_dma64<32>(A, lda, m0, lane, wave_s);
  const DmaStream64<32> dma_b = make_dma64<32>(Bt, ldb, n0, lane, wave_s);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
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
  auto kbytes = [&](int st) { return (st < ns ? st : ns - 1) * BK * 2; };
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma_a.issue(smem + s * W4B_STAGE_BYTES, p, kbytes(s), wave_s);
#pragma unroll
    for (int p = 0; p < 8; ++p)
      dma_b.issue(smem + s * W4B_STAGE_BYTES + W4B_OP_BYTES, p, kbytes(s), wave_s);
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // stage 0 (own pieces) landed
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
  // drain everything (incl. kernel-argument scalar loads) so the compiler's
  // per-register LDS waits inside the loop are exact counts
  __builtin_amdgcn_s_waitcnt(0xC07F);

  constexpr int B3 = LATE ? 96 : 91;          // barrier #3 after MFMA B3
  constexpr int BSP = LATE ? 6 : 4;           // B piece spacing from m 57
  constexpr int NB3 = (B3 - 57) / BSP + 1 < 8 ? (B3 - 57) / BSP + 1 : 8;   // B pieces before it
  for (int s = 0; s < ns; ++s) {
    char* X = smem + (s & 1) * W4B_STAGE_BYTES;
    char* Y = smem + ((s + 1) & 1) * W4B_STAGE_BYTES;
    const int kb2 = kbytes(s + 2);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int w = 0; w < 8; ++w) {
          const int i = MO ? w : u, j = MO ? u : w;
          const int m = h * 64 + u * 8 + w;
          if (h == 0) mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
          else mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
          if (m < 16 && (m & 1)) f1a[m >> 1] = lds_read_b128(X + a_base + (m >> 1) * SUB + off_k1);
          if (m == 19) {
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
          }
          if (m >= 20 && m < 52 && (m & 3) == 1)
            f1b[(m - 21) >> 2] = lds_read_b128(X + b_base + ((m - 21) >> 2) * SUB + off_k1);
          if (m >= 20 && m < 52 && (m & 3) == 3) dma_a.issue(X, (m - 23) >> 2, kb2, wave_s);
          if (m == 55) {
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
          }
          if (m >= 57 && (m - 57) % BSP == 0 && (m - 57) / BSP < 8)
            dma_b.issue(X + W4B_OP_BYTES, (m - 57) / BSP, kb2, wave_s);
          if (m == B3) {
            vm_wait<8 + NB3>();   // stage s+1 (last K-tile's pieces) landed
            __builtin_amdgcn_s_barrier();
          }
          if (m > B3 && m < B3 + 32 && ((m - B3) & 1)) {
            const int r = (m - B3 - 1) >> 1;   // 0..15
            if (MO == 0) {
              if (r < 8) f0b[r] = lds_read_b128(Y + b_base + r * SUB + off_k0);
              else f0a[r - 8] = lds_read_b128(Y + a_base + (r - 8) * SUB + off_k0);
            } else {
              if (r < 8) f0a[r] = lds_read_b128(Y + a_base + r * SUB + off_k0);
              else f0b[r - 8] = lds_read_b128(Y + b_base + (r - 8) * SUB + off_k0);
            }
          }
        }
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  const int crow = lane & 15;
  if constexpr (EPI == 1) {
    const int q = lane >> 4;
    const int ccol = (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + crow;
      uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const uint32_t x0 = mxk::pack2bf(acc[i][j][0], acc[i][j][1]);
        const uint32_t x1 = mxk::pack2bf(acc[i][j][2], acc[i][j][3]);
        const uint32_t y0 = mxk::pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]);
        const uint32_t y1 = mxk::pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        uint4 v;
        v.x = s0[0];
        v.y = s1[0];
        v.z = s0[1];
        v.w = s1[1];
        *reinterpret_cast<uint4*>(cp + j * 16) = v;
      }
    }
  } else {
    const int ccol = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + crow;
      uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4_t v = acc[i][j];
        uint2 pk;
        pk.x = mxk::pack2bf(v[0], v[1]);
        pk.y = mxk::pack2bf(v[2], v[3]);
        *reinterpret_cast<uint2*>(cp + j * 16) = pk;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Schedule 29+ ("w4i"): w4h with the scalar work taken out of the K loop.
// hipcc hoists the per-K-tile address arithmetic of w4h (stage-dependent
// LDS bases for M0, the clamped k offset, a rebuilt buffer descriptor per
// DMA stream) to the top of the loop, ~20 SALU ahead of the first MFMA
// while the matrix pipe drains.  Here
//  * the loop is unrolled by two, so X/Y (and every M0 value) are
//    compile-time per parity;
//  * the k step is the DMA's SGPR soffset on a fixed panel descriptor
//    (one s_add per K-tile) instead of a new descriptor base per stage;
//  * the last two K-tiles run without DMA (no clamped re-reads of the last
//    stage), the last one without the next-k0 reads or barrier #3.
// MODE 1: DMA of stage s+2, vmcnt(8 + NB3) at barrier #3; MODE 2: no DMA,
// vmcnt(0) at barrier #3 (stage s+1 is the last one issued); MODE 3: no
// DMA, no barrier #3, no next-k0 reads (last K-tile).
struct DmaK {
  __amdgpu_buffer_rsrc_t rsrc;   // 256-row panel, whole K
  uint32_t voff[8];              // piece p: row-in-piece * ld * 2 + swizzled chunk + (4p + wave) * 8 rows
  __device__ __forceinline__ void issue(char* lds_op, int p, int k_bytes, int wave_s) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_op + (p * 4 + wave_s) * 1024),
                                             16, voff[p], k_bytes, 0, 0);
  }
};

__device__ __forceinline__ DmaK make_dmak(const uint16_t* src, int ld, int row0, int lane,
                                          int wave) {
  DmaK d;
  const uint16_t* base = src + static_cast<size_t>(row0) * ld;
  d.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, 256 * ld * 2,
                                             0x00020000);
  const int r = lane >> 3;
  const int c = (lane & 7) ^ ((4 * (wave & 1) + (r >> 1)) & 7);
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

using mxk::store_block_wide;
using mxk::store_block_narrow;

template <int MAP, int EPI, int LATE = 0, int R1 = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4i(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
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
  const int fch = (lane >> 4) ^ (frow >> 1);
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
    w4i_ktile<0, 1, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, kb, wave_s);
    w4i_ktile<1, 1, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, kb + BK * 2, wave_s);
    kb += 2 * BK * 2;
  }
  if (s < ns - 2) {   // s even
    w4i_ktile<0, 1, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, kb, wave_s);
    ++s;
  }
  // the last two K-tiles (or the only one): no DMA
  if (ns >= 2) {
    w4i_ktile<2, 2, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                          dma_b, 0, wave_s, s & 1);
    ++s;
  }
  w4i_ktile<2, 3, LATE, R1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                        dma_b, 0, wave_s, s & 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if constexpr (EPI == 1) store_block_wide<false>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
  else if constexpr (EPI == 2) store_block_wide<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
  else store_block_narrow(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
}

// ---------------------------------------------------------------------------
// Schedule 35 ("w4ip"): w4i made persistent (grid <= one workgroup per CU,
// tiles t = blockIdx.x + r * grid).  Between tiles the LDS is free once every
// wave passed the last K-tile (barrier), so the next tile's two prologue
// stages are issued BEFORE the finished tile's store tail and land under it.
// vmcnt at the top of a later tile: 32 DMA pieces then 32 stores per wave
// are outstanding, vmcnt(48) retires exactly stage 0 (16 pieces + 32 stores
// -> vmcnt(32) when K has a single stage).  Every wave runs the same trip
// count, so all reach every barrier and leave the loop together.
template <int MAP, int EPI>
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
      w4i_ktile<0, 1, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                         dma_b, kb, wave_s);
      w4i_ktile<1, 1, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                         dma_b, kb + BK * 2, wave_s);
      kb += 2 * BK * 2;
    }
    if (s < ns - 2) {
      w4i_ktile<0, 1, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                         dma_b, kb, wave_s);
      ++s;
    }
    if (ns >= 2) {
      w4i_ktile<2, 2, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                         dma_b, 0, wave_s, s & 1);
      ++s;
    }
    w4i_ktile<2, 3, 1>(acc, f0a, f0b, f1a, f1b, smem, a_base, b_base, off_k0, off_k1, dma_a,
                       dma_b, 0, wave_s, s & 1);
    // every wave's LDS reads retired (and no DMA is in flight): LDS is free
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();

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
// Schedule 21 ("w4p"): the default w4b schedule (ORD 4, VOFF DMA) made
// persistent — one workgroup per CU walks tiles t = blockIdx.x + r * grid.
// With one 128 KiB workgroup per CU a non-persistent grid leaves the CU idle
// while a tile's store tail drains and the next workgroup refills two
// stages; here the next tile's two prologue stages are issued into the
// (barrier-certified) free LDS right BEFORE the current tile's widened store
// tail (EPI 1), so the refill lands under the stores.  vmcnt bookkeeping at
// the top of a tile: 32 DMA pieces then 32 stores are outstanding per wave;
// vmcnt(48) retires exactly stage 0 (counts retire in issue order).
// The grid is <= one workgroup per CU and every wave runs the same trip
// count, so each wave reaches every barrier and the loop exits for all.
template <int MAP>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4p(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int ntiles = tiles_m * tiles_n;

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
  const int off_k0 = frow * 128 + fch * 16;
  const int off_k1 = frow * 128 + (fch ^ 4) * 16;
  constexpr int SUB = 2048;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4B_OP_BYTES + wn * 8 * SUB;
  const int ns = K / BK;
  auto kbytes = [&](int st) { return (st < ns ? st : ns - 1) * BK * 2; };

  int t = blockIdx.x;
  int m0, n0;
  w4b_tile<MAP>(t, ntiles, tiles_m, tiles_n, &m0, &n0);
  DmaStream64<32> dma_a = make_dma64<32>(A, lda, m0, lane, wave_s);
  DmaStream64<32> dma_b = make_dma64<32>(Bt, ldb, n0, lane, wave_s);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      dma_a.issue(smem + s * W4B_STAGE_BYTES, p, kbytes(s), wave_s);
      dma_b.issue(smem + s * W4B_STAGE_BYTES + W4B_OP_BYTES, p, kbytes(s), wave_s);
    }
  }
  bool first = true;
  while (true) {
    if (first) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    f32x4_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
#pragma unroll
    for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);
    __builtin_amdgcn_s_waitcnt(0xC07F);

    for (int s = 0; s < ns; ++s) {
      char* cur = smem + (s & 1) * W4B_STAGE_BYTES;
      char* nxt = smem + ((s + 1) & 1) * W4B_STAGE_BYTES;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
          const int m = i * 8 + j;
          if (m % 3 == 1 && m / 3 < 16) {
            const int r = m / 3;
            if (r < 8) f1b[r] = lds_read_b128(cur + b_base + r * SUB + off_k1);
            else f1a[r - 8] = lds_read_b128(cur + a_base + (r - 8) * SUB + off_k1);
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
          if ((j & 3) == 1) {
            const int r = i * 2 + (j >> 2);
            if (r < 8) f0b[r] = lds_read_b128(nxt + b_base + r * SUB + off_k0);
            else f0a[r - 8] = lds_read_b128(nxt + a_base + (r - 8) * SUB + off_k0);
          }
          if ((j & 3) == 3) {
            const int p = i * 2 + (j >> 2);
            if (p < 8) dma_a.issue(cur, p, kbytes(s + 2), wave_s);
            else dma_b.issue(cur + W4B_OP_BYTES, p - 8, kbytes(s + 2), wave_s);
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    // every wave's DMA landed and LDS reads retired: the LDS is free
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();

    const int cm0 = m0, cn0 = n0;
    const int tn = t + static_cast<int>(gridDim.x);
    if (tn < ntiles) {
      w4b_tile<MAP>(tn, ntiles, tiles_m, tiles_n, &m0, &n0);
      dma_a = make_dma64<32>(A, lda, m0, lane, wave_s);
      dma_b = make_dma64<32>(Bt, ldb, n0, lane, wave_s);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          dma_a.issue(smem + s * W4B_STAGE_BYTES, p, kbytes(s), wave_s);
          dma_b.issue(smem + s * W4B_STAGE_BYTES + W4B_OP_BYTES, p, kbytes(s), wave_s);
        }
      }
    }

    // widened store tail (EPI 1 of w4b)
    const int crow = lane & 15;
    const int q = lane >> 4;
    const int ccol = (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = cm0 + wm * 128 + i * 16 + crow;
      uint16_t* cp = C + static_cast<size_t>(m) * ldc + cn0 + wn * 128 + ccol;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const uint32_t x0 = mxk::pack2bf(acc[i][j][0], acc[i][j][1]);
        const uint32_t x1 = mxk::pack2bf(acc[i][j][2], acc[i][j][3]);
        const uint32_t y0 = mxk::pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]);
        const uint32_t y1 = mxk::pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        uint4 v;
        v.x = s0[0];
        v.y = s1[0];
        v.z = s0[1];
        v.w = s1[1];
        *reinterpret_cast<uint4*>(cp + j * 16) = v;
      }
    }
    if (tn >= ntiles) break;
    t = tn;
    first = false;
  }
}

// ---------------------------------------------------------------------------
// Schedule 16 ("w4q"): the w4b tile and MFMA stream on a 4-deep ring of
// 32-deep k-steps (4 x 32 KiB LDS) instead of 2 x 64-deep stages.  Every
// k-step issues 8 LDS-DMA pieces per wave (one per 8 MFMAs) for the stage 4
// k-steps ahead, so
//   * the texture path sees a uniform 8 pieces per k-step instead of 16
//     every other k-step (the diagnostic stamps put +300 cycles on the
//     DMA-carrying k-step of w4b), and
//   * a piece has ~2.5 k-steps to land instead of ~1.5;
// at the price of one barrier per k-step (the waves run in near lockstep).
// Stage image: 16-row x 64-B pieces, chunk c of row r at c ^ h((r >> 2) & 3)
// (conflict-free b128 reads: tests/test_gemm_swizzle.py::test_w4b_half_*).
namespace {
constexpr int W4Q_OP_BYTES = 256 * 64;               // 16 KiB per operand per k-step
constexpr int W4Q_STAGE_BYTES = 2 * W4Q_OP_BYTES;    // 32 KiB
constexpr int W4Q_RING = 4;

template <int CP>
struct DmaRing32 {
  static constexpr int AUX = CP & 31;
  const char* base;
  uint32_t bytes;
  uint32_t voff[4];   // piece g = 4p + wave: rows 16g .. 16g+15
  __device__ __forceinline__ void issue(char* lds_op, int p, int k_bytes, int wave_s) const {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(base + k_bytes), 0, static_cast<int>(bytes), 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(lds_op + (p * 4 + wave_s) * 1024), 16,
                                             voff[p], 0, 0, AUX);
  }
};

template <int CP>
__device__ __forceinline__ DmaRing32<CP> make_ring32(const uint16_t* src, int ld, int row0, int lane,
                                                     int wave) {
  DmaRing32<CP> d;
  const uint16_t* base = src + static_cast<size_t>(row0) * ld;
  const int r = lane >> 2;                        // row within the 16-row piece
  const int c = (lane & 3) ^ w4b_h((r >> 2) & 3);
  const uint32_t lane_off = static_cast<uint32_t>(r * ld * 2 + c * 16);
  d.base = reinterpret_cast<const char*>(base);
  d.bytes = static_cast<uint32_t>(256 * ld * 2);
#pragma unroll
  for (int p = 0; p < 4; ++p)
    d.voff[p] = lane_off + static_cast<uint32_t>((p * 4 + wave) * 16 * ld * 2);
  return d;
}

// One k-step: 64 MFMAs on (fa, fb); 16 reads of the next k-step's fragments
// (one per 3 MFMAs, all retired well before the closing lgkmcnt(0)); 8 DMA
// pieces of the stage 4 k-steps ahead into `dma_dst` (one per 8 MFMAs).
template <int ABL, int CP>
__device__ __forceinline__ void w4q_kstep(f32x4_t (&acc)[8][8], const bf16x8_t (&fa)[8],
                                          const bf16x8_t (&fb)[8], bf16x8_t (&na)[8],
                                          bf16x8_t (&nb)[8], const char* nxt, int a_base,
                                          int b_base, int off, const DmaRing32<CP>& da,
                                          const DmaRing32<CP>& db, char* dma_dst, int dma_k,
                                          int wave_s) {
  constexpr int SUB = 1024;
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mfma_16x16x32_agpr(acc[i][j], fb[j], fa[i]);
      const int m = i * 8 + j;
      if (ABL != 2 && m % 3 == 1 && m / 3 < 16) {
        const int r = m / 3;
        if (r < 8) nb[r] = lds_read_b128(nxt + b_base + r * SUB + off);
        else na[r - 8] = lds_read_b128(nxt + a_base + (r - 8) * SUB + off);
      }
      if (ABL != 1 && m % 8 == 5) {
        const int p = m / 8;
        if (p < 4) da.issue(dma_dst, p, dma_k, wave_s);
        else db.issue(dma_dst + W4Q_OP_BYTES, p - 4, dma_k, wave_s);
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
  // the next k-step DMAs into the buffer just read: every wave's reads must
  // have retired; the stage read by the next k-step (issued two k-steps ago)
  // must have landed
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (ABL != 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
}  // namespace

template <int ABL = 0, int CP = 32>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4q(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[W4Q_RING * W4Q_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 1;
  const int wn = wave & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const DmaRing32<CP> da = make_ring32<CP>(A, lda, m0, lane, wave_s);
  const DmaRing32<CP> db = make_ring32<CP>(Bt, ldb, n0, lane, wave_s);

  const int frow = lane & 15;
  const int off = frow * 64 + (((lane >> 4) ^ w4b_h(frow >> 2)) * 16);
  constexpr int SUB = 1024;
  const int a_base = wm * 8 * SUB;
  const int b_base = W4Q_OP_BYTES + wn * 8 * SUB;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / 32;   // even: K % 64 == 0
  // past the end the DMA re-reads the last k-step into a consumed buffer, so
  // every k-step issues the same number of pieces (uniform vmcnt arithmetic)
  auto kbytes = [&](int t) { return (t < nk ? t : nk - 1) * 64; };
  auto stage = [&](int t) { return smem + (t & (W4Q_RING - 1)) * W4Q_STAGE_BYTES; };
#pragma unroll
  for (int t = 0; t < W4Q_RING; ++t) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      da.issue(stage(t), p, kbytes(t), wave_s);
      db.issue(stage(t) + W4Q_OP_BYTES, p, kbytes(t), wave_s);
    }
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // k-steps 0 and 1 landed
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off);
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off);
  __builtin_amdgcn_s_waitcnt(0xC07F);   // incl. scalar loads: exact LDS waits in the loop

  for (int t = 0; t < nk; t += 2) {
    // k-step t: buffer t % 4 was read during k-step t-1 (barrier-certified),
    // so it takes the DMA of k-step t + 4
    w4q_kstep<ABL, CP>(acc, f0a, f0b, f1a, f1b, stage(t + 1), a_base, b_base, off, da, db,
                       stage(t), kbytes(t + 4), wave_s);
    w4q_kstep<ABL, CP>(acc, f1a, f1b, f0a, f0b, stage(t + 2), a_base, b_base, off, da, db,
                       stage(t + 1), kbytes(t + 5), wave_s);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + crow;
    uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4_t v = acc[i][j];
      uint2 pk;
      pk.x = mxk::pack2bf(v[0], v[1]);
      pk.y = mxk::pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(cp + j * 16) = pk;
    }
  }
}

// ---------------------------------------------------------------------------
// Schedule 8 ("early reads"): the w4b tile and LDS image, but each k-step
// issues ALL 16 fragment reads of the next k-step at its start (LDS-bound
// bursts the matrix core hides) instead of one per 4 MFMAs.  k-step 0's
// reads retire after 16 MFMAs; a barrier there certifies that every wave is
// done with the stage's buffer, so the 16 LDS-DMA pieces of stage s+2 are
// spread over BOTH k-steps (8 each) instead of all landing in k-step 1, where
// the diagnostic stamps (variant 12) put +300 cycles.  Stage s+1 is waited
// for with vmcnt(8) (its pieces were issued 1.5-2 k-steps earlier).
// ---------------------------------------------------------------------------
template <int CP = 32>
__global__ void __launch_bounds__(W4_THREADS, 1)
mxk_gemm_bf16_tn_w4e(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 1;
  const int wn = wave_s & 1;

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const DmaStream64<CP> dma_a = make_dma64<CP>(A, lda, m0, lane, wave_s);
  const DmaStream64<CP> dma_b = make_dma64<CP>(Bt, ldb, n0, lane, wave_s);

  const int frow = lane & 15;
  const int fch = (lane >> 4) ^ (frow >> 1);
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
  auto kbytes = [&](int st) { return (st < ns ? st : ns - 1) * BK * 2; };
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    char* buf = smem + s * W4B_STAGE_BYTES;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      dma_a.issue(buf, p, kbytes(s), wave_s);
      dma_b.issue(buf + W4B_OP_BYTES, p, kbytes(s), wave_s);
    }
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);

  for (int s = 0; s < ns; ++s) {
    char* cur = smem + (s & 1) * W4B_STAGE_BYTES;
    char* nxt = smem + ((s + 1) & 1) * W4B_STAGE_BYTES;
    const int kb = kbytes(s + 2);
    // ---- k-step s.0
    __builtin_amdgcn_s_waitcnt(0xC07F);   // set 0 in registers
#pragma unroll
    for (int r = 0; r < 8; ++r) f1b[r] = lds_read_b128(cur + b_base + r * SUB + off_k1);
#pragma unroll
    for (int r = 0; r < 8; ++r) f1a[r] = lds_read_b128(cur + a_base + r * SUB + off_k1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
        if (i == 1 && j == 7) {
          // every wave's reads of `cur` retired -> stage s+2 may land there
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
        }
        if (i >= 2 && i < 6 && (j & 3) == 3) {
          const int p = (i - 2) * 2 + (j >> 2);   // 0..7: A pieces
          dma_a.issue(cur, p, kb, wave_s);
        }
      }
    }
    // stage s+1 (issued 1.5-2 k-steps ago) landed; the 8 newest stay in flight
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- k-step s.1
#pragma unroll
    for (int r = 0; r < 8; ++r) f0b[r] = lds_read_b128(nxt + b_base + r * SUB + off_k0);
#pragma unroll
    for (int r = 0; r < 8; ++r) f0a[r] = lds_read_b128(nxt + a_base + r * SUB + off_k0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
        if (i < 4 && (j & 3) == 3) {
          const int p = i * 2 + (j >> 2);         // 0..7: B pieces
          dma_b.issue(cur + W4B_OP_BYTES, p, kb, wave_s);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + crow;
    uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 128 + ccol;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4_t v = acc[i][j];
      uint2 pk;
      pk.x = mxk::pack2bf(v[0], v[1]);
      pk.y = mxk::pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(cp + j * 16) = pk;
    }
  }
}

// ---------------------------------------------------------------------------
// Schedule 7: the w4b pipeline with 8 waves (2 per SIMD), each owning a
// 128 x 64 block (8 x 4 AGPR tiles).  Every wave issues half the LDS-DMA
// pieces of w4b (8 per stage) and while one wave of a SIMD is held up by a
// DMA issue or an LDS read the other keeps the matrix core busy; the price is
// 1.5x the LDS fragment traffic (each A fragment is read by 4 waves).
// ---------------------------------------------------------------------------
constexpr int W8B_THREADS = 512;

template <int CP>
__device__ __forceinline__ void w8b_issue(const DmaStream64<CP>& d, char* lds_op, int p,
                                          int k_bytes, int wave_s) {
  const int g = p * 8 + wave_s;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(d.rsrc, (lds_void*)(lds_op + g * 1024), 16, d.lane_off,
                                           k_bytes + g * d.piece_stride, 0, CP);
}

template <int CP = 0>
__global__ void __launch_bounds__(W8B_THREADS, 1)
mxk_gemm_bf16_tn_w8b(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                     uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  __shared__ __attribute__((aligned(16))) char smem[2 * W4B_STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave_s >> 2;   // 0..1: 128-row half
  const int wn = wave_s & 3;    // 0..3: 64-column quarter

  const int tiles_m = M / BM, tiles_n = N / BN;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  // DMA pieces g = p*8 + wave (p = 0..3), rows 8g .. 8g+7 -> LDS g*1024;
  // (row >> 1) & 7 = (4 (wave & 1) + (r >> 1)) & 7, so w4b's lane offsets hold
  const DmaStream64<CP> dma_a = make_dma64<CP>(A, lda, m0, lane, wave_s);
  const DmaStream64<CP> dma_b = make_dma64<CP>(Bt, ldb, n0, lane, wave_s);

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

  const int ns = K / BK;
  auto kbytes = [&](int st) { return (st < ns ? st : ns - 1) * BK * 2; };
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    char* buf = smem + s * W4B_STAGE_BYTES;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      w8b_issue<CP>(dma_a, buf, p, kbytes(s), wave_s);
      w8b_issue<CP>(dma_b, buf + W4B_OP_BYTES, p, kbytes(s), wave_s);
    }
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // own pieces of stage 0 landed
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[4], f1a[8], f1b[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = lds_read_b128(smem + a_base + i * SUB + off_k0);
#pragma unroll
  for (int j = 0; j < 4; ++j) f0b[j] = lds_read_b128(smem + b_base + j * SUB + off_k0);

  for (int s = 0; s < ns; ++s) {
    char* cur = smem + (s & 1) * W4B_STAGE_BYTES;
    char* nxt = smem + ((s + 1) & 1) * W4B_STAGE_BYTES;
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mfma_16x16x32_agpr(acc[i][j], f0b[j], f0a[i]);
      }
      if (i < 4) {   // 12 prefetch reads over the first 16 MFMAs of the k-step
        f1b[i] = lds_read_b128(cur + b_base + i * SUB + off_k1);
        f1a[2 * i] = lds_read_b128(cur + a_base + (2 * i) * SUB + off_k1);
        f1a[2 * i + 1] = lds_read_b128(cur + a_base + (2 * i + 1) * SUB + off_k1);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int kb = kbytes(s + 2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mfma_16x16x32_agpr(acc[i][j], f1b[j], f1a[i]);
        if (j == 1) {   // 8 DMA pieces over the k-step: one per 4 MFMAs
          if (i < 4) w8b_issue<CP>(dma_a, cur, i, kb, wave_s);
          else w8b_issue<CP>(dma_b, cur + W4B_OP_BYTES, i - 4, kb, wave_s);
        }
      }
      if (i < 4) {
        f0b[i] = lds_read_b128(nxt + b_base + i * SUB + off_k0);
        f0a[2 * i] = lds_read_b128(nxt + a_base + (2 * i) * SUB + off_k0);
        f0a[2 * i + 1] = lds_read_b128(nxt + a_base + (2 * i + 1) * SUB + off_k0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + crow;
    uint16_t* cp = C + static_cast<size_t>(m) * ldc + n0 + wn * 64 + ccol;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4_t v = acc[i][j];
      uint2 pk;
      pk.x = mxk::pack2bf(v[0], v[1]);
      pk.y = mxk::pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(cp + j * 16) = pk;
    }
  }
}

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
namespace {
// w4i (three-barrier K-tile, scalar-free unrolled loop) + XCD super-block
// map + widened non-temporal stores; 31 (the same with 8-B stores) when C is
// not 16-B aligned or ldc % 8 != 0.  A/B logs: profiles/r1_gemm_w4h/.
constexpr int kDefaultVariant = 34;
constexpr int kDefaultVariantNarrowC = 31;
constexpr int kNumVariants = 36;
// timing ablations and stamp builds: wrong outputs or perturbed schedules
__host__ __device__ constexpr bool is_ablation(int v) {
  return (v >= 9 && v <= 12) || v == 14 || v == 17;
}

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

// the default w4b schedule (ORD 4, VOFF DMA addressing) with tile map MAP and
// epilogue EPI
template <int MAP, int EPI>
void launch_w4b(int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b, uint16_t* c,
                int M, int N, int K, int lda, int ldb, int ldc) {
  hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<0, 4, 32, MAP, EPI>), dim3(nwg), dim3(W4_THREADS), 0,
                     stream, a, b, c, M, N, K, lda, ldb, ldc);
}

template <int MAP, int EPI, int MO = 0, int LATE = 0, int PRIO = 1>
void launch_w4h(int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b, uint16_t* c,
                int M, int N, int K, int lda, int ldb, int ldc) {
  hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4h<MAP, EPI, MO, LATE, PRIO>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b,
                     c, M, N, K, lda, ldb, ldc);
}

template <int MAP, int EPI, int LATE, int R1 = 0>
void launch_w4i(int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b, uint16_t* c,
                int M, int N, int K, int lda, int ldb, int ldc) {
  hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4i<MAP, EPI, LATE, R1>), dim3(nwg), dim3(W4_THREADS), 0, stream,
                     a, b, c, M, N, K, lda, ldb, ldc);
}

void launch_256(int v, int nwg, hipStream_t stream, const void* A, const void* Bt, void* C, int M,
                int N, int K, int lda, int ldb, int ldc) {
  auto* a = static_cast<const uint16_t*>(A);
  auto* b = static_cast<const uint16_t*>(Bt);
  auto* c = static_cast<uint16_t*>(C);
  switch (v) {
    case 0: hipLaunchKernelGGL(mxk_gemm_bf16_tn_256x256<0>, dim3(nwg), dim3(NTHREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 1: hipLaunchKernelGGL(mxk_gemm_bf16_tn_256x256<1>, dim3(nwg), dim3(NTHREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 2: hipLaunchKernelGGL(mxk_gemm_bf16_tn_256x256<2>, dim3(nwg), dim3(NTHREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 3: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4<4, 0>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 4: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w8<4>), dim3(nwg), dim3(W8_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 5: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<0>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 6: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<0, 0, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 7: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w8b<0>), dim3(nwg), dim3(W8B_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 8: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4e<32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 9: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<1>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 10: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<2>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 11: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<3>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 12: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<5, 0, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 13: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<0, 4, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 14: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<5, 4, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 15: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4b<0, 5, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 16: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4q<0, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 17: hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4q<1, 32>), dim3(nwg), dim3(W4_THREADS), 0, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 18: launch_w4b<1, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 19: launch_w4b<0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 20: launch_w4b<1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 21: {
      const int grid = nwg < num_cus() ? nwg : num_cus();
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4p<1>), dim3(grid), dim3(W4_THREADS), 0, stream, a, b,
                         c, M, N, K, lda, ldb, ldc);
      break;
    }
    case 22: launch_w4h<0, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 23: launch_w4h<0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 24: launch_w4h<1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 25: launch_w4h<1, 1, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 26: launch_w4h<1, 1, 0, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 27: launch_w4h<1, 1, 0, 0, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 28: launch_w4h<1, 1, 1, 1, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 29: launch_w4i<1, 1, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 30: launch_w4i<1, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 31: launch_w4i<1, 0, 0>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 32: launch_w4i<1, 1, 1, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 33: launch_w4i<1, 1, 0, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 34: launch_w4i<1, 2, 1>(nwg, stream, a, b, c, M, N, K, lda, ldb, ldc); break;
    case 35: {
      const int grid = nwg < num_cus() ? nwg : num_cus();
      hipLaunchKernelGGL((mxk_gemm_bf16_tn_w4ip<1, 2>), dim3(grid), dim3(W4_THREADS), 0, stream, a,
                         b, c, M, N, K, lda, ldb, ldc);
      break;
    }
  }
}
}  // namespace

// Benchmark hook: run schedule `variant` of the 256x256 kernel (fast shapes only).
MXK_API int mxk_gemm_bf16_tn_variant(const void* A, const void* Bt, void* C, int M, int N, int K,
                                     int lda, int ldb, int ldc, int variant, hipStream_t stream) {
  if (M % BM || N % BN || K % BK || variant < 0 || variant >= kNumVariants)
    return static_cast<int>(hipErrorInvalidValue);
  launch_256(variant, (M / BM) * (N / BN), stream, A, Bt, C, M, N, K, lda, ldb, ldc);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_gemm_bf16_tn_num_variants(void) { return kNumVariants; }

// Diagnostic stamps of variant 12: out[0..2] = summed cycles of k-step 0,
// wait + barrier, k-step 1 over all waves; out[3] = waves.  reset != 0
// clears them.
MXK_API int mxk_gemm_bf16_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_w4b_stamps), sizeof(unsigned long long) * 4);
  if (e == hipSuccess && reset) {
    const unsigned long long z[4] = {0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_w4b_stamps), z, sizeof(z));
  }
  return static_cast<int>(e);
}
MXK_API int mxk_gemm_bf16_tn_is_ablation(int variant) { return is_ablation(variant) ? 1 : 0; }

MXK_API int mxk_gemm_bf16_tn(const void* A, const void* Bt, void* C, int M, int N, int K,
                             int lda, int ldb, int ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return static_cast<int>(hipErrorInvalidValue);
  const bool fast = (M % BM == 0) && (N % BN == 0) && (K % BK == 0) && (lda % 8 == 0) &&
                    (ldb % 8 == 0) && (ldc % 4 == 0) &&
                    (reinterpret_cast<uintptr_t>(A) % 16 == 0) &&
                    (reinterpret_cast<uintptr_t>(Bt) % 16 == 0) &&
                    (reinterpret_cast<uintptr_t>(C) % 8 == 0);
  if (fast) {
    const int nwg = (M / BM) * (N / BN);
    const bool wide_c = (ldc % 8 == 0) && (reinterpret_cast<uintptr_t>(C) % 16 == 0);
    launch_256(wide_c ? kDefaultVariant : kDefaultVariantNarrowC, nwg, stream, A, Bt, C, M, N, K,
               lda, ldb, ldc);
  } else {
    dim3 grid((N + 63) / 64, (M + 63) / 64);
    hipLaunchKernelGGL(mxk_gemm_bf16_tn_generic, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(Bt),
                       static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc);
  }
  MXK_RETURN_LAUNCH_STATUS();
}

// 1 if (M, N, K) takes the tiled MFMA fast path.
MXK_API int mxk_gemm_bf16_tn_is_fast(int M, int N, int K) {
  return (M % BM == 0) && (N % BN == 0) && (K % BK == 0);
}
