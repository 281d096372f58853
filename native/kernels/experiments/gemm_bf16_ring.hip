// CDNA4 bf16 MFMA GEMM, deep-ring variant of gemm_bf16.hip's 256x256 kernel.
//
//   C[M][N] (bf16) = A[M][K] (bf16, K-major) . Bt[N][K]^T (bf16, K-major)
//
// Same workgroup shape as the default schedule (4 waves, one per SIMD, each
// owning 128x128 of C in 256 AGPR accumulators, v_mfma_f32_16x16x32_bf16,
// LDS-DMA staging, LDS-staged C store, XCD-aware super-block tile map), but
// the LDS is a ring of R slots of ONE 32-deep k-step each (32 KiB: A and B
// 256 rows x 64 B) instead of two 64-deep stages:
//
//   * the refill of a slot is issued R steps ahead (R = 5: the whole 160 KiB),
//     so a DMA piece has ~3 k-steps (~3000 cycles) to land before the barrier
//     that publishes it, against ~1.5-3 in the two-stage kernel, whose 16384^3
//     runs lose time when the pieces miss to HBM / MALL (a one-barrier
//     two-stage schedule with ~1.5 steps of slack ran 10 % slower there,
//     profiles/r3_gemm/);
//   * one barrier per k-step (64 MFMAs per wave): behind it every wave's
//     fragment reads of the slot just read retired (lgkmcnt(0)) and the slot
//     two steps ahead landed (counted vmcnt), so the next step reads it and
//     the step after refills the slot this step read;
//   * 8 DMA pieces per wave per step, spread one per 7 MFMAs.
//
// Slot layout: row r at r * 64 B, logical 16-B chunk c (k 8c..8c+7) at
// physical position c ^ G(r), G(r) = {0, 2, 3, 1}[(r >> 2) & 3].  A
// ds_read_b128 fragment (16 rows x 4 chunks) then hits every bank once in
// each of the four 16-lane groups gfx950 services per cycle (MI355X_MICROARCH
// LDS table; tests/test_gemm_swizzle.py checks it).  LDS-DMA writes lane L of
// a piece at piece_base + 16 L, so the swizzle goes on the global side: lane
// L = 4 r + q of a 16-row piece loads logical chunk q ^ G(r).
#include "mx_common.h"

namespace {

constexpr int RB = 256;                 // macro tile M = N
constexpr int RK = 32;                  // k per slot
constexpr int ROP = RB * RK * 2;        // 16 KiB per operand per slot
constexpr int RSLOT = 2 * ROP;          // 32 KiB
constexpr int RTHREADS = 256;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int ring_g(int r) {   // G(r) for r & 15 in a 16-row tile
  return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;   // {0, 2, 3, 1}
}

__device__ __forceinline__ void rmfma(f32x4_t& acc, bf16x8_t a, bf16x8_t b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ bf16x8_t rd128(const char* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// The matrix core is still reading an inline-asm MFMA's A/B registers a few
// cycles after issue, but hipcc (blind to the asm) treats them as free right
// after it and may give them to its own VALU temporaries (seen: an address
// v_add into the B fragment one instruction after its last MFMA; ~1000 wrong
// outputs per 256x256 tile).  One statement that reads every fragment of the
// step and then waits keeps them all live to the end of the step and covers
// the last MFMAs' operand reads (tests/test_isa_hazards.py audits it).
__device__ __forceinline__ void mfma_sources_done(const bf16x8_t (&a)[8], const bf16x8_t (&b)[8]) {
  asm volatile("s_nop 4" ::"v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
               "v"(a[6]), "v"(a[7]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]),
               "v"(b[5]), "v"(b[6]), "v"(b[7]));
}

// One operand's DMA: 256-row panel, 4 pieces of 16 rows per wave per slot.
struct RingDma {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff[4];
  __device__ __forceinline__ void issue(char* lds_op, int j, int wave, int kbytes) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_op + (4 * j + wave) * 1024), 16,
                                             voff[j], kbytes, 0, 0);
  }
};

__device__ __forceinline__ RingDma make_ring_dma(const uint16_t* src, int ld, int row0, int lane,
                                                 int wave) {
  RingDma d;
  d.rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(src + static_cast<size_t>(row0) * ld), 0, RB * ld * 2, 0x00020000);
  const int r = lane >> 2, q = lane & 3;
  const int c = q ^ ring_g(r);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    d.voff[j] = static_cast<uint32_t>(((4 * j + wave) * 16 + r) * ld * 2 + c * 16);
  return d;
}

// Wait until at most N vector-memory ops of this wave are outstanding.
template <int N>
__device__ __forceinline__ void vmwait() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else static_assert(N < 0, "vmwait: add the count");
}

// One k-step: 64 MFMAs on the fragments in (ca, cb); the next step's
// fragments read from `nxt` (slot of step s+1) into (na, nb); DMA of stage
// s+R into `refill` (the slot of step s) when DMA; then lgkmcnt(0) + the
// stage-(s+2) wait + barrier.  VM: the vmcnt of that wait (8 per younger
// stage in flight).
template <bool READ, bool DMA, int VM>
__device__ __forceinline__ void ring_step(f32x4_t (&acc)[8][8], const bf16x8_t (&ca)[8],
                                          const bf16x8_t (&cb)[8], bf16x8_t (&na)[8],
                                          bf16x8_t (&nb)[8], const char* nxt, int a_off, int b_off,
                                          char* refill, const RingDma& da, const RingDma& db,
                                          int wave, int kdma) {
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    const int i = m >> 3, j = m & 7;
    rmfma(acc[i][j], cb[j], ca[i]);
    if (READ && (m & 1) && m < 32) {
      const int r = m >> 1;   // B fragments first (the next step's first MFMAs use B 0..7)
      if (r < 8) nb[r] = rd128(nxt + ROP + b_off + r * 1024);
      else na[r - 8] = rd128(nxt + a_off + (r - 8) * 1024);
    }
    if (DMA && m >= 4 && (m - 4) % 7 == 0 && (m - 4) / 7 < 8) {
      const int p = (m - 4) / 7;
      if (p & 1) db.issue(refill + ROP, p >> 1, wave, kdma);
      else da.issue(refill, p >> 1, wave, kdma);
    }
    if (m == 60) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this step's reads retired
    if (m == 61) vmwait<VM>();                           // stage s+2 landed (this wave's pieces)
    if (m == 62) __builtin_amdgcn_s_barrier();
  }
  mfma_sources_done(ca, cb);
}

// EXTRA = (K / 32 - 1) odd, chosen by the launcher: each instance has one
// tail with fixed fragment registers.  (A runtime branch needs either two
// tails, which spill, or a register copy of one set into the other right in
// front of asm MFMAs, whose operand reads the hazard recognizer does not see:
// acc[0][0] of every wave came out wrong, scripts/gpu/ring_diag.py.)
template <int R, bool EXTRA>
__global__ void __launch_bounds__(RTHREADS, 1)
mxk_gemm_bf16_tn_ring(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                      uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  static_assert(R >= 3 && R * RSLOT <= 160 * 1024, "ring: 3..5 slots");
  constexpr int VM = 8 * (R - 2);       // pieces younger than stage s+2 in steady state
  __shared__ __attribute__((aligned(16))) char smem[R * RSLOT];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int m0, n0;
  mxk::w4b_tile<1>(blockIdx.x, gridDim.x, M / RB, N / RB, &m0, &n0);
  const RingDma da = make_ring_dma(A, lda, m0, lane, wave);
  const RingDma db = make_ring_dma(Bt, ldb, n0, lane, wave);
  const int fr = lane & 15;
  const int foff = fr * 64 + (((lane >> 4) ^ ring_g(fr)) << 4);
  const int a_off = wm * 8 * 1024 + foff;    // the wave's 128 A rows: fragments i at +1 KiB
  const int b_off = wn * 8 * 1024 + foff;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = K / RK;
  // prologue: stages 0 .. R-1 (clamped to the last one when K is short)
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int kb = (t < ns ? t : ns - 1) * RK * 2;
    char* slot = smem + t * RSLOT;
#pragma unroll
    for (int j = 0; j < 4; ++j) da.issue(slot, j, wave, kb);
#pragma unroll
    for (int j = 0; j < 4; ++j) db.issue(slot + ROP, j, wave, kb);
  }
  vmwait<8 * (R - 1)>();                     // stage 0
  __builtin_amdgcn_s_barrier();
  bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = rd128(smem + ROP + b_off + j * 1024);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = rd128(smem + a_off + i * 1024);
  vmwait<VM>();                              // stage 1
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();

  // steady state: step s refills its own slot with stage s + R (clamped)
  int s = 0;
  int slot = 0;                               // slot of step s, in bytes
  auto next_slot = [](int sl) { return sl + RSLOT == R * RSLOT ? 0 : sl + RSLOT; };
  for (; s + 2 <= ns - 1; s += 2) {
    const int sl1 = next_slot(slot), sl2 = next_slot(sl1);
    const int k0 = (s + R < ns ? s + R : ns - 1) * RK * 2;
    const int k1 = (s + 1 + R < ns ? s + 1 + R : ns - 1) * RK * 2;
    ring_step<true, true, VM>(acc, fa0, fb0, fa1, fb1, smem + sl1, a_off, b_off, smem + slot, da,
                              db, wave, k0);
    ring_step<true, true, VM>(acc, fa1, fb1, fa0, fb0, smem + sl2, a_off, b_off, smem + sl1, da,
                              db, wave, k1);
    slot = sl2;
  }
  if constexpr (EXTRA) {   // ns - 1 odd: one more step with a successor (into set 1)
    const int sl1 = next_slot(slot);
    const int k0 = (s + R < ns ? s + R : ns - 1) * RK * 2;
    ring_step<true, true, VM>(acc, fa0, fb0, fa1, fb1, smem + sl1, a_off, b_off, smem + slot, da,
                              db, wave, k0);
    ring_step<false, false, VM>(acc, fa1, fb1, fa0, fb0, smem, a_off, b_off, smem, da, db, wave, 0);
  } else {
    ring_step<false, false, VM>(acc, fa0, fb0, fa1, fb1, smem, a_off, b_off, smem, da, db, wave, 0);
  }
  // every clamped refill has landed and every wave is past its last read
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  mxk::mfma_drain(acc);
  mxk::store_block_lds<true>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane,
                             smem + wave * mxk::kStoreLdsWave);
}

}  // namespace

// Launcher for gemm_bf16.hip's schedule table (M, N multiples of 256, K of
// 32, 16-B aligned operands, ldc % 8 == 0 — checked by the caller).
int mxk_gemm_bf16_tn_ring_launch(int slots, const void* A, const void* Bt, void* C, int M, int N,
                                 int K, int lda, int ldb, int ldc, hipStream_t stream) {
  const dim3 grid((M / RB) * (N / RB));
  auto* a = static_cast<const uint16_t*>(A);
  auto* b = static_cast<const uint16_t*>(Bt);
  auto* c = static_cast<uint16_t*>(C);
  const bool extra = ((K / RK - 1) & 1) != 0;
  if (slots == 4 && extra)
    hipLaunchKernelGGL((mxk_gemm_bf16_tn_ring<4, true>), grid, dim3(RTHREADS), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc);
  else if (slots == 4)
    hipLaunchKernelGGL((mxk_gemm_bf16_tn_ring<4, false>), grid, dim3(RTHREADS), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc);
  else if (slots == 5 && extra)
    hipLaunchKernelGGL((mxk_gemm_bf16_tn_ring<5, true>), grid, dim3(RTHREADS), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc);
  else if (slots == 5)
    hipLaunchKernelGGL((mxk_gemm_bf16_tn_ring<5, false>), grid, dim3(RTHREADS), 0, stream, a, b, c,
                       M, N, K, lda, ldb, ldc);
  else
    return static_cast<int>(hipErrorInvalidValue);
  return static_cast<int>(hipGetLastError());
}
