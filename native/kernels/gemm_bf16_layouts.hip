// CDNA4 bf16 MFMA GEMM for every operand layout of a linear layer's training
// step:  C[M][N] (bf16) = sum_k A(m, k) B(k, n), fp32 accumulation.
//
//   forward  y  = x  W^T : A = x  [M][K] (K-major), B = W  [N][K] (K-major)
//   dgrad    dx = dy W   : A = dy [M][K] (K-major), B = W  [K][N] (N-major)
//   wgrad    dW = dy^T x : A = dy [K][M] (M-major), B = x  [K][N] (N-major)
//
// hipBLASLt runs the N-major ("NT"/"NN") layouts of the Llama-3-8B step at
// 970-1280 TF/s against ~1590 for the K-major forward GEMMs (profiles/r1_ddp),
// so the backward GEMMs get the same 4-wave BK=64 LDS-DMA schedule as
// gemm_bf16.hip's w4b kernel with an operand-layout template:
//
// * K-major operand: LDS-DMA pieces of 8 rows x 128 B, 16-B chunk c of row r
//   at c ^ ((r>>1)&7), fragments by ds_read_b128 (as w4b).
// * N/M-major operand: the stage is 64 k-rows x 256 columns (512 B per row);
//   a DMA piece is 2 k-rows, rows grouped by 8 with a 128-B pad per group
//   (group stride 4224 B) and chunk c of row k at c ^ 2(k&3).  Fragments are
//   the transposed reads ds_read_b64_tr_b16 (two per 16x16x32 operand), which
//   deliver 8 consecutive k of one column exactly like a ds_read_b128 of a
//   K-major row - so both kinds mix in one MFMA.  The pad puts the two 16-lane
//   groups of each half-wave (rows k and k+8) on disjoint bank halves and the
//   XOR separates the four rows of a group: conflict-free
//   (tests/test_gemm_layouts.py).
// LDS: 2 stages x (A + B) <= 132 KiB, one 4-wave workgroup per CU, 128x128
// AGPR accumulators per wave, one barrier per 64-deep stage.
#include <mutex>
#include <map>
#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "mx_common.h"

#include <cstdlib>

namespace {
constexpr int XT = 256;          // threads (4 waves)
constexpr int XBM = 256;         // macro tile M = N = 256
constexpr int XBK = 64;          // k per stage
constexpr int XGROUP_M = 8;
constexpr int TGROUP = 4224;     // bytes per 8 k-rows (4096 + 128 pad)
constexpr int KSTEP_T = 4 * TGROUP;   // 32 k-rows

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void xmfma(f32x4_t& acc, bf16x8_t a, bf16x8_t b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

using mxk::u32x4;
using mxk::make_rsrc;
using mxk::dma16;

__device__ __forceinline__ bf16x4_t tr_b64(const char* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  // a plain address-space cast (not via an integer) keeps `base + constant`
  // visible, so the constant lands in the instruction's offset field
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
}

template <bool NMAJOR>
struct XOp;

// K-major operand [rows][K]: identical to the w4b kernel's operand.
template <>
struct XOp<false> {
  static constexpr int BYTES = 256 * 128;
  u32x4 rsrc;
  uint32_t lane_off, piece_stride;
  uint32_t voff[8];              // lane_off + (p*4 + wave) * piece_stride
  const char* base;
  unsigned bytes;
  int off0, off1;
  __device__ __forceinline__ void init(const uint16_t* src, int ld, int row0, int K, int lane,
                                       int wave) {
    rsrc = make_rsrc(src + static_cast<size_t>(row0) * ld, 256u * ld * 2u);
    base = reinterpret_cast<const char*>(src + static_cast<size_t>(row0) * ld);
    bytes = 256u * ld * 2u;
    const int r = lane >> 3;
    const int c = (lane & 7) ^ ((4 * (wave & 1) + (r >> 1)) & 7);
    lane_off = static_cast<uint32_t>(r * ld * 2 + c * 16);
    piece_stride = static_cast<uint32_t>(8 * ld * 2);
#pragma unroll
    for (int p = 0; p < 8; ++p) voff[p] = lane_off + (p * 4 + wave) * piece_stride;
    const int frow = lane & 15;
    const int fch = (lane >> 4) ^ (frow >> 1);
    off0 = frow * 128 + fch * 16;
    off1 = frow * 128 + (fch ^ 4) * 16;
    (void)K;
  }
  __device__ __forceinline__ void issue(char* lds, int p, int kstage, int wave) const {
    const int g = p * 4 + wave;
    // hipBLASLt-style addressing: per-piece VGPR offset, k folded into the base
    dma16(make_rsrc(base + kstage * (XBK * 2), bytes), lds + g * 1024, voff[p], 0);
  }
  // x2 kernel: fixed panel descriptor, the k offset of the stage as soffset
  __device__ __forceinline__ uint32_t kstep() const { return XBK * 2; }
  // x2 kernel: LDS destinations as smem32 + (lds - smem), scalar arithmetic
  const char* sm = nullptr;
  uint32_t sm32 = 0;
  __device__ __forceinline__ void set_lds(const char* smem, uint32_t smem32) {
    sm = smem;
    sm32 = smem32;
  }
  __device__ __forceinline__ void issue_s(char* lds, int p, uint32_t soff, int wave) const {
    mxk::dma16m(rsrc, sm32 + static_cast<uint32_t>(lds - sm) + (p * 4 + wave) * 1024, voff[p],
                soff);
  }
  // fragment of 16-row subtile i (i = 0..15 over the 256 rows), k-step ks
  __device__ __forceinline__ bf16x8_t frag(const char* lds, int i, int ks) const {
    return *reinterpret_cast<const bf16x8_t*>(lds + i * 2048 + (ks ? off1 : off0));
  }
};

// N/M-major operand [K][cols]: 64 k-rows x 256 columns per stage.
template <>
struct XOp<true> {
  static constexpr int BYTES = 8 * TGROUP;
  u32x4 rsrc;
  uint32_t lane_off, piece_stride, kstride;
  uint32_t voff[8];
  const char* base;
  unsigned bytes;
  int roff[4];                   // read offset of subtile r (mod 4), XOR folded in
  __device__ __forceinline__ void init(const uint16_t* src, int ld, int col0, int K, int lane,
                                       int wave) {
    rsrc = make_rsrc(src + col0, static_cast<unsigned>(K) * ld * 2u);
    base = reinterpret_cast<const char*>(src + col0);
    bytes = static_cast<unsigned>(K) * ld * 2u;
    // piece g = 4p + wave holds k-rows 8p + 2 wave + h (h = lane >> 5)
    const int h = lane >> 5, slot = lane & 31;
    const int c = slot ^ (2 * ((2 * wave + h) & 3));
    lane_off = static_cast<uint32_t>(h * ld * 2 + c * 16);
    piece_stride = static_cast<uint32_t>(2 * ld * 2);
    kstride = static_cast<uint32_t>(XBK * ld * 2);
#pragma unroll
    for (int p = 0; p < 8; ++p) voff[p] = lane_off + (p * 4 + wave) * piece_stride;
    // transposed-read lane constants: group G, row q, column pair b, half-chunk
    const int G = lane >> 4, i16 = lane & 15, q = i16 >> 2;
    // subtile i sits at column byte (32 i) ^ 32q = 32 (i & ~3) + ((32 (i & 3)) ^ 32q):
    // one VGPR per (i & 3), everything else an immediate offset of the read
    const int base_off = G * TGROUP + q * 512 + ((i16 & 3) >> 1) * 16 + 8 * (i16 & 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) roff[r] = base_off + ((32 * r) ^ (32 * q));
  }
  __device__ __forceinline__ void issue(char* lds, int p, int kstage, int wave) const {
    const uint32_t k_off = kstage * kstride;
    dma16(make_rsrc(base + k_off, bytes - k_off), lds + p * TGROUP + wave * 1024, voff[p], 0);
  }
  __device__ __forceinline__ uint32_t kstep() const { return kstride; }
  const char* sm = nullptr;
  uint32_t sm32 = 0;
  __device__ __forceinline__ void set_lds(const char* smem, uint32_t smem32) {
    sm = smem;
    sm32 = smem32;
  }
  __device__ __forceinline__ void issue_s(char* lds, int p, uint32_t soff, int wave) const {
    mxk::dma16m(rsrc, sm32 + static_cast<uint32_t>(lds - sm) + p * TGROUP + wave * 1024, voff[p],
                soff);
  }
  __device__ __forceinline__ bf16x8_t frag(const char* lds, int i, int ks) const {
    const char* p = lds + roff[i & 3] + 32 * (i & ~3) + ks * KSTEP_T;
    const bf16x4_t lo = tr_b64(p);
    const bf16x4_t hi = tr_b64(p + 2048);
    bf16x8_t a;
    a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
    a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
    return a;
  }
};
}  // namespace

template <bool AN, bool BN>
__global__ void __launch_bounds__(XT, 1)
mxk_gemm_bf16_x_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                       uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  constexpr int A_BYTES = XOp<AN>::BYTES;
  constexpr int STAGE = A_BYTES + XOp<BN>::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1;
  const int wn = wave & 1;

  const int tiles_m = M / XBM, tiles_n = N / XBM;
  const int wgid = mxk::xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = XGROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * XGROUP_M;
  const int gsize = min(tiles_m - first_m, XGROUP_M);
  const int in_group = wgid - group * per_group;
  const int m0 = (first_m + in_group % gsize) * XBM;
  const int n0 = (in_group / gsize) * XBM;

  XOp<AN> oa;
  XOp<BN> ob;
  oa.init(A, lda, m0, K, lane, wave);
  ob.init(B, ldb, n0, K, lane, wave);

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = K / XBK;
  auto kst = [&](int st) { return st < ns ? st : ns - 1; };
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    char* buf = smem + s * STAGE;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      oa.issue(buf, p, kst(s), wave);
      ob.issue(buf + A_BYTES, p, kst(s), wave);
    }
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // own pieces of stage 0 landed
  __builtin_amdgcn_s_barrier();

  // wave (wm, wn) owns subtiles wm*8 .. wm*8+7 of A and wn*8 .. of B
  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = oa.frag(smem, wm * 8 + i, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = ob.frag(smem + A_BYTES, wn * 8 + j, 0);

  for (int s = 0; s < ns; ++s) {
    char* cur = smem + (s & 1) * STAGE;
    char* nxt = smem + ((s + 1) & 1) * STAGE;
    // ---- k-step s.0: MFMAs on set 0, prefetch set 1 from `cur`
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xmfma(acc[i][j], f0b[j], f0a[i]);
        if ((j & 3) == 3) {
          const int r = i * 2 + (j >> 2);
          if (r < 8) f1b[r] = ob.frag(cur + A_BYTES, wn * 8 + r, 1);
          else f1a[r - 8] = oa.frag(cur, wm * 8 + r - 8, 1);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // own pieces of stage s+1 landed
    __builtin_amdgcn_s_barrier();
    // ---- k-step s.1: MFMAs on set 1, prefetch set 0 of stage s+1 from
    //      `nxt`, DMA stage s+2 into `cur` (consumed: certified by the barrier)
    const int k2 = kst(s + 2);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xmfma(acc[i][j], f1b[j], f1a[i]);
        if ((j & 3) == 1) {
          const int r = i * 2 + (j >> 2);
          if (r < 8) f0b[r] = ob.frag(nxt + A_BYTES, wn * 8 + r, 0);
          else f0a[r - 8] = oa.frag(nxt, wm * 8 + r - 8, 0);
        }
        if ((j & 3) == 3) {
          const int p = i * 2 + (j >> 2);
          if (p < 8) oa.issue(cur, p, k2, wave);
          else ob.issue(cur + A_BYTES, p - 8, k2, wave);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mxk::mfma_drain(acc);

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
// x2: the layout-generic GEMM on gemm_bf16.hip's w4i schedule (three
// barriers per K-tile with in-place refill of the consumed stage, K loop
// unrolled by two with compile-time LDS bases, the stage's k offset as the
// DMA soffset on a fixed descriptor, DMA-free last two K-tiles, XCD
// super-block tile map, widened store tail).  m = MFMA index 0..127 of a
// K-tile; "read" = one operand fragment (one ds_read_b128 for a K-major
// operand, two ds_read_b64_tr_b16 for an N/M-major one):
//   m 1..15 odd   A k-half-1 fragments from X           m 19  barrier #1
//   m 21..49 /4   B k-half-1 fragments from X
//   m 23..51 /4   DMA of stage s+2, A pieces -> X.A     m 55  barrier #2
//   m 57..99 /6   DMA of stage s+2, B pieces -> X.B
//   m 96          vmcnt(15) + barrier #3 (stage s+1 in Y landed everywhere)
//   m 97..127 odd next k-half-0 fragments from Y (B, then A)
// MODE 1: with DMA; 2: no DMA, vmcnt(0) at barrier #3; 3: last K-tile.
// ---------------------------------------------------------------------------
// VMX >= 0 replaces the stage wait's vmcnt (the trickle kernel's C stores
// sit among the DMA pieces); HOOK(m) runs after MFMA m.
template <bool AN, bool BN, int PAR, int MODE, int VMX = -1, class HOOK = mxk::NoHook,
          int ORDER = 0>
__device__ __forceinline__ void x2_ktile(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                         bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                         bf16x8_t (&f1b)[8], char* smem, const XOp<AN>& oa,
                                         const XOp<BN>& ob, int wm, int wn, uint32_t soa,
                                         uint32_t sob, int wave, int par = 0,
                                         const HOOK& hook = HOOK{}) {
  constexpr int A_BYTES = XOp<AN>::BYTES;
  constexpr int STAGE = A_BYTES + XOp<BN>::BYTES;
  const int px = PAR == 2 ? par : PAR;
  char* X = smem + px * STAGE;
  char* Y = smem + (px ^ 1) * STAGE;
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int o = 0; o < 8; ++o) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int m = h * 64 + o * 8 + q;
        // ORDER 0: A fragment outer; 1: B outer (srcA held for 8 MFMAs)
        const int i = ORDER ? q : o, j = ORDER ? o : q;
        if (h == 0) xmfma(acc[i][j], f0b[j], f0a[i]);
        else xmfma(acc[i][j], f1b[j], f1a[i]);
        hook(m);
        if (m < 16 && (m & 1)) f1a[m >> 1] = oa.frag(X, wm * 8 + (m >> 1), 1);
        if (MODE == 1 && m == 19) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
        }
        if (m >= 20 && m < 52 && (m & 3) == 1)
          f1b[(m - 21) >> 2] = ob.frag(X + A_BYTES, wn * 8 + ((m - 21) >> 2), 1);
        if (MODE == 1 && m >= 20 && m < 52 && (m & 3) == 3) oa.issue_s(X, (m - 23) >> 2, soa, wave);
        if (MODE == 1 && m == 55) {
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
        }
        if (MODE == 1 && m >= 57 && (m - 57) % 6 == 0 && (m - 57) / 6 < 8)
          ob.issue_s(X + A_BYTES, (m - 57) / 6, sob, wave);
        if (MODE != 3 && m == 96) {
          if constexpr (MODE == 1) mxk::vm_wait_n<(VMX >= 0 ? VMX : 15)>();
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        if (MODE != 3 && m > 96 && (m & 1)) {
          const int r = (m - 97) >> 1;
          if (r < 8) f0b[r] = ob.frag(Y + A_BYTES, wn * 8 + r, 0);
          else f0a[r - 8] = oa.frag(Y, wm * 8 + r - 8, 0);
        }
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

// SCHED 1: the same K-tile at hipBLASLt's instruction positions
// (mxk::SchedHB; a "read" is one operand fragment as above).
template <class S, bool AN, bool BN, int PAR, int MODE, int VMX = -1, class HOOK = mxk::NoHook,
          int ORDER = 0>
__device__ __forceinline__ void x2_ktile_tab(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                             bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                             bf16x8_t (&f1b)[8], char* smem, const XOp<AN>& oa,
                                             const XOp<BN>& ob, int wm, int wn, uint32_t soa,
                                             uint32_t sob, int wave, int par = 0,
                                             const HOOK& hook = HOOK{}) {
  constexpr int A_BYTES = XOp<AN>::BYTES;
  constexpr int STAGE = A_BYTES + XOp<BN>::BYTES;
  const int px = PAR == 2 ? par : PAR;
  char* X = smem + px * STAGE;
  char* Y = smem + (px ^ 1) * STAGE;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int o = 0; o < 8; ++o) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int m = h * 64 + o * 8 + q;
        // ORDER 0: A fragment outer; 1: B outer (srcA held for 8 MFMAs)
        const int i = ORDER ? q : o, j = ORDER ? o : q;
        if (h == 0) xmfma(acc[i][j], f0b[j], f0a[i]);
        else xmfma(acc[i][j], f1b[j], f1a[i]);
        hook(m);
        if (S::a1(m) >= 0) f1a[S::a1(m)] = oa.frag(X, wm * 8 + S::a1(m), 1);
        if (MODE == 1 && m == S::W1) __builtin_amdgcn_s_waitcnt(0xC07F);
        if (MODE == 1 && m == S::B1) __builtin_amdgcn_s_barrier();
        if (MODE == 1 && S::adma(m) >= 0) oa.issue_s(X, S::adma(m), soa, wave);
        if (S::b1(m) >= 0) f1b[S::b1(m)] = ob.frag(X + A_BYTES, wn * 8 + S::b1(m), 1);
        if (MODE == 1 && m == S::W2) __builtin_amdgcn_s_waitcnt(0xC07F);
        if (MODE == 1 && m == S::B2) __builtin_amdgcn_s_barrier();
        if (MODE == 1 && S::bdma(m) >= 0) ob.issue_s(X + A_BYTES, S::bdma(m), sob, wave);
        if (MODE != 3 && m == S::W3) {
          if constexpr (MODE == 1) {
            mxk::vm_wait_n<(VMX >= 0 ? VMX : S::VM3)>();
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
        if (MODE != 3 && m == S::B3) __builtin_amdgcn_s_barrier();
        if (MODE != 3 && S::k0(m) >= 0) {
          const int r = S::k0(m);
          if (r < 8) f0b[r] = ob.frag(Y + A_BYTES, wn * 8 + r, 0);
          else f0a[r - 8] = oa.frag(Y, wm * 8 + r - 8, 0);
        }
      }
    }
  }
}

// VMD: how many vector-memory ops beyond the schedule's own pieces are
// younger than the stage being waited for (trickle stores), added to its count.
template <int SCHED, bool AN, bool BN, int PAR, int MODE, int VMD = 0, class HOOK = mxk::NoHook>
__device__ __forceinline__ void x2_ktile_s(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                           bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                           bf16x8_t (&f1b)[8], char* smem, const XOp<AN>& oa,
                                           const XOp<BN>& ob, int wm, int wn, uint32_t soa,
                                           uint32_t sob, int wave, int par = 0,
                                           const HOOK& hook = HOOK{}) {
  // SCHED bit 0: hipBLASLt's positions (x2_ktile_tab); bit 1: B-outer MFMA order
  if constexpr ((SCHED & 1) == 1)
    x2_ktile_tab<mxk::SchedHB, AN, BN, PAR, MODE, (VMD ? mxk::SchedHB::VM3 + VMD : -1), HOOK,
                 (SCHED >> 1) & 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, soa, sob, wave,
                                   par, hook);
  else
    x2_ktile<AN, BN, PAR, MODE, (VMD ? 15 + VMD : -1), HOOK, (SCHED >> 1) & 1>(
        acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, soa, sob, wave, par, hook);
}

// EPI 0: 8-B stores, 1: 16-B stores through LDS (whole lines), 2: SwiGLU backward, 3: SwiGLU
// backward with 16-B g / u accesses (mxk::swiglu_bwd_block_wide), 4: the same
// staged through LDS so each access covers whole lines (swiglu_bwd_block_lds)
// (mxk::swiglu_bwd_block: C = d[g | u], aux = [g | u], both row stride ldc,
// u at column offset N).
// SPLIT (split tail): the launch after the whole-tile one (grid q_full,
// tiles [0, q_full) of the same map) covers the last T - q_full tiles (at
// most half a round) as two K halves each, one workgroup per half
// (blockIdx 2t + h), so the 2(T - q_full) halves fill the final round
// instead of leaving half the CUs idle.  A half writes its fp32 partial
// tile to ws[2t + h] ([256][256]); mxk_gemm_split_fixup sums the pair into
// C.  A separate kernel (not a branch of the whole-tile one): with both
// epilogues in one body the allocator spilled accumulators, and a spill
// store of an AGPR right behind its inline-asm MFMA reads a stale value.
// EPI 4 (SwiGLU backward): pass 0's g / u rows of each wave by LDS-DMA into
// the stage the last K-tile does not read, issued right after the second-to-
// last K-tile's stage barrier (m 96; that stage is free everywhere by then):
// 16 pieces per wave (8 of g, 8 of u), each 4 rows x 256 B, one per MFMA from
// m 97.  The epilogue's vmcnt(0) + barrier covers them.
struct GuPrefetch : mxk::NoHook {
  mxk::u32x4 rsrc;
  uint32_t voff;     // this lane's (row, column) of piece 0, bytes
  uint32_t rowstep;  // 4 rows, bytes
  uint32_t fbytes;   // F columns (g -> u), bytes
  uint32_t lds;      // LDS address of this wave's 16 KiB
  __device__ __forceinline__ void operator()(int m) const {
    if (m >= 97 && m < 113) {
      const int q = m - 97, u = q >> 3, i = q & 7;
      mxk::dma16m(rsrc, lds + u * 8192 + i * 1024, voff + i * rowstep + u * fbytes, 0);
    }
  }
};

// STAG (EPI 4 only, the down projection's dgrad-SwiGLU): rounds staggered by
// XCD group (mx_common.h stagger_part_xcd; TN schedule 57's mapping): XCDs 4-7
// run half a tile out of phase with XCDs 0-3, so the two halves of the chip
// take turns with the epilogue's HBM traffic (1.9 GB per Llama-3-8B layer,
// +19 % over a plain store when every CU bursts at once,
// profiles/r4_step/swiglu_epilogue_price.log) instead of all bursting at once.
// A first K half leaves d as fp32 rows in ws[slot] and raises flags[slot]; the
// second half (later on the same XCD) waits for it, adds it in the epilogue.
template <bool AN, bool BN, int EPI, int SCHED = 0, bool SPLIT = false, bool STAG = false>
__global__ void __launch_bounds__(XT, 1)
mxk_gemm_bf16_x2_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                        uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc,
                        const uint16_t* __restrict__ aux = nullptr, float* __restrict__ ws = nullptr,
                        int q_full = 0, int* __restrict__ flags = nullptr, int stag_cx = 0) {
  constexpr int A_BYTES = XOp<AN>::BYTES;
  constexpr int STAGE = A_BYTES + XOp<BN>::BYTES;
  // EPI 4: 1 KiB more, so the epilogue's acc slices (4 x kSwigluLdsWave from
  // the last K-tile's stage) and the g / u prefetch (64 KiB at the other
  // stage + 1 KiB) never overlap, whichever stage is which
  // EPI 6: EPI 4 with the SwiGLU math removed (timing ablation, wrong values)
  constexpr bool PFEPI = EPI == 4 || EPI == 6;
  static_assert(!PFEPI || (4 * mxk::kSwigluLdsWave <= STAGE + 1024 && 65536 + 1024 <= STAGE),
                "EPI 4 LDS plan");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + (PFEPI ? 1024 : 0)];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1;
  const int wn = wave & 1;
  int tile = blockIdx.x, kbeg = 0, klen = K;
  if constexpr (SPLIT) {
    tile = q_full + (static_cast<int>(blockIdx.x) >> 1);
    klen = K >> 1;
    kbeg = (blockIdx.x & 1) * klen;
  }
  mxk::StaggerPart sp{static_cast<int>(blockIdx.x), 0, -1};
  if constexpr (STAG) {
    static_assert(EPI == 4 && !SPLIT, "STAG: the dgrad-SwiGLU epilogue only");
    sp = mxk::stagger_part_xcd(blockIdx.x, (M / XBM) * (N / XBM), stag_cx);
    if (sp.part < 0) return;
    tile = sp.vtile;
    if (sp.part) {
      klen = K >> 1;
      kbeg = sp.part == 2 ? klen : 0;
    }
  }
  int m0, n0;
  mxk::w4b_tile<1>(tile, (M / XBM) * (N / XBM), M / XBM, N / XBM, &m0, &n0);

  XOp<AN> oa;
  XOp<BN> ob;
  // the K range [kbeg, kbeg + klen): K-major operands start kbeg columns in,
  // N/M-major ones kbeg rows down
  oa.init(AN ? A + static_cast<size_t>(kbeg) * lda : A + kbeg, lda, m0, klen, lane, wave);
  ob.init(BN ? B + static_cast<size_t>(kbeg) * ldb : B + kbeg, ldb, n0, klen, lane, wave);
  oa.set_lds(smem, mxk::lds_addr32(smem));
  ob.set_lds(smem, mxk::lds_addr32(smem));

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int ns = klen / XBK;
  const uint32_t ka = oa.kstep(), kb = ob.kstep();
#pragma unroll
  for (int p = 0; p < 8; ++p) oa.issue_s(smem, p, 0, wave);
#pragma unroll
  for (int p = 0; p < 8; ++p) ob.issue_s(smem + A_BYTES, p, 0, wave);
  if (ns > 1) {
#pragma unroll
    for (int p = 0; p < 8; ++p) oa.issue_s(smem + STAGE, p, ka, wave);
#pragma unroll
    for (int p = 0; p < 8; ++p) ob.issue_s(smem + STAGE + A_BYTES, p, kb, wave);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  bf16x8_t f0a[8], f0b[8], f1a[8], f1b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f0b[j] = ob.frag(smem + A_BYTES, wn * 8 + j, 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) f0a[i] = oa.frag(smem, wm * 8 + i, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);

  int s = 0;
  uint32_t sa = 2 * ka, sb = 2 * kb;
  for (; s + 2 <= ns - 2; s += 2) {
    x2_ktile_s<SCHED, AN, BN, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa, sb, wave);
    x2_ktile_s<SCHED, AN, BN, 1, 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa + ka, sb + kb, wave);
    sa += 2 * ka;
    sb += 2 * kb;
  }
  if (s < ns - 2) {
    x2_ktile_s<SCHED, AN, BN, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa, sb, wave);
    ++s;
  }
  if (ns >= 2) {
    if constexpr (PFEPI && (SCHED & 1) == 0 && !SPLIT) {
      // stage s & 1 is read by this K-tile; the last one reads the other
      GuPrefetch pf;
      pf.rsrc = mxk::make_rsrc(aux, 0xFFFFFFF0u);
      const int rr = lane >> 4, cc = (lane & 15) * 8;
      pf.voff = static_cast<uint32_t>(
          (static_cast<long>(m0 + wm * 128 + rr) * ldc + n0 + wn * 128 + cc) * 2);
      pf.rowstep = static_cast<uint32_t>(4L * ldc * 2);
      pf.fbytes = static_cast<uint32_t>(N * 2);
      pf.lds = mxk::lds_addr32(smem) + (s & 1) * STAGE + 1024 + wave * 16384;
      x2_ktile<AN, BN, 2, 2, -1, GuPrefetch, (SCHED >> 1) & 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob,
                                                               wm, wn, 0, 0,
                                              wave, s & 1, pf);
    } else {
      x2_ktile_s<SCHED, AN, BN, 2, 2>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, 0, 0, wave,
                                      s & 1);
    }
    ++s;
  }
  x2_ktile_s<SCHED, AN, BN, 2, 3>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, 0, 0, wave, s & 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  mxk::mfma_drain(acc);

  if constexpr (SPLIT) {
    // fp32 partial: lane holds 4 consecutive columns of row i*16 + (lane & 15)
    float* wp = ws + static_cast<size_t>(blockIdx.x) * (XBM * XBM);
    const int r0 = wm * 128 + (lane & 15), c0 = wn * 128 + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<f32x4_t*>(wp + (r0 + i * 16) * XBM + c0 + j * 16) = acc[i][j];
  } else if constexpr (EPI == 2)
    mxk::swiglu_bwd_block(acc, aux, C, ldc, N, m0 + wm * 128, n0 + wn * 128, lane);
  else if constexpr (EPI == 3)
    mxk::swiglu_bwd_block_wide(acc, aux, C, ldc, N, m0 + wm * 128, n0 + wn * 128, lane);
  else if constexpr (EPI == 5) {
    // EPI 4 without the g / u prefetch (A/B: MXK_SWIGLU_WIDE=5)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    mxk::swiglu_bwd_block_lds(acc, aux, C, ldc, N, m0 + wm * 128, n0 + wn * 128, lane,
                              smem + wave * mxk::kSwigluLdsWave);
  }
  else if constexpr (PFEPI) {
    static_assert(4 * mxk::kSwigluLdsWave <= 2 * STAGE, "LDS slice per wave");
    // every wave's last-stage fragment reads retired before any slice is written
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    // acc slices in the stage the last K-tile read (s & 1); the g / u rows of
    // pass 0 were prefetched into the other one (ns >= 2)
    // (the launcher takes EPI 4 only for K >= 2 * XBK, so that K-tile ran)
    char* last = smem + (s & 1) * STAGE;
    const char* gul = smem + ((s & 1) ^ 1) * STAGE + 1024 + wave * 16384;
    constexpr bool PFX = (SCHED & 1) == 0 && !SPLIT;
    if constexpr (STAG) {
      float* part = ws + static_cast<size_t>(sp.slot) * (XBM * XBM) + wave * (128 * 128);
      if (sp.part == 1) {
        mxk::swiglu_bwd_block_lds<PFX, false, 1>(acc, aux, C, ldc, N, m0 + wm * 128, n0 + wn * 128,
                                                 lane, last + wave * mxk::kSwigluLdsWave, gul, part);
        __builtin_amdgcn_s_waitcnt(0);            // this wave's partial reached memory
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flags + sp.slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      if (sp.part == 2) {
        if (tid == 0)
          while (__hip_atomic_load(flags + sp.slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
            __builtin_amdgcn_s_sleep(4);
        __syncthreads();
        mxk::swiglu_bwd_block_lds<PFX, false, 2>(acc, aux, C, ldc, N, m0 + wm * 128, n0 + wn * 128,
                                                 lane, last + wave * mxk::kSwigluLdsWave, gul, part);
        __syncthreads();                          // every wave read its partial
        if (tid == 0) __hip_atomic_store(flags + sp.slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
    mxk::swiglu_bwd_block_lds<PFX, EPI == 6>(acc, aux, C, ldc, N, m0 + wm * 128, n0 + wn * 128,
                                             lane, last + wave * mxk::kSwigluLdsWave, gul);
  }
  else if constexpr (EPI == 1) {
    // whole-line stores through LDS (as the TN kernel's default schedule);
    // every wave's last fragment reads retired before a slice is written
    static_assert(4 * mxk::kStoreLdsWave <= 2 * STAGE, "LDS slice per wave");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    mxk::store_block_lds<false>(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane,
                                smem + wave * mxk::kStoreLdsWave);
  }
  else
    mxk::store_block_narrow(acc, C, ldc, m0 + wm * 128, n0 + wn * 128, lane);
}

// x2t: persistent x2 with the C store tail trickled into the next tile's
// main loop (gemm_bf16.hip schedule 31, same mechanism): rows 64..127 of
// each wave block leave as a burst after the next tile's prologue DMA, rows
// 0..63 stay in 64 VGPRs and go out one whole-line store per K-tile in the
// next tile's first 16 K-tiles.  Needs K >= 18 * 64 (the launcher falls
// back to x2 below that).
template <int Q, int NB, int SCHED, bool AN, bool BN>
__device__ __forceinline__ void x2_trickle(f32x4_t (&acc)[8][8], bf16x8_t (&f0a)[8],
                                           bf16x8_t (&f0b)[8], bf16x8_t (&f1a)[8],
                                           bf16x8_t (&f1b)[8], char* smem, const XOp<AN>& oa,
                                           const XOp<BN>& ob, int wm, int wn, uint32_t& sa,
                                           uint32_t& sb, uint32_t ka, uint32_t kb, int wave,
                                           const u32x4_t (&buf)[16], uint16_t* tp, size_t tstride) {
  using H = mxk::TrickleStoreT<false>;
  const H h0{{}, buf[Q], tp + Q * tstride};
  const H h1{{}, buf[Q + 1], tp + (Q + 1) * tstride};
  // K-tile 0: the 16 burst stores and its own trickle store are younger than stage 1
  x2_ktile_s<SCHED, AN, BN, 0, 1, (Q == 0 ? 17 : 1), H>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm,
                                                        wn, sa, sb, wave, 0, h0);
  x2_ktile_s<SCHED, AN, BN, 1, 1, 1, H>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa + ka,
                                        sb + kb, wave, 0, h1);
  sa += 2 * ka;
  sb += 2 * kb;
  if constexpr (Q + 2 < NB)
    x2_trickle<Q + 2, NB, SCHED, AN, BN>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa, sb, ka, kb,
                                     wave, buf, tp, tstride);
}

template <bool AN, bool BN, int SCHED, int NB = (AN && BN ? 8 : AN ? 12 : 16)>
__global__ void __launch_bounds__(XT, 1)
mxk_gemm_bf16_x2t_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                         uint16_t* __restrict__ C, int M, int N, int K, int lda, int ldb, int ldc) {
  constexpr int A_BYTES = XOp<AN>::BYTES;
  constexpr int STAGE = A_BYTES + XOp<BN>::BYTES;
  static_assert(4 * mxk::kStoreLdsWave <= 2 * STAGE, "LDS slice per wave");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1;
  const int wn = wave & 1;
  const int tiles_m = M / XBM, tiles_n = N / XBM;
  const int ntiles = tiles_m * tiles_n;
  const int ns = K / XBK;                       // >= 18 (launcher)
  const int rr = lane >> 4, cc = (lane & 15) * 8;
  const size_t tstride = static_cast<size_t>(4) * ldc;

  int t = blockIdx.x;
  int m0, n0;
  mxk::w4b_tile<1>(t, ntiles, tiles_m, tiles_n, &m0, &n0);
  XOp<AN> oa;
  XOp<BN> ob;
  auto setup = [&]() {
    oa.init(A, lda, m0, K, lane, wave);
    ob.init(B, ldb, n0, K, lane, wave);
    oa.set_lds(smem, mxk::lds_addr32(smem));
    ob.set_lds(smem, mxk::lds_addr32(smem));
  };
  setup();
  const uint32_t ka = oa.kstep(), kb = ob.kstep();
  auto prologue = [&]() {
#pragma unroll
    for (int p = 0; p < 8; ++p) oa.issue_s(smem, p, 0, wave);
#pragma unroll
    for (int p = 0; p < 8; ++p) ob.issue_s(smem + A_BYTES, p, 0, wave);
#pragma unroll
    for (int p = 0; p < 8; ++p) oa.issue_s(smem + STAGE, p, ka, wave);
#pragma unroll
    for (int p = 0; p < 8; ++p) ob.issue_s(smem + STAGE + A_BYTES, p, kb, wave);
  };
  prologue();
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  static_assert(NB % 2 == 0 && NB <= 16, "trickle vectors");
  u32x4_t buf[16];                                    // 0..NB-1 trickled
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
    for (int j = 0; j < 8; ++j) f0b[j] = ob.frag(smem + A_BYTES, wn * 8 + j, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) f0a[i] = oa.frag(smem, wm * 8 + i, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);

    int s = 0;
    uint32_t sa = 2 * ka, sb = 2 * kb;
    if (trickle) {
      x2_trickle<0, NB, SCHED, AN, BN>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa, sb, ka,
                                       kb, wave, buf, tp, tstride);
      s = NB;
    }
    for (; s + 2 <= ns - 2; s += 2) {
      x2_ktile_s<SCHED, AN, BN, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa, sb, wave);
      x2_ktile_s<SCHED, AN, BN, 1, 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa + ka,
                                      sb + kb, wave);
      sa += 2 * ka;
      sb += 2 * kb;
    }
    if (s < ns - 2) {
      x2_ktile_s<SCHED, AN, BN, 0, 1>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, sa, sb, wave);
      ++s;
    }
    x2_ktile_s<SCHED, AN, BN, 2, 2>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, 0, 0, wave, s & 1);
    ++s;
    x2_ktile_s<SCHED, AN, BN, 2, 3>(acc, f0a, f0b, f1a, f1b, smem, oa, ob, wm, wn, 0, 0, wave, s & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mxk::mfma_drain(acc);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();

    char* lds = smem + wave * mxk::kStoreLdsWave;
    uint16_t* row0 = C + static_cast<size_t>(m0 + wm * 128 + rr) * ldc + n0 + wn * 128 + cc;
    const int tn = t + static_cast<int>(gridDim.x);
    u32x4_t hi[16];
    mxk::stage_half(acc, 0, lane, lds, buf);
    mxk::stage_half(acc, 1, lane, lds, hi);
    if (tn >= ntiles) {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        *reinterpret_cast<u32x4_t*>(row0 + it * tstride) = buf[it];
        *reinterpret_cast<u32x4_t*>(row0 + (16 + it) * tstride) = hi[it];
      }
      break;
    }
    // vectors beyond NB go out now, ahead of the next prologue (the stage-0
    // wait then covers them, so no count below changes)
#pragma unroll
    for (int it = NB; it < 16; ++it) *reinterpret_cast<u32x4_t*>(row0 + it * tstride) = buf[it];
    tp = row0;
    __builtin_amdgcn_s_barrier();                     // every wave read its slice back
    t = tn;
    mxk::w4b_tile<1>(t, ntiles, tiles_m, tiles_n, &m0, &n0);
    setup();
    prologue();
#pragma unroll
    for (int it = 0; it < 16; ++it) *reinterpret_cast<u32x4_t*>(tp + (16 + it) * tstride) = hi[it];
    asm volatile("s_waitcnt vmcnt(32)" ::: "memory");  // stage 0 (stage 1 + 16 stores in flight)
    __builtin_amdgcn_s_barrier();
    trickle = true;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// C tile of split pair t = ws[2t] + ws[2t + 1]; grid (32, tail tiles), each
// thread 8 consecutive columns of one row (two 8-B stores: ldc % 4 == 0).
__global__ void __launch_bounds__(256)
mxk_gemm_split_fixup(const float* __restrict__ ws, uint16_t* __restrict__ C, int M, int N, int ldc,
                     int q_full) {
  const int t = blockIdx.y;
  int m0, n0;
  mxk::w4b_tile<1>(q_full + t, (M / XBM) * (N / XBM), M / XBM, N / XBM, &m0, &n0);
  const int e = (blockIdx.x * 256 + threadIdx.x) * 8;
  const int r = e / XBM, c = e % XBM;
  const float* p0 = ws + static_cast<size_t>(2 * t) * (XBM * XBM) + e;
  const float* p1 = p0 + XBM * XBM;
  const f32x4_t a0 = *reinterpret_cast<const f32x4_t*>(p0);
  const f32x4_t a1 = *reinterpret_cast<const f32x4_t*>(p0 + 4);
  const f32x4_t b0 = *reinterpret_cast<const f32x4_t*>(p1);
  const f32x4_t b1 = *reinterpret_cast<const f32x4_t*>(p1 + 4);
  uint2 lo, hi;
  lo.x = mxk::pack2bf(a0[0] + b0[0], a0[1] + b0[1]);
  lo.y = mxk::pack2bf(a0[2] + b0[2], a0[3] + b0[3]);
  hi.x = mxk::pack2bf(a1[0] + b1[0], a1[1] + b1[1]);
  hi.y = mxk::pack2bf(a1[2] + b1[2], a1[3] + b1[3]);
  uint16_t* cp = C + static_cast<size_t>(m0 + r) * ldc + n0 + c;
  *reinterpret_cast<uint2*>(cp) = lo;
  *reinterpret_cast<uint2*>(cp + 4) = hi;
}

namespace {
std::atomic<int> g_x2_order{-1};
int x2_order() {
#ifndef MXK_GEMM_EXPERIMENTS
  return 0;   // the B-outer order is built into the experiments library only
#endif
  int v = g_x2_order.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("MXK_X2_ORDER");
    v = e && std::atoi(e) == 1 ? 1 : 0;
    g_x2_order.store(v, std::memory_order_relaxed);
  }
  return v;
}
}  // namespace

// MFMA order of the layout kernel's K-tile: 0 A-fragment outer (default), 1
// B-fragment outer (env MXK_X2_ORDER)
MXK_API void mxk_gemm_x2_set_order(int v) { g_x2_order.store(v == 1 ? 1 : 0); }

template <bool AN, bool BN>
static void launch_x(int sched, bool wide, int nwg, hipStream_t stream, const uint16_t* a,
                     const uint16_t* b, uint16_t* c, int M, int N, int K, int lda, int ldb,
                     int ldc) {
  // sched: -1 = the one-barrier x kernel, 0 = x2, 1 = x2 at hipBLASLt positions;
  // x2_order() adds bit 1 (B-outer MFMA order, MXK_X2_ORDER=1)
  if (sched < 0) {
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x_kernel<AN, BN>), dim3(nwg), dim3(XT), stream, a, b, c,
                    M, N, K, lda, ldb, ldc);
    return;
  }
  switch ((sched | (x2_order() ? 2 : 0)) * 2 + (wide ? 1 : 0)) {
#define MXK_X2_CASE(S, W)                                                                        \
  case S * 2 + W:                                                                                \
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<AN, BN, W, S>), dim3(nwg), dim3(XT), stream, a, b, c, \
                    M, N, K, lda, ldb, ldc);                                                     \
    break;
    MXK_X2_CASE(0, 0) MXK_X2_CASE(0, 1) MXK_X2_CASE(1, 0) MXK_X2_CASE(1, 1)
#ifdef MXK_GEMM_EXPERIMENTS
    // B-outer order: step-neutral (profiles/r4_step/step_ab_set2.txt), A/B only
    MXK_X2_CASE(2, 0) MXK_X2_CASE(2, 1) MXK_X2_CASE(3, 0) MXK_X2_CASE(3, 1)
#endif
#undef MXK_X2_CASE
    default: break;
  }
}

// 1 if layout-kernel variant v is in this build (4, x2t: experiments only)
MXK_API int mxk_gemm_bf16_ex_variant_built(int v) {
#ifdef MXK_GEMM_EXPERIMENTS
  return v >= 0 && v <= 4;
#else
  return v >= 0 && v <= 3;
#endif
}

MXK_API int mxk_gemm_bf16_tn(const void* A, const void* Bt, void* C, int M, int N, int K,
                             int lda, int ldb, int ldc, hipStream_t stream);

namespace {
int device_cus();
}

// x2t: persistent trickle-store layout kernel, one workgroup per CU at most
template <bool AN, bool BN>
static void launch_xt(int sched, int nwg, hipStream_t stream, const uint16_t* a, const uint16_t* b,
                      uint16_t* c, int M, int N, int K, int lda, int ldb, int ldc) {
  const int cus = device_cus();
  const int grid = nwg < cus ? nwg : cus;
  if (sched == 1)
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2t_kernel<AN, BN, 1>), dim3(grid), dim3(XT), stream, a, b,
                       c, M, N, K, lda, ldb, ldc);
  else
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2t_kernel<AN, BN, 0>), dim3(grid), dim3(XT), stream, a, b,
                       c, M, N, K, lda, ldb, ldc);
}

// a_kmajor: A stored [M][K] (1) or [K][M] (0); b_kmajor: B stored [N][K] (1)
// or [K][N] (0).  Row strides lda/ldb/ldc in elements.  Tiles exactly:
// M % 256, N % 256, K % 64; returns hipErrorInvalidValue otherwise (callers
// keep the library GEMM for other shapes).  variant:
//   1 (default) both K-major -> the validator's TN kernel (gemm_bf16.hip);
//     both N/M-major (weight gradients) -> x2 at hipBLASLt's positions
//     (+2-10 % on the Llama-3-8B wgrad shapes); mixed (dgrad) -> x2
//   2 x2 at hipBLASLt's positions, 3 x2, 0 the one-barrier x kernel
//   (2, 3 and 0 run every layout on the layout kernel, for A/B)
//   4 x2t (persistent, trickled C stores; variant 1's schedule per layout,
//     hipBLASLt positions for TN; x2 when K < 18 * 64)
MXK_API int mxk_gemm_bf16_ex_variant(const void* A, const void* B, void* C, int M, int N, int K,
                                     int lda, int ldb, int ldc, int a_kmajor, int b_kmajor,
                                     int variant, hipStream_t stream) {
  const auto bytes = [](long rows, long ld) { return rows * ld * 2; };
  const bool ok = M > 0 && N > 0 && K > 0 && M % XBM == 0 && N % XBM == 0 && K % XBK == 0 &&
                  lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 &&
                  (a_kmajor ? lda >= K : lda >= M) && (b_kmajor ? ldb >= K : ldb >= N) &&
                  ldc >= N && (a_kmajor || bytes(K, lda) < (1L << 32)) &&
                  (b_kmajor || bytes(K, ldb) < (1L << 32)) &&
                  reinterpret_cast<uintptr_t>(A) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(B) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(C) % 8 == 0 && variant >= 0 && variant <= 4;
  if (!ok) return static_cast<int>(hipErrorInvalidValue);
  if (variant == 1 && a_kmajor && b_kmajor)
    return mxk_gemm_bf16_tn(A, B, C, M, N, K, lda, ldb, ldc, stream);
#ifdef MXK_GEMM_EXPERIMENTS
  // x2t, the persistent trickle-store kernel: an A/B record (mixed against
  // x2 on the Llama-3-8B step shapes, profiles/r3_pass1/layouts_ab.log)
  if (variant == 4 && K >= 18 * XBK && (ldc % 8 == 0) && reinterpret_cast<uintptr_t>(C) % 16 == 0) {
    const int xs = (a_kmajor == b_kmajor) ? 1 : 0;
    const int xn = (M / XBM) * (N / XBM);
    auto a = static_cast<const uint16_t*>(A);
    auto b = static_cast<const uint16_t*>(B);
    auto c = static_cast<uint16_t*>(C);
    if (a_kmajor && b_kmajor)
      launch_xt<false, false>(xs, xn, stream, a, b, c, M, N, K, lda, ldb, ldc);
    else if (a_kmajor)
      launch_xt<false, true>(xs, xn, stream, a, b, c, M, N, K, lda, ldb, ldc);
    else if (b_kmajor)
      launch_xt<true, false>(xs, xn, stream, a, b, c, M, N, K, lda, ldb, ldc);
    else
      launch_xt<true, true>(xs, xn, stream, a, b, c, M, N, K, lda, ldb, ldc);
    MXK_RETURN_LAUNCH_STATUS();
  }
#endif
  if (variant == 4) variant = 1;
  if (variant == 1 && a_kmajor && b_kmajor)
    return mxk_gemm_bf16_tn(A, B, C, M, N, K, lda, ldb, ldc, stream);
  const int sched = variant == 0 ? -1 : variant == 2 ? 1 : variant == 3 ? 0
                  : (!a_kmajor && !b_kmajor) ? 1 : 0;
  const int nwg = (M / XBM) * (N / XBM);
  const bool wide = (ldc % 8 == 0) && (reinterpret_cast<uintptr_t>(C) % 16 == 0);
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  if (a_kmajor && b_kmajor)
    launch_x<false, false>(sched, wide, nwg, stream, a, b, c, M, N, K, lda, ldb, ldc);
  else if (a_kmajor)
    launch_x<false, true>(sched, wide, nwg, stream, a, b, c, M, N, K, lda, ldb, ldc);
  else if (b_kmajor)
    launch_x<true, false>(sched, wide, nwg, stream, a, b, c, M, N, K, lda, ldb, ldc);
  else
    launch_x<true, true>(sched, wide, nwg, stream, a, b, c, M, N, K, lda, ldb, ldc);
  MXK_RETURN_LAUNCH_STATUS();
}

namespace {
std::atomic<int> g_swiglu_epi{-1};
int swiglu_epi() {
  int v = g_swiglu_epi.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("MXK_SWIGLU_WIDE");
    v = e ? std::atoi(e) : 4;
    g_swiglu_epi.store(v, std::memory_order_relaxed);
  }
  return v;
}
}  // namespace

// dgrad-SwiGLU epilogue mode (MXK_SWIGLU_WIDE; see mxk_gemm_bf16_dgrad_swiglu)
MXK_API void mxk_gemm_swiglu_set_epi(int v) { g_swiglu_epi.store(v); }

#ifdef MXK_GEMM_EXPERIMENTS
namespace {
// Per-(device, stream) uncached workspace of the staggered dgrad-SwiGLU GEMM:
// fp32 partial tiles (256 KiB each) and their flags, zeroed once; each
// consumer resets its flag, so later launches and graph replays start clean.
struct SwigluStagWs {
  float* ws = nullptr;
  int* flags = nullptr;
  int slots = 0;
};
std::mutex g_sstag_mu;
std::map<std::pair<int, hipStream_t>, SwigluStagWs> g_sstag;

const SwigluStagWs* swiglu_stag_ws(hipStream_t stream, int slots) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_sstag_mu);
  SwigluStagWs& w = g_sstag[{dev, stream}];
  if (w.slots >= slots) return &w;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
    return nullptr;
  if (w.ws) (void)hipFree(w.ws);
  if (w.flags) (void)hipFree(w.flags);
  w = SwigluStagWs{};
  void *ws = nullptr, *fl = nullptr;
  if (hipExtMallocWithFlags(&ws, static_cast<size_t>(slots) * XBM * XBM * 4,
                            hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags(&fl, static_cast<size_t>(slots) * 4, hipDeviceMallocUncached) != hipSuccess ||
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
}  // namespace
#endif

// Down-projection input gradient with the SwiGLU backward fused into the
// epilogue: d(act) = dy W2 (dy [M][K] K-major, W2 [K][F] F-major) never
// reaches memory; dgu [M][2F] = d[g | u] is written from gu [M][2F].
// Tiles exactly (M % 256, F % 256, K % 64); hipErrorInvalidValue otherwise.
MXK_API int mxk_gemm_bf16_dgrad_swiglu(const void* dy, const void* w2, const void* gu, void* dgu,
                                       int M, int F, int K, int ld_dy, int ld_w2,
                                       hipStream_t stream) {
  const bool ok = M > 0 && F > 0 && K > 0 && M % XBM == 0 && F % XBM == 0 && K % XBK == 0 &&
                  ld_dy % 8 == 0 && ld_w2 % 8 == 0 && ld_dy >= K && ld_w2 >= F &&
                  static_cast<long>(K) * ld_w2 * 2 < (1L << 32) &&
                  reinterpret_cast<uintptr_t>(dy) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w2) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(gu) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(dgu) % 8 == 0;
  if (!ok) return static_cast<int>(hipErrorInvalidValue);
  const int nwg = (M / XBM) * (F / XBM);
  // 16-B g/u accesses: EPI 4 (LDS-staged, whole lines, pass 0's g/u
  // prefetched during the last K-tiles) by default, EPI 5 (the same without
  // the prefetch) with MXK_SWIGLU_WIDE=5, EPI 3 (permlane pairs) with =3, the
  // 8-B form with =0 (A/B); 6 = EPI 4 without the SwiGLU math (timing only);
  // 8 = EPI 4 staggered by XCD group (STAG)
  const int wide_mode = swiglu_epi();
  const bool wide = wide_mode != 0 && reinterpret_cast<uintptr_t>(gu) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(dgu) % 16 == 0 && K >= 2 * XBK;
#ifdef MXK_GEMM_EXPERIMENTS
  // A/B records (experiments library): 8 = staggered by XCD group (+0.8 %,
  // profiles/r4_step/swiglu_epilogue_stagger.log), 6 = no SwiGLU math (timing
  // ablation), 5 = no g/u prefetch, and the B-outer MFMA order
  if (wide && wide_mode == 8) {
    const int cx = device_cus() / 8;
    const long T = nwg;
    const bool fits = T % 8 == 0 && cx > 0 && T / 8 >= 2 * cx && K % (2 * XBK) == 0;
    const SwigluStagWs* w = fits ? swiglu_stag_ws(stream, 4 * cx) : nullptr;
    if (w) {
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 4, 0, false, true>), dim3(nwg + 8 * cx),
                      dim3(XT), stream, static_cast<const uint16_t*>(dy),
                      static_cast<const uint16_t*>(w2), static_cast<uint16_t*>(dgu), M, F, K, ld_dy,
                      ld_w2, 2 * F, static_cast<const uint16_t*>(gu), w->ws, 0, w->flags, cx);
      MXK_RETURN_LAUNCH_STATUS();
    }
  }
  if (wide && (wide_mode == 6 || wide_mode == 5 || x2_order())) {
    if (wide_mode == 6)
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 6, 0>), dim3(nwg), dim3(XT), stream,
                      static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w2),
                      static_cast<uint16_t*>(dgu), M, F, K, ld_dy, ld_w2, 2 * F,
                      static_cast<const uint16_t*>(gu));
    else if (wide_mode == 5)
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 5, 0>), dim3(nwg), dim3(XT), stream,
                      static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w2),
                      static_cast<uint16_t*>(dgu), M, F, K, ld_dy, ld_w2, 2 * F,
                      static_cast<const uint16_t*>(gu));
    else
      MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 4, 2>), dim3(nwg), dim3(XT), stream,
                      static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w2),
                      static_cast<uint16_t*>(dgu), M, F, K, ld_dy, ld_w2, 2 * F,
                      static_cast<const uint16_t*>(gu));
    MXK_RETURN_LAUNCH_STATUS();
  }
#endif
  if (wide && wide_mode == 3)
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 3, 0>), dim3(nwg), dim3(XT), stream,
                       static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w2),
                       static_cast<uint16_t*>(dgu), M, F, K, ld_dy, ld_w2, 2 * F,
                       static_cast<const uint16_t*>(gu));
  else if (wide)
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 4, 0>), dim3(nwg), dim3(XT), stream,
                       static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w2),
                       static_cast<uint16_t*>(dgu), M, F, K, ld_dy, ld_w2, 2 * F,
                       static_cast<const uint16_t*>(gu));
  else
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<false, true, 2, 0>), dim3(nwg), dim3(XT), stream,
                       static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w2),
                       static_cast<uint16_t*>(dgu), M, F, K, ld_dy, ld_w2, 2 * F,
                       static_cast<const uint16_t*>(gu));
  MXK_RETURN_LAUNCH_STATUS();
}

// ---- compute units the GEMMs may plan for -------------------------------
// Every round / split-tail decision below assumes `cus` workgroups run at
// once.  With collectives in flight (the ZeRO-1 reduce-scatter under the
// backward, the parameter all-gather under the forward) RCCL's kernels hold
// some CUs for the whole collective, and a GEMM whose tiles exactly fill the
// chip then runs one extra, nearly empty round.  mxk_gemm_set_reserved_cus(k)
// (or MXK_GEMM_RESERVED_CUS=k) tells the planner that k CUs are taken: rounds
// and the split tail are sized for the CUs that are left.
namespace {
std::atomic<int> g_reserved_cus{-1};

int hw_cus() {
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

int reserved_cus() {
  int r = g_reserved_cus.load(std::memory_order_relaxed);
  if (r < 0) {
    const char* e = std::getenv("MXK_GEMM_RESERVED_CUS");
    r = e ? std::max(0, std::atoi(e)) : 0;
    g_reserved_cus.store(r, std::memory_order_relaxed);
  }
  return r;
}

int device_cus() { return std::max(1, hw_cus() - reserved_cus()); }

std::atomic<int> g_exclusive{-1};
int exclusive() {
  int e = g_exclusive.load(std::memory_order_relaxed);
  if (e < 0) {
    const char* v = std::getenv("MXK_GEMM_EXCLUSIVE");
    e = v && std::atoi(v) ? 1 : 0;
    g_exclusive.store(e, std::memory_order_relaxed);
  }
  return e;
}
std::mutex g_excl_mu;
std::map<std::pair<int, const void*>, size_t> g_excl;
}  // namespace

size_t mxk_excl_lds(const void* kernel) {
  if (!exclusive()) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(g_excl_mu);
  auto it = g_excl.find({dev, kernel});
  if (it != g_excl.end()) return it->second;
  hipFuncAttributes fa{};
  int max_lds = 0;
  size_t add = 0;
  if (hipFuncGetAttributes(&fa, kernel) == hipSuccess &&
      hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess &&
      fa.sharedSizeBytes < static_cast<size_t>(max_lds))
    add = static_cast<size_t>(max_lds) - fa.sharedSizeBytes;
  g_excl[{dev, kernel}] = add;
  return add;
}

MXK_API void mxk_gemm_set_exclusive(int on) { g_exclusive.store(on ? 1 : 0); }
MXK_API int mxk_gemm_exclusive(void) { return exclusive(); }

MXK_API void mxk_gemm_set_reserved_cus(int n) { g_reserved_cus.store(std::max(0, n)); }
MXK_API int mxk_gemm_reserved_cus(void) { return reserved_cus(); }
MXK_API int mxk_gemm_available_cus(void) { return device_cus(); }

// The split-tail plan for nwg 256^2 output tiles over `cus` CUs and depth K
// (pure host arithmetic; tests/test_gemm_plan.py checks it on the CPU):
// returns the number of tail tiles run as K halves (0: no split) and sets
// *q_full to the tiles that run whole.
MXK_API int mxk_gemm_split_plan(long nwg, int K, int cus, long* q_full) {
  const int tail = nwg > 0 && cus > 0 ? static_cast<int>(nwg % cus) : 0;
  const bool want = tail > 0 && 2 * tail <= cus && K % (2 * XBK) == 0 && K >= 16 * XBK;
  if (q_full) *q_full = want ? nwg - tail : nwg;
  return want ? tail : 0;
}

namespace {

template <bool AN, bool BN>
void launch_split(int sched, bool wide, int nwg, int q_full, hipStream_t stream, const uint16_t* a,
                  const uint16_t* b, uint16_t* c, int M, int N, int K, int lda, int ldb, int ldc,
                  float* ws) {
  // whole tiles [0, q_full) (the tile map is over all nwg tiles, not the grid)
  if (q_full > 0) launch_x<AN, BN>(sched, wide, q_full, stream, a, b, c, M, N, K, lda, ldb, ldc);
  const dim3 grid(2 * (nwg - q_full));
  if (sched == 1)
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<AN, BN, 0, 1, true>), grid, dim3(XT), stream, a,
                       b, c, M, N, K, lda, ldb, ldc, nullptr, ws, q_full);
  else
    MXK_LAUNCH_GEMM((mxk_gemm_bf16_x2_kernel<AN, BN, 0, 0, true>), grid, dim3(XT), stream, a,
                       b, c, M, N, K, lda, ldb, ldc, nullptr, ws, q_full);
  hipLaunchKernelGGL(mxk_gemm_split_fixup, dim3(XBM * XBM / (256 * 8), nwg - q_full), dim3(256), 0,
                     stream, ws, c, M, N, ldc, q_full);
}
}  // namespace

// Bytes of fp32 workspace the split tail of an (M, N) output needs at most
// (half a round of tiles, two partial tiles each).
MXK_API long mxk_gemm_bf16_split_workspace(void) {
  return static_cast<long>(hw_cus() / 2) * 2 * XBM * XBM * 4;   // any reservation fits
}

// mxk_gemm_bf16_ex (variant 1) with the split tail: when the output's 256^2
// tiles fill q whole rounds of the CUs plus a last round at most half full
// (e.g. 384 tiles on 256 CUs), the tail tiles run as K halves on twice as
// many workgroups (fp32 partials in ws, summed by a fixup kernel) instead of
// leaving half the chip idle for a whole round.  Layouts other than both
// K-major only; every other case runs mxk_gemm_bf16_ex unchanged.  `ws`
// holds >= ws_bytes (mxk_gemm_bf16_split_workspace()); sets *split to 1
// when the split path ran.
MXK_API int mxk_gemm_bf16_ex_ws(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                                int ldb, int ldc, int a_kmajor, int b_kmajor, void* ws,
                                long ws_bytes, int* split, hipStream_t stream) {
  if (split) *split = 0;
  const int cus = device_cus();
  const long nwg = M > 0 && N > 0 ? static_cast<long>(M / XBM) * (N / XBM) : 0;
  long q_plan = nwg;
  const int tail = static_cast<int>(mxk_gemm_split_plan(nwg, K, cus, &q_plan));
  const bool want = tail > 0 && ws != nullptr &&
                    ws_bytes >= static_cast<long>(2 * tail) * XBM * XBM * 4 &&
                    reinterpret_cast<uintptr_t>(ws) % 16 == 0;
  if (!want)
    return mxk_gemm_bf16_ex_variant(A, B, C, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor, 1, stream);
  const auto bytes = [](long rows, long ld) { return rows * ld * 2; };
  const bool ok = M % XBM == 0 && N % XBM == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 &&
                  (a_kmajor ? lda >= K : lda >= M) && (b_kmajor ? ldb >= K : ldb >= N) &&
                  ldc >= N && (a_kmajor || bytes(K, lda) < (1L << 32)) &&
                  (b_kmajor || bytes(K, ldb) < (1L << 32)) &&
                  reinterpret_cast<uintptr_t>(A) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(B) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(C) % 8 == 0;
  if (!ok) return static_cast<int>(hipErrorInvalidValue);
  const int sched = (!a_kmajor && !b_kmajor) ? 1 : 0;
  const bool wide = (ldc % 8 == 0) && (reinterpret_cast<uintptr_t>(C) % 16 == 0);
  const int q_full = static_cast<int>(nwg) - tail;
  auto a = static_cast<const uint16_t*>(A);
  auto b = static_cast<const uint16_t*>(B);
  auto c = static_cast<uint16_t*>(C);
  auto w = static_cast<float*>(ws);
  if (a_kmajor && b_kmajor)   // forward y = x W^T: the TN tail
    launch_split<false, false>(sched, wide, nwg, q_full, stream, a, b, c, M, N, K, lda, ldb, ldc, w);
  else if (a_kmajor)
    launch_split<false, true>(sched, wide, nwg, q_full, stream, a, b, c, M, N, K, lda, ldb, ldc, w);
  else if (b_kmajor)
    launch_split<true, false>(sched, wide, nwg, q_full, stream, a, b, c, M, N, K, lda, ldb, ldc, w);
  else
    launch_split<true, true>(sched, wide, nwg, q_full, stream, a, b, c, M, N, K, lda, ldb, ldc, w);
  if (split) *split = 1;
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_gemm_bf16_ex(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                             int ldb, int ldc, int a_kmajor, int b_kmajor, hipStream_t stream) {
  return mxk_gemm_bf16_ex_variant(A, B, C, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor, 1, stream);
}
