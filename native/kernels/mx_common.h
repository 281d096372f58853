// Shared helpers for the mxk8s CDNA4 (gfx950) kernels.
//
// Everything here is written for MI355X only: 64-lane wavefronts, MFMA
// matrix cores, 160 KiB LDS per CU, 8 XCDs with private L2s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MXK_API extern "C" __attribute__((visibility("default")))

// Dynamic LDS to add to a one-workgroup-per-CU GEMM launch so that it claims
// the CU's whole LDS while exclusive mode is on (mxk_gemm_set_exclusive,
// MXK_GEMM_EXCLUSIVE=1; gemm_bf16_layouts.hip): then no other kernel's
// workgroup (an RCCL collective's, say) can share a CU with a GEMM tile and
// slow it; it takes a CU between tiles instead, and the planner sized for
// the CUs left (mxk_gemm_set_reserved_cus) absorbs that.  0 when off.
size_t mxk_excl_lds(const void* kernel);
#define MXK_LAUNCH_GEMM(kern, grid, block, stream, ...)                                         \
  hipLaunchKernelGGL(kern, grid, block, mxk_excl_lds(reinterpret_cast<const void*>(kern)), stream, \
                     __VA_ARGS__)

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
  // one v_cvt_pk_bf16_f32 for the pair (two scalar casts cost two converts
  // and an SDWA or)
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const b2_t b = __builtin_convertvector(f2_t{lo, hi}, b2_t);
  return __builtin_bit_cast(uint32_t, b);
}

// Rotary embedding of one (i, i + D/2) pair ("rotate-half"): a' = a cos -
// b s, b' = b cos + a s, with s = sign * sin (sign -1: the inverse rotation,
// the backward).  Explicit fmas, so the stand-alone kernel (fused_ops.hip)
// and the epilogues that fuse it (attention backward) round identically.
__device__ __forceinline__ void rope_pair(float a, float b, float c, float s, float& oa,
                                          float& ob) {
  oa = __builtin_fmaf(a, c, -(b * s));
  ob = __builtin_fmaf(b, c, a * s);
}

// Eight bf16 elements of one rotate-half row rotated: `own` holds dims
// i0 .. i0 + 7 of the lower half (lo) or of the upper half, `par` the same
// dims of the other half; cs / sn: cos / sin at the row's position for
// frequencies i0 .. i0 + 7 (8 floats each, 16-B aligned); sign -1: the
// inverse rotation.  Returns the 8 rotated elements of `own`'s half, rounded
// as the stand-alone pass (fused_ops.hip) rounds them.
__device__ __forceinline__ u32x4_t rope8_bf16(u32x4_t own, u32x4_t par, bool lo, const float* cs,
                                              const float* sn, float sign) {
  const float4 c0 = *reinterpret_cast<const float4*>(cs);
  const float4 c1 = *reinterpret_cast<const float4*>(cs + 4);
  const float4 s0 = *reinterpret_cast<const float4*>(sn);
  const float4 s1 = *reinterpret_cast<const float4*>(sn + 4);
  const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  u32x4_t out;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float o2[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float x = __uint_as_float(e ? own[w] & 0xFFFF0000u : own[w] << 16);
      const float y = __uint_as_float(e ? par[w] & 0xFFFF0000u : par[w] << 16);
      float oa, ob;
      rope_pair(lo ? x : y, lo ? y : x, c[2 * w + e], sign * sv[2 * w + e], oa, ob);
      o2[e] = lo ? oa : ob;
    }
    out[w] = pack2bf(o2[0], o2[1]);
  }
  return out;
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

// Inline-asm MFMAs (used to pin accumulators to AGPRs) are invisible to
// hipcc's hazard recognizer: it knows the asm's "+a" outputs but not that the
// MFMA writes them ~16 cycles after issue.  Nothing then stops the register
// allocator from copying an accumulator to a VGPR (v_accvgpr_read) right
// behind the asm MFMA that last writes it — seen on two GEMM schedules after
// unrelated edits: acc[0][0..1] resp. acc[7][7] read one instruction after
// their final MFMA, wrong outputs.  Call after the last MFMA, before the
// accumulators are read: the s_nops cover the write latency and the empty
// asms redefine every accumulator behind them, so each later read (and any
// register copy of it) depends on a value that only exists after the nops.
template <int NI, int NJ>
__device__ __forceinline__ void mfma_drain(f32x4_t (&acc)[NI][NJ]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" : "+a"(acc[i][j]));
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
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 4\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(m), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

// dma16 with the LDS destination given as a 32-bit LDS address that the
// caller keeps scalar, bound straight to M0 ("{m0}"): the compiler writes M0
// with the address arithmetic itself (one s_add into m0), with no
// v_readfirstlane and no save/restore of M0 around every piece.  The LDS
// write stays invisible to the compiler (inline asm), so it inserts no
// conservative vmcnt(0) before transposed LDS reads, which the builtin
// __builtin_amdgcn_raw_ptr_buffer_load_lds does.
//
// Opens with s_nop 4: a descriptor / offset SGPR that a VALU instruction has
// just written (v_readlane of an SGPR spilled to VGPR lanes, v_readfirstlane)
// needs 5 wait states before a vector-memory instruction reads it, and hipcc
// pads that only for its own loads.  Seen in the causal 256-row forward: a
// descriptor word restored right before the DMA was read stale (keys of whole
// tiles missing from O, then a memory fault).  tests/test_isa_hazards.py
// (valu_sgpr_to_vmem) audits the listings.
__device__ __forceinline__ void dma16m(const u32x4& rsrc, uint32_t lds_addr, uint32_t voff,
                                       uint32_t soff) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(rsrc), "s"(soff), "{m0}"(lds_addr)
               : "memory");
}

// 32-bit LDS address of a __shared__ array (a constant after folding)
template <class T>
__device__ __forceinline__ uint32_t lds_addr32(T* shared_array) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) char*)shared_array));
}

// Block -> 256x256 output tile of the MFMA GEMMs (gemm_bf16*.hip).
//  MAP 0: XCD remap + GROUP_M column sweep (each XCD owns GROUP_M tile rows
//         and walks the columns; chip-wide every A panel is live at once).
//  MAP 1: XCD-aware super-blocks.  The 8 XCDs x 32 CUs = 256 resident
//         workgroups cover one 16x16-tile super-block per "round"; XCD x
//         takes the 8 (M) x 4 (N) sub-block (x >> 2, x & 3) of it, so an XCD's
//         L2 serves 12 panels to 32 tiles (the 81 % reuse of MAP 0) while the
//         chip as a whole touches only 16 A + 16 B panels per round (Infinity
//         Cache-sized at 16384^2) instead of every A panel.  Rounds snake over
//         the super-block grid so consecutive rounds share their A panels.
//         Needs tiles_m % 16 == tiles_n % 16 == 0; MAP 0 otherwise.
//  MAP 2 / 3 / 4 (A/B records): the MAP 1 super-block with the XCD sub-block
//         4 x 8 / 2 x 16 / 16 x 2 tiles (M x N) instead of 8 x 4.
template <int MAP>
__device__ __forceinline__ void w4b_tile(int bid, int nwg, int tiles_m, int tiles_n, int* m0,
                                         int* n0) {
  if (MAP >= 2 && MAP <= 4 && (tiles_m & 15) == 0 && (tiles_n & 15) == 0) {
    constexpr int SM = MAP == 2 ? 4 : MAP == 3 ? 2 : 16;   // sub-block rows; SM * SN = 32
    constexpr int XM = 16 / SM;                             // XCD grid: XM x (8 / XM)
    const int xcd = bid & 7, l = bid >> 3;
    const int round = l >> 5, pos = l & 31;
    const int sbn = tiles_n >> 4;
    const int sm = round / sbn;
    int sn = round - sm * sbn;
    if (sm & 1) sn = sbn - 1 - sn;
    *m0 = (sm * 16 + (xcd % XM) * SM + pos % SM) * 256;
    *n0 = (sn * 16 + (xcd / XM) * (32 / SM) + pos / SM) * 256;
    return;
  }
  if (MAP == 1 && (tiles_m & 15) == 0 && (tiles_n & 15) == 0) {
    const int xcd = bid & 7, l = bid >> 3;
    const int round = l >> 5, pos = l & 31;
    const int sbn = tiles_n >> 4;
    const int sm = round / sbn;
    int sn = round - sm * sbn;
    if (sm & 1) sn = sbn - 1 - sn;
    *m0 = (sm * 16 + (xcd >> 2) * 8 + (pos & 7)) * 256;
    *n0 = (sn * 16 + (xcd & 3) * 4 + (pos >> 3)) * 256;
    return;
  }
  const int wgid = xcd_remap(bid, nwg);
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wgid - group * per_group;
  *m0 = (first_m + in_group % gsize) * 256;
  *n0 = (in_group / gsize) * 256;
}

// ---- staggered rounds (gemm_tn_core.h schedules 54-57; the dgrad-SwiGLU
// layout GEMM) ----------------------------------------------------------------
struct StaggerPart {
  int vtile;   // tile index fed to the tile map
  int part;    // 0 whole tile, 1 first K half, 2 second K half, -1 idle
  int slot;    // partial slot (parts 1, 2), else -1
};

// XCD-group stagger (schedule 57): the PMC of the per-CU stagger above shows
// +43 % fetch beyond L2 at 8192^3 - half of an XCD's CUs half a tile out of
// phase no longer read each panel slice together, so the XCD's L2 stops
// sharing it.  Here whole XCDs are out of phase instead: XCDs 0-3 run whole
// tiles, XCDs 4-7 start with the first K halves of their first cx tiles (one
// per CU) and end with the second halves.  Inside an XCD every CU stays in
// phase (L2 reuse kept); XCDs 0-3 and 4-7 share no A panel of the super-block
// (rows x >> 2) and their shared B panels are half a tile apart (MALL hits);
// the C-store bursts of the two halves of the chip alternate.  Workgroup b on
// XCD x = b & 7, local index i = b >> 3, tx = T / 8, grid 8 (tx + cx):
//   x < 4:  i < tx whole tile i; i >= tx nothing (part -1)
//   x >= 4: i < cx first half of tile i (slot (x - 4) cx + i); cx <= i < tx
//           whole tile i; tx <= i second half of tile i - tx
__host__ __device__ inline StaggerPart stagger_part_xcd(int b, int T, int cx) {
  const int x = b & 7, i = b >> 3;
  const int tx = T >> 3;
  StaggerPart r;
  r.slot = -1;
  if (x < 4) {
    r.part = i < tx ? 0 : -1;
    r.vtile = x + 8 * (i < tx ? i : 0);
  } else if (i < cx) {
    r.part = 1; r.slot = (x - 4) * cx + i; r.vtile = x + 8 * i;
  } else if (i < tx) {
    r.part = 0; r.vtile = x + 8 * i;
  } else {
    r.part = 2; r.slot = (x - 4) * cx + (i - tx); r.vtile = x + 8 * (i - tx);
  }
  return r;
}

// bf16 store of a wave's 128x128 accumulator block, widened to dwordx4 by
// v_permlane16_swap (w4b EPI 1).  NT: non-temporal stores (C is written once
// and not re-read by this kernel; keeps it from displacing A/B panels).
template <bool NT = false, int NI = 8, int NJ = 8>
__device__ __forceinline__ void store_block_wide(const f32x4_t (&acc)[NI][NJ], uint16_t* C, int ldc,
                                                 int row0, int col0, int lane) {
  const int crow = lane & 15;
  const int q = lane >> 4;
  const int ccol = (q & 1) * 16 + (q >> 1) * 8;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    uint16_t* cp = C + static_cast<size_t>(row0 + i * 16 + crow) * ldc + col0 + ccol;
#pragma unroll
    for (int j = 0; j < NJ; j += 2) {
      const uint32_t x0 = pack2bf(acc[i][j][0], acc[i][j][1]);
      const uint32_t x1 = pack2bf(acc[i][j][2], acc[i][j][3]);
      const uint32_t y0 = pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]);
      const uint32_t y1 = pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      if constexpr (NT) {
        const u32x4_t v = {s0[0], s1[0], s0[1], s1[1]};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(cp + j * 16));
      } else {
        uint4 v;
        v.x = s0[0];
        v.y = s1[0];
        v.z = s0[1];
        v.w = s1[1];
        *reinterpret_cast<uint4*>(cp + j * 16) = v;
      }
    }
  }
}

__device__ __forceinline__ void store_block_narrow(const f32x4_t (&acc)[8][8], uint16_t* C, int ldc,
                                                   int row0, int col0, int lane) {
  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint16_t* cp = C + static_cast<size_t>(row0 + i * 16 + crow) * ldc + col0 + ccol;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint2 pk;
      pk.x = pack2bf(acc[i][j][0], acc[i][j][1]);
      pk.y = pack2bf(acc[i][j][2], acc[i][j][3]);
      *reinterpret_cast<uint2*>(cp + j * 16) = pk;
    }
  }
}

// bf16 store of a wave's 128x128 accumulator block through its own LDS
// slice (two 64-row passes, 272-B padded rows), read back row-major so each
// global store covers 4 rows x 256 B (whole lines) instead of the 16 rows x
// 64 B of store_block_wide.  The caller barriers before the first call (the
// slices overlap the GEMM's stages).  lds: 64 x 272 B per wave.
constexpr int kStoreLdsRow = 272;
constexpr int kStoreLdsWave = 64 * kStoreLdsRow;
// rot 1: acc[4p..4p+3] hold rows 64 (p ^ 1) .. (the w13 SwiGLU kernel's
// rotated up waves); the two passes then write each other's rows.
template <bool NT = true>
__device__ __forceinline__ void store_block_lds(const f32x4_t (&acc)[8][8], uint16_t* C, int ldc,
                                                int row0, int col0, int lane, char* lds,
                                                int rot = 0) {
  const int crow = lane & 15, q = lane >> 4;
  const int rr = lane >> 4, cc = (lane & 15) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint2 pk;
        pk.x = pack2bf(acc[4 * p + ii][j][0], acc[4 * p + ii][j][1]);
        pk.y = pack2bf(acc[4 * p + ii][j][2], acc[4 * p + ii][j][3]);
        *reinterpret_cast<uint2*>(lds + (ii * 16 + crow) * kStoreLdsRow + (j * 16 + q * 4) * 2) = pk;
      }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int r = it * 4 + rr;
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(lds + r * kStoreLdsRow + cc * 2);
      uint16_t* cp = C + static_cast<size_t>(row0 + (p ^ rot) * 64 + r) * ldc + col0 + cc;
      if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(cp));
      else *reinterpret_cast<u32x4_t*>(cp) = v;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __asm__ volatile("" ::: "memory");
  }
}

// store_block_lds with the rotary embedding applied on the way out: the
// block's 128 columns are one head (col0 % 128 == 0), row t (token) sits at
// position t % S of its sequence (S % 64 == 0, row0 % 64 == 0); each lane
// reads its 16-B chunk and the partner 64 columns away from the LDS rows and
// stores its chunk rotated (rcos / rsin: [S][64] fp32).
// rope false (wave-uniform): store_block_lds itself.
template <bool NT = true>
__device__ __forceinline__ void store_block_lds_rope(const f32x4_t (&acc)[8][8], uint16_t* C,
                                                     int ldc, int row0, int col0, int lane,
                                                     char* lds, const float* rcos,
                                                     const float* rsin, int S, bool rope) {
  const int crow = lane & 15, q = lane >> 4;
  const int rr = lane >> 4, cc = (lane & 15) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint2 pk;
        pk.x = pack2bf(acc[4 * p + ii][j][0], acc[4 * p + ii][j][1]);
        pk.y = pack2bf(acc[4 * p + ii][j][2], acc[4 * p + ii][j][3]);
        *reinterpret_cast<uint2*>(lds + (ii * 16 + crow) * kStoreLdsRow + (j * 16 + q * 4) * 2) = pk;
      }
    const int pos0 = (row0 + p * 64) % S;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int r = it * 4 + rr;
      u32x4_t o = *reinterpret_cast<const u32x4_t*>(lds + r * kStoreLdsRow + cc * 2);
      if (rope) {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(lds + r * kStoreLdsRow + (cc ^ 64) * 2);
        const long tb = static_cast<long>(pos0 + r) * 64 + (cc & 63);
        o = rope8_bf16(o, w, cc < 64, rcos + tb, rsin + tb, 1.f);
      }
      uint16_t* cp = C + static_cast<size_t>(row0 + p * 64 + r) * ldc + col0 + cc;
      if constexpr (NT) __builtin_nontemporal_store(o, reinterpret_cast<u32x4_t*>(cp));
      else *reinterpret_cast<u32x4_t*>(cp) = o;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __asm__ volatile("" ::: "memory");
  }
}

// s_waitcnt vmcnt(N) with a compile-time N (the "memory" clobber keeps the
// compiler from moving LDS / global accesses across it)
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// K-tile hook that does nothing (the K-tile bodies call hook(m) after MFMA m,
// and hook.at(p) around the waits: p 0 / 1 before wait #1 / after barrier #1,
// 2 / 3 around #2, 4 / 5 around #3)
struct NoHook {
  __device__ __forceinline__ void operator()(int) const {}
  __device__ __forceinline__ void at(int) const {}
};

// ---- trickled C stores (persistent GEMMs, gemm_bf16.hip schedule 31/32 and
// the layout kernel's x2t): a finished tile's C leaves partly as one
// whole-line store per K-tile of the next tile.
template <bool NT = true>
struct TrickleStoreT : NoHook {
  u32x4_t v;
  uint16_t* p;
  __device__ __forceinline__ void operator()(int m) const {
    if (m == 3) {
      if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
      else *reinterpret_cast<u32x4_t*>(p) = v;
    }
  }
};
using TrickleStore = TrickleStoreT<true>;

// LDS-held part (schedule 32): read after MFMA 1, stored after MFMA 9
struct TrickleLds : NoHook {
  const char* src;
  uint16_t* p;
  u32x4_t& v;
  __device__ __forceinline__ void operator()(int m) const {
    if (m == 1) v = *reinterpret_cast<const u32x4_t*>(src);
    if (m == 9) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
  }
};

// rows 64 p .. 64 p + 63 of the wave's 128 x 128 block through the LDS slice
// (schedule 26's layout, mx_common.h store_block_lds) into 16 whole-line
// vectors per lane: vector it is row 4 it + (lane >> 4), 8 columns at
// 8 (lane & 15).
__device__ __forceinline__ void stage_half(const f32x4_t (&acc)[8][8], int p, int lane, char* lds,
                                           u32x4_t (&out)[16]) {
  const int crow = lane & 15, q = lane >> 4;
  const int rr = lane >> 4, cc = (lane & 15) * 8;
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint2 pk;
      pk.x = pack2bf(acc[4 * p + ii][j][0], acc[4 * p + ii][j][1]);
      pk.y = pack2bf(acc[4 * p + ii][j][2], acc[4 * p + ii][j][3]);
      *reinterpret_cast<uint2*>(lds + (ii * 16 + crow) * kStoreLdsRow + (j * 16 + q * 4) * 2) = pk;
    }
#pragma unroll
  for (int it = 0; it < 16; ++it)
    out[it] = *reinterpret_cast<const u32x4_t*>(lds + (it * 4 + rr) * kStoreLdsRow + cc * 2);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __asm__ volatile("" ::: "memory");
}

// Fused SwiGLU-backward epilogue of the down-projection's input-gradient GEMM:
// the block's accumulators are d(act) = dY W2 for act = silu(g) * u, and the
// lane's 4 consecutive columns of row r are combined with g, u read from
// gu = [g | u] (row stride ld, u at column offset F) into
//   dg = d u s (1 + g (1 - s)),  du = d g s,   s = sigmoid(g)
// written to dgu (same layout as gu).  d(act) itself never reaches memory.
// The g / u loads run two 16-row blocks ahead of the math (software
// pipeline), so their latency overlaps the previous block's math and stores.
__device__ __forceinline__ void swiglu_bwd_rows(const f32x4_t (&acc)[8][8], int i,
                                                const uint2 (&gw)[8], const uint2 (&uw)[8],
                                                uint16_t* dgu, long off, int F) {
  // element pairs in packed fp32 (v_pk_mul/fma_f32: two elements per VALU
  // op); exp and rcp stay per element.  With 1 + g (1 - s) = (1 + g) - g s:
  //   t = d s,  du = t g,  dg = t u ((1 + g) - g s)
  typedef float f2_t __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t gp[2] = {gw[j].x, gw[j].y};
    const uint32_t up[2] = {uw[j].x, uw[j].y};
    uint32_t pg[2], pu[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f2_t g = {__uint_as_float(gp[h] << 16), __uint_as_float(gp[h] & 0xFFFF0000u)};
      const f2_t u = {__uint_as_float(up[h] << 16), __uint_as_float(up[h] & 0xFFFF0000u)};
      const f2_t d = {acc[i][j][2 * h], acc[i][j][2 * h + 1]};
      const f2_t x = g * -1.44269504f;
      // v_rcp_f32 (1 ulp) instead of the IEEE division sequence (~10 VALU
      // ops per element); the result is rounded to bf16 anyway
      const f2_t sg = {__builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x[0])),
                       __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x[1]))};
      const f2_t t = d * sg;
      const f2_t du = t * g;
      const f2_t dg = t * u * ((g + 1.f) - g * sg);
      pg[h] = pack2bf(dg[0], dg[1]);
      pu[h] = pack2bf(du[0], du[1]);
    }
    *reinterpret_cast<uint2*>(dgu + off + j * 16) = make_uint2(pg[0], pg[1]);
    *reinterpret_cast<uint2*>(dgu + off + F + j * 16) = make_uint2(pu[0], pu[1]);
  }
}

__device__ __forceinline__ void swiglu_bwd_block(const f32x4_t (&acc)[8][8], const uint16_t* gu,
                                                 uint16_t* dgu, long ld, int F, int row0,
                                                 int col0, int lane) {
  const int crow = lane & 15;
  const int ccol = (lane >> 4) * 4;
  const long off0 = static_cast<long>(row0 + crow) * ld + col0 + ccol;
  const long step = 16 * ld;
  uint2 gw[2][8], uw[2][8];
  auto load = [&](int i, int b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gw[b][j] = *reinterpret_cast<const uint2*>(gu + off0 + i * step + j * 16);
      uw[b][j] = *reinterpret_cast<const uint2*>(gu + off0 + i * step + F + j * 16);
    }
  };
  load(0, 0);
  load(1, 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    swiglu_bwd_rows(acc, i, gw[i & 1], uw[i & 1], dgu, off0 + i * step, F);
    if (i + 2 < 8) load(i + 2, i & 1);
  }
}

// Widened form of swiglu_bwd_block: v_permlane16_swap pairs the 16x16 tiles
// j and j+1 (as store_block_wide does for bf16 C), so each lane owns 8
// consecutive columns and every g / u load and dg / du store is 16 B (one
// wave-instruction = 16 rows x 64 B instead of 16 rows x 32 B): half the
// memory instructions.  Lanes q = lane >> 4: columns j*16 + (q&1)*16 +
// (q>>1)*8 + 0..7; swap(a_e, b_e) of tile j / j+1 element e gives columns e
// and 4 + e of that run.  Needs gu, dgu 16-B aligned and ld % 8 == 0.
__device__ __forceinline__ void swiglu_bwd_block_wide(const f32x4_t (&acc)[8][8],
                                                      const uint16_t* gu, uint16_t* dgu, long ld,
                                                      int F, int row0, int col0, int lane) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const int crow = lane & 15;
  const int q = lane >> 4;
  const int ccol = (q & 1) * 16 + (q >> 1) * 8;
  const long off0 = static_cast<long>(row0 + crow) * ld + col0 + ccol;
  const long step = 16 * ld;
  uint4 gw[2][4], uw[2][4];
  auto load = [&](int i, int b) {
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      gw[b][jp] = *reinterpret_cast<const uint4*>(gu + off0 + i * step + jp * 32);
      uw[b][jp] = *reinterpret_cast<const uint4*>(gu + off0 + i * step + F + jp * 32);
    }
  };
  load(0, 0);
  load(1, 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int b = i & 1;
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      float d[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][e]),
                                                        __float_as_uint(acc[i][2 * jp + 1][e]),
                                                        false, false);
        d[e] = __uint_as_float(p[0]);
        d[4 + e] = __uint_as_float(p[1]);
      }
      const uint32_t gp[4] = {gw[b][jp].x, gw[b][jp].y, gw[b][jp].z, gw[b][jp].w};
      const uint32_t up[4] = {uw[b][jp].x, uw[b][jp].y, uw[b][jp].z, uw[b][jp].w};
      uint32_t pg[4], pu[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const f2_t g = {__uint_as_float(gp[h] << 16), __uint_as_float(gp[h] & 0xFFFF0000u)};
        const f2_t u = {__uint_as_float(up[h] << 16), __uint_as_float(up[h] & 0xFFFF0000u)};
        const f2_t dd = {d[2 * h], d[2 * h + 1]};
        const f2_t x = g * -1.44269504f;
        const f2_t sg = {__builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x[0])),
                         __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x[1]))};
        const f2_t t = dd * sg;
        const f2_t du = t * g;
        const f2_t dg = t * u * ((g + 1.f) - g * sg);
        pg[h] = pack2bf(dg[0], dg[1]);
        pu[h] = pack2bf(du[0], du[1]);
      }
      *reinterpret_cast<uint4*>(dgu + off0 + i * step + jp * 32) = make_uint4(pg[0], pg[1], pg[2], pg[3]);
      *reinterpret_cast<uint4*>(dgu + off0 + i * step + F + jp * 32) =
          make_uint4(pu[0], pu[1], pu[2], pu[3]);
    }
    if (i + 2 < 8) load(i + 2, b);
  }
}

// LDS-staged form: the wave's d block goes through its own LDS slice (the
// stages are free after the K loop; the caller barriers first) in four
// 32-row passes, and is read back row-major so that every g / u load and
// dg / du store covers 4 rows x 256 B (16 lanes x 16 B per row) - whole
// 128-B lines instead of the 16 rows x 64 B of the permlane form.  The g / u
// loads of pass p + 1 are in flight while pass p is written and computed.
// lds: 32 x 528 B per wave (512-B fp32 rows + 16-B pad: the 16 rows of a
// ds_write_b128 group land 4 banks apart).
constexpr int kSwigluLdsRow = 528;
constexpr int kSwigluLdsWave = 32 * kSwigluLdsRow;
// gu_lds (optional): this wave's pass-0 g / u rows already in LDS (32 rows x
// 256 B of g, then 32 x 256 B of u; the layout GEMM DMAs them during its last
// K-tiles, x2 EPI 4), so pass 0 does not wait for HBM after the K loop.
// NOMATH (timing ablation, wrong values): dg = d u, du = d g - the same
// memory traffic without the sigmoid's exp / rcp and its products.
// PM (staggered dgrad-SwiGLU, x2 STAG): 1 = this is a first K half: store d
// as fp32 rows to part (this wave's [128][128] block, row-major) and nothing
// else; 2 = a second K half: d += part before the SwiGLU backward.
template <bool PF = false, bool NOMATH = false, int PM = 0>
__device__ __forceinline__ void swiglu_bwd_block_lds(const f32x4_t (&acc)[8][8],
                                                     const uint16_t* gu, uint16_t* dgu, long ld,
                                                     int F, int row0, int col0, int lane,
                                                     char* lds, const char* gu_lds = nullptr,
                                                     float* part = nullptr) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const int crow = lane & 15, q = lane >> 4;
  const int rr = lane >> 4, cc = (lane & 15) * 8;   // read phase: row rr of 4, 8 columns
  uint4 gw[2][8], uw[2][8];
  auto load = [&](int p, int b) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const long off = static_cast<long>(row0 + p * 32 + it * 4 + rr) * ld + col0 + cc;
      gw[b][it] = *reinterpret_cast<const uint4*>(gu + off);
      uw[b][it] = *reinterpret_cast<const uint4*>(gu + off + F);
    }
  };
  if constexpr (PM == 1) {
  } else if constexpr (PF) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const char* gp = gu_lds + (it * 4 + rr) * 256 + cc * 2;
      gw[0][it] = *reinterpret_cast<const uint4*>(gp);
      uw[0][it] = *reinterpret_cast<const uint4*>(gp + 8192);
    }
  } else {
    load(0, 0);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int b = p & 1;
    if (PM != 1 && p + 1 < 4) load(p + 1, b ^ 1);
    // d rows [32p, 32p + 32) = accumulator rows i = 2p, 2p + 1
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<f32x4_t*>(lds + (ii * 16 + crow) * kSwigluLdsRow + (j * 16 + q * 4) * 4) =
            acc[2 * p + ii][j];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int r = it * 4 + rr;
      const char* dp = lds + r * kSwigluLdsRow + cc * 4;
      f32x4_t d0 = *reinterpret_cast<const f32x4_t*>(dp);
      f32x4_t d1 = *reinterpret_cast<const f32x4_t*>(dp + 16);
      float* pp = part + (p * 32 + r) * 128 + cc;
      if constexpr (PM == 1) {
        *reinterpret_cast<f32x4_t*>(pp) = d0;
        *reinterpret_cast<f32x4_t*>(pp + 4) = d1;
        continue;
      } else if constexpr (PM == 2) {
        d0 += *reinterpret_cast<const f32x4_t*>(pp);
        d1 += *reinterpret_cast<const f32x4_t*>(pp + 4);
      }
      const float d[8] = {d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
      const uint32_t gp[4] = {gw[b][it].x, gw[b][it].y, gw[b][it].z, gw[b][it].w};
      const uint32_t up[4] = {uw[b][it].x, uw[b][it].y, uw[b][it].z, uw[b][it].w};
      uint32_t pg[4], pu[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const f2_t g = {__uint_as_float(gp[h] << 16), __uint_as_float(gp[h] & 0xFFFF0000u)};
        const f2_t u = {__uint_as_float(up[h] << 16), __uint_as_float(up[h] & 0xFFFF0000u)};
        const f2_t dd = {d[2 * h], d[2 * h + 1]};
        f2_t dg, du;
        if constexpr (NOMATH) {
          dg = dd * u;
          du = dd * g;
        } else {
          const f2_t x = g * -1.44269504f;
          const f2_t sg = {__builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x[0])),
                           __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x[1]))};
          const f2_t t = dd * sg;
          du = t * g;
          dg = t * u * ((g + 1.f) - g * sg);
        }
        pg[h] = pack2bf(dg[0], dg[1]);
        pu[h] = pack2bf(du[0], du[1]);
      }
      const long off = static_cast<long>(row0 + p * 32 + r) * ld + col0 + cc;
      *reinterpret_cast<uint4*>(dgu + off) = make_uint4(pg[0], pg[1], pg[2], pg[3]);
      *reinterpret_cast<uint4*>(dgu + off + F) = make_uint4(pu[0], pu[1], pu[2], pu[3]);
    }
    // this pass's LDS reads retire before the next pass overwrites the slice
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __asm__ volatile("" ::: "memory");
  }
}

// Per-K-tile instruction positions of the three-barrier GEMM schedules (see
// gemm_bf16.hip): for MFMA index m (0..127) the fragment read / DMA piece
// index that follows it (-1: none), and the MFMA after which each wait and
// barrier sits.
struct SchedHB {
  static constexpr int W1 = 20, B1 = 21, W2 = 50, B2 = 51, W3 = 91, VM3 = 13, B3 = 92;
  __host__ __device__ static constexpr int a1(int m) { return m < 16 && (m & 1) == 0 ? m >> 1 : -1; }
  __host__ __device__ static constexpr int b1(int m) {
    return m == 24 ? 0 : m == 27 ? 1 : m == 30 ? 2 : m == 33 ? 3 : m == 36 ? 4 : m == 38 ? 5
         : m == 40 ? 6 : m == 42 ? 7 : -1;
  }
  __host__ __device__ static constexpr int adma(int m) {
    return m == 22 ? 0 : m == 25 ? 1 : m == 28 ? 2 : m == 31 ? 3 : m == 34 ? 4 : m == 52 ? 5
         : m == 55 ? 6 : m == 58 ? 7 : -1;
  }
  __host__ __device__ static constexpr int bdma(int m) {
    return m == 61 ? 0 : m == 64 ? 1 : m == 85 ? 2 : m == 87 ? 3 : m == 89 ? 4 : m == 96 ? 5
         : m == 100 ? 6 : m == 124 ? 7 : -1;
  }
  __host__ __device__ static constexpr int k0(int m) {
    return m == 93 ? 0 : m == 94 ? 1 : m == 95 ? 2 : m == 97 ? 3 : m == 98 ? 4 : m == 102 ? 5
         : m == 103 ? 6 : m == 104 ? 7 : m == 105 ? 8 : m == 106 ? 9 : m == 109 ? 10
         : m == 112 ? 11 : m == 114 ? 12 : m == 117 ? 13 : m == 120 ? 14 : m == 123 ? 15 : -1;
  }
};

// SCHED 3 ("HB-earlyB"): SchedHB with every B piece of stage s+2 issued
// before the stage-(s+1) wait (59..80 every 3), so that wait covers only
// pieces issued a full K-tile earlier: vmcnt(16).
struct SchedEarlyB : SchedHB {
  static constexpr int VM3 = 16;
  __host__ __device__ static constexpr int bdma(int m) {
    return m >= 59 && m <= 80 && (m - 59) % 3 == 0 ? (m - 59) / 3 : -1;
  }
};

// SCHED 4 ("HB-spread"): SchedHB with the 16 next-k0 fragment reads spread
// one per two MFMAs (odd m 93..123) instead of front-loaded.
struct SchedSpreadK0 : SchedHB {
  __host__ __device__ static constexpr int k0(int m) {
    return m >= 93 && m <= 123 && (m & 1) ? (m - 93) >> 1 : -1;
  }
};

// SCHED 2: two barriers per K-tile — all k-half-1 fragments (A at even m
// 0..14, B at even m 16..30) retire before ONE barrier after m 35, then the
// 16 pieces of stage s+2 go out interleaved (A at 36 + 6p, B at 39 + 6p);
// vmcnt(16) + barrier #3 after m 96; next-k0 reads at odd m 97..127.
struct SchedTwoBarrier {
  static constexpr int W1 = 34, B1 = 35, W2 = -1, B2 = -1, W3 = 95, VM3 = 16, B3 = 96;
  __host__ __device__ static constexpr int a1(int m) { return m < 16 && (m & 1) == 0 ? m >> 1 : -1; }
  __host__ __device__ static constexpr int b1(int m) {
    return m >= 16 && m < 32 && (m & 1) == 0 ? (m - 16) >> 1 : -1;
  }
  __host__ __device__ static constexpr int adma(int m) {
    return m >= 36 && (m - 36) % 6 == 0 && (m - 36) / 6 < 8 ? (m - 36) / 6 : -1;
  }
  __host__ __device__ static constexpr int bdma(int m) {
    return m >= 39 && (m - 39) % 6 == 0 && (m - 39) / 6 < 8 ? (m - 39) / 6 : -1;
  }
  __host__ __device__ static constexpr int k0(int m) {
    return m >= 97 && (m & 1) ? (m - 97) >> 1 : -1;
  }
};

// SCHED 7: ONE barrier per K-tile.  The two 64 KiB stages alternate per
// K-tile (tile t reads buffer t & 1); the barrier sits in the MIDDLE of the
// tile, after the k-half-1 fragments of stage t were read (m 0..30, retired
// by the lgkmcnt(0) before it) and after this wave's pieces of stage t+1
// landed (vmcnt(0): the only DMA in flight is stage t+1's, issued one K-tile
// earlier).  Past it every wave is done with buffer t & 1 (-> refill with
// stage t+2, m 64..94 even) and stage t+1 is visible everywhere (-> its
// k-half-0 fragments, m 65..95 odd).  The DMA gets a whole K-tile to land.
struct SchedOneBarrier {
  static constexpr int W1 = 62, B1 = -1, W2 = -1, B2 = -1, W3 = 62, VM3 = 0, B3 = 63;
  __host__ __device__ static constexpr int a1(int m) { return m < 16 && (m & 1) == 0 ? m >> 1 : -1; }
  __host__ __device__ static constexpr int b1(int m) {
    return m >= 16 && m < 32 && (m & 1) == 0 ? (m - 16) >> 1 : -1;
  }
  __host__ __device__ static constexpr int adma(int m) {
    return m >= 64 && m < 80 && (m & 1) == 0 ? (m - 64) >> 1 : -1;
  }
  __host__ __device__ static constexpr int bdma(int m) {
    return m >= 80 && m < 96 && (m & 1) == 0 ? (m - 80) >> 1 : -1;
  }
  __host__ __device__ static constexpr int k0(int m) {
    return m >= 65 && m < 96 && (m & 1) ? (m - 65) >> 1 : -1;
  }
};

// SCHED 8: SchedOneBarrier with the 16 pieces spread one per three MFMAs
// (m 64..109) and the k-half-0 reads one per two (odd m 65..95).
struct SchedOneBarrierSpread : SchedOneBarrier {
  __host__ __device__ static constexpr int adma(int m) {
    return m >= 64 && (m - 64) % 6 == 0 && (m - 64) / 6 < 8 ? (m - 64) / 6 : -1;
  }
  __host__ __device__ static constexpr int bdma(int m) {
    return m >= 67 && (m - 67) % 6 == 0 && (m - 67) / 6 < 8 ? (m - 67) / 6 : -1;
  }
};

}  // namespace mxk

// Host-side error plumbing: every launcher returns hipError_t as int so the
// Python (ctypes) side can raise with the HIP error string.
#define MXK_RETURN_LAUNCH_STATUS() return static_cast<int>(hipGetLastError())
