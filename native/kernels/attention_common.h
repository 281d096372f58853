// Helpers shared by the flash-attention kernels (attention.hip) and the
// experiments-only forward A/B records (experiments/attention_fwd_exp.hip).
#pragma once
#include <type_traits>

#include "mx_common.h"

namespace {
constexpr int D = 128;          // head dim
constexpr int BQ = 128;         // query rows per workgroup (4 waves x 32)
constexpr int BKV = 64;         // keys per block
constexpr int NT = 256;         // threads per workgroup
constexpr int TILE_BYTES = BKV * D * 2;   // 16 KiB

// byte offset of 16-B chunk `ch` (0..15) of row `row` in a [rows][128 bf16] image
__device__ __forceinline__ int swz(int row, int ch) {
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

__device__ __forceinline__ bf16x8_t lds_b128(const char* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

// s_waitcnt vmcnt(0) through the builtin rather than inline asm: the
// compiler's wait-insertion pass then knows every earlier load has landed and
// adds no waits of its own further on (with inline asm it re-waits, e.g. on a
// register a finished load wrote - and such a wait also waits for the DMA of
// the next tile, which the compiler cannot see).
__device__ __forceinline__ void vm_wait0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ bf16x4_t lds_tr_b64(const char* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  // plain address-space cast (not via an integer): `base + constant` stays
  // visible and the constant folds into the instruction's offset field
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
  return v;
}

__device__ __forceinline__ f32x16_t mfma32(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// max / sum of a lane's value with the same lane of the other 32-lane half
__device__ __forceinline__ float half_max(float x) {
  const unsigned u = __float_as_uint(x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const unsigned u = __float_as_uint(x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// v_exp_f32 directly: inputs are <= 0 (or -inf for masked keys), where the
// libm exp2f's denormal range fix-up (cmp/cndmask/ldexp) is dead weight.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 8-element MFMA operand from two transposed 4-element reads
__device__ __forceinline__ bf16x8_t cat8(bf16x4_t lo, bf16x4_t hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// row of a 32x32 accumulator register r (0..15) for lane half h
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8_t pack8(const f32x16_t& x, int base) {
  bf16x8_t o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = static_cast<short>(mxk::f2bf(x[base + j]));
  return o;
}

// Work order: first half of the grid = heaviest query blocks (descending),
// second half = lightest (ascending); block b and b + n/2 are complementary.
__device__ __forceinline__ void map_block(int w, int nbh, int nqb, bool causal, int* bh, int* qb) {
  if (!causal) {
    *bh = w % nbh;
    *qb = w / nbh;
    return;
  }
  if (nqb & 1) {   // heaviest first
    *bh = w % nbh;
    *qb = nqb - 1 - w / nbh;
    return;
  }
  const int half = (nbh * nqb) / 2;
  if (w < half) {
    *bh = w % nbh;
    *qb = nqb - 1 - w / nbh;
  } else {
    const int v = w - half;
    *bh = v % nbh;
    *qb = v / nbh;
  }
}

// XCD-local work order.  Workgroups are dispatched round-robin over the 8
// XCDs (each with its own L2), so with map_block the blocks resident on one
// XCD at a time belong to many different heads and share little.  Here
// mxk::xcd_remap gives each XCD a contiguous range of logical ids, and
// consecutive logical ids are the `grp` query heads of one KV head x all
// their blocks (heaviest first when causal): about one such group is
// resident per XCD, so its K/V (1 MiB) stays in that L2.  Forward 0.408 ->
// 0.368 ms, dQ 570 -> 526 us per Llama-3-8B layer (profiles/r1_attention/).
// Not used by dK/dV: its per-group Q/dO (4 MiB) is the whole L2, and the same
// order there ran 8 % slower.
__device__ __forceinline__ void map_block_xcd(int w, int nwg, int nqb, int grp, bool causal,
                                              int* bh, int* qb) {
  const int L = mxk::xcd_remap(w, nwg);
  const int per = grp * nqb;
  const int g = L / per, r = L - g * per;
  const int j = r / grp;
  *bh = g * grp + (r - j * grp);
  *qb = causal ? nqb - 1 - j : j;
}
}  // namespace

namespace {
typedef float f32x2_t __attribute__((ext_vector_type(2)));
}

// dK / dV with 256 keys per workgroup (attention_bwd256.hip; backward variant 6)
MXK_API int mxk_attn_bwd_dkdv256(const void* q, const void* k, const void* v, const void* dout,
                                 const float* rowc, void* dk, void* dv, int B, int S, int Hq,
                                 int Hkv, long q_tok, long k_tok, long v_tok, long dk_tok,
                                 long dv_tok, float scale, int causal, hipStream_t stream);
MXK_API long mxk_attn_bwd_onepass_workspace(int B, int S, int Hq, int bf16_atomics);
MXK_API int mxk_attn_bwd_onepass(const void* q, const void* k, const void* v, const void* o,
                                 const void* dout, const float* lse, void* dq, void* dk, void* dv,
                                 void* workspace, int B, int S, int Hq, int Hkv, long q_tok,
                                 long k_tok, long v_tok, long dk_tok, long dv_tok, float scale,
                                 int causal, int bf16_atomics, hipStream_t stream);
// dQ of backward variant 9 (attention_dq256.hip): 4 query heads x 64 rows per
// workgroup, one wave per SIMD; writes the rowc pairs for mxk_attn_bwd_dkdv256
MXK_API int mxk_attn_bwd_dq256(const void* q, const void* k, const void* v, const void* o,
                               const void* dout, const float* lse, void* dq, float* rowc, int B,
                               int S, int Hq, int Hkv, long q_tok, long k_tok, long v_tok,
                               float scale, int causal, hipStream_t stream);
// the same two kernels with the rotary-embedding backward fused into their
// stores (rcos / rsin: [S][D/2] fp32 tables; dQ / dK leave un-rotated, i.e.
// as the gradient of the pre-RoPE projection) and dQ at a token stride
MXK_API int mxk_attn_bwd_dkdv256_rope(const void* q, const void* k, const void* v, const void* dout,
                                      const float* rowc, void* dk, void* dv, int B, int S, int Hq,
                                      int Hkv, long q_tok, long k_tok, long v_tok, long dk_tok,
                                      long dv_tok, const float* rcos, const float* rsin,
                                      float scale, int causal, hipStream_t stream);
MXK_API int mxk_attn_bwd_dq256_rope(const void* q, const void* k, const void* v, const void* o,
                                    const void* dout, const float* lse, void* dq, float* rowc,
                                    int B, int S, int Hq, int Hkv, long q_tok, long k_tok,
                                    long v_tok, long dq_tok, const float* rcos, const float* rsin,
                                    float scale, int causal, hipStream_t stream);
// forward variant 10 (attention_fwd256.hip)
MXK_API int mxk_attn_fwd256(const void* q, const void* k, const void* v, void* o, float* lse,
                            int B, int S, int Hq, int Hkv, long q_tok, long k_tok, long v_tok,
                            float scale, int causal, hipStream_t stream);
