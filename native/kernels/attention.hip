// Flash attention (causal / full, GQA, head_dim 128, bf16) for gfx950.
//
// The Llama-3-8B DDP validator step (BASELINE config 5) spends ~16 % of its
// time in attention; torch's SDPA backends on this image reach 140-150 TF/s.
// These kernels keep the S x S scores on chip (online softmax) and are
// written around CDNA4's 32x32x16 bf16 MFMA and 64-lane waves:
//
// Forward (mxk_attn_fwd): one workgroup = 4 waves = 128 query rows of one
// (batch, q-head); each wave owns 32 query rows.  Per 64-key block:
//   * S^T = K . Q^T with the KEY as the MFMA row and the QUERY on the lane
//     ("swapped" QK^T): every lane holds 32 of its query's 64 scores, so the
//     row max / row sum are in-lane plus ONE permlane32_swap with the other
//     lane half - no LDS, no shuffles;
//   * P^T (bf16, straight from the accumulator registers) is the B operand
//     of O^T += V^T . P^T, whose A operand comes from LDS with the gfx950
//     transposed read ds_read_b64_tr_b16 - V is stored row-major as loaded;
//   * O^T accumulates with the query on the lane, so the online-softmax
//     rescale is a per-lane scalar multiply.
// K and V tiles are staged through registers into a double-buffered,
// XOR-swizzled LDS image (256-B rows, chunk c of row r at
// c ^ ((r&3)<<2 | (r>>2)&3)), conflict-free for both the row reads of K and
// the transposed reads of V (tests/test_attention_layout.py).
// Causal work is balanced by launching the heaviest query blocks first and
// pairing block i with block n-1-i across the two halves of the grid.
//
// Layouts: q [B, S, Hq, 128], k/v [B, S, Hkv, 128] with arbitrary token
// strides (so q/k/v can be views of the fused QKV projection), o
// [B, S, Hq, 128] contiguous, lse [B, Hq, S] fp32 (natural log of the row's
// sum of exp(scale * s)) for the backward pass.
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

__device__ __forceinline__ bf16x4_t lds_tr_b64(const char* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(reinterpret_cast<uintptr_t>(p)));
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
}  // namespace

template <bool CAUSAL>
__global__ void __launch_bounds__(NT, 2)
mxk_attn_fwd_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                    const uint16_t* __restrict__ v, uint16_t* __restrict__ o,
                    float* __restrict__ lse, int S, int Hq, int Hkv, long q_tok, long k_tok,
                    long v_tok, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[2][2 * TILE_BYTES];   // [buf][K | V]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nqb = S / BQ;
  int bh, qb;
  map_block(blockIdx.x, gridDim.x / nqb, nqb, CAUSAL, &bh, &qb);
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int q0 = qb * BQ;
  const int qw0 = q0 + wave * 32;
  const int myq = qw0 + r32;

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  // Q^T fragments (B operand): lane holds Q[myq][16s + 8h .. +7]
  bf16x8_t qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
    qf[s] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + static_cast<long>(myq) * q_tok + 16 * s + 8 * h);

  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int nkv = kv_end / BKV;

  // loader: thread t moves chunks t + 256 i (i = 0..3) of the 64 x 16-chunk tile
  const int ld_row = tid >> 4, ld_ch = tid & 15;
  bf16x8_t kst[4], vst[4];
  auto load_tile = [&](int j) {
    const long r0 = static_cast<long>(j) * BKV + ld_row;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kst[i] = *reinterpret_cast<const bf16x8_t*>(kb_ptr + (r0 + 16 * i) * k_tok + ld_ch * 8);
      vst[i] = *reinterpret_cast<const bf16x8_t*>(vb_ptr + (r0 + 16 * i) * v_tok + ld_ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    char* kt = smem[buf];
    char* vt = smem[buf] + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = swz(ld_row + 16 * i, ld_ch);
      *reinterpret_cast<bf16x8_t*>(kt + off) = kst[i];
      *reinterpret_cast<bf16x8_t*>(vt + off) = vst[i];
    }
  };
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const float c = scale * 1.4426950408889634f;   // scores -> log2 domain
  float m = -INFINITY, l = 0.f;
  f32x16_t acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[db][r] = 0.f;

  // per-lane parts of the transposed-read addresses of V (see header)
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * h + (i16 >> 2);                          // + 32kb + 16s' + 8jh
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);               // + 4db
  const int tr_byte = 8 * (i16 & 1);

  for (int j = 0; j < nkv; ++j) {
    const int buf = j & 1;
    if (j + 1 < nkv) load_tile(j + 1);
    const int kv0 = j * BKV;
    const bool active = !CAUSAL || kv0 <= qw0 + 31;
    if (active) {
      const char* kt = smem[buf];
      const char* vt = smem[buf] + TILE_BYTES;
      // ---- S^T = K . Q^T : two 32-key halves
      f32x16_t s0, s1;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] = 0.f; s1[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8_t a0 = lds_b128(kt + swz(r32, 2 * s + h));
        const bf16x8_t a1 = lds_b128(kt + swz(32 + r32, 2 * s + h));
        s0 = mfma32(a0, qf[s], s0);
        s1 = mfma32(a1, qf[s], s1);
      }
      if (CAUSAL && kv0 + BKV - 1 > qw0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kv0 + crow(r, h);
          if (key > myq) s0[r] = -INFINITY;
          if (key + 32 > myq) s1[r] = -INFINITY;
        }
      }
      // ---- online softmax (query = lane, keys in registers + other half)
      float mx = s0[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s0[r]);
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s1[r]);
      mx = half_max(mx);
      const float m_new = fmaxf(m, mx);
      const float alpha = exp2f((m - m_new) * c);
      m = m_new;
      const float mc = m_new * c;
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = exp2f(fmaf(s0[r], c, -mc));
        s1[r] = exp2f(fmaf(s1[r], c, -mc));
        ls += s0[r] + s1[r];
      }
      l = l * alpha + ls;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[db][r] *= alpha;
      // P^T fragments for the 4 16-key k-steps
      bf16x8_t pf[4];
      pf[0] = pack8(s0, 0);
      pf[1] = pack8(s0, 8);
      pf[2] = pack8(s1, 0);
      pf[3] = pack8(s1, 8);
      // ---- O^T += V^T . P^T
#pragma unroll
      for (int db = 0; db < 4; ++db) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int key = 16 * ks + tr_key;
          const int ch = 4 * db + tr_ch;
          const bf16x4_t lo = lds_tr_b64(vt + swz(key, ch) + tr_byte);
          const bf16x4_t hi = lds_tr_b64(vt + swz(key + 8, ch) + tr_byte);
          bf16x8_t a;
          a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
          a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
          acc[db] = mfma32(a, pf[ks], acc[db]);
        }
      }
    }
    if (j + 1 < nkv) store_tile(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: normalise, store O[b][myq][hq][:] and the row LSE
  const float lt = half_sum(l);
  const float inv = 1.f / lt;
  uint16_t* orow = o + (static_cast<long>(b) * S + myq) * Hq * D + static_cast<long>(hq) * D;
#pragma unroll
  for (int db = 0; db < 4; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * db + 8 * g + 4 * h;
      uint2 pk;
      pk.x = mxk::pack2bf(acc[db][4 * g] * inv, acc[db][4 * g + 1] * inv);
      pk.y = mxk::pack2bf(acc[db][4 * g + 2] * inv, acc[db][4 * g + 3] * inv);
      *reinterpret_cast<uint2*>(orow + d) = pk;
    }
  }
  if (h == 0) lse[(static_cast<long>(b) * Hq + hq) * S + myq] = m * scale + logf(lt);
}

// ---------------------------------------------------------------------------
MXK_API int mxk_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B,
                         int S, int Hq, int Hkv, int head_dim, long q_tok, long k_tok, long v_tok,
                         float scale, int causal, hipStream_t stream) {
  if (head_dim != D || B < 1 || S < BQ || S % BQ || Hkv < 1 || Hq % Hkv ||
      q_tok % 8 || k_tok % 8 || v_tok % 8 ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * Hq * (S / BQ);
  if (causal)
    hipLaunchKernelGGL(mxk_attn_fwd_kernel<true>, dim3(nwg), dim3(NT), 0, stream,
                       static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k),
                       static_cast<const uint16_t*>(v), static_cast<uint16_t*>(o), lse, S, Hq, Hkv,
                       q_tok, k_tok, v_tok, scale);
  else
    hipLaunchKernelGGL(mxk_attn_fwd_kernel<false>, dim3(nwg), dim3(NT), 0, stream,
                       static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k),
                       static_cast<const uint16_t*>(v), static_cast<uint16_t*>(o), lse, S, Hq, Hkv,
                       q_tok, k_tok, v_tok, scale);
  MXK_RETURN_LAUNCH_STATUS();
}
