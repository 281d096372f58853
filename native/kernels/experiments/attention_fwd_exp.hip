// Flash-attention forward A/B records (variants 5-9), built only into the
// experiments library (`make gemm-exp` -> libmxkernels_exp.so, selected with
// MXK_KERNELS_LIB); mxk_attn_fwd_variant (attention.hip) dispatches here in that
// build.  Measured slower than the production variant 4 (docs/ARCHITECTURE.md,
// profiles/r3_attn/, profiles/r3_pmc/): kept so the records can be re-run.
#include "attention_common.h"

// ---------------------------------------------------------------------------
// Forward, 8-wave ping-pong (variant 5).  The kernels above run each wave's
// QK^T MFMAs, its softmax (VALU, ~700 issue cycles per 64-key tile: 32 v_exp
// at 8 cycles each, scale/shift, row max and sum, bf16 packs) and its PV
// MFMAs back to back, and all four waves of a workgroup pass the same
// barriers, so a SIMD's matrix pipe idles whenever its waves are in the
// softmax (PMC: MFMA busy 40 %, VALU/MFMA co-execution 13 %).
// Here one 512-thread workgroup = 8 waves x 32 query rows (256 rows of one
// (batch, q-head)); SIMD s holds wave s (group A, rows 32 s ..) and wave s + 4
// (group B, rows 128 + 32 s ..).  Both groups run the same per-tile sequence
//     M_j: S_j = K_j . Q^T (16 MFMAs) and O += V_{j-1}^T . P_{j-1} (16 MFMAs)
//     S_j: mask, row max, lazy rescale of O, exp2, row sum, P_j to bf16
// one phase apart, with one workgroup barrier per phase: while group A is in
// M_j, group B is in S_{j-1}, and the other way round, so every SIMD pairs
// one wave's matrix work with its partner's softmax (the FA3 ping-pong, here
// between the two waves of a SIMD).  K and V tiles arrive by LDS-DMA into
// 3-slot rings (K_j is read in phases 2j / 2j+1, V_j in 2j+2 / 2j+3): at
// every even phase 2i each wave issues its 4 pieces of K_{i+2} and V_{i+1},
// and waits for them (counted vmcnt, 4 pieces left in flight) at the end of
// phase 2i+3.  Math, LDS image, swizzle and operand mapping are variant 4's.
// Causal: tile j is skipped by a wave whose 32 rows all precede key 64 j
// (the workgroup still walks every phase: one barrier schedule).
namespace {
constexpr int PP_BQ = 256;     // query rows per workgroup (8 waves x 32)
constexpr int PP_NT = 512;
constexpr int PP_SLOTS = 3;    // K ring and V ring depth
}  // namespace

template <bool CAUSAL, bool PRIO = false, int DIAG = 0>
__global__ void __launch_bounds__(PP_NT, 1)
mxk_attn_fwd_pp_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                       const uint16_t* __restrict__ v, uint16_t* __restrict__ o,
                       float* __restrict__ lse, int S, int Hq, int Hkv, long q_tok, long k_tok,
                       long v_tok, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PP_SLOTS * TILE_BYTES];   // K ring | V ring
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nqb = S / PP_BQ;
  int bh, qb;
  map_block_xcd(blockIdx.x, gridDim.x, nqb, Hq / Hkv, CAUSAL, &bh, &qb);
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int q0 = qb * PP_BQ;
  const int qw0 = q0 + wave * 32;
  const int myq = qw0 + r32;

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  bf16x8_t qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
    qf[s] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + static_cast<long>(myq) * q_tok + 16 * s + 8 * h);

  const int n = (CAUSAL ? min(S, q0 + PP_BQ) : S) / BKV;

  // DMA: wave w moves the 1-KiB pieces g = 2w, 2w + 1 (rows 4g .. 4g + 3) of
  // each tile; lane i lands at row 4g + (i >> 4), slot i & 15, so it fetches
  // chunk (i & 15) ^ ((i >> 4) << 2 | (g & 3)) (the swz() image).
  const mxk::u32x4 rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
  const mxk::u32x4 rv = mxk::make_rsrc(vb_ptr, static_cast<unsigned>(S * v_tok * 2));
  const int prow = lane >> 4, pslot = lane & 15;
  uint32_t kvo[2], vvo[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int g = 2 * wave + p;
    const int row = 4 * g + prow;
    const int ch = pslot ^ ((prow << 2) | (g & 3));
    kvo[p] = static_cast<uint32_t>(row * k_tok * 2 + ch * 16);
    vvo[p] = static_cast<uint32_t>(row * v_tok * 2 + ch * 16);
  }
  const uint32_t k_step = static_cast<uint32_t>(BKV * k_tok * 2);
  const uint32_t v_step = static_cast<uint32_t>(BKV * v_tok * 2);
  const uint32_t sm32 = mxk::lds_addr32(&smem[0]);
  auto issue_k = [&](int j) {
    const uint32_t d = sm32 + (j % PP_SLOTS) * TILE_BYTES + (2 * wave) * 1024;
#pragma unroll
    for (int p = 0; p < 2; ++p) mxk::dma16m(rk, d + p * 1024, kvo[p], j * k_step);
  };
  auto issue_v = [&](int j) {
    const uint32_t d = sm32 + (PP_SLOTS + j % PP_SLOTS) * TILE_BYTES + (2 * wave) * 1024;
#pragma unroll
    for (int p = 0; p < 2; ++p) mxk::dma16m(rv, d + p * 1024, vvo[p], j * v_step);
  };
  issue_k(0);
  issue_v(0);
  if (n > 1) issue_k(1);

  int koff[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) koff[s] = swz(r32, 2 * s + h);
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * h + (i16 >> 2);
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);
  const int tr_byte = 8 * (i16 & 1);
  int voff[4][2];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    voff[db][0] = swz(tr_key, 4 * db + tr_ch) + tr_byte;
    voff[db][1] = swz(tr_key + 8, 4 * db + tr_ch) + tr_byte;
  }

  const float c = scale * 1.4426950408889634f;   // scores -> log2 domain
  const f32x2_t cc = {c, c};
  float m = -INFINITY, l = 0.f;
  f32x16_t acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[db][r] = 0.f;
  f32x16_t s0, s1;
  bf16x8_t pf[4];

#pragma unroll
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]));
  vm_wait0();   // Q, K_0, V_0, K_1
  __syncthreads();

  // tile j is active for this wave unless all its rows precede key 64 j;
  // the active tiles are a prefix 0 .. na - 1
  const int na = CAUSAL ? min(n, (qw0 + 31) / BKV + 1) : n;

  // end of global phase ph: counted wait for the DMA this wave issued at
  // phase ph - 3 (odd ph), the workgroup barrier, then the next even phase's
  // DMA (K_{i+2}, V_{i+1} at phase 2i)
  auto issue_for = [&](int ph) {
    const int i = ph >> 1;
    if (i + 2 < n) issue_k(i + 2);
    if (i + 1 < n) issue_v(i + 1);
  };
  auto end_phase = [&](int ph) {
    if ((ph & 1) && ph >= 3) {
      if (((ph - 3) >> 1) + 3 < n) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS reads retired
    __builtin_amdgcn_s_barrier();
    if (ph & 1) issue_for(ph + 1);
  };

  // operands are read one group ahead of their MFMAs (two-slot rings:
  // K 4 x b128 per k-step pair, V^T 4 x (2 transposed b64) per db); the
  // sched_barrier fences keep the compiler from hoisting every read of the
  // phase (64 + 64 VGPRs) ahead of the first MFMA
  auto qk = [&](int j) {
    if constexpr (DIAG == 2) {   // timing ablation: no MFMAs
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] = qf[r >> 1][r & 7] * 1e-3f; s1[r] = s0[r] + j; }
      return;
    }
    const char* kt = smem + (j % PP_SLOTS) * TILE_BYTES;
#pragma unroll
    for (int r = 0; r < 16; ++r) { s0[r] = 0.f; s1[r] = 0.f; }
    bf16x8_t ka[2][4];
    auto read_k = [&](int pr, int slot) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        ka[slot][2 * e] = lds_b128(kt + koff[2 * pr + e]);
        ka[slot][2 * e + 1] = lds_b128(kt + koff[2 * pr + e] + 32 * 256);
      }
    };
    read_k(0, 0);
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) {
      if (pr < 3) read_k(pr + 1, (pr + 1) & 1);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        s0 = mfma32(ka[pr & 1][2 * e], qf[2 * pr + e], s0);
        s1 = mfma32(ka[pr & 1][2 * e + 1], qf[2 * pr + e], s1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto pv = [&](int j) {
    if constexpr (DIAG == 2) {
#pragma unroll
      for (int db = 0; db < 4; ++db) acc[db][0] += static_cast<float>(pf[db][0]);
      return;
    }
    const char* vt = smem + (PP_SLOTS + j % PP_SLOTS) * TILE_BYTES;
    bf16x8_t va[2][4];
    auto read_v = [&](int db, int slot) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        va[slot][ks] = cat8(lds_tr_b64(vt + voff[db][0] + ks * 4096),
                            lds_tr_b64(vt + voff[db][1] + ks * 4096));
    };
    read_v(0, 0);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      if (db < 3) read_v(db + 1, (db + 1) & 1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc[db] = mfma32(va[db & 1][ks], pf[ks], acc[db]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  auto softmax = [&](int j) {
    if constexpr (DIAG == 1) {   // timing ablation: P = packed raw scores
      pf[0] = pack8(s0, 0);
      pf[1] = pack8(s0, 8);
      pf[2] = pack8(s1, 0);
      pf[3] = pack8(s1, 8);
      l += s0[0];
      return;
    }
    const int kv0 = j * BKV;
    if (CAUSAL && kv0 + BKV - 1 > qw0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kv0 + crow(r, h);
        if (key > myq) s0[r] = -INFINITY;
        if (key + 32 > myq) s1[r] = -INFINITY;
      }
    }
    float mx = s0[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s0[r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s1[r]);
    mx = half_max(mx);
    float m_new = fmaxf(m, mx);
    // lazy rescale (variant 4): keep the stale max unless the new one
    // exceeds it by more than 2^8 in the exp2 domain
    const bool grow = (m_new - m) * c > 8.f;
    if (!grow) m_new = m;
    const float alpha = grow ? fexp2((m - m_new) * c) : 1.f;
    m = m_new;
    if (__builtin_amdgcn_ballot_w64(grow)) {
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[db][r] *= alpha;
    }
    const f32x2_t nmc = {-m_new * c, -m_new * c};
    f32x2_t ls2 = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      f32x2_t x0 = {s0[r], s0[r + 1]};
      f32x2_t x1 = {s1[r], s1[r + 1]};
      x0 = __builtin_elementwise_fma(x0, cc, nmc);
      x1 = __builtin_elementwise_fma(x1, cc, nmc);
      x0[0] = fexp2(x0[0]);
      x0[1] = fexp2(x0[1]);
      x1[0] = fexp2(x1[0]);
      x1[1] = fexp2(x1[1]);
      ls2 += x0 + x1;
      s0[r] = x0[0];
      s0[r + 1] = x0[1];
      s1[r] = x1[0];
      s1[r + 1] = x1[1];
    }
    l = l * alpha + (ls2[0] + ls2[1]);
    pf[0] = pack8(s0, 0);
    pf[1] = pack8(s0, 8);
    pf[2] = pack8(s1, 0);
    pf[3] = pack8(s1, 8);
  };

  // global phase ph: group A runs its local phase ph, group B ph - 1; local
  // phase 2j is M_j = {QK_j, PV_{j-1}}, 2j + 1 is S_j; M_na is PV_{na-1}
  // alone.  Barriers follow global phases 0 .. 2n (phase 2n + 1 is B's M_n).
  // PRIO (variant 6): a wave raises its priority for its MFMA phase.  The
  // SIMD's vector-issue arbiter prefers the older wave at equal priority, so
  // without it group A's softmax VALU (waves 0-3, older) takes the issue
  // slots group B's MFMAs need and the two phases serialise (PMC of variant
  // 5: MFMA busy 29 %, co-execution 4 % of SIMD cycles).
  auto prio_hi = [&]() { if constexpr (PRIO) __builtin_amdgcn_s_setprio(1); };
  auto prio_lo = [&]() { if constexpr (PRIO) __builtin_amdgcn_s_setprio(0); };
  issue_for(0);
  int ph = 0;
  if (grp) end_phase(ph++);
  prio_hi();
  qk(0);
  prio_lo();
  end_phase(ph++);
  softmax(0);
  end_phase(ph++);
  for (int j = 1; j < na; ++j) {
    prio_hi();
    qk(j);
    pv(j - 1);
    prio_lo();
    end_phase(ph++);
    softmax(j);
    end_phase(ph++);
  }
  prio_hi();
  pv(na - 1);
  prio_lo();
  for (; ph <= 2 * n; ++ph) end_phase(ph);

  const float lt = half_sum(l);
  const float inv = 1.f / lt;
  uint16_t* orow = o + (static_cast<long>(b) * S + myq) * Hq * D + static_cast<long>(hq) * D;
#pragma unroll
  for (int db = 0; db < 4; ++db) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int g0 = 2 * kk, g1 = 2 * kk + 1;
      const uint32_t x0 = mxk::pack2bf(acc[db][4 * g0] * inv, acc[db][4 * g0 + 1] * inv);
      const uint32_t x1 = mxk::pack2bf(acc[db][4 * g0 + 2] * inv, acc[db][4 * g0 + 3] * inv);
      const uint32_t y0 = mxk::pack2bf(acc[db][4 * g1] * inv, acc[db][4 * g1 + 1] * inv);
      const uint32_t y1 = mxk::pack2bf(acc[db][4 * g1 + 2] * inv, acc[db][4 * g1 + 3] * inv);
      const auto p0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
      const auto p1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
      uint4 vv;
      vv.x = p0[0];
      vv.y = p1[0];
      vv.z = p0[1];
      vv.w = p1[1];
      *reinterpret_cast<uint4*>(orow + 32 * db + 16 * kk + 8 * h) = vv;
    }
  }
  if (h == 0) lse[(static_cast<long>(b) * Hq + hq) * S + myq] = m * scale + logf(lt);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outlives the workgroup
}

// ---------------------------------------------------------------------------
// Forward, one wave per SIMD with two interleaved row groups (variant 9).
// One 256-thread workgroup = 4 waves x 64 query rows; a wave owns two 32-row
// groups, g0 = rows 32 w .. and g1 = rows 32 (7 - w) .. of the block
// (mirrored, so every wave has the same causal work), and the whole 512
// registers of its SIMD.  Per 64-key tile j the wave issues four blocks of
// 16 v_mfma_f32_32x32x16_bf16
//     B1 QK(g0, K_j)  B2 PV(g1, V_{j-1})  B3 QK(g1, K_j)  B4 PV(g0, V_j)
// and places the softmax of the OTHER group's scores between them, one
// short VALU chunk behind each MFMA (<= ~6 issues: the MFMA holds the SIMD's
// vector issue for 8 of its 32 cycles, the rest is free): softmax(g0, j) in
// B2 + B3, softmax(g1, j) in B4 + B1 of the next tile.  Each group's rare
// lazy rescale (variant 4's 2^8 threshold) is a branch between blocks, so
// the interleaved blocks stay branch-free.  K ring 2 slots, V ring 3 slots
// (V_j is read in B4 of tile j and B2 of tile j + 1), LDS-DMA issued after
// the tile's barrier and waited one tile later.  Diagonal tiles mask S with
// selects before the softmax (groups whose rows all precede the tile still
// run it: P = 0).
namespace {
constexpr int W1_BQ = 256;

typedef unsigned u32x4v_t __attribute__((ext_vector_type(4)));

struct W1Grp {
  f32x16_t s0, s1;      // S^T of the two 32-key halves (query on the lane)
  f32x16_t o[4];        // O^T accumulators
  u32x4v_t p[4];        // P^T operands of the PV MFMAs (bf16 pairs)
  float m, l;           // running row max (stale by <= 2^8) and row sum
  float mq[4], mx, alpha, nmc;
  float la[4];
  bool grow;
};

__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// softmax chunk k (0..31) of a group whose scores s0 / s1 are final; chunks
// 0-15 run beside one MFMA block, 16-31 beside the next
__device__ __forceinline__ void w1_sm(W1Grp& g, int k, float cs) {
  if (k < 4) {                       // row max, four chains (v_max3)
    const int r = 4 * k;
    if (k == 0) {
      g.mq[0] = fmaxf(g.s0[0], g.s0[1]);
      g.mq[1] = fmaxf(g.s0[2], g.s0[3]);
      g.mq[2] = fmaxf(g.s1[0], g.s1[1]);
      g.mq[3] = fmaxf(g.s1[2], g.s1[3]);
    } else {
      g.mq[0] = max3(g.mq[0], g.s0[r], g.s0[r + 1]);
      g.mq[1] = max3(g.mq[1], g.s0[r + 2], g.s0[r + 3]);
      g.mq[2] = max3(g.mq[2], g.s1[r], g.s1[r + 1]);
      g.mq[3] = max3(g.mq[3], g.s1[r + 2], g.s1[r + 3]);
    }
  } else if (k == 4) {
    g.mx = half_max(max3(g.mq[0], g.mq[1], fmaxf(g.mq[2], g.mq[3])));
  } else if (k == 5) {
    float m_new = fmaxf(g.m, g.mx);
    g.grow = (m_new - g.m) * cs > 8.f;
    if (!g.grow) m_new = g.m;
    g.alpha = g.grow ? fexp2((g.m - m_new) * cs) : 1.f;
    g.m = m_new;
    g.nmc = -m_new * cs;
    g.la[0] = g.la[1] = g.la[2] = g.la[3] = 0.f;
  } else if (k < 22) {               // exp2 of two scores per chunk, packed to bf16
    const int e = k - 6;             // 0..15: pair (r, r + 1) of s0 (e < 8) or s1
    const f32x16_t& x = e < 8 ? g.s0 : g.s1;
    const int r = 2 * (e & 7);
    const float e0 = fexp2(fmaf(x[r], cs, g.nmc));
    const float e1 = fexp2(fmaf(x[r + 1], cs, g.nmc));
    g.la[e & 3] += e0 + e1;
    // pack8(s, base) order: P operand t = 2 (e >> 3) + ((e & 7) >> 2), word e & 3
    g.p[2 * (e >> 3) + ((e & 7) >> 2)][e & 3] = mxk::pack2bf(e0, e1);
  } else if (k == 26) {
    g.l = g.l * g.alpha + ((g.la[0] + g.la[1]) + (g.la[2] + g.la[3]));
  }
}
}  // namespace

template <bool CAUSAL>
__global__ void __launch_bounds__(NT, 1)
mxk_attn_fwd_w1_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                       const uint16_t* __restrict__ v, uint16_t* __restrict__ o,
                       float* __restrict__ lse, int S, int Hq, int Hkv, long q_tok, long k_tok,
                       long v_tok, float scale) {
  constexpr int VS = 3, KS = 3;
  // LDS: K ring [0, 48 KiB), V ring [48, 96 KiB); the V ring's base is folded
  // into the per-lane V read offsets, so every LDS read is base VGPR +
  // immediate < 64 KiB (a larger constant costs an extra address register per
  // read stream: the build spills)
  constexpr int VB = KS * TILE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[(VS + KS) * TILE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nqb = S / W1_BQ;
  int bh, qb;
  map_block_xcd(blockIdx.x, gridDim.x, nqb, Hq / Hkv, CAUSAL, &bh, &qb);
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int q0 = qb * W1_BQ;
  const int qw0 = q0 + 32 * wave, qw1 = q0 + 32 * (7 - wave);
  const int myq0 = qw0 + r32, myq1 = qw1 + r32;

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  bf16x8_t qf0[8], qf1[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    qf0[s] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + static_cast<long>(myq0) * q_tok + 16 * s + 8 * h);
    qf1[s] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + static_cast<long>(myq1) * q_tok + 16 * s + 8 * h);
  }
  const int n = (CAUSAL ? min(S, q0 + W1_BQ) : S) / BKV;

  // DMA: wave w moves pieces 4w + p of each tile (variant 4's map)
  const mxk::u32x4 rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
  const mxk::u32x4 rv = mxk::make_rsrc(vb_ptr, static_cast<unsigned>(S * v_tok * 2));
  const int prow = lane >> 4, pslot = lane & 15;
  const uint32_t k_row = static_cast<uint32_t>(k_tok) * 2u, v_row = static_cast<uint32_t>(v_tok) * 2u;
  uint32_t kvo[4], vvo[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t row = static_cast<uint32_t>(4 * (4 * wave + p) + prow);
    const uint32_t ch = static_cast<uint32_t>(pslot ^ ((prow << 2) | p));
    kvo[p] = row * k_row + ch * 16u;
    vvo[p] = row * v_row + ch * 16u;
  }
  const uint32_t k_step = static_cast<uint32_t>(BKV) * k_row;
  const uint32_t v_step = static_cast<uint32_t>(BKV) * v_row;
  const uint32_t sm32 = mxk::lds_addr32(&smem[0]);
  auto issue = [&](int j) __attribute__((always_inline)) {
    const uint32_t dk = sm32 + (j % KS) * TILE_BYTES + (4 * wave) * 1024;
    const uint32_t dv = sm32 + VB + (j % VS) * TILE_BYTES + (4 * wave) * 1024;
    const uint32_t ks = __builtin_amdgcn_readfirstlane(j * k_step);
    const uint32_t vs = __builtin_amdgcn_readfirstlane(j * v_step);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      mxk::dma16m(rk, __builtin_amdgcn_readfirstlane(dk + p * 1024), kvo[p], ks);
      mxk::dma16m(rv, __builtin_amdgcn_readfirstlane(dv + p * 1024), vvo[p], vs);
    }
  };
  issue(0);
  if (n > 1) issue(1);

  int koff[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) koff[s] = swz(r32, 2 * s + h);
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * h + (i16 >> 2);
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);
  const int tr_byte = 8 * (i16 & 1);
  int voff[4][2];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    voff[db][0] = VB + swz(tr_key, 4 * db + tr_ch) + tr_byte;
    voff[db][1] = VB + swz(tr_key + 8, 4 * db + tr_ch) + tr_byte;
  }

  const float cs = scale * 1.4426950408889634f;   // scores -> log2 domain
  W1Grp g0, g1;
  g0.m = g1.m = -INFINITY;
  g0.l = g1.l = 0.f;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) { g0.o[db][r] = 0.f; g1.o[db][r] = 0.f; }

#pragma unroll
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf0[s]), "v"(qf1[s]));
  if (n > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // tile 0 (tile 1 flies on)
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // MFMA blocks, operands read one group of 4 MFMAs ahead; SM(c) runs the
  // softmax chunk that follows MFMA c of the block (c = 0..15)
  auto qk_block = [&](W1Grp& g, const bf16x8_t (&qf)[8], int kslot, auto&& SM) __attribute__((always_inline)) {
    const char* kt = smem + kslot * TILE_BYTES;
#pragma unroll
    for (int r = 0; r < 16; ++r) { g.s0[r] = 0.f; g.s1[r] = 0.f; }
    bf16x8_t ka[2][4];
    auto rd = [&](int pr, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        ka[slot][2 * e] = lds_b128(kt + koff[2 * pr + e]);
        ka[slot][2 * e + 1] = lds_b128(kt + koff[2 * pr + e] + 32 * 256);
      }
    };
    rd(0, 0);
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) {
      if (pr < 3) rd(pr + 1, (pr + 1) & 1);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        g.s0 = mfma32(ka[pr & 1][2 * e], qf[2 * pr + e], g.s0);
        SM(4 * pr + 2 * e);
        __builtin_amdgcn_sched_barrier(0);
        g.s1 = mfma32(ka[pr & 1][2 * e + 1], qf[2 * pr + e], g.s1);
        SM(4 * pr + 2 * e + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto pv_block = [&](W1Grp& g, int vslot, auto&& SM) __attribute__((always_inline)) {
    const char* vt = smem + vslot * TILE_BYTES;   // VB is inside voff
    bf16x8_t va[2][4];
    auto rd = [&](int db, int slot) __attribute__((always_inline)) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        va[slot][ks] = cat8(lds_tr_b64(vt + voff[db][0] + ks * 4096),
                            lds_tr_b64(vt + voff[db][1] + ks * 4096));
    };
    rd(0, 0);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      if (db < 3) rd(db + 1, (db + 1) & 1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        g.o[db] = mfma32(va[db & 1][ks], __builtin_bit_cast(bf16x8_t, g.p[ks]), g.o[db]);
        SM(4 * db + ks);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto rescale = [&](W1Grp& g) __attribute__((always_inline)) {
    if (__builtin_amdgcn_ballot_w64(g.grow)) {
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) g.o[db][r] *= g.alpha;
    }
  };
  auto mask = [&](W1Grp& g, int kv0, int myq) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kv0 + crow(r, h);
      g.s0[r] = key > myq ? -INFINITY : g.s0[r];
      g.s1[r] = key + 32 > myq ? -INFINITY : g.s1[r];
    }
  };
  auto none = [&](int) __attribute__((always_inline)) {};
  auto sm0a = [&](int c) __attribute__((always_inline)) { w1_sm(g0, c, cs); };
  auto sm0b = [&](int c) __attribute__((always_inline)) { w1_sm(g0, 16 + c, cs); };
  auto sm1a = [&](int c) __attribute__((always_inline)) { w1_sm(g1, c, cs); };
  auto sm1b = [&](int c) __attribute__((always_inline)) { w1_sm(g1, 16 + c, cs); };

  const int jd = CAUSAL ? q0 / BKV : n;   // tiles j >= jd are diagonal (masked)
  // one tile: K_j and V_j in ring slot j % 3
  auto tile = [&](int sl, int j, auto firstc) __attribute__((always_inline)) {
    constexpr bool first = decltype(firstc)::value;
    const int sp = sl == 0 ? 2 : sl - 1;
    const bool diag = CAUSAL && j >= jd;
    // B1: QK(g0, K_j) beside the second half of softmax(g1, j - 1)
    if constexpr (first) qk_block(g0, qf0, sl, none);
    else qk_block(g0, qf0, sl, sm1b);
    if (diag) mask(g0, j * BKV, myq0);
    if constexpr (!first) {
      rescale(g1);
      // B2: PV(g1, V_{j-1}) beside the first half of softmax(g0, j)
      pv_block(g1, sp, sm0a);
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) sm0a(c);
    }
    // B3: QK(g1, K_j) beside the second half of softmax(g0, j)
    qk_block(g1, qf1, sl, sm0b);
    if (diag) mask(g1, j * BKV, myq1);
    rescale(g0);
    // B4: PV(g0, V_j) beside the first half of softmax(g1, j)
    pv_block(g0, sl, sm1a);
    // K_{j+1}, V_{j+1} landed (issued one tile ago); the barrier also
    // certifies that K_j's and V_{j-1}'s slots are no longer read
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (j + 2 < n) issue(j + 2);
  };
  // one loop body with a runtime ring slot (a v_add per LDS read stream and
  // tile; unrolled by the ring depth the register allocator spills)
  tile(0, 0, std::true_type{});
  for (int j = 1, sl = 1; j < n; ++j, sl = sl == 2 ? 0 : sl + 1) tile(sl, j, std::false_type{});
#pragma unroll
  for (int c = 0; c < 16; ++c) sm1b(c);
  rescale(g1);
  pv_block(g1, (n - 1) % 3, none);

  auto store = [&](W1Grp& g, int myq) __attribute__((always_inline)) {
    const float lt = half_sum(g.l);
    const float inv = 1.f / lt;
    uint16_t* orow = o + (static_cast<long>(b) * S + myq) * Hq * D + static_cast<long>(hq) * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int a0 = 2 * kk, a1 = 2 * kk + 1;
        const uint32_t x0 = mxk::pack2bf(g.o[db][4 * a0] * inv, g.o[db][4 * a0 + 1] * inv);
        const uint32_t x1 = mxk::pack2bf(g.o[db][4 * a0 + 2] * inv, g.o[db][4 * a0 + 3] * inv);
        const uint32_t y0 = mxk::pack2bf(g.o[db][4 * a1] * inv, g.o[db][4 * a1 + 1] * inv);
        const uint32_t y1 = mxk::pack2bf(g.o[db][4 * a1 + 2] * inv, g.o[db][4 * a1 + 3] * inv);
        const auto p0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto p1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        uint4 vv;
        vv.x = p0[0];
        vv.y = p1[0];
        vv.z = p0[1];
        vv.w = p1[1];
        *reinterpret_cast<uint4*>(orow + 32 * db + 16 * kk + 8 * h) = vv;
      }
    }
    if (h == 0) lse[(static_cast<long>(b) * Hq + hq) * S + myq] = g.m * scale + logf(lt);
  };
  store(g0, myq0);
  store(g1, myq1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// Launcher of the A/B records, called by mxk_attn_fwd_variant (attention.hip)
// in the experiments build: the status, or -1 when the variant does not tile
// the shape (the caller then runs variant 4).
int mxk_attn_fwd_exp_launch(int variant, const uint16_t* qp, const uint16_t* kp, const uint16_t* vp,
                            uint16_t* op, float* lse, int B, int S, int Hq, int Hkv, long q_tok,
                            long k_tok, long v_tok, float scale, int causal, hipStream_t stream) {
  if (variant == 9) {
    if (S % W1_BQ) return -1;
    {
      const int nwg9 = B * Hq * (S / W1_BQ);
      if (causal)
        hipLaunchKernelGGL(mxk_attn_fwd_w1_kernel<true>, dim3(nwg9), dim3(NT), 0, stream, qp, kp, vp,
                           op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
      else
        hipLaunchKernelGGL(mxk_attn_fwd_w1_kernel<false>, dim3(nwg9), dim3(NT), 0, stream, qp, kp,
                           vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
      return static_cast<int>(hipGetLastError());
    }
  }
  if (S % PP_BQ) return -1;
  if (variant >= 5) {
    const int nwg5 = B * Hq * (S / PP_BQ);
    if (variant == 7 || variant == 8) {   // timing ablations (wrong outputs)
      if (variant == 7)
        hipLaunchKernelGGL((mxk_attn_fwd_pp_kernel<true, false, 1>), dim3(nwg5), dim3(PP_NT), 0,
                           stream, qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
      else
        hipLaunchKernelGGL((mxk_attn_fwd_pp_kernel<true, false, 2>), dim3(nwg5), dim3(PP_NT), 0,
                           stream, qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    } else if (variant == 6) {
      if (causal)
        hipLaunchKernelGGL((mxk_attn_fwd_pp_kernel<true, true>), dim3(nwg5), dim3(PP_NT), 0, stream,
                           qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
      else
        hipLaunchKernelGGL((mxk_attn_fwd_pp_kernel<false, true>), dim3(nwg5), dim3(PP_NT), 0, stream,
                           qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    } else if (causal) {
      hipLaunchKernelGGL(mxk_attn_fwd_pp_kernel<true>, dim3(nwg5), dim3(PP_NT), 0, stream, qp, kp,
                         vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    } else {
      hipLaunchKernelGGL(mxk_attn_fwd_pp_kernel<false>, dim3(nwg5), dim3(PP_NT), 0, stream, qp, kp,
                         vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    }
    return static_cast<int>(hipGetLastError());
  }
  return -1;
}
