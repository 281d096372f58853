// Flash attention forward, one wave per SIMD with two 32-row groups per wave
// (gfx950; forward variant 10).
//
// The default forward (attention.hip variant 4: 4 waves x 32 rows, two
// workgroups per CU) keeps the matrix cores 45 % busy: each wave runs its
// QK^T MFMAs, then its softmax, then its PV MFMAs, and only the other wave
// of the SIMD can fill the gaps (profiles/r4_attention/pmc_fwd4_bwd5.txt).
// Here a workgroup is 4 waves = 256 query rows of one (batch, q-head), one
// wave per SIMD, and each wave owns two independent 32-row groups g0 / g1
// (/opt/skills/guides/cdna_hip_programming.md Appendix B, 'Fused attention
// prefill', the 4-wave one-wave-per-SIMD structure).  Per 64-key K / V tile
// j the wave runs four phases, each pairing one group's MFMAs with the other
// group's softmax on the VALU:
//
//   1  S^T(g0, j) = K Q(g0)^T          beside  softmax(g1, j-1) part B
//   2  O^T(g1) += V^T P^T(g1, j-1)     beside  softmax(g0, j)   part A
//   -- barrier: tile j+1 landed, slot of tile j-1 free: DMA of tile j+3 --
//   3  S^T(g1, j) = K Q(g1)^T          beside  softmax(g0, j)   part B
//   4  O^T(g0) += V^T P^T(g0, j)       beside  softmax(g1, j)   part A
//
// part A: causal mask, row max (in-lane + one permlane32_swap), lazy
// rescale decision (the row max only moves when it grew by more than 2^8),
// first half of the exps; part B: second half, row sums, the bf16 P^T
// operands and the (rare) O rescale.
//
// Registers: O^T of both groups (2 x 4 x 16) in AGPRs, pinned by inline-asm
// MFMAs; S^T of both groups (2 x 2 x 16) in VGPRs, also asm MFMAs (the VALU
// reads them), with explicit XDL-write -> VALU-read wait states; Q in VGPRs.
// Swapped QK^T as in attention.hip: the query is the MFMA lane, so the row
// statistics are per lane and P^T leaves the accumulator as the B operand of
// O^T += V^T P^T with V^T by ds_read_b64_tr_b16 from the row-major V image.
// K / V tiles by LDS-DMA into a 4-slot ring (two tiles of lead), one barrier
// per tile.  Causal: every wave walks every tile of its block (a wave past
// its diagonal sees only masked keys) - no divergent control flow.
//
// Layouts as attention.hip: q [B, S, Hq, 128] (token stride q_tok), k / v
// [B, S, Hkv, 128] (k_tok / v_tok), o [B, S, Hq, 128] contiguous, lse
// [B, Hq, S] fp32 (natural log).  S % 256 == 0.
#include "attention_common.h"

namespace {
constexpr int QB = 256;                        // query rows per workgroup
constexpr int KT = 64;                         // keys per tile
constexpr int FSLOT = 2 * TILE_BYTES;          // K | V image of one tile (32 KiB)
constexpr int FNSLOT = 4;
constexpr int FLDS = FNSLOT * FSLOT;           // 128 KiB

// MFMA with a VGPR accumulator (S^T): FENCE for the first of a chain whose
// C / operands a VALU instruction may just have written
template <bool FENCE = false>
__device__ __forceinline__ void fmfma_v(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  if constexpr (FENCE)
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// S^T chain with the B operand (Q^T fragment) held in AGPRs: the 64
// registers of both groups' Q live in the accumulator file for the whole
// kernel, beside O^T, leaving the arch VGPRs to S^T, P^T and the operands
template <bool FENCE = false>
__device__ __forceinline__ void fmfma_vq(f32x16_t& acc, const bf16x8_t& a, bf16x8_t& bq) {
  // "+a" on the Q fragment: the AGPR copy is the live value (an "a" input
  // alone lets the allocator keep Q in VGPRs and copy it in per MFMA)
  if constexpr (FENCE)
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %2, %1, %0" : "+v"(acc), "+a"(bq) : "v"(a));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %2, %1, %0" : "+v"(acc), "+a"(bq) : "v"(a));
}
// first MFMA of an S^T chain: C = 0 as an inline constant (no VALU
// zeroing, so no VALU-write -> MFMA wait either); early-clobber output, as
// an MFMA's D must not overlap its A / B
__device__ __forceinline__ void fmfma_vq0(f32x16_t& acc, const bf16x8_t& a, bf16x8_t& bq) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %2, %1, 0" : "=&v"(acc), "+a"(bq) : "v"(a));
}
// MFMA with the accumulator pinned to AGPRs (O^T)
__device__ __forceinline__ void fmfma_a(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// 8-pass XDL write -> VALU read: 12 wait states, results redefined behind them
__device__ __forceinline__ void ffence2(f32x16_t& x, f32x16_t& y) {
  asm volatile("s_nop 7\n\ts_nop 4" : "+v"(x), "+v"(y));
}
// VALU-written MFMA operands (P^T) and accumulators (a rescaled O^T) ->
// MFMA read: the wait states, with both named so nothing of either is
// written behind the nops
__device__ __forceinline__ void fops_ready(const bf16x8_t (&p)[4], f32x16_t (&acc)[4]) {
  asm volatile("s_nop 2"
               : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3])
               : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]));
}
// acc *= a for a 16-register accumulator tile held in AGPRs, inside one asm
// statement (read, multiply, write back through one VGPR): the allocator
// then never materialises a VGPR copy of the O tiles for the (rare) rescale
#define MXK_AS1(i) "v_accvgpr_read_b32 %16, %" #i "\n\tv_mul_f32 %16, %16, %17\n\tv_accvgpr_write_b32 %" #i ", %16\n\t"
__device__ __forceinline__ void agpr_scale16(f32x16_t& x, float a) {
  float t;
  asm volatile(MXK_AS1(0) MXK_AS1(1) MXK_AS1(2) MXK_AS1(3) MXK_AS1(4) MXK_AS1(5) MXK_AS1(6)
               MXK_AS1(7) MXK_AS1(8) MXK_AS1(9) MXK_AS1(10) MXK_AS1(11) MXK_AS1(12) MXK_AS1(13)
               MXK_AS1(14) MXK_AS1(15) "s_nop 1"
               : "+a"(x[0]), "+a"(x[1]), "+a"(x[2]), "+a"(x[3]), "+a"(x[4]), "+a"(x[5]),
                 "+a"(x[6]), "+a"(x[7]), "+a"(x[8]), "+a"(x[9]), "+a"(x[10]), "+a"(x[11]),
                 "+a"(x[12]), "+a"(x[13]), "+a"(x[14]), "+a"(x[15]), "=&v"(t)
               : "v"(a));
}
#undef MXK_AS1
__device__ __forceinline__ void vm_wait_n8() { __builtin_amdgcn_s_waitcnt(8 | (7 << 4) | (15 << 8)); }
}  // namespace

// STAMP (diagnostic build, mxk_attn_fwd256_stamps): each wave adds up the
// shader cycles of its phase 1, phase 2 and barrier segments and writes
// them with its total, its prologue and its time to the tail's end to
// stamps[wave id][6]; the
// production instance has none
template <bool CAUSAL, bool STAMP = false>
__global__ void __launch_bounds__(256, 1)
mxk_attn_fwd256_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                       const uint16_t* __restrict__ v, uint16_t* __restrict__ o,
                       float* __restrict__ lse, int S, int Hq, int Hkv, long q_tok, long k_tok,
                       long v_tok, float scale, unsigned long long* __restrict__ stamps = nullptr) {
  __shared__ __attribute__((aligned(16))) char smem[FLDS];
  unsigned long long st_p1 = 0, st_p2 = 0, st_bar = 0, st_0 = 0, st_pro = 0, st_tail = 0;
  if constexpr (STAMP) st_0 = __builtin_readcyclecounter();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nqb = S / QB;
  int bh, qb;
  map_block_xcd(blockIdx.x, gridDim.x, nqb, Hq / Hkv, CAUSAL, &bh, &qb);
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int q0 = qb * QB;
  const int qw0 = q0 + wave * 64;              // g0: qw0 + r32, g1: qw0 + 32 + r32

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  const int J = CAUSAL ? (q0 + QB) / KT : S / KT;   // tiles of this block

  // ---- DMA: wave w moves pieces 4 w .. 4 w + 3 of K and of V (1 KiB, 4 rows
  // each; lane i at row 4 g + (i >> 4), chunk (i & 15) ^ swizzle(row))
  const mxk::u32x4 rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
  const mxk::u32x4 rv = mxk::make_rsrc(vb_ptr, static_cast<unsigned>(S * v_tok * 2));
  // per piece p: row 4 (4 wave + p) + prow, chunk (pslot ^ (prow << 2)) ^ p,
  // formed at issue time (2 VALU per piece) rather than held in 8 VGPRs
  // through the loop (the arch VGPRs are S^T's double buffer's)
  const int prow = lane >> 4, cbase = (lane & 15) ^ (prow << 2);
  const uint32_t krow0 = static_cast<uint32_t>((16 * wave + prow) * k_tok * 2);
  const uint32_t vrow0 = static_cast<uint32_t>((16 * wave + prow) * v_tok * 2);
  const uint32_t k_step = static_cast<uint32_t>(KT * k_tok * 2);
  const uint32_t v_step = static_cast<uint32_t>(KT * v_tok * 2);
  const uint32_t sm32 = mxk::lds_addr32(smem);
  // piece p (0..3) of tile j: one K and one V LDS-DMA instruction
  auto issue_piece = [&](int j, int p) {
    uint32_t d0 = sm32 + (j % FNSLOT) * FSLOT + (4 * wave + p) * 1024;
    // opaque base: the piece addresses are one s_add each here, not 32
    // loop-invariant SGPRs (4 slots x 8 pieces) hoisted and spilled
    asm volatile("" : "+s"(d0));
    const uint32_t ch16 = static_cast<uint32_t>((cbase ^ p) << 4);
    mxk::dma16m(rk, d0, krow0 + static_cast<uint32_t>(p * 4 * k_tok * 2) + ch16, j * k_step);
    mxk::dma16m(rv, d0 + TILE_BYTES, vrow0 + static_cast<uint32_t>(p * 4 * v_tok * 2) + ch16,
                j * v_step);
  };
  auto issue = [&](int j) {
#pragma unroll
    for (int p = 0; p < 4; ++p) issue_piece(j, p);
  };
  // Prologue: tile 0's DMA, Q (asm loads: a compiler-visible load's first
  // use would carry a vmcnt(0) that also waits for tiles 1 and 2), then
  // tiles 1 and 2; the loop starts once Q and tile 0 are in (vmcnt 16: the
  // 16 pieces of tiles 1 and 2 may still fly; barrier B_0 waits for tile 1)
  issue(0);
  // Q^T fragments (B operand of S^T = K Q^T): lane holds Q[row][16 s + 8 h .. + 7]
  bf16x8_t qf[2][8];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      asm volatile("global_load_dwordx4 %0, %1, off"
                   : "=v"(qf[g][s])
                   : "v"(qb_ptr + static_cast<long>(qw0 + 32 * g + r32) * q_tok + 16 * s + 8 * h)
                   : "memory");
  // J >= 4 always (S % 256 == 0): no branch here, whose merge would copy
  // the Q registers before their loads land
  issue(1);
  issue(2);
  asm volatile("s_waitcnt vmcnt(16)"
               : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[0][2]), "+v"(qf[0][3]), "+v"(qf[0][4]),
                 "+v"(qf[0][5]), "+v"(qf[0][6]), "+v"(qf[0][7]), "+v"(qf[1][0]), "+v"(qf[1][1]),
                 "+v"(qf[1][2]), "+v"(qf[1][3]), "+v"(qf[1][4]), "+v"(qf[1][5]), "+v"(qf[1][6]),
                 "+v"(qf[1][7]));
  __syncthreads();

  // LDS read offsets (loop invariants + slot immediates): K rows r32 (+32
  // for key half 1 = +8 KiB), chunk 2 s + h; V^T transposed reads at keys
  // tr_key (+8) of k-step ks (+4 KiB each), chunk 4 db + tr_ch
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
    voff[db][0] = TILE_BYTES + swz(tr_key, 4 * db + tr_ch) + tr_byte;
    voff[db][1] = TILE_BYTES + swz(tr_key + 8, 4 * db + tr_ch) + tr_byte;
  }

  const float c = scale * 1.4426950408889634f;   // scores -> log2 domain
  f32x16_t oacc[2][4];                           // O^T: rows d = 32 db + crow, lane = query
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[g][db][r] = 0.f;
  // S^T of both groups, double-buffered by tile parity: buffer j & 1 takes
  // S(j) in phase 1 of tile j while the other finishes P(j-1)
  f32x16_t sacc[2][2][2];                        // [buf][g][kh]: rows key = 32 kh + crow, lane = query
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f}, alpha[2] = {1.f, 1.f};
  // P^T operands [buf][g][ks] (k-step ks = keys 16 ks ..), double-buffered
  // by tile parity: tile j's key half 0 is packed in phase 2 of tile j while
  // phase 2 reads tile j-1's
  bf16x8_t pf[2][2][4];

  // ---- the two phase bodies, each 32 MFMAs.  Each MFMA is followed by
  // beside(u) and a sched region boundary: one unit of the softmax (about
  // one exp and three other VALU ops) then issues in that MFMA's shadow.
  // (Coarser regions - a unit beside four MFMAs - let the scheduler emit
  // the VALU block first and the MFMAs back to back behind it: measured
  // 2281 cycles for phase 1's 1024 MFMA cycles.)  Both groups share every
  // K / V fragment read: each feeds one MFMA per group.  Operands are read
  // one k-step ahead.
  //
  // phase 1: S^T(g, j) = K Q(g)^T for both groups
  auto qk2 = [&](auto buf_c, const char* kt, auto&& beside) {
    constexpr int B = decltype(buf_c)::value;
    bf16x8_t a[2] = {lds_b128(kt + koff[0]), lds_b128(kt + koff[0] + 32 * 256)};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      bf16x8_t n[2] = {a[0], a[1]};
      if (s < 7) {
        n[0] = lds_b128(kt + koff[s + 1]);
        n[1] = lds_b128(kt + koff[s + 1] + 32 * 256);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = u >> 1, kh = u & 1;
        if (s == 0)   // C = 0: no VALU zeroing of S^T
          fmfma_vq0(sacc[B][g][kh], a[kh], qf[g][s]);
        else
          fmfma_vq(sacc[B][g][kh], a[kh], qf[g][s]);
        beside(4 * s + u);
        __builtin_amdgcn_sched_barrier(0);
      }
      a[0] = n[0];
      a[1] = n[1];
    }
    ffence2(sacc[B][0][0], sacc[B][0][1]);
    ffence2(sacc[B][1][0], sacc[B][1][1]);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto vread = [&](const char* vt, int i) {
    const int db = i >> 2, ks = i & 3;
    return cat8(lds_tr_b64(vt + voff[db][0] + ks * 4096), lds_tr_b64(vt + voff[db][1] + ks * 4096));
  };
  // phase 2: O^T(g) += V^T P^T(g, j-1) for both groups
  auto pv2 = [&](auto buf_c, const char* vt, auto&& beside) {
    constexpr int B = decltype(buf_c)::value;
    fops_ready(pf[B][0], oacc[0]);
    fops_ready(pf[B][1], oacc[1]);
    bf16x8_t a = vread(vt, 0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const bf16x8_t n = i < 15 ? vread(vt, i + 1) : a;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        fmfma_a(oacc[g][i >> 2], a, pf[B][g][i & 3]);
        beside(2 * i + g);
        __builtin_amdgcn_sched_barrier(0);
      }
      a = n;
    }
  };
  // softmax start of tile j, unit u of 32 (beside phase 2's MFMAs):
  // 0-7 causal mask and row max over 8 scores each ((g, kh) = (u >> 2,
  // (u >> 1) & 1), registers 8 (u & 1) ..); 8 / 9 the max across the lane
  // halves, the lazy rescale decision and alpha of g0 / g1; 10-31 the exps
  // of key half 0 (2 per unit in 10-19, then 1) with the row sums, each
  // group's bf16 P^T operands of k-steps 0 / 1 once their 8 registers are done
  float mx[2] = {-INFINITY, -INFINITY}, nmc[2] = {0.f, 0.f};
  float ls[2] = {0.f, 0.f};
  auto start = [&](auto buf_c, int j, int u, auto mask_c) {
    constexpr int B = decltype(buf_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    if (u < 8) {
      const int g = u >> 2, kh = (u >> 1) & 1, r0 = 8 * (u & 1);
      // causal: key 32 kh + crow(r, h) of the tile is masked past the lane's
      // query, i.e. when (r & 3) + 8 (r >> 2) > lim - one compare against a
      // constant per score (VCC only: no SGPR mask pairs to spill)
      if (MASK) {
        const int lim = qw0 + 32 * g + r32 - j * KT - 32 * kh - 4 * h;
#pragma unroll
        for (int r = r0; r < r0 + 8; ++r)
          // a scalar select written back: an `if (...) v[r] = x` on the
          // 16-wide vector compiles to a select of the whole vector
          sacc[B][g][kh][r] = (r & 3) + 8 * (r >> 2) > lim ? -INFINITY : sacc[B][g][kh][r];
      }
      const bool first = (u & 3) == 0;
      float x = first ? sacc[B][g][kh][r0] : mx[g];
#pragma unroll
      for (int r = first ? r0 + 1 : r0; r < r0 + 8; ++r) x = fmaxf(x, sacc[B][g][kh][r]);
      mx[g] = x;
    } else if (u < 10) {
      const int g = u - 8;
      const float mm = half_max(mx[g]);
      float m_new = fmaxf(m[g], mm);
      // lazy rescale: keep the stale max unless the new one exceeds it by
      // more than 2^8 (P stays <= 256, exact in bf16's exponent range)
      const bool grow = (m_new - m[g]) * c > 8.f;
      if (!grow) m_new = m[g];
      alpha[g] = grow ? fexp2((m[g] - m_new) * c) : 1.f;
      m[g] = m_new;
      nmc[g] = -m_new * c;
    } else {
      const int e0 = u < 20 ? 2 * (u - 10) : u, e1 = u < 20 ? e0 + 2 : u + 1;
#pragma unroll
      for (int e = e0; e < e1; ++e) {
        const int g = e >> 4, r = e & 15;
        sacc[B][g][0][r] = fexp2(fmaf(sacc[B][g][0][r], c, nmc[g]));
        ls[g] = (r == 0 ? 0.f : ls[g]) + sacc[B][g][0][r];
        if ((r & 7) == 7) pf[B][g][r >> 3] = pack8(sacc[B][g][0], r & 8);
      }
    }
  };
  // softmax finish of tile j-1, unit u of 32 (beside phase 1's MFMAs): the
  // exp of key half 1's register u >> 1 of group u & 1 and its row sum;
  // the bf16 P^T operands of k-steps 2 / 3 once their 8 registers are done;
  // after the last, l and the rare O rescale of both groups
  auto finish = [&](auto buf_c, int u) {
    constexpr int B = decltype(buf_c)::value;
    const int g = u & 1, r = u >> 1;
    sacc[B][g][1][r] = fexp2(fmaf(sacc[B][g][1][r], c, nmc[g]));
    ls[g] += sacc[B][g][1][r];
    if (u == 15) {
      // pack behind the sums (packed first, P's fp32 stays live for them
      // and spills)
      asm volatile("" : "+v"(sacc[B][0][1]), "+v"(sacc[B][1][1]) : "v"(ls[0]), "v"(ls[1]));
      pf[B][0][2] = pack8(sacc[B][0][1], 0);
      pf[B][1][2] = pack8(sacc[B][1][1], 0);
    }
    if (r == 15) {
      pf[B][g][3] = pack8(sacc[B][g][1], 8);
      // packed here, ahead of the rescale branch (sunk below it, the fp32
      // P was copied whole into the registers of the branch merge)
      asm volatile("" : "+v"(pf[B][g][3]));
    }
    if (u == 31) {
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        l[gg] = l[gg] * alpha[gg] + ls[gg];
        if (__builtin_amdgcn_ballot_w64(alpha[gg] != 1.f)) {   // rare after the first tiles
#pragma unroll
          for (int db = 0; db < 4; ++db) agpr_scale16(oacc[gg][db], alpha[gg]);
        }
      }
    }
  };
  // barrier B_j (after phase 2 of tile j): tile j+1 landed (own pieces;
  // tile j+2's 8 may be in flight), every wave is past phase 2 of tile j
  // (the last reader of tile j-1's slot, its V), then tile j+3's DMA.
  // (Spreading the 8 DMA instructions over phase 1 instead, one per 4
  // MFMAs, measured +1030 cycles in phase 1 against -430 here.)
  auto barrier_j = [&](int j) {
    if (j + 2 < J) vm_wait_n8();
    else vm_wait0();
    __builtin_amdgcn_s_barrier();
    if (j + 3 < J) issue(j + 3);
  };

  // Tile 0's phase 1 finishes a tile -1 and its phase 2 adds it to O: made
  // a no-op by P(-1) = 0 (key half 0's operands packed as 0; half 1 at -inf
  // with nmc = 0: exp 0, ls stays 0), so l stays 0 and alpha 1, against a
  // zeroed V image in slot 3 (no NaN from uninitialised LDS)
#pragma unroll
  for (int g = 0; g < 2; ++g) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[1][g][1][r] = -INFINITY;
    pf[1][g][0] = bf16x8_t{};
    pf[1][g][1] = bf16x8_t{};
  }
  {
    uint4* z = reinterpret_cast<uint4*>(smem + 3 * FSLOT + TILE_BYTES);
#pragma unroll
    for (int i = 0; i < 4; ++i) z[tid + 256 * i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
  auto tile = [&](int j, auto slot_c, auto mask_c) {
    constexpr int SL = decltype(slot_c)::value;        // == j % 4
    constexpr int PSL = (SL + FNSLOT - 1) % FNSLOT;    // tile j-1's slot
    const char* tj = smem + SL * FSLOT;
    const char* tp = smem + PSL * FSLOT;
    using cur = std::integral_constant<int, SL & 1>;
    using prv = std::integral_constant<int, (SL & 1) ^ 1>;
    // phase 1: S^T(j) beside the finish of softmax(j-1)
    unsigned long long ta = 0, tb = 0;
    if constexpr (STAMP) ta = __builtin_readcyclecounter();
    qk2(cur{}, tj, [&](int u) { finish(prv{}, u); });
    if constexpr (STAMP) {
      tb = __builtin_readcyclecounter();
      st_p1 += tb - ta;
    }
    // phase 2: O^T += V^T P^T(j-1) beside the start of softmax(j)
    pv2(prv{}, tp, [&](int cc) { start(cur{}, j, cc, mask_c); });
    if constexpr (STAMP) {
      ta = __builtin_readcyclecounter();
      st_p2 += ta - tb;
    }
    barrier_j(j);
    if constexpr (STAMP) st_bar += __builtin_readcyclecounter() - ta;
  };
  // J is a multiple of 4 (S % 256 == 0): one body of four tiles, the ring's
  // slots as compile-time immediates.  Causal: every diagonal tile of the
  // block's four waves is one of its last four (wave w's first is J - 4 + w),
  // so only the last body carries the mask
  auto body = [&](int j, auto mask_c) {
    tile(j, std::integral_constant<int, 0>{}, mask_c);
    tile(j + 1, std::integral_constant<int, 1>{}, mask_c);
    tile(j + 2, std::integral_constant<int, 2>{}, mask_c);
    tile(j + 3, std::integral_constant<int, 3>{}, mask_c);
  };
  // 8-pass XDL -> accumulator read: the register allocator may copy O^T
  // (just written by phase 2's MFMAs) on the loop's exit edge
#define MXK_O_FENCE                                                                    \
  asm volatile("s_nop 7\n\ts_nop 4"                                                    \
               : "+a"(oacc[0][0]), "+a"(oacc[0][1]), "+a"(oacc[0][2]), "+a"(oacc[0][3]), \
                 "+a"(oacc[1][0]), "+a"(oacc[1][1]), "+a"(oacc[1][2]), "+a"(oacc[1][3]))
  const int Jm = CAUSAL ? J - 4 : J;
  if constexpr (STAMP) st_pro = __builtin_readcyclecounter() - st_0;
  for (int j = 0; j < Jm; j += 4) {
    body(j, std::false_type{});
    MXK_O_FENCE;
  }
  if constexpr (CAUSAL) {
    body(Jm, std::true_type{});
    MXK_O_FENCE;
  }
#undef MXK_O_FENCE
  // tail: finish the last tile (J-1, slot 3, buffer 1) and add it
#pragma unroll
  for (int u = 0; u < 32; ++u) finish(std::integral_constant<int, 1>{}, u);
  __builtin_amdgcn_sched_barrier(0);
  pv2(std::integral_constant<int, 1>{}, smem + 3 * FSLOT, [](int) {});
  if constexpr (STAMP) st_tail = __builtin_readcyclecounter() - st_0;
  // O accumulators final: drain the asm MFMAs before reading them
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int db = 0; db < 4; ++db) asm volatile("" : "+a"(oacc[g][db]));

  // ---- epilogue: O = O^T / l, staged through LDS so every global store
  // instruction writes 4 whole 256-B rows (8 full lines) - stored straight
  // from the lanes, each instruction touched 32 rows with 32 B each; lse.
  // The wave's 64 x 256 B image goes to slots 0-1 (its 16 KiB at 16 KiB x
  // wave), free since the last barrier (the tail reads slot 3 only); the
  // 16-B chunk index is XORed with the row's low 4 bits (conflict-free).
  char* img = smem + wave * 16384;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int row = 32 * g + r32;
    const float lt = half_sum(l[g]);
    const float inv = 1.f / lt;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int g0 = 2 * kk, g1 = 2 * kk + 1;
        const uint32_t x0 = mxk::pack2bf(oacc[g][db][4 * g0] * inv, oacc[g][db][4 * g0 + 1] * inv);
        const uint32_t x1 = mxk::pack2bf(oacc[g][db][4 * g0 + 2] * inv, oacc[g][db][4 * g0 + 3] * inv);
        const uint32_t y0 = mxk::pack2bf(oacc[g][db][4 * g1] * inv, oacc[g][db][4 * g1 + 1] * inv);
        const uint32_t y1 = mxk::pack2bf(oacc[g][db][4 * g1 + 2] * inv, oacc[g][db][4 * g1 + 3] * inv);
        const auto p0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto p1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        uint4 ov;
        ov.x = p0[0];
        ov.y = p1[0];
        ov.z = p0[1];
        ov.w = p1[1];
        const int ch = 4 * db + 2 * kk + h;   // 16-B chunk: d = 8 ch ..
        *reinterpret_cast<uint4*>(img + row * 256 + ((ch ^ (row & 15)) << 4)) = ov;
      }
    }
    if (h == 0) lse[(static_cast<long>(b) * Hq + hq) * S + qw0 + row] = m[g] * scale + logf(lt);
  }
  {
    const int ch = lane & 15;
    uint16_t* obase = o + (static_cast<long>(b) * S + qw0) * Hq * D + static_cast<long>(hq) * D + 8 * ch;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int row = 4 * t + (lane >> 4);
      const uint4 ov = *reinterpret_cast<const uint4*>(img + row * 256 + ((ch ^ (row & 15)) << 4));
      *reinterpret_cast<uint4*>(obase + static_cast<long>(row) * Hq * D) = ov;
    }
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* w = stamps + (static_cast<long>(blockIdx.x) * 4 + wave) * 6;
      w[0] = __builtin_readcyclecounter() - st_0;
      w[1] = st_p1;
      w[2] = st_p2;
      w[3] = st_bar;
      w[4] = st_pro;
      w[5] = st_tail;
    }
  }
}

// Forward variant 10.  Returns hipErrorInvalidValue for layouts it does not
// take (S % 256, 32-bit buffer offsets); attention.hip then falls back.
MXK_API int mxk_attn_fwd256(const void* q, const void* k, const void* v, void* o, float* lse,
                            int B, int S, int Hq, int Hkv, long q_tok, long k_tok, long v_tok,
                            float scale, int causal, hipStream_t stream) {
  if (B < 1 || S < QB || S % QB || Hkv < 1 || Hq % Hkv || q_tok % 8 || k_tok % 8 || v_tok % 8 ||
      static_cast<long>(S) * k_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * v_tok * 2 >= (1L << 32) ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * Hq * (S / QB);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  auto* O = static_cast<uint16_t*>(o);
  if (causal)
    hipLaunchKernelGGL(mxk_attn_fwd256_kernel<true>, dim3(nwg), dim3(256), 0, stream, Q, K, V, O,
                       lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else
    hipLaunchKernelGGL(mxk_attn_fwd256_kernel<false>, dim3(nwg), dim3(256), 0, stream, Q, K, V, O,
                       lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  MXK_RETURN_LAUNCH_STATUS();
}

// Diagnostic: forward variant 10 with per-wave segment cycle counts
// (stamps: [B * Hq * S / 256 workgroups][4 waves][total, phase 1, phase 2,
// barrier, prologue, start -> end of the tail]); same arguments as
// mxk_attn_fwd256 otherwise.
MXK_API int mxk_attn_fwd256_stamps(const void* q, const void* k, const void* v, void* o,
                                   float* lse, int B, int S, int Hq, int Hkv, long q_tok,
                                   long k_tok, long v_tok, float scale, int causal,
                                   unsigned long long* stamps, hipStream_t stream) {
  if (B < 1 || S < QB || S % QB || Hkv < 1 || Hq % Hkv || q_tok % 8 || k_tok % 8 || v_tok % 8 ||
      !stamps)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * Hq * (S / QB);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  auto* O = static_cast<uint16_t*>(o);
  if (causal)
    hipLaunchKernelGGL((mxk_attn_fwd256_kernel<true, true>), dim3(nwg), dim3(256), 0, stream, Q, K,
                       V, O, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale, stamps);
  else
    hipLaunchKernelGGL((mxk_attn_fwd256_kernel<false, true>), dim3(nwg), dim3(256), 0, stream, Q,
                       K, V, O, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale, stamps);
  MXK_RETURN_LAUNCH_STATUS();
}
