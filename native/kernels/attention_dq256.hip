// Flash attention backward, dQ with one wave per SIMD (gfx950; backward
// variant 9).
//
// The dQ kernel of variants 5 / 6 (attention.hip, mxk_attn_bwd_dq_kernel:
// 4 waves x 32 query rows, two workgroups per CU) takes 459.5 us of the
// 1.018 ms Llama-3-8B layer backward at 44.8 % MFMA busy and 81.9 % L2 hit
// (profiles/r5_attention/pmc_default_fwd4_bwd6_and_v8.txt): every K / V
// fragment it reads from LDS feeds ONE MFMA, and every 128 query rows
// re-stream the head's keys.  Here (the one-wave-per-SIMD structure of the
// 256-key dK / dV kernel, attention_bwd256.hip, applied to the query side):
//
//   * one workgroup = 4 waves = the 4 query heads of one GQA quad x the same
//     64 query rows: the waves share every K / V tile (one LDS-DMA stream per
//     quad instead of one per head) and, being on the same rows, the same
//     causal key range - no wave idles past its diagonal;
//   * a wave owns its 64 rows as two 32-row tiles g0 / g1: every K / V / K^T
//     fragment read from LDS feeds one MFMA per tile (two per read);
//   * Q and dO of the 64 rows are resident for the whole sweep as MFMA B
//     operands in the accumulator file (2 x 64 AGPRs), beside dQ^T (128
//     AGPRs), so the arch VGPRs hold only S^T / dP^T and operands;
//   * key on the register, query on the lane (S^T = K Q^T, dP^T = V dO^T):
//     the row constants -lse and -delta are per lane, and dS^T converted to
//     bf16 IS the B operand of dQ^T += K^T dS^T (K^T by ds_read_b64_tr_b16
//     from the row-major K image), no LDS round trip;
//   * per 32-key step j two phases, each with VALU work beside its MFMAs:
//       A(j)    S^T, dP^T of step j (32 MFMAs)   beside softmax(j-1) of g1
//       B(j-1)  dQ^T += K^T dS^T(j-1) (16)       beside softmax(j)   of g0
//     (softmax: P = exp2(c S - lse log2 e), the causal mask on the two
//     diagonal steps, dS = P (dP - delta), bf16 pairs);
//   * K / V tiles of 64 keys by LDS-DMA into a 4-slot ring (two tiles of
//     lead), one barrier per tile (two steps).
//
// The delta pass is folded in (delta = dO . O from the row's own dO
// fragments and O), and the kernel writes the {-lse/scale, -delta} row pairs
// that the 256-key dK / dV kernel streams, so variant 9 is this kernel then
// mxk_attn_bwd_dkdv256 - deterministic, no atomics.
//
// Layouts as attention.hip: q [B, S, Hq, 128] (token stride q_tok), k / v
// [B, S, Hkv, 128] (k_tok / v_tok), o / dout / dq [B, S, Hq, 128] contiguous,
// lse [B, Hq, S] fp32 (natural log), rowc [B, Hq, S] x float2.  Hq / Hkv a
// multiple of 4, S % 64 == 0, K / V panels within a 32-bit buffer range.
#include "attention_common.h"

namespace {
constexpr int QW = 64;                     // query rows per wave (and workgroup)
constexpr int KT = 64;                     // keys per DMA tile (two steps of 32)
constexpr int QSLOT = 2 * TILE_BYTES;      // K | V image of one tile (32 KiB)
constexpr int QNSLOT = 4;
constexpr int QLDS = QNSLOT * QSLOT;       // 128 KiB

// S^T / dP^T chains: accumulator in VGPRs (the VALU reads it), B operand (a
// Q / dO fragment) pinned in AGPRs ("+a": the AGPR copy is the live value).
// First of a chain: C = 0 as an inline constant (no VALU zeroing, so no
// VALU-write -> MFMA-read wait); early-clobber, D must not overlap A / B.
__device__ __forceinline__ void mq0(f32x16_t& acc, const bf16x8_t& a, bf16x8_t& bq) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %2, %1, 0" : "=&v"(acc), "+a"(bq) : "v"(a));
}
__device__ __forceinline__ void mq(f32x16_t& acc, const bf16x8_t& a, bf16x8_t& bq) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %2, %1, %0" : "+v"(acc), "+a"(bq) : "v"(a));
}
// the last k-step of phase A: four MFMAs and the XDL-write -> VALU-read wait
// states (8-pass 32x32x16: 12) in ONE statement, so the allocator cannot
// copy a result between the MFMA and the nops
__device__ __forceinline__ void mq4_fenced(f32x16_t& s0, f32x16_t& s1, f32x16_t& p0, f32x16_t& p1,
                                           bf16x8_t& q0, bf16x8_t& q1, bf16x8_t& d0, bf16x8_t& d1,
                                           const bf16x8_t& ka, const bf16x8_t& va) {
  asm volatile(
      "v_mfma_f32_32x32x16_bf16 %0, %8, %4, %0\n\t"
      "v_mfma_f32_32x32x16_bf16 %1, %8, %5, %1\n\t"
      "v_mfma_f32_32x32x16_bf16 %2, %9, %6, %2\n\t"
      "v_mfma_f32_32x32x16_bf16 %3, %9, %7, %3\n\t"
      "s_nop 7\n\ts_nop 4"
      : "+v"(s0), "+v"(s1), "+v"(p0), "+v"(p1), "+a"(q0), "+a"(q1), "+a"(d0), "+a"(d1)
      : "v"(ka), "v"(va));
}
// dQ^T accumulation, accumulator pinned to AGPRs
__device__ __forceinline__ void ma(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// VALU-written dS^T operands -> MFMA read: the wait states, with the operands
// named so none of them is written behind the nops.  The dQ^T tiles are named
// too ("+a"): the allocator shuffles them between the loop and the tail's
// MFMA instance with v_accvgpr_write / _mov, which an inline-asm MFMA right
// behind would read stale (register 0 of a tile, seen); a copy it needs now
// sits in front of these nops
__device__ __forceinline__ void ds_ready(const bf16x8_t (&x)[2][2], f32x16_t (&acc)[2][4]) {
  asm volatile("s_nop 2"
               : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]),
                 "+a"(acc[1][0]), "+a"(acc[1][1]), "+a"(acc[1][2]), "+a"(acc[1][3])
               : "v"(x[0][0]), "v"(x[0][1]), "v"(x[1][0]), "v"(x[1][1]));
}
// the same for the Q / dO fragments (MFMA B operands in AGPRs) in front of a
// phase A: any allocator copy of them lands before the nops
__device__ __forceinline__ void qd_ready(bf16x8_t (&qf)[2][8], bf16x8_t (&df)[2][8]) {
  asm volatile(""
               : "+a"(qf[0][0]), "+a"(qf[0][1]), "+a"(qf[0][2]), "+a"(qf[0][3]), "+a"(qf[0][4]),
                 "+a"(qf[0][5]), "+a"(qf[0][6]), "+a"(qf[0][7]), "+a"(qf[1][0]), "+a"(qf[1][1]),
                 "+a"(qf[1][2]), "+a"(qf[1][3]), "+a"(qf[1][4]), "+a"(qf[1][5]), "+a"(qf[1][6]),
                 "+a"(qf[1][7]));
  asm volatile("s_nop 1"
               : "+a"(df[0][0]), "+a"(df[0][1]), "+a"(df[0][2]), "+a"(df[0][3]), "+a"(df[0][4]),
                 "+a"(df[0][5]), "+a"(df[0][6]), "+a"(df[0][7]), "+a"(df[1][0]), "+a"(df[1][1]),
                 "+a"(df[1][2]), "+a"(df[1][3]), "+a"(df[1][4]), "+a"(df[1][5]), "+a"(df[1][6]),
                 "+a"(df[1][7]));
}
template <int N>
__device__ __forceinline__ void vmw() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ uint32_t pk2(float lo, float hi) { return mxk::pack2bf(lo, hi); }
}  // namespace

// DBG (diagnostic instances, mxk_attn_bwd_dq256_dbg): the dS^T operand
// replaced by 1 (1), by S (2) or by dP (3) wherever P > 0, so a wrong dQ
// can be pinned on phase B, on the S or on the dP product.  STAMP
// (mxk_attn_bwd_dq256_stamps): each wave adds up the shader cycles of its
// prologue, phases A, phases B, barrier segments and tail, and writes them
// with its total to stamps[wave id][6]
//
// (A persistent form - one workgroup per CU looping over heavy / light
// paired row blocks, with an L2 prefetch of the next block's Q / dO / O -
// measured within 0.2 % of this launch, 1.0275 vs 1.0293 ms per layer
// backward, and spilled once the prologue staged through LDS; not kept,
// profiles/r6_dq256/.)
// ROPE: dQ leaves through the rotary-embedding backward (each lane reads
// its 16-B chunk and the pair partner 64 dims away from the row image and
// writes its own chunk rotated back at the row's position), rounded to bf16
// before and after exactly as the stand-alone pass (fused_ops.hip) does;
// dq_tok (> 0): dQ's token stride (a slice of a fused d(QKV) buffer).
template <bool CAUSAL, int DBG = 0, bool STAMP = false, bool ROPE = false>
__global__ void __launch_bounds__(256, 1)
mxk_attn_bwd_dq256_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                          const uint16_t* __restrict__ v, const uint16_t* __restrict__ o,
                          const uint16_t* __restrict__ dout, const float* __restrict__ lse,
                          uint16_t* __restrict__ dq, float* __restrict__ rowc, int S, int Hq,
                          int Hkv, long q_tok, long k_tok, long v_tok, float scale,
                          unsigned long long* __restrict__ stamps = nullptr, int succ = 0,
                          long dq_tok = 0, const float* __restrict__ rcos = nullptr,
                          const float* __restrict__ rsin = nullptr) {
  __shared__ __attribute__((aligned(16))) char smem[QLDS + 4 * 256];   // ring | prefetch sinks
  unsigned long long st_0 = 0, st_c = 0, st_seg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (STAMP) st_0 = st_c = __builtin_readcyclecounter();
  // segment e ends here: 0 prologue (offsets, zeroing), 1 phase A, 2 phase
  // B, 3 barrier, 4 tail + dQ store, 5 prologue load issue, 6 wait for dO /
  // O, 7 delta + rowc + wait for Q / tile 0 + barrier
  auto stamp = [&](int e) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_readcyclecounter();
      st_seg[e] += t - st_c;
      st_c = t;
    }
  };
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  // workgroup -> (batch, quad of query heads, 64-row block): the quads of one
  // KV head and all their blocks are consecutive logical ids of one XCD,
  // heaviest block first (map_block_xcd), so a KV head's K / V stays in its L2
  const int grp = Hq / Hkv;
  const int nq4 = Hq / 4;
  const int nqb = S / QW;
  const long tokd = static_cast<long>(Hq) * D;
  const uint32_t sm32 = mxk::lds_addr32(smem);
  const int prow = lane >> 4, cbase = (lane & 15) ^ (prow << 2);
  // one (quad, row block) item; (nbq4, nqb_): the item of the workgroup
  // `succ` ids later (-1: none), which this one prefetches
  auto run_item = [&](int bq4, int qb, int nbq4, int nqb_) {
  const int b = bq4 / nq4;
  const int hq = (bq4 - b * nq4) * 4 + wave;
  const int hkv = hq / grp;                    // the same for the 4 waves
  const int q0 = qb * QW;

  const uint16_t* qh = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* doh = dout + static_cast<long>(b) * S * tokd + static_cast<long>(hq) * D;
  const uint16_t* oh = o + static_cast<long>(b) * S * tokd + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;
  const long lrow0 = (static_cast<long>(b) * Hq + hq) * S + q0;

  const int T = CAUSAL ? qb + 1 : S / KT;      // 64-key tiles (keys 0 .. q0 + 63 when causal)

  // ---- DMA: wave w moves pieces 4 w .. 4 w + 3 of K and of V (1 KiB, 4 rows
  // each; lane i at row 4 g + (i >> 4), chunk (i & 15) ^ swizzle(row))
  const mxk::u32x4 rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
  const mxk::u32x4 rv = mxk::make_rsrc(vb_ptr, static_cast<unsigned>(S * v_tok * 2));
  const uint32_t krow0 = static_cast<uint32_t>((16 * wave + prow) * k_tok * 2);
  const uint32_t vrow0 = static_cast<uint32_t>((16 * wave + prow) * v_tok * 2);
  const uint32_t k_step = static_cast<uint32_t>(KT * k_tok * 2);
  const uint32_t v_step = static_cast<uint32_t>(KT * v_tok * 2);
  // piece i (0..7) of tile t: K (i even) or V (i odd) rows 4 (4 wave + i / 2)
  // .. + 3.  No s_nop in front (mxk::dma16m opens with one for VALU-written
  // descriptor / offset SGPRs; here every one is SALU-made, which
  // tests/test_isa_hazards.py's valu_sgpr_to_vmem audits)
  auto issue_piece = [&](int t, int i) {
    const int p = i >> 1;
    uint32_t d0 = sm32 + ((t + 2) & 3) * QSLOT + (4 * wave + p) * 1024 + (i & 1) * TILE_BYTES;
    asm volatile("" : "+s"(d0));
    const uint32_t ch16 = static_cast<uint32_t>((cbase ^ p) << 4);
    const uint32_t voff = (i & 1) ? vrow0 + static_cast<uint32_t>(p * 4 * v_tok * 2) + ch16
                                  : krow0 + static_cast<uint32_t>(p * 4 * k_tok * 2) + ch16;
    const uint32_t soff = (i & 1) ? t * v_step : t * k_step;
    if (i & 1)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                   :
                   : "v"(voff), "s"(rv), "s"(soff), "{m0}"(d0)
                   : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                   :
                   : "v"(voff), "s"(rk), "s"(soff), "{m0}"(d0)
                   : "memory");
  };
  auto issue = [&](int t) {
#pragma unroll
    for (int i = 0; i < 8; ++i) issue_piece(t, i);
  };
  // the successor's Q / dO / O rows of this wave's head into L2 / MALL: 3 x
  // 64 rows x 2 lines of 128 B, one dword each, 6 LDS-DMA loads into the
  // wave's 256-B sink (never read).  The successor - the workgroup `succ`
  // (= CU count) ids later - runs on this XCD (8 | succ), about when this
  // one ends; its prologue then streams from cache what it would have
  // fetched from HBM with nothing else to do
  auto prefetch_next = [&]() {
    if (nbq4 < 0) return;
    const int nb = nbq4 / nq4, nh = (nbq4 - nb * nq4) * 4 + wave, nr0 = nqb_ * QW;
    const uint16_t* bases[3] = {q + (static_cast<long>(nb) * S + nr0) * q_tok + static_cast<long>(nh) * D,
                                dout + (static_cast<long>(nb) * S + nr0) * tokd + static_cast<long>(nh) * D,
                                o + (static_cast<long>(nb) * S + nr0) * tokd + static_cast<long>(nh) * D};
    const long strides[3] = {q_tok, tokd, tokd};
    uint32_t sink = sm32 + QLDS + wave * 256;
    asm volatile("" : "+s"(sink));
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      const int tsr = m >> 1;
      const int line = (m & 1) * 64 + lane;          // row line >> 1, 128-B half line & 1
      const mxk::u32x4 rs = mxk::make_rsrc(bases[tsr], static_cast<unsigned>(QW * strides[tsr] * 2));
      const uint32_t voff = static_cast<uint32_t>((line >> 1) * strides[tsr] * 2 + (line & 1) * 128);
      asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, 0 offen lds"
                   :
                   : "v"(voff), "s"(rs), "{m0}"(sink)
                   : "memory");
    }
  };
  // ---- per-row operands, staged through LDS by full-row LDS-DMA (the
  // K-tile piece mapping, swizzled images): as direct loads in the MFMA
  // fragment layout every load instruction touched 32 B of 32 rows, and
  // just issuing the 50 loads took 21 % of the kernel's cycles - the
  // vector-memory path, not HBM, was the limit (an L2 prefetch of the next
  // item changed nothing; profiles/r6_dq256/).  Each wave moves its own
  // head's 64 rows (16 KiB a tensor) into its own region, so only the K / V
  // tiles need the barrier:
  //   1. dO -> region A_w (slots 0-1 area), O -> region B_w (slots 2-3 area)
  //   2. dO fragments -> AGPRs, O fragments -> VGPRs; Q -> region A_w
  //   3. delta, rowc; barrier (every wave done with its B region) ->
  //      K / V tiles 0, 1 into slots 2, 3 (tile t lives in slot (t + 2) & 3)
  //   4. Q fragments -> AGPRs; tile 0 landed; barrier
  const uint32_t regA = sm32 + wave * 16384, regB = sm32 + 65536 + wave * 16384;
  auto stage = [&](const uint16_t* base, long tok, uint32_t reg) {
    const mxk::u32x4 rs = mxk::make_rsrc(base, static_cast<unsigned>(QW * tok * 2));
#pragma unroll
    for (int pc = 0; pc < 16; ++pc) {
      uint32_t d0 = reg + pc * 1024;
      asm volatile("" : "+s"(d0));
      const uint32_t voff = static_cast<uint32_t>((4 * pc + prow) * tok * 2 + ((cbase ^ (pc & 3)) << 4));
      asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                   :
                   : "v"(voff), "s"(rs), "{m0}"(d0)
                   : "memory");
    }
  };
  const uint16_t* qrow = qh + static_cast<long>(q0) * q_tok;
  const uint16_t* dorow = doh + static_cast<long>(q0) * tokd;
  const uint16_t* orow = oh + static_cast<long>(q0) * tokd;
  float lv[2];
#pragma unroll
  for (int g = 0; g < 2; ++g)
    asm volatile("global_load_dword %0, %1, off"
                 : "=v"(lv[g])
                 : "v"(lse + lrow0 + 32 * g + r32)
                 : "memory");
  stage(dorow, tokd, regA);
  stage(orow, tokd, regB);
  stamp(5);
  vmw<0>();                          // own pieces (no other wave reads them)
  asm volatile("" : "+v"(lv[0]), "+v"(lv[1]) :: "memory");
  int koff[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) koff[s] = swz(r32, 2 * s + h);
  const char* imA = smem + wave * 16384;
  const char* imB = smem + 65536 + wave * 16384;
  bf16x8_t qf[2][8], df[2][8];
  float part[2] = {0.f, 0.f};
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      df[g][s] = lds_b128(imA + koff[s] + g * 8192);
      const bf16x8_t of = lds_b128(imB + koff[s] + g * 8192);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        part[g] += mxk::bf2f(static_cast<uint16_t>(df[g][s][e])) * mxk::bf2f(static_cast<uint16_t>(of[e]));
    }
  // region A_w is read: Q goes there (LDS traffic retired first)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  stage(qrow, q_tok, regA);
  stamp(6);
  // delta = dO . O of the row (the two lane halves hold 64 dims each)
  float nl[2], dl[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const float delta = half_sum(part[g]);
    nl[g] = -lv[g] * 1.4426950408889634f;
    dl[g] = delta;
    if (h == 0)
      *reinterpret_cast<float2*>(rowc + 2 * (lrow0 + 32 * g + r32)) =
          make_float2(-lv[g] / scale, -delta);
  }
  // every wave done with its O region (slots 2-3): tiles 0 and 1 go there
  __builtin_amdgcn_s_barrier();
  issue(0);
  issue(1);
  // Q (own) landed: 16 pieces of tiles 0 / 1 and the two rowc stores may fly
  vmw<18>();
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[g][s] = lds_b128(imA + koff[s] + g * 8192);
  // Q read (tile 2 goes into slot 0 during tile 0) and tile 0 landed
  // (tile 1's 8 may fly; the rowc stores are older than tile 0)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  vmw<8>();
  __builtin_amdgcn_s_barrier();
  stamp(7);

  // ---- LDS read offsets: K / V rows r32 (+ 8 KiB for the step's key half),
  // chunk 2 s + h; K^T transposed reads at keys tr_key (+8) of k-step kk
  // (+ 4 KiB), chunk 4 db + tr_ch
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * h + (i16 >> 2);
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);
  const int tr_byte = 8 * (i16 & 1);
  int ktr[4][2];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    ktr[db][0] = swz(tr_key, 4 * db + tr_ch) + tr_byte;
    ktr[db][1] = swz(tr_key + 8, 4 * db + tr_ch) + tr_byte;
  }

  const float c = scale * 1.4426950408889634f;
  f32x16_t dqa[2][4];                 // dQ^T: rows d = 32 db + crow, lane = query (AGPRs)
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) dqa[g][db][r] = 0.f;
  f32x16_t sacc[2][2], pacc[2][2];    // [step parity][g]: rows key = crow, lane = query
  bf16x8_t dsf[2][2][2];              // dS^T operands [step parity][g][k-step of 16 keys]
  // step -1 (a no-op): its g1 softmax sees S = -inf (P = 0, dS = 0) and its
  // g0 operands are zero, so B(-1) adds K^T . 0 (tile 0's finite keys)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    sacc[1][1][r] = -INFINITY;
    pacc[1][1][r] = 0.f;
  }
  dsf[1][0][0] = bf16x8_t{};
  dsf[1][0][1] = bf16x8_t{};

  // softmax of step j's tile g as 24 items (unit u = 0..7: item 3 u element
  // 2 u, 3 u + 1 element 2 u + 1, 3 u + 2 their bf16 pair; the k-step operand
  // is complete after units 3 / 7), placed one or two per MFMA gap: an item
  // costs <= 20 issue cycles (fma, exp, sub, mul; the guide's one-wave
  // budget is ~24 per 32-cycle gap with at most one 8-cycle exp), where whole
  // units (two exps) made the gaps they sat in ~50 cycles.  MASK (the two
  // diagonal steps): key kv0 + crow(r, h) past query q0 + 32 g + r32, i.e.
  // (r & 3) + 8 (r >> 2) > lim, one compare a score.
  uint32_t dsw[2][2][2][4];           // the operands as bf16 pairs, [parity][g][kk][word]
  float xe[2];                        // the unit's two elements between their items
  auto smi = [&](auto par_c, int g, int n, int lim, auto mask_c) {
    constexpr int P = decltype(par_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const int u = n / 3, kind = n - 3 * u;
    if (kind < 2) {
      const int r = 2 * u + kind;
      float p = fexp2(fmaf(sacc[P][g][r], c, nl[g]));
      if (MASK) p = (r & 3) + 8 * (r >> 2) > lim ? 0.f : p;
      float x = p * (pacc[P][g][r] - dl[g]);
      if constexpr (DBG == 1) x = p > 0.f ? 1.f : 0.f;
      if constexpr (DBG == 2) x = p > 0.f ? sacc[P][g][r] : 0.f;
      if constexpr (DBG == 3) x = p > 0.f ? pacc[P][g][r] : 0.f;
      xe[kind] = x;
    } else {
      dsw[P][g][u >> 2][u & 3] = pk2(xe[0], xe[1]);
      if ((u & 3) == 3) {
        const uint32_t* w = dsw[P][g][u >> 2];
        dsf[P][g][u >> 2] = __builtin_bit_cast(bf16x8_t, u32x4_t{w[0], w[1], w[2], w[3]});
      }
    }
  };
  auto lim_of = [&](int j, int g) { return q0 + 32 * g + r32 - 32 * j - 4 * h; };

  // operands carried across phases: phase A's first K / V rows (read during
  // the preceding phase B when both read the same tile) and phase B's first
  // two K^T operands (read during the preceding phase A), so no phase opens
  // with an exposed LDS latency
  bf16x8_t pre_k, pre_v, pre_b0, pre_b1;
  auto kread = [&](const char* kt, int i) {
    const int db = i >> 1, kk = i & 1;
    return cat8(lds_tr_b64(kt + ktr[db][0] + kk * 4096), lds_tr_b64(kt + ktr[db][1] + kk * 4096));
  };

  // phase A(j): S^T, dP^T of step j (parity PA) from the K / V rows at kt;
  // beside: softmax(j-1) of g1 (parity PA ^ 1), items 0..23 after MFMAs
  // 0..23.  PRE: the s = 0 operands are in pre_k / pre_v.  NEXTB (non-null):
  // read the first two operands of the phase B that follows from there.
  auto phaseA = [&](auto par_c, const char* kt, int j, auto mask_c, auto pre_c,
                    const char* nextb, int dma_t, bool pf = false) {
    constexpr int PA = decltype(par_c)::value;
    constexpr bool PRE = decltype(pre_c)::value;
    using prv = std::integral_constant<int, PA ^ 1>;
    const int lim = lim_of(j - 1, 1);
    // the successor prefetch goes out ahead of this phase's DMA pieces: the
    // tile's barrier (vmcnt 8: only the pieces may fly) then covers it
    if (pf) prefetch_next();
    qd_ready(qf, df);
    bf16x8_t ka = PRE ? pre_k : lds_b128(kt + koff[0]);
    bf16x8_t va = PRE ? pre_v : lds_b128(kt + TILE_BYTES + koff[0]);
    int item = 0;
    auto beside = [&]() {
      if (item < 24) smi(prv{}, 1, item, lim, mask_c);
      ++item;
    };
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      bf16x8_t nk = ka, nv = va;
      // DMA_T >= 0: one piece of that tile per k-step (8 pieces): spread
      // over the phase instead of a burst behind the tile's barrier
      if (dma_t >= 0) issue_piece(dma_t, s);
      if (s < 7) {
        nk = lds_b128(kt + koff[s + 1]);
        nv = lds_b128(kt + TILE_BYTES + koff[s + 1]);
      } else {
        pre_b0 = kread(nextb, 0);
        pre_b1 = kread(nextb, 1);
      }
      if (s == 0) {
        mq0(sacc[PA][0], ka, qf[0][0]);
        beside();
        __builtin_amdgcn_sched_barrier(0);
        mq0(sacc[PA][1], ka, qf[1][0]);
        beside();
        __builtin_amdgcn_sched_barrier(0);
        mq0(pacc[PA][0], va, df[0][0]);
        beside();
        __builtin_amdgcn_sched_barrier(0);
        mq0(pacc[PA][1], va, df[1][0]);
        beside();
      } else if (s < 7) {
        mq(sacc[PA][0], ka, qf[0][s]);
        beside();
        __builtin_amdgcn_sched_barrier(0);
        mq(sacc[PA][1], ka, qf[1][s]);
        beside();
        __builtin_amdgcn_sched_barrier(0);
        mq(pacc[PA][0], va, df[0][s]);
        beside();
        __builtin_amdgcn_sched_barrier(0);
        mq(pacc[PA][1], va, df[1][s]);
        beside();
      } else {
        mq4_fenced(sacc[PA][0], sacc[PA][1], pacc[PA][0], pacc[PA][1], qf[0][7], qf[1][7],
                   df[0][7], df[1][7], ka, va);
      }
      __builtin_amdgcn_sched_barrier(0);
      ka = nk;
      va = nv;
    }
  };
  // phase B(j-1): dQ^T += K^T dS^T of step j-1 (parity PB) with K^T from the
  // K image at kt (its first two operands in pre_b0 / pre_b1); beside:
  // softmax(j) of g0 (parity PB ^ 1), items 3 u / 3 u + 1 after MFMAs 2 u /
  // 2 u + 1 and 3 u + 2 beside the latter.  SOFT false: nothing beside (the
  // tail).  NEXTA (non-null): read the next phase A's s = 0 operands from
  // there during the last MFMA pair.
  auto phaseB = [&](auto par_c, const char* kt, int j, auto mask_c, auto soft_c,
                    const char* nexta) {
    constexpr int PB = decltype(par_c)::value;
    constexpr bool SOFT = decltype(soft_c)::value;
    using cur = std::integral_constant<int, PB ^ 1>;
    const int lim = lim_of(j, 0);
    ds_ready(dsf[PB], dqa);
    // K^T operands two MFMA pairs ahead (one pair ahead exposed the
    // transposed reads' latency: one wave per SIMD, nothing else hides it)
    bf16x8_t a = pre_b0, a1 = pre_b1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x8_t n = a;
      if (i < 6) {
        n = kread(kt, i + 2);
      } else if (i == 6 && nexta != nullptr) {
        pre_k = lds_b128(nexta + koff[0]);
        pre_v = lds_b128(nexta + TILE_BYTES + koff[0]);
      }
      ma(dqa[0][i >> 1], a, dsf[PB][0][i & 1]);
      if (SOFT) smi(cur{}, 0, 3 * i, lim, mask_c);
      __builtin_amdgcn_sched_barrier(0);
      ma(dqa[1][i >> 1], a, dsf[PB][1][i & 1]);
      if (SOFT) {
        smi(cur{}, 0, 3 * i + 1, lim, mask_c);
        smi(cur{}, 0, 3 * i + 2, lim, mask_c);
      }
      __builtin_amdgcn_sched_barrier(0);
      a = a1;
      a1 = n;
    }
  };

  // tile t = steps 2 t (parity 0) and 2 t + 1 (parity 1).  MASK: the
  // causal block's last tile (its two steps are the diagonal ones).
  auto tile = [&](int t, auto mask_c) {
    using F = std::false_type;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    const char* cur = smem + ((t + 2) & 3) * QSLOT;
    const char* prv = t ? smem + ((t + 1) & 3) * QSLOT : cur;
    // step 2t: A(2t) beside softmax(2t-1, g1) (never diagonal); B(2t-1)
    // beside softmax(2t, g0)
    using T_ = std::true_type;
    // tile t + 2's DMA during phase A(2t): its slot's tile t - 2 was last
    // read in step 2t - 2, before the barrier that ended tile t - 1
    // (the causal block's last tile has no next tile to move: none, which
    // also keeps hipcc from computing the DMA's SGPR operands in VGPRs there)
    phaseA(P0{}, cur, 2 * t, F{}, F{}, prv + 32 * 256, decltype(mask_c)::value ? -1 : t + 2,
           t == (T > 4 ? T - 4 : 0));
    stamp(1);
    phaseB(P1{}, prv + 32 * 256, 2 * t, mask_c, T_{}, cur + 32 * 256);
    stamp(2);
    // step 2t+1: A(2t+1) beside softmax(2t, g1); B(2t) beside softmax(2t+1, g0)
    phaseA(P1{}, cur + 32 * 256, 2 * t + 1, mask_c, T_{}, cur, -1);
    stamp(1);
    phaseB(P0{}, cur, 2 * t + 1, mask_c, T_{}, nullptr);
    stamp(2);
    // 8-pass XDL write -> accumulator read: the allocator may copy dQ^T (just
    // written by phase B's MFMAs) on the loop's exit edge - seen: register 0
    // of the last tile read one instruction behind its MFMA, stale in every
    // non-causal block; the nops cover the latency and the accumulators are
    // redefined behind them
    asm volatile("s_nop 7\n\ts_nop 4"
                 : "+a"(dqa[0][0]), "+a"(dqa[0][1]), "+a"(dqa[0][2]), "+a"(dqa[0][3]),
                   "+a"(dqa[1][0]), "+a"(dqa[1][1]), "+a"(dqa[1][2]), "+a"(dqa[1][3]));
    // barrier: tile t+1 landed (own pieces; tile t+2's 8 may fly) and
    // every wave past B(2t-1), the last reader of tile t-1's slot
    vmw<8>();
    __builtin_amdgcn_s_barrier();
    stamp(3);
  };
  stamp(0);
  const int Tm = CAUSAL ? T - 1 : T;
  for (int t = 0; t < Tm; ++t) tile(t, std::false_type{});
  if constexpr (CAUSAL) tile(T - 1, std::true_type{});
  // tail: softmax(J-1) of g1, then B(J-1)
  {
    const int j = 2 * T - 1;
    const int lim = lim_of(j, 1);
    const char* kt = smem + ((T + 1) & 3) * QSLOT + 32 * 256;
    pre_b0 = kread(kt, 0);
    pre_b1 = kread(kt, 1);
#pragma unroll
    for (int n = 0; n < 24; ++n)
      smi(std::integral_constant<int, 1>{}, 1, n, lim, std::integral_constant<bool, CAUSAL>{});
    __builtin_amdgcn_sched_barrier(0);
    phaseB(std::integral_constant<int, 1>{}, kt, j + 1, std::false_type{}, std::false_type{},
           nullptr);
  }
  // the DMA of tiles past the block (T and T + 1) must land before the
  // workgroup ends and its LDS goes to another one
  vmw<0>();
  // dQ^T final: drain the asm MFMAs before the accumulators are read
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int db = 0; db < 4; ++db) asm volatile("" : "+a"(dqa[g][db]));

  // ---- dQ = scale (dQ^T)^T, staged through LDS so every global store
  // writes 4 whole 256-B rows (straight from the lanes each store touched 32
  // rows with 16 B each: store-bound, 8 % of the kernel's cycles).  Lane
  // (r32, h) holds row 32 g + r32, dims 32 db + 8 rg + 4 h .. + 3: one 8-B
  // LDS write each into the wave's 16-KiB row-major image (16-B chunks
  // XOR-swizzled by swz()); every wave is past its tail first (the last
  // tile's slot may be any wave's image region).
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  // ROPE: the cos / sin rows of the block's 64 positions (16 KiB each,
  // shared by the 4 heads) by LDS-DMA into slots 2-3 (free now), 8 pieces a
  // wave, read from LDS by the row loop instead of one L2 round trip per row
  const char* rtab = smem + 65536;
  if constexpr (ROPE) {
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) {
      const int tbl = pc >> 2, piece = 4 * wave + (pc & 3);
      const mxk::u32x4 rs = mxk::make_rsrc((tbl ? rsin : rcos) + static_cast<long>(q0) * (D / 2),
                                           static_cast<unsigned>(QW * (D / 2) * 4));
      uint32_t d0 = sm32 + 65536 + tbl * 16384 + piece * 1024;
      asm volatile("" : "+s"(d0));
      asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                   :
                   : "v"(static_cast<uint32_t>(piece * 1024 + lane * 16)), "s"(rs), "{m0}"(d0)
                   : "memory");
    }
  }
  char* img = smem + wave * 16384;
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        uint2 pk;
        pk.x = pk2(dqa[g][db][4 * rg] * scale, dqa[g][db][4 * rg + 1] * scale);
        pk.y = pk2(dqa[g][db][4 * rg + 2] * scale, dqa[g][db][4 * rg + 3] * scale);
        *reinterpret_cast<uint2*>(img + swz(32 * g + r32, 4 * db + rg) + 8 * h) = pk;
      }
  __builtin_amdgcn_s_waitcnt(0xC07F);   // own image: no other wave reads it
  if constexpr (ROPE) {
    vmw<0>();                            // the table pieces, every wave's
    __builtin_amdgcn_s_barrier();
  }
  // lane l: chunk l & 15 of rows (l >> 4) + 4 i
  const int crow0 = lane >> 4, cch = lane & 15;
  const long dqt = dq_tok > 0 ? dq_tok : tokd;
  uint16_t* dbase = dq + (static_cast<long>(b) * S + q0) * dqt + static_cast<long>(hq) * D + cch * 8;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = crow0 + 4 * i;
    uint4 x = *reinterpret_cast<const uint4*>(img + swz(row, cch));
    if constexpr (ROPE) {
      // chunks cch < 8 hold a (dims 8 cch ..), the partner cch ^ 8 holds b
      const uint4 y = *reinterpret_cast<const uint4*>(img + swz(row, cch ^ 8));
      const float* ct = reinterpret_cast<const float*>(rtab) + row * (D / 2) + 8 * (cch & 7);
      const u32x4_t o = mxk::rope8_bf16(u32x4_t{x.x, x.y, x.z, x.w}, u32x4_t{y.x, y.y, y.z, y.w},
                                        cch < 8, ct, ct + QW * (D / 2), -1.f);
      x = make_uint4(o[0], o[1], o[2], o[3]);
    }
    *reinterpret_cast<uint4*>(dbase + static_cast<long>(row) * dqt) = x;
  }
  stamp(4);
  };   // run_item

  int bq4, qb, nbq4 = -1, nqb_ = -1;
  map_block_xcd(blockIdx.x, gridDim.x, nqb, grp / 4, CAUSAL, &bq4, &qb);
  if (succ > 0 && static_cast<int>(blockIdx.x) + succ < static_cast<int>(gridDim.x))
    map_block_xcd(blockIdx.x + succ, gridDim.x, nqb, grp / 4, CAUSAL, &nbq4, &nqb_);
  run_item(bq4, qb, nbq4, nqb_);
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* w = stamps + (static_cast<long>(blockIdx.x) * 4 + wave) * 9;
      w[0] = __builtin_readcyclecounter() - st_0;
#pragma unroll
      for (int e = 0; e < 8; ++e) w[1 + e] = st_seg[e];
    }
  }
}

#include <atomic>
#include <cstdlib>

namespace {
// the successor distance of the prefetch: the CU count (workgroups of one
// XCD are ids congruent mod 8, so the id `CUs` later runs on the same XCD
// about when this one ends); MXK_DQ256_PREFETCH=0 turns the prefetch off (A/B)
int dq256_succ() {
  static std::atomic<int> v{-1};
  int n = v.load(std::memory_order_relaxed);
  if (n < 0) {
    const char* e = std::getenv("MXK_DQ256_PREFETCH");
    n = 0;
    if (!(e && e[0] == '0')) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      n -= n % 8;
    }
    v.store(n, std::memory_order_relaxed);
  }
  return n;
}
}  // namespace

// dQ of backward variant 9 (+ the rowc pairs for mxk_attn_bwd_dkdv256).
// Returns a HIP status; hipErrorInvalidValue for a layout it does not take.
MXK_API int mxk_attn_bwd_dq256(const void* q, const void* k, const void* v, const void* o,
                               const void* dout, const float* lse, void* dq, float* rowc, int B,
                               int S, int Hq, int Hkv, long q_tok, long k_tok, long v_tok,
                               float scale, int causal, hipStream_t stream) {
  if (B < 1 || S < QW || S % QW || Hkv < 1 || Hq % Hkv || (Hq / Hkv) % 4 || q_tok % 8 ||
      k_tok % 8 || v_tok % 8 || static_cast<long>(S) * k_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * v_tok * 2 >= (1L << 32) ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
       reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
       reinterpret_cast<uintptr_t>(rowc)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * (Hq / 4) * (S / QW);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* O = static_cast<const uint16_t*>(o);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dQ = static_cast<uint16_t*>(dq);
  const int succ = dq256_succ();
  if (causal)
    hipLaunchKernelGGL(mxk_attn_bwd_dq256_kernel<true>, dim3(nwg), dim3(256), 0, stream, Q, K, V, O,
                       dO, lse, dQ, rowc, S, Hq, Hkv, q_tok, k_tok, v_tok, scale, nullptr, succ);
  else
    hipLaunchKernelGGL(mxk_attn_bwd_dq256_kernel<false>, dim3(nwg), dim3(256), 0, stream, Q, K, V,
                       O, dO, lse, dQ, rowc, S, Hq, Hkv, q_tok, k_tok, v_tok, scale, nullptr, succ);
  MXK_RETURN_LAUNCH_STATUS();
}

// mxk_attn_bwd_dq256 with the rotary-embedding backward fused into the dQ
// store (rcos / rsin: [S][D/2] fp32) and dQ at token stride dq_tok
MXK_API int mxk_attn_bwd_dq256_rope(const void* q, const void* k, const void* v, const void* o,
                                    const void* dout, const float* lse, void* dq, float* rowc,
                                    int B, int S, int Hq, int Hkv, long q_tok, long k_tok,
                                    long v_tok, long dq_tok, const float* rcos, const float* rsin,
                                    float scale, int causal, hipStream_t stream) {
  if (B < 1 || S < QW || S % QW || Hkv < 1 || Hq % Hkv || (Hq / Hkv) % 4 || q_tok % 8 ||
      k_tok % 8 || v_tok % 8 || dq_tok < static_cast<long>(Hq) * D || dq_tok % 8 || !rcos ||
      !rsin || static_cast<long>(S) * k_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * v_tok * 2 >= (1L << 32) ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
       reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
       reinterpret_cast<uintptr_t>(rowc) | reinterpret_cast<uintptr_t>(rcos) |
       reinterpret_cast<uintptr_t>(rsin)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * (Hq / 4) * (S / QW);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* O = static_cast<const uint16_t*>(o);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dQ = static_cast<uint16_t*>(dq);
  const int succ = dq256_succ();
  if (causal)
    hipLaunchKernelGGL((mxk_attn_bwd_dq256_kernel<true, 0, false, true>), dim3(nwg), dim3(256), 0,
                       stream, Q, K, V, O, dO, lse, dQ, rowc, S, Hq, Hkv, q_tok, k_tok, v_tok, scale,
                       nullptr, succ, dq_tok, rcos, rsin);
  else
    hipLaunchKernelGGL((mxk_attn_bwd_dq256_kernel<false, 0, false, true>), dim3(nwg), dim3(256), 0,
                       stream, Q, K, V, O, dO, lse, dQ, rowc, S, Hq, Hkv, q_tok, k_tok, v_tok, scale,
                       nullptr, succ, dq_tok, rcos, rsin);
  MXK_RETURN_LAUNCH_STATUS();
}

// Diagnostic: mxk_attn_bwd_dq256 with the dS^T operand replaced (dbg 1: 1,
// 2: S, 3: dP wherever P > 0); non-causal only.
MXK_API int mxk_attn_bwd_dq256_dbg(const void* q, const void* k, const void* v, const void* o,
                                   const void* dout, const float* lse, void* dq, float* rowc, int B,
                                   int S, int Hq, int Hkv, long q_tok, long k_tok, long v_tok,
                                   float scale, int dbg, hipStream_t stream) {
  if (B < 1 || S < QW || S % QW || Hkv < 1 || Hq % Hkv || (Hq / Hkv) % 4 || dbg < 1 || dbg > 3)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * (Hq / 4) * (S / QW);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* O = static_cast<const uint16_t*>(o);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dQ = static_cast<uint16_t*>(dq);
#define MXK_DQ256_DBG(N)                                                                         \
  hipLaunchKernelGGL((mxk_attn_bwd_dq256_kernel<false, N>), dim3(nwg), dim3(256), 0, stream, Q, K, \
                     V, O, dO, lse, dQ, rowc, S, Hq, Hkv, q_tok, k_tok, v_tok, scale)
  if (dbg == 1) MXK_DQ256_DBG(1);
  else if (dbg == 2) MXK_DQ256_DBG(2);
  else MXK_DQ256_DBG(3);
#undef MXK_DQ256_DBG
  MXK_RETURN_LAUNCH_STATUS();
}

// Diagnostic: mxk_attn_bwd_dq256 (causal) with per-wave segment cycle counts,
// stamps: [workgroups of the launch][4 waves][total, the 8 segments of the
// kernel's stamp()]
MXK_API int mxk_attn_bwd_dq256_stamps(const void* q, const void* k, const void* v, const void* o,
                                      const void* dout, const float* lse, void* dq, float* rowc,
                                      int B, int S, int Hq, int Hkv, long q_tok, long k_tok,
                                      long v_tok, float scale, unsigned long long* stamps,
                                      hipStream_t stream) {
  if (B < 1 || S < QW || S % QW || Hkv < 1 || Hq % Hkv || (Hq / Hkv) % 4 || !stamps)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * (Hq / 4) * (S / QW);
  hipLaunchKernelGGL((mxk_attn_bwd_dq256_kernel<true, 0, true>), dim3(nwg), dim3(256), 0, stream,
                     static_cast<const uint16_t*>(q), static_cast<const uint16_t*>(k),
                     static_cast<const uint16_t*>(v), static_cast<const uint16_t*>(o),
                     static_cast<const uint16_t*>(dout), lse, static_cast<uint16_t*>(dq), rowc, S,
                     Hq, Hkv, q_tok, k_tok, v_tok, scale, stamps, dq256_succ());
  MXK_RETURN_LAUNCH_STATUS();
}
