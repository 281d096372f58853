// Flash attention backward, dK/dV with 256 keys per workgroup (gfx950).
//
// The round-4 PMC of the GQA dK/dV kernel (attention.hip, mxk_attn_bwd_dkdv16:
// 8 waves x 16 keys = 128 keys per workgroup, 16x16x32 MFMAs) shows it as the
// slowest piece of the backward: 39 % MFMA busy, 16 % of its wave cycles
// waiting on LDS, and 857 MB per Llama-3-8B layer fetched from beyond L2
// (31 % hit rate) because every 128-key block re-streams the whole Q / dO of
// its query-head group (profiles/r4_attention/pmc_fwd4_bwd5.txt).  This
// kernel is the structure of /opt/skills/guides/cdna_hip_programming.md
// Appendix B 'Attention backward':
//
//   * one workgroup = 4 waves = 256 keys of one (batch, KV head); a wave owns
//     64 keys and keeps dK^T and dV^T of them (2 x 128 x 64 fp32) in its 256
//     accumulator registers for the whole sweep over the group's query heads
//     x 32-row query slices - so the Q / dO stream per FLOP is half the
//     128-key kernel's, and each operand fragment feeds a 32x32 MFMA tile
//     (four times the FLOPs per LDS byte of the 16x16 tiles);
//   * key on the MFMA lane: S = Q K^T and dP = dO V^T come out of
//     v_mfma_f32_32x32x16_bf16 with the query in the registers and the key
//     on the lane, so the accumulators converted to bf16 ARE the B operands
//     of dV^T += dO^T P and dK^T += Q^T dS (no LDS round trip for P / dS);
//   * the row constants are the initial accumulators: S starts at -LSE/scale
//     and dP at -delta, so P = exp2(c S') and dS = P dP' need no subtraction
//     and no row maximum (c = scale log2 e);
//   * one LDS image per tile: the K block (64 KiB, resident for the whole
//     kernel) is read by rows for S; the Q / dO slices by rows for S / dP and
//     by ds_read_b64_tr_b16 columns for dV^T / dK^T; V's B fragments live in
//     registers;
//   * Q / dO slices (and their {-LSE/scale, -delta} rows) arrive by LDS-DMA
//     two items ahead into a 3-slot ring: one barrier per item, counted
//     vmcnt waits.
//
// This file computes dK and dV only; dQ comes from the query-parallel dQ
// kernel of attention.hip (variant 5's, with the delta pass folded in),
// which writes the {-LSE/scale, -delta} row pairs this kernel streams.  The
// split costs two MFMA products per tile over a single pass (S and dP are
// recomputed) but needs no dQ atomics: at 256 keys per workgroup a single
// pass adds one byte of fp32 atomics per 640 FLOPs, and at the chip-wide
// ~1.3 TB/s atomic rate (MI355X_MICROARCH.md 'Global float atomics') that
// floor alone is ~0.93 ms per Llama-3-8B layer (B 8, S 2048, causal) - more
// than the whole two-kernel backward.
//
// Layouts as attention.hip: q [B, S, Hq, 128] (token stride q_tok), k / v
// [B, S, Hkv, 128] (k_tok / v_tok), dout [B, S, Hq, 128] contiguous, rowc
// [B, Hq, S] x {-lse/scale, -delta} fp32, dk / dv [B, S, Hkv, 128] (token
// strides dk_tok / dv_tok).  S % 256 == 0; every Q / K / V / dO panel must
// fit a 32-bit buffer offset.
#include "attention_common.h"

namespace {
constexpr int KW = 64;                        // keys per wave
constexpr int KBLK = 256;                     // keys per workgroup
constexpr int QS = 32;                        // query rows per item
constexpr int NSLOT = 3;                      // Q / dO ring depth
constexpr int QIMG = QS * 256;                // 8 KiB: one 32-row slice image
constexpr int SLOT = 2 * QIMG + QS * 8;       // Q | dO | rowc (32 x float2)
constexpr int KIMG = KBLK * 256;              // 64 KiB
// ring first: every ring offset (< 49920) fits a ds_read's 16-bit immediate
constexpr int KOFF = NSLOT * SLOT;             // K image after the ring
constexpr int LDS_BYTES = KOFF + KIMG;

__device__ __forceinline__ void dma4m(const mxk::u32x4& rsrc, uint32_t lds_addr, uint32_t voff,
                                      uint32_t soff) {
  asm volatile("s_nop 0\n\tbuffer_load_dword %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(rsrc), "s"(soff), "{m0}"(lds_addr)
               : "memory");
}

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt untouched)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// dK^T / dV^T accumulation with the accumulators pinned to AGPRs (inline
// asm, "+a"): all 256 accumulator registers hold dK^T / dV^T for the whole
// kernel, so S / dP - which the VALU reads - stay in VGPRs.  The asm is
// opaque to hipcc's hazard recognizer; its operands are either LDS-read
// results (no VALU hazard) or the bf16 P / dS operands, which
// mfma_operands_ready() fences with the VALU-write -> MFMA-read wait states.
__device__ __forceinline__ void mfma_acc(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// S / dP chains, accumulators pinned to VGPRs ("+v"): the VALU reads them,
// so they must not be allocated in (or shuffled through) the accumulator
// file.  FENCE: the first MFMA of a chain whose C or operands a VALU
// instruction may just have written.
template <bool FENCE = false>
__device__ __forceinline__ void mfma_v(f32x16_t& acc, const bf16x8_t& a, const bf16x8_t& b) {
  if constexpr (FENCE)
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// after the last MFMA of an S / dP chain: the XDL-write -> VALU-read wait
// states (8-pass 32x32x16: 12) before anything reads the results, and the
// results redefined behind the nops so no reader is scheduled above them
__device__ __forceinline__ void mfma_result_fence(f32x16_t& x, f32x16_t& y) {
  asm volatile("s_nop 7\n\ts_nop 4" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void mfma_operands_ready(const bf16x8_t (&pf)[2], const bf16x8_t (&sf)[2]) {
  asm volatile("s_nop 2" ::"v"(pf[0]), "v"(pf[1]), "v"(sf[0]), "v"(sf[1]));
}
// after the last accumulating MFMA, before the accumulators are read: cover
// the 16-pass MFMA's write latency, and make every later read depend on a
// value defined behind the nops (cf. mxk::mfma_drain)
template <int NI, int NJ>
__device__ __forceinline__ void mfma_drain_acc(f32x16_t (&x)[NI][NJ], f32x16_t (&y)[NI][NJ]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" : "+a"(x[i][j]), "+a"(y[i][j]));
}

__device__ __forceinline__ void zero16(f32x16_t& x) {
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = 0.f;
}
}  // namespace

// One workgroup = (batch b, KV head hkv, key block kb of 256 keys).
// Heaviest key blocks first (causal: block kb has S - 256 kb query rows per
// head): with two rounds of workgroups per CU that is the longest-job-first
// order, which balances exactly at Llama's 8 key blocks.
template <bool CAUSAL>
__global__ void __launch_bounds__(256, 1)
mxk_attn_bwd_dkdv256_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                            const uint16_t* __restrict__ v, const uint16_t* __restrict__ dout,
                            const float* __restrict__ rowc, uint16_t* __restrict__ dk,
                            uint16_t* __restrict__ dv, int S, int Hq, int Hkv, long q_tok,
                            long k_tok, long v_tok, long dk_tok, long dv_tok, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nkb = S / KBLK;
  const int nbh = gridDim.x / nkb;
  const int bh = blockIdx.x % nbh;
  const int kb = blockIdx.x / nbh;     // heaviest (kb 0) first
  const int grp = Hq / Hkv;
  const int b = bh / Hkv, hkv = bh % Hkv;
  const int hq0 = hkv * grp;
  const int k0 = kb * KBLK;
  const int kw0 = k0 + wave * KW;

  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;
  const uint16_t* qg_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq0) * D;
  const uint16_t* dog_ptr = dout + static_cast<long>(b) * S * Hq * D + static_cast<long>(hq0) * D;
  const float* rowc_g = rowc + (static_cast<long>(b) * Hq + hq0) * S * 2;

  const uint32_t sm32 = mxk::lds_addr32(smem);
  const uint32_t ring = sm32;
  const uint32_t kimg = sm32 + KOFF;          // K image [256 keys][256 B], swizzled

  // ---- DMA sources (swizzle on the source address: lane i of a 1-KiB piece
  // lands at row 4p + (i >> 4), slot i & 15, and fetches chunk
  // slot ^ ((row & 3) << 2 | (row >> 2) & 3) so the image is swz()-ordered)
  const mxk::u32x4 rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
  const mxk::u32x4 rq = mxk::make_rsrc(qg_ptr, static_cast<unsigned>(S * q_tok * 2));
  const mxk::u32x4 rd = mxk::make_rsrc(dog_ptr, static_cast<unsigned>(static_cast<long>(S) * Hq * D * 2));
  const mxk::u32x4 rr = mxk::make_rsrc(rowc_g, static_cast<unsigned>(grp * S * 8));
  const int prow = lane >> 4, pslot = lane & 15;

  // K image: 64 pieces of 4 rows; wave w moves pieces 16 w .. 16 w + 15
  for (int j = 0; j < 16; ++j) {
    const int p = 16 * wave + j;
    const int row = 4 * p + prow;
    const int ch = pslot ^ ((prow << 2) | (p & 3));
    mxk::dma16m(rk, kimg + p * 1024, static_cast<uint32_t>(row * k_tok * 2 + ch * 16),
                static_cast<uint32_t>(k0 * k_tok * 2));
  }

  // Q / dO slice pieces: wave 0 / 1 move Q pieces 0-3 / 4-7, wave 2 / 3 dO
  // pieces 0-3 / 4-7; wave 0 also moves the 256-B rowc block (32 float2)
  const bool is_q = wave < 2;
  const long tok = is_q ? q_tok : static_cast<long>(Hq) * D;
  const mxk::u32x4 rsl = is_q ? rq : rd;
  uint32_t svo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = 4 * (wave & 1) + j;
    const int row = 4 * p + prow;
    const int ch = pslot ^ ((prow << 2) | (p & 3));
    svo[j] = static_cast<uint32_t>(row * tok * 2 + ch * 16);
  }
  const uint32_t sdst = (is_q ? 0 : QIMG) + 4 * (wave & 1) * 1024;

  // work items: (query head gq of the group, 32-row slice t), head-outer,
  // slices ascending from the key block's diagonal (causal)
  const int q_begin = CAUSAL ? k0 : 0;
  const int nsl = (S - q_begin) / QS;
  const int niter = nsl * grp;
  auto issue = [&](int i) {
    const int gq = i / nsl;
    const int qs0 = q_begin + (i - gq * nsl) * QS;
    const uint32_t slot = ring + (i % NSLOT) * SLOT;
    const uint32_t so = static_cast<uint32_t>((qs0 * tok + gq * D) * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) mxk::dma16m(rsl, slot + sdst + j * 1024, svo[j], so);
    if (wave == 0)   // lanes 0-31: -lse/scale of rows 0..31, lanes 32-63: -delta
      dma4m(rr, slot + 2 * QIMG, static_cast<uint32_t>(r32 * 8 + h * 4),
            static_cast<uint32_t>((gq * S + qs0) * 8));
  };
  issue(0);
  if (niter > 1) issue(1);

  // V's B fragments (dP = dO V^T, key on the lane): lane holds
  // V[kw0 + 32 kt + r32][16 s + 8 h .. + 7]
  bf16x8_t vf[2][8];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      vf[kt][s] = *reinterpret_cast<const bf16x8_t*>(
          vb_ptr + static_cast<long>(kw0 + 32 * kt + r32) * v_tok + 16 * s + 8 * h);
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(vf[kt][s]));
  vm_wait<0>();
  __syncthreads();

  const float c = scale * 1.4426950408889634f;
  f32x16_t dva[4][2], dka[4][2];   // [d tile][key tile]: rows d, lane = key
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      zero16(dva[db][kt]);
      zero16(dka[db][kt]);
    }

  // per-lane LDS offsets: row reads (A of S / dP: row r32, chunk 2 s + h;
  // B of S: K row 64 w + 32 kt + r32), transposed reads (A of dV^T / dK^T:
  // query rows 16 s' + tr_row (+8), chunk 4 db + tr_ch)
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_row = 4 * h + (i16 >> 2);
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);
  const int tr_byte = 8 * (i16 & 1);
  // row-read offsets: chunk 2 s + h of row r32 (Q / dO slices: + slot
  // immediates; K: + the wave's 64-row block of the image)
  int roff[8], koff[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    roff[s] = swz(r32, 2 * s + h);
    koff[s] = KOFF + wave * KW * 256 + roff[s];
  }

  // softmax of one 32-key tile: P = exp2(c S'), dS = P dP' (causal mask on
  // the diagonal slices), converted to the bf16 B operands of the two
  // k-steps of 16 queries
  auto softmax = [&](f32x16_t& sacc, f32x16_t& pacc, int kt, int qs0, bool diag,
                     bf16x8_t (&pf)[2], bf16x8_t (&sf)[2]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = fexp2(sacc[r] * c);
      if (diag && kw0 + 32 * kt + r32 > qs0 + crow(r, h)) p = 0.f;
      sacc[r] = p;
      pacc[r] = p * pacc[r];
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      pf[s2] = pack8(sacc, 8 * s2);
      sf[s2] = pack8(pacc, 8 * s2);
    }
  };
  // dV^T[., kt] += dO^T P, dK^T[., kt] += Q^T dS (A: transposed reads)
  auto dkdv = [&](const char* qt, const char* dt, int kt, const bf16x8_t (&pf)[2],
                  const bf16x8_t (&sf)[2]) {
    mfma_operands_ready(pf, sf);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int row = 16 * s2 + tr_row;
        const int ch = 4 * db + tr_ch;
        const bf16x8_t ao = cat8(lds_tr_b64(dt + swz(row, ch) + tr_byte),
                                 lds_tr_b64(dt + swz(row + 8, ch) + tr_byte));
        const bf16x8_t aq = cat8(lds_tr_b64(qt + swz(row, ch) + tr_byte),
                                 lds_tr_b64(qt + swz(row + 8, ch) + tr_byte));
        mfma_acc(dva[db][kt], ao, pf[s2]);
        mfma_acc(dka[db][kt], aq, sf[s2]);
      }
    }
  };

  auto step = [&](int i, auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;   // == i % NSLOT
    // slot (i + 2) % 3 was last read in item i - 1 (barrier-certified)
    if (i + 2 < niter) issue(i + 2);
    const int gq = i / nsl;
    const int qs0 = q_begin + (i - gq * nsl) * QS;
    if (!CAUSAL || qs0 + QS - 1 >= kw0) {     // else every key of this wave is masked
      const char* qt = smem + SL * SLOT;
      const char* dt = qt + QIMG;
      const float* rc = reinterpret_cast<const float*>(qt + 2 * QIMG);
      const bool diag = CAUSAL && qs0 < kw0 + KW - 1;

      // initial accumulators straight from LDS (no VALU write in front of
      // the MFMA chains): rows 8 g + 4 h + 0..3 of the slice's -lse/scale
      // block (floats 0..31) and -delta block (32..63)
      f32x16_t s0, p0, s1, p1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(rc + 8 * g + 4 * h);
        const float4 d4 = *reinterpret_cast<const float4*>(rc + 32 + 8 * g + 4 * h);
        s0[4 * g + 0] = l4.x; s0[4 * g + 1] = l4.y; s0[4 * g + 2] = l4.z; s0[4 * g + 3] = l4.w;
        p0[4 * g + 0] = d4.x; p0[4 * g + 1] = d4.y; p0[4 * g + 2] = d4.z; p0[4 * g + 3] = d4.w;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(rc + 8 * g + 4 * h);
        const float4 d4 = *reinterpret_cast<const float4*>(rc + 32 + 8 * g + 4 * h);
        s1[4 * g + 0] = l4.x; s1[4 * g + 1] = l4.y; s1[4 * g + 2] = l4.z; s1[4 * g + 3] = l4.w;
        p1[4 * g + 0] = d4.x; p1[4 * g + 1] = d4.y; p1[4 * g + 2] = d4.z; p1[4 * g + 3] = d4.w;
      }
      __builtin_amdgcn_sched_barrier(0);
      // phase A: S' / dP' of key tile 0
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8_t qa = lds_b128(qt + roff[s]);
        const bf16x8_t da = lds_b128(dt + roff[s]);
        const bf16x8_t kf = lds_b128(smem + koff[s]);
        mfma_v(s0, qa, kf);
        mfma_v(p0, da, vf[0][s]);
      }
      mfma_result_fence(s0, p0);
      __builtin_amdgcn_sched_barrier(0);
      // phase B: S' / dP' of key tile 1 beside the softmax of tile 0
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8_t qa = lds_b128(qt + roff[s]);
        const bf16x8_t da = lds_b128(dt + roff[s]);
        const bf16x8_t kf = lds_b128(smem + koff[s] + 32 * 256);
        mfma_v(s1, qa, kf);
        mfma_v(p1, da, vf[1][s]);
      }
      mfma_result_fence(s1, p1);
      bf16x8_t pf0[2], sf0[2], pf1[2], sf1[2];
      softmax(s0, p0, 0, qs0, diag, pf0, sf0);
      __builtin_amdgcn_sched_barrier(0);
      // phase C: dK / dV of tile 0 beside the softmax of tile 1
      dkdv(qt, dt, 0, pf0, sf0);
      softmax(s1, p1, 1, qs0, diag, pf1, sf1);
      __builtin_amdgcn_sched_barrier(0);
      // phase D: dK / dV of tile 1
      dkdv(qt, dt, 1, pf1, sf1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // item i + 1 landed (own pieces); the barrier publishes every wave's
    // pieces and certifies slot i % 3 is no longer read
    if (i + 2 < niter) {
      if (wave == 0) vm_wait<5>();
      else vm_wait<4>();
    } else {
      vm_wait<0>();
    }
    __syncthreads();
  };
  // unrolled by the ring depth: every slot offset is a compile-time immediate
  for (int i = 0; i < niter; i += NSLOT) {
    step(i, std::integral_constant<int, 0>{});
    if (i + 1 < niter) step(i + 1, std::integral_constant<int, 1>{});
    if (i + 2 < niter) step(i + 2, std::integral_constant<int, 2>{});
  }
  mfma_drain_acc(dva, dka);

  // ---- dK = scale * (dK^T)^T, dV: lane = key, registers r -> d = 32 db + crow(r, h)
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const long key = kw0 + 32 * kt + r32;
    uint16_t* dkr = dk + (static_cast<long>(b) * S + key) * dk_tok + static_cast<long>(hkv) * D;
    uint16_t* dvr = dv + (static_cast<long>(b) * S + key) * dv_tok + static_cast<long>(hkv) * D;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * db + 8 * g + 4 * h;
        uint2 pk;
        pk.x = mxk::pack2bf(dka[db][kt][4 * g] * scale, dka[db][kt][4 * g + 1] * scale);
        pk.y = mxk::pack2bf(dka[db][kt][4 * g + 2] * scale, dka[db][kt][4 * g + 3] * scale);
        *reinterpret_cast<uint2*>(dkr + d) = pk;
        pk.x = mxk::pack2bf(dva[db][kt][4 * g], dva[db][kt][4 * g + 1]);
        pk.y = mxk::pack2bf(dva[db][kt][4 * g + 2], dva[db][kt][4 * g + 3]);
        *reinterpret_cast<uint2*>(dvr + d) = pk;
      }
    }
  }
}

// dK / dV of the 256-key kernel.  rowc: [B, Hq, S] x {-lse/scale, -delta}
// (written by the dQ kernel of attention.hip with ROWC).  Returns a HIP
// status; hipErrorInvalidValue when a layout does not fit.
MXK_API int mxk_attn_bwd_dkdv256(const void* q, const void* k, const void* v, const void* dout,
                                 const float* rowc, void* dk, void* dv, int B, int S, int Hq,
                                 int Hkv, long q_tok, long k_tok, long v_tok, long dk_tok,
                                 long dv_tok, float scale, int causal, hipStream_t stream) {
  if (B < 1 || S < KBLK || S % KBLK || Hkv < 1 || Hq % Hkv || q_tok % 8 || k_tok % 8 ||
      v_tok % 8 || dk_tok % 4 || dv_tok % 4 ||
      static_cast<long>(S) * q_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * k_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * Hq * D * 2 >= (1L << 32) ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(dout) |
       reinterpret_cast<uintptr_t>(rowc)) % 16 ||
      (reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) % 8)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * Hkv * (S / KBLK);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dK = static_cast<uint16_t*>(dk);
  auto* dV = static_cast<uint16_t*>(dv);
  if (causal)
    hipLaunchKernelGGL(mxk_attn_bwd_dkdv256_kernel<true>, dim3(nwg), dim3(256), 0, stream,
                       Q, K, V, dO, rowc, dK, dV, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok, dv_tok,
                       scale);
  else
    hipLaunchKernelGGL(mxk_attn_bwd_dkdv256_kernel<false>, dim3(nwg), dim3(256), 0, stream,
                       Q, K, V, dO, rowc, dK, dV, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok, dv_tok,
                       scale);
  MXK_RETURN_LAUNCH_STATUS();
}
