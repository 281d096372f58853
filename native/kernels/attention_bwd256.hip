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
constexpr int QIMG = QS * 256;                // 8 KiB: one 32-row slice image
constexpr int KIMG = KBLK * 256;              // 64 KiB
constexpr int DSIMG = QS * 512;               // 16 KiB: [32 q][256 key positions]
// LDS layout: the ring's rowc blocks (32 x float2 per slot), the ring's
// Q | dO slice images, the K image; the one-pass variants (DQ != 0) add a
// double-buffered image of the workgroup's dS (32 queries x 256 keys, bf16)
// for the dQ product.  Ring depth 4 (three items of DMA lead) without dQ, 3
// with it (LDS: 132 / 145 KiB); every ring offset stays a ds_read immediate
// (< 65536): rowc first, then the slices.
template <int DQ>
struct Lay {
  static constexpr int NS = DQ ? 3 : 4;                 // Q / dO ring depth
  static constexpr int RCB = NS * QS * 8;               // rowc blocks
  static constexpr int KOFF = RCB + NS * 2 * QIMG;      // K image after the ring
  static constexpr int DSOFF = KOFF + KIMG;
  static constexpr int BYTES = DQ ? DSOFF + 2 * DSIMG : KOFF + KIMG;
  static_assert(RCB + (NS - 1) * 2 * QIMG + QIMG < 65536, "ring immediates");
};

__device__ __forceinline__ void dma4m(const mxk::u32x4& rsrc, uint32_t lds_addr, uint32_t voff,
                                      uint32_t soff) {
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2 offen lds"
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
// S' / dP' of both key tiles for one k-step, then 12 wait states, in one
// statement
__device__ __forceinline__ void mfma4_fenced(f32x16_t& s0, f32x16_t& p0, f32x16_t& s1,
                                             f32x16_t& p1, const bf16x8_t& qa,
                                             const bf16x8_t& da, const bf16x8_t& k0,
                                             const bf16x8_t& k1, const bf16x8_t& v0,
                                             const bf16x8_t& v1) {
  asm volatile(
      "v_mfma_f32_32x32x16_bf16 %0, %4, %6, %0\n\t"
      "v_mfma_f32_32x32x16_bf16 %1, %5, %8, %1\n\t"
      "v_mfma_f32_32x32x16_bf16 %2, %4, %7, %2\n\t"
      "v_mfma_f32_32x32x16_bf16 %3, %5, %9, %3\n\t"
      "s_nop 7\n\ts_nop 4"
      : "+v"(s0), "+v"(p0), "+v"(s1), "+v"(p1)
      : "v"(qa), "v"(da), "v"(k0), "v"(k1), "v"(v0), "v"(v1));
}
__device__ __forceinline__ void mfma_result_fence1(f32x16_t& x) {
  asm volatile("s_nop 7\n\ts_nop 4" : "+v"(x));
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

// s_waitcnt vmcnt(n) for the few counts the ring uses (n: ring pieces plus
// the dQ atomics issued after the awaited piece); anything else waits for all
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
    case 4: vm_wait<4>(); break;
    case 5: vm_wait<5>(); break;
    case 8: vm_wait<8>(); break;
    case 10: vm_wait<10>(); break;
    case 12: vm_wait<12>(); break;
    case 13: vm_wait<13>(); break;
    case 16: vm_wait<16>(); break;
    case 20: vm_wait<20>(); break;
    case 21: vm_wait<21>(); break;
    case 32: vm_wait<32>(); break;
    case 36: vm_wait<36>(); break;
    case 37: vm_wait<37>(); break;
    default: vm_wait<0>(); break;
  }
}
// the ring's barrier: LDS traffic retired, then s_barrier (no vmcnt wait:
// __syncthreads() would drain the dQ atomics, and with them the DMA ring)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
}
// key position in the dS image: bits 2 and 3 of the key swapped, so that a
// row read of 8 consecutive positions yields the keys in the order the
// transposed K reads (the V^T pattern of the forward) deliver them
__device__ __forceinline__ int dspos(int key) {
  return (key & ~12) | ((key & 4) << 1) | ((key & 8) >> 1);
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
//
// DQ (one-pass variants 7 / 8): the same workgroup also computes its 256
// keys' share of dQ = dS K: each wave writes its dS (bf16) into an LDS image
// [32 queries][256 key positions], and one item later (after the item's
// barrier) wave w multiplies the whole 256-key dS by K[., 32 w .. 32 w + 31]
// (transposed reads of the resident K image) and adds the 32 x 32 result to
// global memory: DQ 1 fp32 atomics into dq_acc [B, S, Hq, 128] (then a
// convert pass), DQ 2 packed-bf16 atomics straight into dq (scaled here).
// STAMP (diagnostic build, mxk_attn_bwd_dkdv256_stamps): each wave adds up
// the shader cycles of the step's phases (AB, softmax 0, C, D) and its
// end-of-step wait + barrier, and writes them with its total to
// stamps[wave id][9] (+ prologue, the last pending tile, the stores)
// ROPE: dK leaves through the rotary-embedding backward (the inverse
// rotation of its (d, d + 64) pairs at the key's position; both halves of a
// pair are in the same lane, d tiles db and db + 2), rounded to bf16 before
// and after exactly as the stand-alone pass (fused_ops.hip) does.
template <bool CAUSAL, int DQ = 0, bool STAMP = false, bool ROPE = false>
__global__ void __launch_bounds__(256, 1)
mxk_attn_bwd_dkdv256_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                            const uint16_t* __restrict__ v, const uint16_t* __restrict__ dout,
                            const float* __restrict__ rowc, uint16_t* __restrict__ dk,
                            uint16_t* __restrict__ dv, int S, int Hq, int Hkv, long q_tok,
                            long k_tok, long v_tok, long dk_tok, long dv_tok, float scale,
                            void* __restrict__ dqo = nullptr,
                            unsigned long long* __restrict__ stamps = nullptr,
                            const float* __restrict__ rcos = nullptr,
                            const float* __restrict__ rsin = nullptr) {
  unsigned long long st_t0 = 0, st_ph[5] = {0, 0, 0, 0, 0}, st_c = 0, st_loop = 0, st_tail = 0,
                     st_drain = 0;
  if constexpr (STAMP) st_t0 = __builtin_readcyclecounter();
  auto stamp = [&](int ph) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_readcyclecounter();
      if (ph >= 0) st_ph[ph] += t - st_c;
      st_c = t;
    }
  };
  using L = Lay<DQ>;
  constexpr int NSLOT = L::NS, KOFF = L::KOFF, DSOFF = L::DSOFF;
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
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
    const uint32_t slot = ring + L::RCB + (i % NSLOT) * 2 * QIMG;
    const uint32_t so = static_cast<uint32_t>((qs0 * tok + gq * D) * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) mxk::dma16m(rsl, slot + sdst + j * 1024, svo[j], so);
    if (wave == 0)   // lanes 0-31: -lse/scale of rows 0..31, lanes 32-63: -delta
      dma4m(rr, ring + (i % NSLOT) * QS * 8, static_cast<uint32_t>(r32 * 8 + h * 4),
            static_cast<uint32_t>((gq * S + qs0) * 8));
  };
  // items of DMA lead: DQ == 0 keeps an item's slices one step longer (its
  // key tile 1 is finished in the next step, see the step body), so the
  // ring of 4 holds the pending item, the current one and two ahead
  constexpr int LEAD = DQ ? NSLOT - 1 : NSLOT - 2;
#pragma unroll
  for (int i = 0; i < LEAD; ++i)
    if (i < niter) issue(i);

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
  if constexpr (DQ == 0) {
    // the slices the first step's no-op pending tile reads (slot NSLOT - 1,
    // not filled before step 1): zeros, not uninitialised LDS
    uint4* z = reinterpret_cast<uint4*>(smem + L::RCB + (NSLOT - 1) * 2 * QIMG);
#pragma unroll
    for (int e = 0; e < 4; ++e) z[tid + 256 * e] = make_uint4(0, 0, 0, 0);
  }
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
  // DQ: dS image writes (per key tile kt and row class j & 3; + (2 s2 +
  // (j >> 2)) * 4096 immediates), reads of the A operand of dQ (per key
  // step class s'' & 3; + (s'' >> 2) * 128), transposed reads of K as the B
  // operand (d = 32 wave + r32; + s'' * 4096)
  int dsw[2][4] = {}, dsr[4] = {}, ktr0 = 0, ktr1 = 0;
  if constexpr (DQ != 0) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int pos = dspos(wave * KW + 32 * kt + r32);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int q7 = jj + 4 * h;
        dsw[kt][jj] = DSOFF + q7 * 512 + (((pos >> 3) ^ q7) << 4) + (pos & 7) * 2;
      }
    }
    const int m = (r32 >> 1) & 3;
#pragma unroll
    for (int sl = 0; sl < 4; ++sl)
      dsr[sl] = DSOFF + r32 * 512 + ((2 * (sl ^ m) + (h ^ (r32 & 1))) << 4);
    ktr0 = KOFF + swz(tr_row, 4 * wave + tr_ch) + tr_byte;
    ktr1 = KOFF + swz(tr_row + 8, 4 * wave + tr_ch) + tr_byte;
  }

  // DQ: item j's share of dQ - rows qs0 .. qs0 + 31 of head gq, columns
  // 32 wave .. + 31 - from the whole workgroup's dS image (buffer j & 1)
  auto dq_item = [&](int j) {
    const int gq = j / nsl;
    const int qs0 = q_begin + (j - gq * nsl) * QS;
    const int buf = (j & 1) * DSIMG;
    // key steps holding an unmasked key (a fully masked wave wrote nothing)
    const int s_end = CAUSAL ? min(16, (qs0 + QS - k0 + 15) >> 4) : 16;
    f32x16_t acc;
    zero16(acc);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (t < s_end) {
        const bf16x8_t a = lds_b128(smem + buf + dsr[t & 3] + (t >> 2) * 128);
        const bf16x8_t bk = cat8(lds_tr_b64(smem + ktr0 + t * 4096), lds_tr_b64(smem + ktr1 + t * 4096));
        if (t == 0) mfma_v<true>(acc, a, bk);
        else mfma_v(acc, a, bk);
      }
      if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // bound the operand look-ahead
    }
    mfma_result_fence1(acc);
    // wave-uniform row base + one lane offset, so the atomics take the
    // SGPR-base + VGPR-offset form (no 64-bit address per register)
    const long row0 = (static_cast<long>(b) * S + qs0) * Hq + hq0 + gq;   // (b, qs0, head)
    const long rstride = static_cast<long>(Hq) * D;                       // elements per token
    if constexpr (DQ == 1) {
      float* rb = static_cast<float*>(dqo) + row0 * D;
      const uint32_t lo = static_cast<uint32_t>(4 * h * rstride + 32 * wave + r32);
#pragma unroll
      for (int r = 0; r < 16; ++r)
        __hip_atomic_fetch_add(rb + ((r & 3) + 8 * (r >> 2)) * rstride + lo, acc[r],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      // packed bf16 pairs: lanes 2m and 2m + 1 swap one value of a register
      // pair, so the even lane holds columns (2m, 2m + 1) of row crow(r) and
      // the odd lane the same columns of row crow(r + 1)
      typedef short s2_t __attribute__((ext_vector_type(2)));
      uint16_t* rb = static_cast<uint16_t*>(dqo) + row0 * D;
      const bool odd = r32 & 1;
      const uint32_t lo = static_cast<uint32_t>((4 * h + (odd ? 1 : 0)) * rstride + 32 * wave +
                                                (r32 & ~1));
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float x = odd ? acc[r] : acc[r + 1];
        const float y = __builtin_bit_cast(
            float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, true));
        const float vlo = odd ? y : acc[r];
        const float vhi = odd ? acc[r + 1] : y;
        const uint32_t pk = mxk::pack2bf(vlo * scale, vhi * scale);
        __builtin_amdgcn_global_atomic_fadd_v2bf16(
            reinterpret_cast<s2_t*>(rb + ((r & 3) + 8 * (r >> 2)) * rstride + lo),
            __builtin_bit_cast(s2_t, pk));
      }
    }
  };
  constexpr int NATOM = DQ == 1 ? 16 : DQ == 2 ? 8 : 0;   // atomics per dq_item

  // softmax of one 32-key tile: P = exp2(c S'), dS = P dP' (causal mask on
  // the diagonal slices), converted to the bf16 B operands of the two
  // k-steps of 16 queries
  // softmax of one 32-key tile, chunk cc (0..7) of 8: registers 2 cc and
  // 2 cc + 1 of P = exp2(c S') (causal mask on the diagonal slices) and
  // dS = P dP'; after chunks 3 and 7 the bf16 B operands of the k-step of
  // 16 queries they complete.  The chunks are placed between the MFMA pairs
  // of the neighbouring phase (one sched region each), so the VALU work
  // issues in the MFMAs' shadow instead of as one block between them.
  auto softmax_chunk = [&](f32x16_t& sacc, f32x16_t& pacc, int kt, int qs0, bool diag,
                           bf16x8_t (&pf)[2], bf16x8_t (&sf)[2], int cc) {
    // key kw0 + 32 kt + r32 is past query qs0 + crow(r, h) when lim >
    // (r & 3) + 8 (r >> 2): one compare against a constant per score (off
    // the diagonal lim is below every constant)
    const int lim = diag ? kw0 + 32 * kt + r32 - qs0 - 4 * h : -1;
#pragma unroll
    for (int r = 2 * cc; r < 2 * cc + 2; ++r) {
      float p = fexp2(sacc[r] * c);
      if (lim > (r & 3) + 8 * (r >> 2)) p = 0.f;
      sacc[r] = p;
      pacc[r] = p * pacc[r];
    }
    if ((cc & 3) == 3) {
      const int s2 = cc >> 2;
      pf[s2] = pack8(sacc, 8 * s2);
      sf[s2] = pack8(pacc, 8 * s2);
    }
  };
  // dV^T[., kt] += dO^T P, dK^T[., kt] += Q^T dS (A: transposed reads)
  auto dkdv = [&](const char* qt, const char* dt, int kt, const bf16x8_t (&pf)[2],
                  const bf16x8_t (&sf)[2], auto&& beside) {
    mfma_operands_ready(pf, sf);
    // transposed operands one MFMA pair ahead (as phase AB)
    auto tread = [&](const char* base, int i) {
      const int row = 16 * (i & 1) + tr_row;
      const int ch = 4 * (i >> 1) + tr_ch;
      return cat8(lds_tr_b64(base + swz(row, ch) + tr_byte),
                  lds_tr_b64(base + swz(row + 8, ch) + tr_byte));
    };
    bf16x8_t ao = tread(dt, 0), aq = tread(qt, 0);
#pragma unroll
    for (int db = 0; db < 4; ++db) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int i = 2 * db + s2;
        bf16x8_t no = ao, nq = aq;
        if (i < 7) {
          no = tread(dt, i + 1);
          nq = tread(qt, i + 1);
        }
        mfma_acc(dva[db][kt], ao, pf[s2]);
        mfma_acc(dka[db][kt], aq, sf[s2]);
        beside(2 * db + s2);
        __builtin_amdgcn_sched_barrier(0);
        ao = no;
        aq = nq;
      }
    }
  };

  // DQ == 0: the pending item's key tile 1 (S' / dP' accumulators, the
  // first query row of its slice, its diagonal flag).  Before the first
  // item a no-op tile: P = exp2(-inf) = 0 and dP' = 0, so dS = 0 (its dK /
  // dV MFMAs add zeros; the slices they read are the zeroed slot NSLOT - 1).
  f32x16_t ps1, pp1;
  int p_qs0 = 0;
  bool p_diag = false;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    ps1[r] = -INFINITY;
    pp1[r] = 0.f;
  }
  auto step = [&](int i, auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;   // == i % NSLOT
    // slot (i + LEAD) % NSLOT was last read in step i - 1 (barrier-certified)
    if (i + LEAD < niter) issue(i + LEAD);
    if constexpr (DQ != 0) {
      if (i > 0) dq_item(i - 1);    // its dS image was completed before this item's barrier
    }
    const int gq = i / nsl;
    const int qs0 = q_begin + (i - gq * nsl) * QS;
    // DQ != 0: a wave whose keys are all masked skips the item.  DQ == 0
    // runs it anyway (the mask zeroes P and dS): the barrier makes the step
    // as long as its busiest wave either way, and a skip branch made the
    // allocator spill the pending tile across its merge
    if (DQ == 0 || !CAUSAL || qs0 + QS - 1 >= kw0) {
      const char* qt = smem + L::RCB + SL * 2 * QIMG;
      const char* dt = qt + QIMG;
      const float* rc = reinterpret_cast<const float*>(smem + SL * QS * 8);
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
      stamp(-1);
      // phase AB: S' / dP' of both key tiles, each Q / dO fragment read once
      // for both (split into a tile-0 and a tile-1 phase, the fragments were
      // read twice: 48 b128 reads a step instead of 32), operands one k-step
      // ahead.  Measured before: phase A 954 and phase B 1132 cycles a step
      // for 16 MFMAs each (512 at the MFMA roof).
      //
      // DQ == 0 pipelines across steps: beside phase AB the softmax of the
      // PREVIOUS item's key tile 1, then its dK / dV beside this item's tile-0
      // softmax, then this item's tile-0 dK / dV; tile 1 stays pending (its
      // S' / dP' in ps1 / pp1) until the next step.  Every MFMA phase then has
      // VALU work beside it but the last (run alone, the tile-0 softmax
      // measured 721 cycles a step).  DQ != 0: the item's softmax of tile 0
      // alone, dK / dV of tile 0 beside the softmax of tile 1, then tile 1.
      bf16x8_t pf0[2], sf0[2], pf1[2], sf1[2];
      {
        bf16x8_t qa = lds_b128(qt + roff[0]);
        bf16x8_t da = lds_b128(dt + roff[0]);
        bf16x8_t k0 = lds_b128(smem + koff[0]);
        bf16x8_t k1 = lds_b128(smem + koff[0] + 32 * 256);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          bf16x8_t nq = qa, nd = da, n0 = k0, n1 = k1;
          if (s < 7) {
            nq = lds_b128(qt + roff[s + 1]);
            nd = lds_b128(dt + roff[s + 1]);
            n0 = lds_b128(smem + koff[s + 1]);
            n1 = lds_b128(smem + koff[s + 1] + 32 * 256);
          }
          if (s == 0) {   // each chain's C may be a VALU copy made just before it
            mfma_v<true>(s0, qa, k0);
            mfma_v<true>(p0, da, vf[0][s]);
            mfma_v<true>(s1, qa, k1);
            mfma_v<true>(p1, da, vf[1][s]);
          } else if (s < 7) {
            mfma_v(s0, qa, k0);
            mfma_v(p0, da, vf[0][s]);
            mfma_v(s1, qa, k1);
            mfma_v(p1, da, vf[1][s]);
          } else {
            // the last four with the XDL-write -> VALU wait states inside the
            // same statement: with a separate fence statement the allocator
            // moved the results into the fence's registers ahead of it (the
            // pending tile's copies), reading them 10 states after the MFMA
            mfma4_fenced(s0, p0, s1, p1, qa, da, k0, k1, vf[0][s], vf[1][s]);
          }
          if constexpr (DQ == 0) softmax_chunk(ps1, pp1, 1, p_qs0, p_diag, pf1, sf1, s);
          __builtin_amdgcn_sched_barrier(0);
          qa = nq;
          da = nd;
          k0 = n0;
          k1 = n1;
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // (k-step 7's statement carried the wait states)
      stamp(0);
      if constexpr (DQ == 0) {
        constexpr int PSL = (SL + NSLOT - 1) % NSLOT;   // the pending item's slot
        const char* pq = smem + L::RCB + PSL * 2 * QIMG;
        dkdv(pq, pq + QIMG, 1, pf1, sf1,
             [&](int cc) { softmax_chunk(s0, p0, 0, qs0, diag, pf0, sf0, cc); });
        stamp(1);
        dkdv(qt, dt, 0, pf0, sf0, [](int) {});
        stamp(2);
        ps1 = s1;
        pp1 = p1;
        p_qs0 = qs0;
        p_diag = diag;
        stamp(3);
      } else {
        // softmax of tile 0 (no MFMA beside it)
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) softmax_chunk(s0, p0, 0, qs0, diag, pf0, sf0, cc);
        __builtin_amdgcn_sched_barrier(0);
        stamp(1);
        // phase C: dK / dV of tile 0 beside the softmax of tile 1
        dkdv(qt, dt, 0, pf0, sf0,
             [&](int cc) { softmax_chunk(s1, p1, 1, qs0, diag, pf1, sf1, cc); });
        stamp(2);
        // phase D: dK / dV of tile 1
        dkdv(qt, dt, 1, pf1, sf1, [](int) {});
        stamp(3);
      }
      if constexpr (DQ != 0) {
        // dS into the image (buffer i & 1; its previous item's dQ reads
        // ended before the last barrier): element j of sf[kt][s2] is row
        // crow(8 s2 + j, h) = (j & 3) + 4 h + 8 (2 s2 + (j >> 2))
        char* dsb = smem + (i & 1) * DSIMG;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int imm = (2 * s2 + (j >> 2)) * 4096;
            *reinterpret_cast<short*>(dsb + dsw[0][j & 3] + imm) = sf0[s2][j];
            *reinterpret_cast<short*>(dsb + dsw[1][j & 3] + imm) = sf1[s2][j];
          }
      }
    }
    // item i + 1 landed (own pieces: all but the pieces of item i + 2 and
    // the dQ atomics issued after item i + 1's pieces); the barrier publishes
    // every wave's pieces (and dS image) and certifies slot i % 3 is no
    // longer read
    const int pieces = wave == 0 ? 5 : 4;
    const int younger = min(LEAD - 1, max(0, niter - 2 - i));   // items issued after i + 1
    if constexpr (STAMP) {
      if (st_c == 0) st_c = __builtin_readcyclecounter();   // a skipped (masked) item
    }
    vm_wait_n(pieces * younger + (i >= 1 ? NATOM : 0) + (i >= 2 ? NATOM : 0));
    lds_barrier();
    stamp(4);
    if constexpr (STAMP) st_c = 0;
  };
  if constexpr (STAMP) st_loop = __builtin_readcyclecounter();
  // unrolled by the ring depth: every slot offset is a compile-time immediate
  for (int i = 0; i < niter; i += NSLOT) {
    step(i, std::integral_constant<int, 0>{});
    if (i + 1 < niter) step(i + 1, std::integral_constant<int, 1>{});
    if (i + 2 < niter) step(i + 2, std::integral_constant<int, 2>{});
    if constexpr (NSLOT > 3)
      if (i + 3 < niter) step(i + 3, std::integral_constant<int, 3>{});
  }
  if constexpr (STAMP) st_tail = __builtin_readcyclecounter();
  if constexpr (DQ != 0) dq_item(niter - 1);
  if constexpr (DQ == 0) {   // the last pending tile 1
    const char* pq = smem + L::RCB + ((niter - 1) % NSLOT) * 2 * QIMG;
    bf16x8_t pf1[2], sf1[2];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) softmax_chunk(ps1, pp1, 1, p_qs0, p_diag, pf1, sf1, cc);
    __builtin_amdgcn_sched_barrier(0);
    dkdv(pq, pq + QIMG, 1, pf1, sf1, [](int) {});
  }
  mfma_drain_acc(dva, dka);
  if constexpr (STAMP) st_drain = __builtin_readcyclecounter();

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
        if (!ROPE) {
          pk.x = mxk::pack2bf(dka[db][kt][4 * g] * scale, dka[db][kt][4 * g + 1] * scale);
          pk.y = mxk::pack2bf(dka[db][kt][4 * g + 2] * scale, dka[db][kt][4 * g + 3] * scale);
          *reinterpret_cast<uint2*>(dkr + d) = pk;
        } else if (db < 2) {
          // pair (d, d + 64): tiles db, db + 2, same register
          const float4 c4 = *reinterpret_cast<const float4*>(rcos + key * (D / 2) + d);
          const float4 s4 = *reinterpret_cast<const float4*>(rsin + key * (D / 2) + d);
          const float cs[4] = {c4.x, c4.y, c4.z, c4.w}, sn[4] = {s4.x, s4.y, s4.z, s4.w};
          float oa[4], ob[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float a = mxk::bf2f(mxk::f2bf(dka[db][kt][4 * g + j] * scale));
            const float bb = mxk::bf2f(mxk::f2bf(dka[db + 2][kt][4 * g + j] * scale));
            mxk::rope_pair(a, bb, cs[j], -sn[j], oa[j], ob[j]);
          }
          pk.x = mxk::pack2bf(oa[0], oa[1]);
          pk.y = mxk::pack2bf(oa[2], oa[3]);
          *reinterpret_cast<uint2*>(dkr + d) = pk;
          pk.x = mxk::pack2bf(ob[0], ob[1]);
          pk.y = mxk::pack2bf(ob[2], ob[3]);
          *reinterpret_cast<uint2*>(dkr + d + 64) = pk;
        }
        pk.x = mxk::pack2bf(dva[db][kt][4 * g], dva[db][kt][4 * g + 1]);
        pk.y = mxk::pack2bf(dva[db][kt][4 * g + 2], dva[db][kt][4 * g + 3]);
        *reinterpret_cast<uint2*>(dvr + d) = pk;
      }
    }
  }
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* w = stamps + (static_cast<long>(blockIdx.x) * 4 + wave) * 9;
      w[0] = __builtin_readcyclecounter() - st_t0;
#pragma unroll
      for (int e = 0; e < 5; ++e) w[1 + e] = st_ph[e];
      w[6] = st_loop - st_t0;                // prologue
      w[7] = st_drain - st_tail;             // last pending tile + drain
      w[8] = w[0] - (st_drain - st_t0);      // dK / dV stores
    }
  }
}

// dK / dV of the 256-key kernel.  rowc: [B, Hq, S] x {-lse/scale, -delta}
// (written by the dQ kernel of attention.hip with ROWC).  rcos / rsin
// (both or neither): the rotary-embedding backward fused into the dK store.
// Returns a HIP status; hipErrorInvalidValue when a layout does not fit.
static int dkdv256_launch(const void* q, const void* k, const void* v, const void* dout,
                          const float* rowc, void* dk, void* dv, int B, int S, int Hq, int Hkv,
                          long q_tok, long k_tok, long v_tok, long dk_tok, long dv_tok,
                          const float* rcos, const float* rsin, float scale, int causal,
                          hipStream_t stream) {
  if (B < 1 || S < KBLK || S % KBLK || Hkv < 1 || Hq % Hkv || q_tok % 8 || k_tok % 8 ||
      v_tok % 8 || dk_tok % 4 || dv_tok % 4 ||
      static_cast<long>(S) * q_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * k_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * Hq * D * 2 >= (1L << 32) ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(dout) |
       reinterpret_cast<uintptr_t>(rowc) | reinterpret_cast<uintptr_t>(rcos) |
       reinterpret_cast<uintptr_t>(rsin)) % 16 ||
      (reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) % 8 ||
      (rcos == nullptr) != (rsin == nullptr))
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * Hkv * (S / KBLK);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dK = static_cast<uint16_t*>(dk);
  auto* dV = static_cast<uint16_t*>(dv);
#define MXK_DKDV256(C, R)                                                                    \
  hipLaunchKernelGGL((mxk_attn_bwd_dkdv256_kernel<C, 0, false, R>), dim3(nwg), dim3(256), 0, \
                     stream, Q, K, V, dO, rowc, dK, dV, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok, \
                     dv_tok, scale, nullptr, nullptr, rcos, rsin)
  if (rcos) {
    if (causal) MXK_DKDV256(true, true);
    else MXK_DKDV256(false, true);
  } else {
    if (causal) MXK_DKDV256(true, false);
    else MXK_DKDV256(false, false);
  }
#undef MXK_DKDV256
  MXK_RETURN_LAUNCH_STATUS();
}
MXK_API int mxk_attn_bwd_dkdv256(const void* q, const void* k, const void* v, const void* dout,
                                 const float* rowc, void* dk, void* dv, int B, int S, int Hq,
                                 int Hkv, long q_tok, long k_tok, long v_tok, long dk_tok,
                                 long dv_tok, float scale, int causal, hipStream_t stream) {
  return dkdv256_launch(q, k, v, dout, rowc, dk, dv, B, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok,
                        dv_tok, nullptr, nullptr, scale, causal, stream);
}
MXK_API int mxk_attn_bwd_dkdv256_rope(const void* q, const void* k, const void* v, const void* dout,
                                      const float* rowc, void* dk, void* dv, int B, int S, int Hq,
                                      int Hkv, long q_tok, long k_tok, long v_tok, long dk_tok,
                                      long dv_tok, const float* rcos, const float* rsin,
                                      float scale, int causal, hipStream_t stream) {
  if (!rcos || !rsin) return static_cast<int>(hipErrorInvalidValue);
  return dkdv256_launch(q, k, v, dout, rowc, dk, dv, B, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok,
                        dv_tok, rcos, rsin, scale, causal, stream);
}

// ---------------------------------------------------------------------------
// One-pass backward (variants 7 / 8): prep -> the 256-key kernel with DQ ->
// (fp32: convert).
//
// prep: one 16-lane group per (b, q, head) row of 128 dims: delta = dO . O,
// the row pair {-lse/scale, -delta}, and the row's dQ accumulator zeroed
// (ZERO 1: fp32 dq_acc; 2: the bf16 dq the packed atomics add into).
template <int ZERO>
__global__ void __launch_bounds__(256)
mxk_attn_bwd_prep_kernel(const uint16_t* __restrict__ o, const uint16_t* __restrict__ dout,
                         const float* __restrict__ lse, float* __restrict__ rowc,
                         void* __restrict__ dqz, int S, int Hq, long rows, float inv_scale) {
  const long row = (static_cast<long>(blockIdx.x) * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  if (row >= rows) return;
  const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(o + row * D + sub * 8);
  const bf16x8_t g = *reinterpret_cast<const bf16x8_t*>(dout + row * D + sub * 8);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    sum += mxk::bf2f(static_cast<uint16_t>(a[e])) * mxk::bf2f(static_cast<uint16_t>(g[e]));
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 16);
  if constexpr (ZERO == 1) {
    float4* z = reinterpret_cast<float4*>(static_cast<float*>(dqz) + row * D) + 2 * sub;
    z[0] = make_float4(0.f, 0.f, 0.f, 0.f);
    z[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  } else if constexpr (ZERO == 2) {
    reinterpret_cast<uint4*>(static_cast<uint16_t*>(dqz) + row * D)[sub] = make_uint4(0, 0, 0, 0);
  }
  if (sub == 0) {
    const long bq = row / Hq;               // row = (b S + q) Hq + hq
    const int hq = static_cast<int>(row - bq * Hq);
    const long bb = bq / S, qi = bq - bb * S;
    const long ri = (bb * Hq + hq) * S + qi;
    *reinterpret_cast<float2*>(rowc + 2 * ri) = make_float2(-lse[ri] * inv_scale, -sum);
  }
}

// dq = bf16(scale * dq_acc), 8 elements per thread
__global__ void __launch_bounds__(256)
mxk_attn_bwd_dq_convert_kernel(const float* __restrict__ acc, uint16_t* __restrict__ dq, long n8,
                               float scale) {
  const long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  const float4 x = reinterpret_cast<const float4*>(acc)[2 * i];
  const float4 y = reinterpret_cast<const float4*>(acc)[2 * i + 1];
  uint4 o;
  o.x = mxk::pack2bf(x.x * scale, x.y * scale);
  o.y = mxk::pack2bf(x.z * scale, x.w * scale);
  o.z = mxk::pack2bf(y.x * scale, y.y * scale);
  o.w = mxk::pack2bf(y.z * scale, y.w * scale);
  reinterpret_cast<uint4*>(dq)[i] = o;
}

// Workspace bytes of the one-pass backward: rowc (8 B per row) and, for the
// fp32 atomics, dq_acc (512 B per row).
MXK_API long mxk_attn_bwd_onepass_workspace(int B, int S, int Hq, int bf16_atomics) {
  const long rows = static_cast<long>(B) * Hq * S;
  return rows * 8 + (bf16_atomics ? 0 : rows * D * 4);
}

// One-pass backward: dq [B, S, Hq, 128] contiguous.  bf16_atomics 0: fp32
// atomics into a zeroed dq_acc, then dq = bf16(scale dq_acc); 1: packed bf16
// atomics straight into the zeroed dq (half the atomic bytes, each partial
// sum rounded to bf16).  Results depend on the atomics' arrival order.
MXK_API int mxk_attn_bwd_onepass(const void* q, const void* k, const void* v, const void* o,
                                 const void* dout, const float* lse, void* dq, void* dk, void* dv,
                                 void* workspace, int B, int S, int Hq, int Hkv, long q_tok,
                                 long k_tok, long v_tok, long dk_tok, long dv_tok, float scale,
                                 int causal, int bf16_atomics, hipStream_t stream) {
  if (B < 1 || S < KBLK || S % KBLK || Hkv < 1 || Hq % Hkv || q_tok % 8 || k_tok % 8 ||
      v_tok % 8 || dk_tok % 4 || dv_tok % 4 ||
      static_cast<long>(S) * q_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * k_tok * 2 >= (1L << 32) ||
      static_cast<long>(S) * Hq * D * 2 >= (1L << 32) ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
       reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
       reinterpret_cast<uintptr_t>(workspace)) % 16 ||
      (reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) % 8)
    return static_cast<int>(hipErrorInvalidValue);
  const long rows = static_cast<long>(B) * Hq * S;
  float* rowc = static_cast<float*>(workspace);
  float* dq_acc = rowc + 2 * rows;
  const auto* O = static_cast<const uint16_t*>(o);
  const auto* dO = static_cast<const uint16_t*>(dout);
  const unsigned pblocks = static_cast<unsigned>((rows * 16 + 255) / 256);
  if (bf16_atomics)
    hipLaunchKernelGGL(mxk_attn_bwd_prep_kernel<2>, dim3(pblocks), dim3(256), 0, stream, O, dO, lse,
                       rowc, dq, S, Hq, rows, 1.f / scale);
  else
    hipLaunchKernelGGL(mxk_attn_bwd_prep_kernel<1>, dim3(pblocks), dim3(256), 0, stream, O, dO, lse,
                       rowc, static_cast<void*>(dq_acc), S, Hq, rows, 1.f / scale);
  const int nwg = B * Hkv * (S / KBLK);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  auto* dK = static_cast<uint16_t*>(dk);
  auto* dV = static_cast<uint16_t*>(dv);
  void* dqo = bf16_atomics ? dq : static_cast<void*>(dq_acc);
#define MXK_ONEPASS_LAUNCH(C, M)                                                                  \
  hipLaunchKernelGGL((mxk_attn_bwd_dkdv256_kernel<C, M>), dim3(nwg), dim3(256), 0, stream, Q, K,   \
                     V, dO, rowc, dK, dV, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok, dv_tok, scale, \
                     dqo)
  if (causal && bf16_atomics) MXK_ONEPASS_LAUNCH(true, 2);
  else if (causal) MXK_ONEPASS_LAUNCH(true, 1);
  else if (bf16_atomics) MXK_ONEPASS_LAUNCH(false, 2);
  else MXK_ONEPASS_LAUNCH(false, 1);
#undef MXK_ONEPASS_LAUNCH
  if (!bf16_atomics) {
    const long n8 = rows * D / 8;
    hipLaunchKernelGGL(mxk_attn_bwd_dq_convert_kernel, dim3(static_cast<unsigned>((n8 + 255) / 256)),
                       dim3(256), 0, stream, dq_acc, static_cast<uint16_t*>(dq), n8, scale);
  }
  MXK_RETURN_LAUNCH_STATUS();
}

// Diagnostic: the dK / dV kernel with per-wave segment cycle counts
// (stamps: [B * Hkv * S / 256 workgroups][4 waves][9]: total, AB, C, D, copies,
// end-of-step wait + barrier, prologue, last pending tile, stores]); arguments as
// mxk_attn_bwd_dkdv256.
MXK_API int mxk_attn_bwd_dkdv256_stamps(const void* q, const void* k, const void* v,
                                        const void* dout, const float* rowc, void* dk, void* dv,
                                        int B, int S, int Hq, int Hkv, long q_tok, long k_tok,
                                        long v_tok, long dk_tok, long dv_tok, float scale,
                                        int causal, unsigned long long* stamps, hipStream_t stream) {
  if (B < 1 || S < KBLK || S % KBLK || Hkv < 1 || Hq % Hkv || !stamps)
    return static_cast<int>(hipErrorInvalidValue);
  const int nwg = B * Hkv * (S / KBLK);
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dK = static_cast<uint16_t*>(dk);
  auto* dV = static_cast<uint16_t*>(dv);
  if (causal)
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv256_kernel<true, 0, true>), dim3(nwg), dim3(256), 0,
                       stream, Q, K, V, dO, rowc, dK, dV, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok,
                       dv_tok, scale, nullptr, stamps);
  else
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv256_kernel<false, 0, true>), dim3(nwg), dim3(256), 0,
                       stream, Q, K, V, dO, rowc, dK, dV, S, Hq, Hkv, q_tok, k_tok, v_tok, dk_tok,
                       dv_tok, scale, nullptr, stamps);
  MXK_RETURN_LAUNCH_STATUS();
}
