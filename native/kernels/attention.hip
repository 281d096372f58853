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
#include "attention_common.h"

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
      const float alpha = fexp2((m - m_new) * c);
      m = m_new;
      const float mc = m_new * c;
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = fexp2(fmaf(s0[r], c, -mc));
        s1[r] = fexp2(fmaf(s1[r], c, -mc));
        ls += s0[r] + s1[r];
      }
      l = l * alpha + ls;
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {   // wave-uniform: some row max moved
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[db][r] *= alpha;
      }
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
          const bf16x8_t a = cat8(lo, hi);
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
// Forward, DMA-fed (the default): the same math and LDS image, but
//   * K/V tiles land in LDS by LDS-DMA (`buffer_load ... lds`, swizzle applied
//     on the source address) issued at the top of the iteration for the next
//     tile: no staging VGPRs, no ds_writes, and no 64-bit address arithmetic
//     per tile (one SGPR offset);
//   * the per-lane LDS read offsets of K (8) and V (8) are loop invariants;
//   * scale-and-shift and the row sum use packed fp32 (v_pk_fma_f32,
//     v_pk_add_f32), halving the softmax's full-rate VALU work.
// Requires S * token_stride * 2 < 2^32 for K and V (buffer offsets).

template <bool CAUSAL, bool UNROLL, bool PIPE = false>
__global__ void __launch_bounds__(NT, 2)
mxk_attn_fwd_dma_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
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
  map_block_xcd(blockIdx.x, gridDim.x, nqb, Hq / Hkv, CAUSAL, &bh, &qb);
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int q0 = qb * BQ;
  const int qw0 = q0 + wave * 32;
  const int myq = qw0 + r32;

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  bf16x8_t qf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
    qf[s] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + static_cast<long>(myq) * q_tok + 16 * s + 8 * h);

  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int nkv = kv_end / BKV;

  // DMA: wave w moves the 1-KiB pieces g = 4w + p (rows 4g .. 4g+3) of K and
  // V; lane i lands at row 4g + (i >> 4), slot i & 15, so it fetches chunk
  // (i & 15) ^ f(row) with f(row) = (row & 3) << 2 | (row >> 2) & 3
  // = (i >> 4) << 2 | p.
  const mxk::u32x4 rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
  const mxk::u32x4 rv = mxk::make_rsrc(vb_ptr, static_cast<unsigned>(S * v_tok * 2));
  const int prow = lane >> 4, pslot = lane & 15;
  uint32_t kvo[4], vvo[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int row = 4 * (4 * wave + p) + prow;
    const int ch = pslot ^ ((prow << 2) | p);
    kvo[p] = static_cast<uint32_t>(row * k_tok * 2 + ch * 16);
    vvo[p] = static_cast<uint32_t>(row * v_tok * 2 + ch * 16);
  }
  const uint32_t k_step = static_cast<uint32_t>(BKV * k_tok * 2);
  const uint32_t v_step = static_cast<uint32_t>(BKV * v_tok * 2);
  // LDS destinations as scalar 32-bit addresses bound to M0 (mxk::dma16m)
  const uint32_t sm32 = mxk::lds_addr32(&smem[0][0]);
  auto issue = [&](int j, int buf) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t d = sm32 + buf * (2 * TILE_BYTES) + (4 * wave + p) * 1024;
      mxk::dma16m(rk, d, kvo[p], j * k_step);
      mxk::dma16m(rv, d + TILE_BYTES, vvo[p], j * v_step);
    }
  };
  issue(0, 0);

  // loop-invariant LDS read offsets: K rows r32 (+32 rows = +8 KiB), chunk
  // 2s + h; V transposed reads at keys tr_key (+8), chunk 4db + tr_ch, with
  // +16 keys = +4 KiB per k-step
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

  // Consume the Q fragments here: the compiler then waits for their loads
  // before the loop instead of placing vmcnt waits inside it, where they
  // would also wait for the next tile's (untracked) DMA.
#pragma unroll
  for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]));
  vm_wait0();   // tile 0
  __syncthreads();

  // the loop body; UNROLL makes the LDS buffer a compile-time constant (read
  // addresses are then loop-invariant VGPRs + immediate offsets)
  auto step = [&](int j, int buf) {
    // buffer buf^1 was last read in iteration j-1 (barrier-certified)
    if (j + 1 < nkv) issue(j + 1, buf ^ 1);
    const int kv0 = j * BKV;
    const bool active = !CAUSAL || kv0 <= qw0 + 31;
    if (active) {
      const char* kt = smem[buf];
      const char* vt = smem[buf] + TILE_BYTES;
      f32x16_t s0, s1;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] = 0.f; s1[r] = 0.f; }
      bf16x8_t vop[16];   // V^T operands [4 db + ks] (PIPE)
      auto read_v = [&](int x) {
        vop[x] = cat8(lds_tr_b64(vt + voff[x >> 2][0] + (x & 3) * 4096),
                      lds_tr_b64(vt + voff[x >> 2][1] + (x & 3) * 4096));
      };
      if constexpr (PIPE) {
        // K operands a k-step pair ahead (two-slot ring), the first V^T
        // operands under the last S MFMAs and the softmax, the rest one db
        // ahead of the PV MFMAs; sched_barrier fences keep the order (the
        // plain loop below gets read -> lgkmcnt(0) -> MFMA per instruction)
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
          else
#pragma unroll
            for (int x = 0; x < 4; ++x) read_v(x);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            s0 = mfma32(ka[pr & 1][2 * e], qf[2 * pr + e], s0);
            s1 = mfma32(ka[pr & 1][2 * e + 1], qf[2 * pr + e], s1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int x = 4; x < 8; ++x) read_v(x);
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8_t a0 = lds_b128(kt + koff[s]);
          const bf16x8_t a1 = lds_b128(kt + koff[s] + 32 * 256);
          s0 = mfma32(a0, qf[s], s0);
          s1 = mfma32(a1, qf[s], s1);
        }
      }
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
      bool grow = true;
      if constexpr (PIPE) {
        // Lazy rescale: keep the stale row max unless the new one exceeds it
        // by more than 2^8 (log2 units).  P = exp2((s - m) c) then stays
        // <= 256 - exact in bf16's exponent range - and l / acc stay
        // consistent with the m they were built with (final o = acc / l,
        // lse = m scale + ln l).  On random data almost every block after the
        // first skips the 32 v_pk_mul of the accumulator rescale.
        grow = (m_new - m) * c > 8.f;
        if (!grow) m_new = m;
      }
      const float alpha = grow ? fexp2((m - m_new) * c) : 1.f;
      m = m_new;
      const f32x2_t nmc = {-m_new * c, -m_new * c};
      if constexpr (PIPE) {
        // P in four 16-key chunks: the exp of chunk ks + 1 runs on the VALU
        // while the four PV MFMAs of chunk ks run on the matrix core (one
        // wave overlaps its own softmax with its own MFMAs)
#pragma unroll
        for (int x = 8; x < 16; ++x) read_v(x);
        if (__builtin_amdgcn_ballot_w64(grow)) {
#pragma unroll
          for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[db][r] *= alpha;
        }
        f32x2_t ls2 = {0.f, 0.f};
        auto chunk = [&](int ks) {
          f32x16_t& x = ks < 2 ? s0 : s1;
          const int base = (ks & 1) * 8;
#pragma unroll
          for (int r = 0; r < 8; r += 2) {
            f32x2_t y = {x[base + r], x[base + r + 1]};
            y = __builtin_elementwise_fma(y, cc, nmc);
            y[0] = fexp2(y[0]);
            y[1] = fexp2(y[1]);
            ls2 += y;
            x[base + r] = y[0];
            x[base + r + 1] = y[1];
          }
          return pack8(x, base);
        };
        bf16x8_t pf[4];
        pf[0] = chunk(0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
          for (int db = 0; db < 4; ++db) acc[db] = mfma32(vop[4 * db + ks], pf[ks], acc[db]);
          if (ks < 3) pf[ks + 1] = chunk(ks + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        l = l * alpha + (ls2[0] + ls2[1]);
      } else {
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
        if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
          for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[db][r] *= alpha;
        }
        bf16x8_t pf[4];
        pf[0] = pack8(s0, 0);
        pf[1] = pack8(s0, 8);
        pf[2] = pack8(s1, 0);
        pf[3] = pack8(s1, 8);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const bf16x4_t lo = lds_tr_b64(vt + voff[db][0] + ks * 4096);
            const bf16x4_t hi = lds_tr_b64(vt + voff[db][1] + ks * 4096);
            acc[db] = mfma32(cat8(lo, hi), pf[ks], acc[db]);
          }
        }
      }
    }
    // tile j+1 (own pieces) landed; the barrier publishes every wave's pieces
    // and certifies that buffer buf is no longer read
    vm_wait0();
    __syncthreads();
  };
  if constexpr (UNROLL) {
    for (int j = 0; j < nkv; j += 2) {
      step(j, 0);
      if (j + 1 < nkv) step(j + 1, 1);
    }
  } else {
    for (int j = 0; j < nkv; ++j) step(j, j & 1);
  }

  const float lt = half_sum(l);
  const float inv = 1.f / lt;
  uint16_t* orow = o + (static_cast<long>(b) * S + myq) * Hq * D + static_cast<long>(hq) * D;
  // 16-B stores: v_permlane32_swap pairs groups g = 2k, 2k+1 across the lane
  // halves, so lane half h holds d = 32 db + 16 k + 8 h + 0..7 (half h of
  // group g holds 4 h + 0..3 of its 8)
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
      uint4 ov;
      ov.x = p0[0];
      ov.y = p1[0];
      ov.z = p0[1];
      ov.w = p1[1];
      *reinterpret_cast<uint4*>(orow + 32 * db + 16 * kk + 8 * h) = ov;
    }
  }
  if (h == 0) lse[(static_cast<long>(b) * Hq + hq) * S + myq] = m * scale + logf(lt);
}

// ---------------------------------------------------------------------------
// variant: 0 = register-staged K/V, 1 = LDS-DMA with the loop unrolled by 2
// (static LDS buffer), 2 = LDS-DMA, 3 = 2 with the PIPE body (operands read a
// group ahead, exp of P chunk ks+1 under the PV MFMAs of chunk ks, lazy
// rescale), 4 = 3 unrolled by 2 (default: the per-iteration v_or of the
// buffer base into 22 LDS addresses disappears).  1-4 fall back to 0 when a
// K/V panel exceeds the 32-bit buffer range.  B=8 Llama shape: 0.42 / 0.43 /
// 0.38 ms (profiles/r1_attention/); round 2: 2 / 3 / 4 = 0.3387 / 0.3218 /
// 0.3133 ms (profiles/r2_attention/fwd_lazy_rescale_unroll_ab.log).
#ifdef MXK_GEMM_EXPERIMENTS
int mxk_attn_fwd_exp_launch(int variant, const uint16_t* qp, const uint16_t* kp, const uint16_t* vp,
                            uint16_t* op, float* lse, int B, int S, int Hq, int Hkv, long q_tok,
                            long k_tok, long v_tok, float scale, int causal, hipStream_t stream);
#endif

MXK_API int mxk_attn_fwd_variant(const void* q, const void* k, const void* v, void* o, float* lse,
                                 int B, int S, int Hq, int Hkv, int head_dim, long q_tok,
                                 long k_tok, long v_tok, float scale, int causal, int variant,
                                 hipStream_t stream) {
  if (head_dim != D || B < 1 || S < BQ || S % BQ || Hkv < 1 || Hq % Hkv ||
      q_tok % 8 || k_tok % 8 || v_tok % 8 || variant < 0 || variant > 10 ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  if (variant == 10) {
    // one wave per SIMD, two 32-row groups per wave (attention_fwd256.hip);
    // shapes it does not take (S % 256, 32-bit offsets) run variant 4
    const int st = mxk_attn_fwd256(q, k, v, o, lse, B, S, Hq, Hkv, q_tok, k_tok, v_tok, scale,
                                   causal, stream);
    if (st != static_cast<int>(hipErrorInvalidValue)) return st;
    variant = 4;
  }
  const int nwg = B * Hq * (S / BQ);
  const long span = static_cast<long>(S) * (k_tok > v_tok ? k_tok : v_tok) * 2;
  if (variant != 0 && span >= (1L << 32)) variant = 0;
  const auto* qp = static_cast<const uint16_t*>(q);
  const auto* kp = static_cast<const uint16_t*>(k);
  const auto* vp = static_cast<const uint16_t*>(v);
  auto* op = static_cast<uint16_t*>(o);
  if (variant >= 5) {
#ifdef MXK_GEMM_EXPERIMENTS
    // A/B records 5-9 (experiments/attention_fwd_exp.hip); -1: shape not
    // tiled by that variant, run variant 4
    const int st = mxk_attn_fwd_exp_launch(variant, qp, kp, vp, op, lse, B, S, Hq, Hkv, q_tok, k_tok,
                                           v_tok, scale, causal, stream);
    if (st >= 0) return st;
    variant = 4;
#else
    return static_cast<int>(hipErrorNotSupported);
#endif
  }
  if (variant == 4) {
    if (causal)
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<true, true, true>), dim3(nwg), dim3(NT), 0, stream,
                         qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    else
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<false, true, true>), dim3(nwg), dim3(NT), 0,
                         stream, qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  } else if (variant == 3) {
    if (causal)
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<true, false, true>), dim3(nwg), dim3(NT), 0, stream,
                         qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    else
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<false, false, true>), dim3(nwg), dim3(NT), 0,
                         stream, qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  } else if (variant == 1) {
    if (causal)
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<true, true>), dim3(nwg), dim3(NT), 0, stream, qp,
                         kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    else
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<false, true>), dim3(nwg), dim3(NT), 0, stream, qp,
                         kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  } else if (variant == 2) {
    if (causal)
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<true, false>), dim3(nwg), dim3(NT), 0, stream, qp,
                         kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    else
      hipLaunchKernelGGL((mxk_attn_fwd_dma_kernel<false, false>), dim3(nwg), dim3(NT), 0, stream,
                         qp, kp, vp, op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  } else {
    if (causal)
      hipLaunchKernelGGL(mxk_attn_fwd_kernel<true>, dim3(nwg), dim3(NT), 0, stream, qp, kp, vp, op,
                         lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
    else
      hipLaunchKernelGGL(mxk_attn_fwd_kernel<false>, dim3(nwg), dim3(NT), 0, stream, qp, kp, vp,
                         op, lse, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  }
  MXK_RETURN_LAUNCH_STATUS();
}

// 1 if forward variant v is in this build (5-9 only in the experiments library)
MXK_API int mxk_attn_fwd_variant_built(int v) {
  if (v == 10) return 1;
#ifdef MXK_GEMM_EXPERIMENTS
  return v >= 0 && v <= 9;
#else
  return v >= 0 && v <= 4;
#endif
}

MXK_API int mxk_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B,
                         int S, int Hq, int Hkv, int head_dim, long q_tok, long k_tok, long v_tok,
                         float scale, int causal, hipStream_t stream) {
  return mxk_attn_fwd_variant(q, k, v, o, lse, B, S, Hq, Hkv, head_dim, q_tok, k_tok, v_tok,
                              scale, causal, 2, stream);
}

// ===========================================================================
// Backward.  Three passes, no atomics (deterministic):
//   1. delta[b][hq][q] = sum_d dO . O                       (mxk_attn_bwd_delta)
//   2. dQ, query-parallel, structured like the forward: per 64-key block
//      S^T = K.Q^T and dP^T = V.dO^T with the query on the lane, P^T from the
//      saved LSE (no max/sum), dS^T = P^T (dP^T - delta), dQ^T += K^T.dS^T
//      (K^T by ds_read_b64_tr_b16 from the same swizzled image).
//   3. dK/dV, key-parallel: one workgroup = 4 waves x 32 keys of one
//      (batch, q-head), sweeping 64-query slices: S = Q.K^T and dP = dO.V^T
//      with the KEY on the lane, so P and dS are already the B operands of
//      dV^T += dO^T.P and dK^T += Q^T.dS (dO^T, Q^T by transposed reads);
//      the accumulator init carries -LSE/scale and -delta, so
//      p = exp2(c * acc) and dS = p * acc' need no extra subtraction.
//      Per-q-head partial dK/dV (fp32) are summed over each GQA group by
//      mxk_attn_bwd_gqa_reduce.
// Recomputing S and dP in both passes costs 7 instead of 5 MFMA products
// per tile but removes the dQ atomics (1.3 TB/s chip-wide would bound the
// pass) and keeps every kernel deterministic.
// ===========================================================================
namespace {
constexpr int BQB = 64;   // queries per slice in the dK/dV kernel

__device__ __forceinline__ void zero16(f32x16_t& x) {
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = 0.f;
}
}  // namespace

__global__ void __launch_bounds__(256)
mxk_attn_bwd_delta_kernel(const uint16_t* __restrict__ o, const uint16_t* __restrict__ dout,
                          float* __restrict__ delta, int S, int Hq, long rows) {
  // one 16-lane group per (b, q, hq) row of 128 dims: 8 bf16 per lane
  const long row = (static_cast<long>(blockIdx.x) * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  if (row >= rows) return;
  const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(o + row * D + sub * 8);
  const bf16x8_t g = *reinterpret_cast<const bf16x8_t*>(dout + row * D + sub * 8);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    s += mxk::bf2f(static_cast<uint16_t>(a[e])) * mxk::bf2f(static_cast<uint16_t>(g[e]));
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) s += __shfl_xor(s, off, 16);
  if (sub == 0) {
    // row = (b * S + q) * Hq + hq  ->  delta[b][hq][q]
    const long bq = row / Hq;
    const int hq = static_cast<int>(row % Hq);
    const long b = bq / S, qi = bq % S;
    delta[(b * Hq + hq) * S + qi] = s;
  }
}

// DMA: K/V tiles by LDS-DMA straight into the swizzled image (the forward
// kernel's piece mapping, destinations bound to M0) instead of register
// staging - frees the 32 staging VGPRs that made this kernel spill at two
// waves per SIMD, and the ds_writes.  Requires S * token_stride * 2 < 2^32.
// FOLD (backward variant 5): the delta pass folded in - each query row's
// delta = dO . O is computed here from the row's own dO fragments and O (the
// two lanes of a row hold 64 columns each) and written to delta_w for the
// dK/dV kernel, which then runs after this one; no separate delta kernel.
// ROWC (with FOLD; backward variant 6): instead of delta, write the row
// pair {-lse/scale, -delta} that the 256-key dK/dV kernel
// (attention_bwd256.hip) loads as the initial S' / dP' accumulators.
template <bool CAUSAL, bool DMA = false, bool PIPE = false, bool UNROLL = false, bool FOLD = false,
          bool ROWC = false>
__global__ void __launch_bounds__(NT, 2)
mxk_attn_bwd_dq_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                       const uint16_t* __restrict__ v, const uint16_t* __restrict__ dout,
                       const float* __restrict__ lse, const float* __restrict__ delta,
                       uint16_t* __restrict__ dq, int S, int Hq, int Hkv, long q_tok, long k_tok,
                       long v_tok, float scale, const uint16_t* __restrict__ o = nullptr,
                       float* __restrict__ delta_w = nullptr) {
  __shared__ __attribute__((aligned(16))) char smem[2][2 * TILE_BYTES];   // [buf][K | V]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nqb = S / BQ;
  int bh, qb;
  map_block_xcd(blockIdx.x, gridDim.x, nqb, Hq / Hkv, CAUSAL, &bh, &qb);
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int q0 = qb * BQ;
  const int qw0 = q0 + wave * 32;
  const int myq = qw0 + r32;

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* dob_ptr = dout + static_cast<long>(b) * S * Hq * D + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  bf16x8_t qf[8], dof[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + static_cast<long>(myq) * q_tok + 16 * s + 8 * h);
    dof[s] = *reinterpret_cast<const bf16x8_t*>(dob_ptr + static_cast<long>(myq) * Hq * D + 16 * s + 8 * h);
  }
  const float c = scale * 1.4426950408889634f;
  const long lrow = (static_cast<long>(b) * Hq + hq) * S + myq;
  const float lse2 = lse[lrow] * 1.4426950408889634f;
  float dlt;
  if constexpr (FOLD) {
    const uint16_t* ob_ptr = o + static_cast<long>(b) * S * Hq * D + static_cast<long>(hq) * D;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const bf16x8_t of = *reinterpret_cast<const bf16x8_t*>(ob_ptr + static_cast<long>(myq) * Hq * D +
                                                              16 * s + 8 * h);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        part += mxk::bf2f(static_cast<uint16_t>(dof[s][e])) * mxk::bf2f(static_cast<uint16_t>(of[e]));
    }
    dlt = part + __shfl_xor(part, 32);       // the row's other 64 columns
    if constexpr (ROWC) {
      if (h == 0)
        *reinterpret_cast<float2*>(delta_w + 2 * lrow) = make_float2(-lse[lrow] / scale, -dlt);
    } else {
      if (h == 0) delta_w[lrow] = dlt;
    }
  } else {
    dlt = delta[lrow];
  }

  const int kv_end = CAUSAL ? min(S, q0 + BQ) : S;
  const int nkv = kv_end / BKV;
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
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = swz(ld_row + 16 * i, ld_ch);
      *reinterpret_cast<bf16x8_t*>(smem[buf] + off) = kst[i];
      *reinterpret_cast<bf16x8_t*>(smem[buf] + TILE_BYTES + off) = vst[i];
    }
  };
  // DMA pieces: wave w moves 1-KiB pieces g = 4w + p (rows 4g .. 4g+3) of K
  // and V, lane i at row 4g + (i >> 4), chunk (i & 15) ^ ((i >> 4) << 2 | p)
  mxk::u32x4 rk{}, rv{};
  uint32_t kvo[4] = {}, vvo[4] = {};
  const uint32_t sm32 = mxk::lds_addr32(&smem[0][0]);
  const uint32_t k_step = static_cast<uint32_t>(BKV * k_tok * 2);
  const uint32_t v_step = static_cast<uint32_t>(BKV * v_tok * 2);
  if constexpr (DMA) {
    rk = mxk::make_rsrc(kb_ptr, static_cast<unsigned>(S * k_tok * 2));
    rv = mxk::make_rsrc(vb_ptr, static_cast<unsigned>(S * v_tok * 2));
    const int prow = lane >> 4, pslot = lane & 15;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = 4 * (4 * wave + p) + prow;
      const int ch = pslot ^ ((prow << 2) | p);
      kvo[p] = static_cast<uint32_t>(r * k_tok * 2 + ch * 16);
      vvo[p] = static_cast<uint32_t>(r * v_tok * 2 + ch * 16);
    }
  }
  auto issue = [&](int j, int buf) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t d = sm32 + buf * (2 * TILE_BYTES) + (4 * wave + p) * 1024;
      mxk::dma16m(rk, d, kvo[p], j * k_step);
      mxk::dma16m(rv, d + TILE_BYTES, vvo[p], j * v_step);
    }
  };
  if constexpr (DMA) {
    issue(0, 0);
    // consume the per-query loads here, so the compiler's vmcnt waits for
    // them sit before the loop and not inside it (where they would also wait
    // for the next tile's untracked DMA)
#pragma unroll
    for (int s = 0; s < 8; ++s) asm volatile("" ::"v"(qf[s]), "v"(dof[s]));
    asm volatile("" ::"v"(lse2), "v"(dlt));
    vm_wait0();
  } else {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  f32x16_t acc[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) zero16(acc[db]);
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_key = 4 * h + (i16 >> 2);
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);
  const int tr_byte = 8 * (i16 & 1);

  if constexpr (!UNROLL) {
  for (int j = 0; j < nkv; ++j) {
    const int buf = j & 1;
    // DMA: buffer buf^1 was last read in iteration j-1 (barrier-certified)
    if (j + 1 < nkv) {
      if constexpr (DMA) issue(j + 1, buf ^ 1);
      else load_tile(j + 1);
    }
    const int kv0 = j * BKV;
    if (!CAUSAL || kv0 <= qw0 + 31) {
      const char* kt = smem[buf];
      const char* vt = smem[buf] + TILE_BYTES;
      const bool diag = CAUSAL && kv0 + BKV - 1 > qw0;
      if constexpr (PIPE) {
        // software-pipelined as the dK/dV kernel's PIPE body: S / dP operands
        // read a half (4 k-steps) ahead, dS-side transposed reads issued
        // under the exp, the next half's first operands under the dQ MFMAs
        bf16x8_t ka[2][2], va[2][2];    // ring of two k-step pairs
        auto read_p = [&](int kh, int pr, int slot) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int s = 2 * pr + e;
            ka[slot][e] = lds_b128(kt + swz(32 * kh + r32, 2 * s + h));
            va[slot][e] = lds_b128(vt + swz(32 * kh + r32, 2 * s + h));
          }
        };
        auto read_t = [&](int kh, int db, int kk) {
          const int key = 32 * kh + 16 * kk + tr_key;
          const int ch = 4 * db + tr_ch;
          return cat8(lds_tr_b64(kt + swz(key, ch) + tr_byte), lds_tr_b64(kt + swz(key + 8, ch) + tr_byte));
        };
        read_p(0, 0, 0);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          __builtin_amdgcn_sched_barrier(0);
          f32x16_t s0, p0;
          zero16(s0);
          zero16(p0);
          bf16x8_t ta[8];
#pragma unroll
          for (int pr = 0; pr < 4; ++pr) {
            if (pr < 3) {
              read_p(kh, pr + 1, (pr + 1) & 1);
            } else {
#pragma unroll
              for (int x = 0; x < 4; ++x) ta[x] = read_t(kh, x >> 1, x & 1);
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              s0 = mfma32(ka[pr & 1][e], qf[2 * pr + e], s0);
              p0 = mfma32(va[pr & 1][e], dof[2 * pr + e], p0);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int x = 4; x < 8; ++x) ta[x] = read_t(kh, x >> 1, x & 1);
          // packed fp32 (v_pk_fma / v_pk_add / v_pk_mul): half the VALU issues
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            f32x2_t x = {s0[r], s0[r + 1]};
            x = __builtin_elementwise_fma(x, f32x2_t{c, c}, f32x2_t{-lse2, -lse2});
            s0[r] = fexp2(x[0]);   // P^T
            s0[r + 1] = fexp2(x[1]);
          }
          if (diag) {   // wave-uniform: only diagonal tiles pay for the mask
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (kv0 + 32 * kh + crow(r, h) > myq) s0[r] = 0.f;
          }
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const f32x2_t pp = f32x2_t{p0[r], p0[r + 1]} - f32x2_t{dlt, dlt};
            const f32x2_t d = f32x2_t{s0[r], s0[r + 1]} * pp;   // dS^T
            s0[r] = d[0];
            s0[r + 1] = d[1];
          }
          bf16x8_t df[2];
          df[0] = pack8(s0, 0);
          df[1] = pack8(s0, 8);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int x = 0; x < 8; ++x) {
            acc[x >> 1] = mfma32(ta[x], df[x & 1], acc[x >> 1]);
            if (kh == 0 && x == 5) {
              read_p(1, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      } else {
      // one 32-key half at a time keeps S^T / dP^T to 32 registers
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        f32x16_t s0, p0;
        zero16(s0);
        zero16(p0);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8_t kf = lds_b128(kt + swz(32 * kh + r32, 2 * s + h));
          const bf16x8_t vf = lds_b128(vt + swz(32 * kh + r32, 2 * s + h));
          s0 = mfma32(kf, qf[s], s0);
          p0 = mfma32(vf, dof[s], p0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float e0 = fexp2(fmaf(s0[r], c, -lse2));
          if (diag && kv0 + 32 * kh + crow(r, h) > myq) e0 = 0.f;
          s0[r] = e0 * (p0[r] - dlt);   // dS^T
        }
        bf16x8_t df[2];
        df[0] = pack8(s0, 0);
        df[1] = pack8(s0, 8);
        // dQ^T += K^T . dS^T  (K^T by transposed reads of the K image)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const int key = 32 * kh + 16 * kk + tr_key;
            const int ch = 4 * db + tr_ch;
            const bf16x4_t lo = lds_tr_b64(kt + swz(key, ch) + tr_byte);
            const bf16x4_t hi = lds_tr_b64(kt + swz(key + 8, ch) + tr_byte);
            const bf16x8_t a = cat8(lo, hi);
            acc[db] = mfma32(a, df[kk], acc[db]);
          }
        }
      }
      }
    }
    if constexpr (DMA) {
      vm_wait0();   // own pieces of tile j+1
    } else {
      if (j + 1 < nkv) store_tile(buf ^ 1);
    }
    __syncthreads();
  }
  } else {
  // UNROLL: the loop body as a lambda called with a compile-time buffer, so
  // the LDS read addresses are loop invariants (as in the forward's variant 4)
  auto step = [&](int j, int buf) {
    // DMA: buffer buf^1 was last read in iteration j-1 (barrier-certified)
    if (j + 1 < nkv) {
      if constexpr (DMA) issue(j + 1, buf ^ 1);
      else load_tile(j + 1);
    }
    const int kv0 = j * BKV;
    if (!CAUSAL || kv0 <= qw0 + 31) {
      const char* kt = smem[buf];
      const char* vt = smem[buf] + TILE_BYTES;
      const bool diag = CAUSAL && kv0 + BKV - 1 > qw0;
      if constexpr (PIPE) {
        // software-pipelined as the dK/dV kernel's PIPE body: S / dP operands
        // read a half (4 k-steps) ahead, dS-side transposed reads issued
        // under the exp, the next half's first operands under the dQ MFMAs
        bf16x8_t ka[2][2], va[2][2];    // ring of two k-step pairs
        auto read_p = [&](int kh, int pr, int slot) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int s = 2 * pr + e;
            ka[slot][e] = lds_b128(kt + swz(32 * kh + r32, 2 * s + h));
            va[slot][e] = lds_b128(vt + swz(32 * kh + r32, 2 * s + h));
          }
        };
        auto read_t = [&](int kh, int db, int kk) {
          const int key = 32 * kh + 16 * kk + tr_key;
          const int ch = 4 * db + tr_ch;
          return cat8(lds_tr_b64(kt + swz(key, ch) + tr_byte), lds_tr_b64(kt + swz(key + 8, ch) + tr_byte));
        };
        read_p(0, 0, 0);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          __builtin_amdgcn_sched_barrier(0);
          f32x16_t s0, p0;
          zero16(s0);
          zero16(p0);
          bf16x8_t ta[8];
#pragma unroll
          for (int pr = 0; pr < 4; ++pr) {
            if (pr < 3) {
              read_p(kh, pr + 1, (pr + 1) & 1);
            } else {
#pragma unroll
              for (int x = 0; x < 4; ++x) ta[x] = read_t(kh, x >> 1, x & 1);
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              s0 = mfma32(ka[pr & 1][e], qf[2 * pr + e], s0);
              p0 = mfma32(va[pr & 1][e], dof[2 * pr + e], p0);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int x = 4; x < 8; ++x) ta[x] = read_t(kh, x >> 1, x & 1);
          // packed fp32 (v_pk_fma / v_pk_add / v_pk_mul): half the VALU issues
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            f32x2_t x = {s0[r], s0[r + 1]};
            x = __builtin_elementwise_fma(x, f32x2_t{c, c}, f32x2_t{-lse2, -lse2});
            s0[r] = fexp2(x[0]);   // P^T
            s0[r + 1] = fexp2(x[1]);
          }
          if (diag) {   // wave-uniform: only diagonal tiles pay for the mask
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (kv0 + 32 * kh + crow(r, h) > myq) s0[r] = 0.f;
          }
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const f32x2_t pp = f32x2_t{p0[r], p0[r + 1]} - f32x2_t{dlt, dlt};
            const f32x2_t d = f32x2_t{s0[r], s0[r + 1]} * pp;   // dS^T
            s0[r] = d[0];
            s0[r + 1] = d[1];
          }
          bf16x8_t df[2];
          df[0] = pack8(s0, 0);
          df[1] = pack8(s0, 8);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int x = 0; x < 8; ++x) {
            acc[x >> 1] = mfma32(ta[x], df[x & 1], acc[x >> 1]);
            if (kh == 0 && x == 5) {
              read_p(1, 0, 0);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      } else {
      // one 32-key half at a time keeps S^T / dP^T to 32 registers
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        f32x16_t s0, p0;
        zero16(s0);
        zero16(p0);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const bf16x8_t kf = lds_b128(kt + swz(32 * kh + r32, 2 * s + h));
          const bf16x8_t vf = lds_b128(vt + swz(32 * kh + r32, 2 * s + h));
          s0 = mfma32(kf, qf[s], s0);
          p0 = mfma32(vf, dof[s], p0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float e0 = fexp2(fmaf(s0[r], c, -lse2));
          if (diag && kv0 + 32 * kh + crow(r, h) > myq) e0 = 0.f;
          s0[r] = e0 * (p0[r] - dlt);   // dS^T
        }
        bf16x8_t df[2];
        df[0] = pack8(s0, 0);
        df[1] = pack8(s0, 8);
        // dQ^T += K^T . dS^T  (K^T by transposed reads of the K image)
#pragma unroll
        for (int db = 0; db < 4; ++db) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const int key = 32 * kh + 16 * kk + tr_key;
            const int ch = 4 * db + tr_ch;
            const bf16x4_t lo = lds_tr_b64(kt + swz(key, ch) + tr_byte);
            const bf16x4_t hi = lds_tr_b64(kt + swz(key + 8, ch) + tr_byte);
            const bf16x8_t a = cat8(lo, hi);
            acc[db] = mfma32(a, df[kk], acc[db]);
          }
        }
      }
      }
    }
    if constexpr (DMA) {
      vm_wait0();   // own pieces of tile j+1
    } else {
      if (j + 1 < nkv) store_tile(buf ^ 1);
    }
    __syncthreads();
  };
  for (int j = 0; j < nkv; j += 2) {
    step(j, 0);
    if (j + 1 < nkv) step(j + 1, 1);
  }
  }
  uint16_t* row = dq + (static_cast<long>(b) * S + myq) * Hq * D + static_cast<long>(hq) * D;
  // 16-B stores, lane halves paired by v_permlane32_swap (as the forward's O)
#pragma unroll
  for (int db = 0; db < 4; ++db) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int g0 = 2 * kk, g1 = 2 * kk + 1;
      const uint32_t x0 = mxk::pack2bf(acc[db][4 * g0] * scale, acc[db][4 * g0 + 1] * scale);
      const uint32_t x1 = mxk::pack2bf(acc[db][4 * g0 + 2] * scale, acc[db][4 * g0 + 3] * scale);
      const uint32_t y0 = mxk::pack2bf(acc[db][4 * g1] * scale, acc[db][4 * g1 + 1] * scale);
      const uint32_t y1 = mxk::pack2bf(acc[db][4 * g1 + 2] * scale, acc[db][4 * g1 + 3] * scale);
      const auto p0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
      const auto p1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
      uint4 ov;
      ov.x = p0[0];
      ov.y = p1[0];
      ov.z = p0[1];
      ov.w = p1[1];
      *reinterpret_cast<uint4*>(row + 32 * db + 16 * kk + 8 * h) = ov;
    }
  }
}

// dK/dV for 128 keys of one (batch, q-head); partials dk_p/dv_p are fp32
// [B, S, Hq, 128] (summed over the GQA group afterwards).
template <bool CAUSAL>
__global__ void __launch_bounds__(NT, 1)
mxk_attn_bwd_dkdv_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                         const uint16_t* __restrict__ v, const uint16_t* __restrict__ dout,
                         const float* __restrict__ lse, const float* __restrict__ delta,
                         float* __restrict__ dk_p, float* __restrict__ dv_p, int S, int Hq,
                         int Hkv, long q_tok, long k_tok, long v_tok, float scale) {
  // [buf][Q tile 64x128 | dO tile 64x128] + lse/delta slices
  __shared__ __attribute__((aligned(16))) char smem[2][2 * BQB * 256];
  __shared__ __attribute__((aligned(16))) float srow[2][2][BQB];   // [buf][lse*log2e/c | delta]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int nkb = S / BQ;   // 128-key blocks
  int bh, kb;
  {
    // key block kb has (nkb - kb) query blocks of work: heaviest = kb 0
    int qbi;
    map_block(blockIdx.x, gridDim.x / nkb, nkb, CAUSAL, &bh, &qbi);
    kb = CAUSAL ? nkb - 1 - qbi : qbi;
  }
  const int b = bh / Hq, hq = bh % Hq;
  const int hkv = hq / (Hq / Hkv);
  const int k0 = kb * BQ;
  const int kw0 = k0 + wave * 32;
  const int mykey = kw0 + r32;

  const uint16_t* qb_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq) * D;
  const uint16_t* dob_ptr = dout + static_cast<long>(b) * S * Hq * D + static_cast<long>(hq) * D;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;
  const float* lse_b = lse + (static_cast<long>(b) * Hq + hq) * S;
  const float* dl_b = delta + (static_cast<long>(b) * Hq + hq) * S;

  // K^T / V^T fragments (B operands of S = Q.K^T and dP = dO.V^T)
  bf16x8_t kf[8], vf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8_t*>(kb_ptr + static_cast<long>(mykey) * k_tok + 16 * s + 8 * h);
    vf[s] = *reinterpret_cast<const bf16x8_t*>(vb_ptr + static_cast<long>(mykey) * v_tok + 16 * s + 8 * h);
  }
  const float c = scale * 1.4426950408889634f;
  const float inv_c = 1.f / c;

  const int q_begin = CAUSAL ? k0 : 0;
  const int nsl = (S - q_begin) / BQB;
  const int ld_row = tid >> 4, ld_ch = tid & 15;
  bf16x8_t qst[4], dst[4];
  float rst = 0.f;
  auto load_slice = [&](int t) {
    const long r0 = q_begin + static_cast<long>(t) * BQB + ld_row;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      qst[i] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + (r0 + 16 * i) * q_tok + ld_ch * 8);
      dst[i] = *reinterpret_cast<const bf16x8_t*>(dob_ptr + (r0 + 16 * i) * Hq * D + ld_ch * 8);
    }
    if (tid < 2 * BQB) {
      const long qi = q_begin + static_cast<long>(t) * BQB + (tid & (BQB - 1));
      rst = tid < BQB ? -lse_b[qi] * 1.4426950408889634f * inv_c : -dl_b[qi];
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = swz(ld_row + 16 * i, ld_ch);
      *reinterpret_cast<bf16x8_t*>(smem[buf] + off) = qst[i];
      *reinterpret_cast<bf16x8_t*>(smem[buf] + BQB * 256 + off) = dst[i];
    }
    if (tid < 2 * BQB) srow[buf][tid / BQB][tid & (BQB - 1)] = rst;
  };
  load_slice(0);
  store_slice(0);
  __syncthreads();

  f32x16_t dka[4], dva[4];
#pragma unroll
  for (int db = 0; db < 4; ++db) { zero16(dka[db]); zero16(dva[db]); }
  const int G = lane >> 4, i16 = lane & 15;
  const int tr_row = 4 * h + (i16 >> 2);
  const int tr_ch = 2 * (G & 1) + ((i16 & 3) >> 1);
  const int tr_byte = 8 * (i16 & 1);

  for (int t = 0; t < nsl; ++t) {
    const int buf = t & 1;
    if (t + 1 < nsl) load_slice(t + 1);
    const int qs0 = q_begin + t * BQB;
    if (!CAUSAL || qs0 + BQB - 1 >= kw0) {
      const char* qt = smem[buf];
      const char* dt = smem[buf] + BQB * 256;
      // accumulator init: -LSE/scale (S) and -delta (dP) per query row
      f32x16_t s0, s1, p0, p1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int qr = 8 * g + 4 * h;
        const float4 l0 = *reinterpret_cast<const float4*>(&srow[buf][0][qr]);
        const float4 l1 = *reinterpret_cast<const float4*>(&srow[buf][0][32 + qr]);
        const float4 d0 = *reinterpret_cast<const float4*>(&srow[buf][1][qr]);
        const float4 d1 = *reinterpret_cast<const float4*>(&srow[buf][1][32 + qr]);
        s0[4 * g] = l0.x; s0[4 * g + 1] = l0.y; s0[4 * g + 2] = l0.z; s0[4 * g + 3] = l0.w;
        s1[4 * g] = l1.x; s1[4 * g + 1] = l1.y; s1[4 * g + 2] = l1.z; s1[4 * g + 3] = l1.w;
        p0[4 * g] = d0.x; p0[4 * g + 1] = d0.y; p0[4 * g + 2] = d0.z; p0[4 * g + 3] = d0.w;
        p1[4 * g] = d1.x; p1[4 * g + 1] = d1.y; p1[4 * g + 2] = d1.z; p1[4 * g + 3] = d1.w;
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bf16x8_t q0f = lds_b128(qt + swz(r32, 2 * s + h));
        const bf16x8_t q1f = lds_b128(qt + swz(32 + r32, 2 * s + h));
        const bf16x8_t o0f = lds_b128(dt + swz(r32, 2 * s + h));
        const bf16x8_t o1f = lds_b128(dt + swz(32 + r32, 2 * s + h));
        s0 = mfma32(q0f, kf[s], s0);
        s1 = mfma32(q1f, kf[s], s1);
        p0 = mfma32(o0f, vf[s], p0);
        p1 = mfma32(o1f, vf[s], p1);
      }
      const bool diag = CAUSAL && qs0 < kw0 + 31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = qs0 + crow(r, h);
        float e0 = fexp2(s0[r] * c);
        float e1 = fexp2(s1[r] * c);
        if (diag && mykey > qi) e0 = 0.f;
        if (diag && mykey > qi + 32) e1 = 0.f;
        s0[r] = e0;                 // P
        s1[r] = e1;
        p0[r] = e0 * p0[r];         // dS = P (dP - delta)
        p1[r] = e1 * p1[r];
      }
      bf16x8_t pf[4], sf[4];
      pf[0] = pack8(s0, 0); pf[1] = pack8(s0, 8); pf[2] = pack8(s1, 0); pf[3] = pack8(s1, 8);
      sf[0] = pack8(p0, 0); sf[1] = pack8(p0, 8); sf[2] = pack8(p1, 0); sf[3] = pack8(p1, 8);
      // dV^T += dO^T . P ; dK^T += Q^T . dS   (transposed reads of dO / Q)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int row = 16 * ks + tr_row;
          const int ch = 4 * db + tr_ch;
          const bf16x4_t olo = lds_tr_b64(dt + swz(row, ch) + tr_byte);
          const bf16x4_t ohi = lds_tr_b64(dt + swz(row + 8, ch) + tr_byte);
          const bf16x4_t qlo = lds_tr_b64(qt + swz(row, ch) + tr_byte);
          const bf16x4_t qhi = lds_tr_b64(qt + swz(row + 8, ch) + tr_byte);
          const bf16x8_t ao = cat8(olo, ohi);
          const bf16x8_t aq = cat8(qlo, qhi);
          dva[db] = mfma32(ao, pf[ks], dva[db]);
          dka[db] = mfma32(aq, sf[ks], dka[db]);
        }
      }
    }
    if (t + 1 < nsl) store_slice(buf ^ 1);
    __syncthreads();
  }
  // partials: lane = key, registers = dims
  const long prow = ((static_cast<long>(b) * S + mykey) * Hq + hq) * D;
#pragma unroll
  for (int db = 0; db < 4; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * db + 8 * g + 4 * h;
      *reinterpret_cast<float4*>(dk_p + prow + d) =
          make_float4(dka[db][4 * g] * scale, dka[db][4 * g + 1] * scale,
                      dka[db][4 * g + 2] * scale, dka[db][4 * g + 3] * scale);
      *reinterpret_cast<float4*>(dv_p + prow + d) =
          make_float4(dva[db][4 * g], dva[db][4 * g + 1], dva[db][4 * g + 2], dva[db][4 * g + 3]);
    }
  }
}

// Round-2 alternatives measured against the PIPE body of this kernel
// (profiles/r2_attention/): a four-buffer LDS ring with every load three
// items ahead (lse / delta rows by DMA too) 1.129 vs 1.099 ms per layer, and
// a pipelined 32-key-per-wave kernel (4 waves, one per SIMD, half the LDS
// operand traffic, dK / dV pinned to AGPRs, softmax overlapped in-wave)
// 1.182 vs 1.107 ms - two waves per SIMD hide more than the halved LDS
// traffic saves.  Also neutral: 128-query slices (half the barriers and
// pipeline drains; 1.1249 vs 1.1215 ms, bit-identical).  A staggered order
// for waves 4-7 (both S / dP groups first, so the SIMD partners' exp phases
// do not coincide) needs ~16 more VGPRs than the 223 of this body and
// spilled (119 VGPRs, 4.17 ms).
// dK/dV with 16x16x32 MFMAs: one workgroup = 8 waves x 16 keys (128 keys of
// one (batch, q-head)), so a wave holds dK^T / dV^T of its keys in 64
// registers (32x32 tiles need 128) and two waves share each SIMD - the
// 32-key kernel above runs one wave per SIMD and leaves the matrix core idle
// through its exp / pack / LDS phases.  Per 32-query k-step:
//   S  = Q.K^T, dP = dO.V^T    (A: Q / dO rows, ds_read_b128; B: K / V in registers)
//   P  = exp2(c S'), dS = P dP' (accumulators pre-loaded with -LSE/scale, -delta)
//   dV^T += dO^T.P, dK^T += Q^T.dS  (A: transposed reads of the same images;
//   B: two 16x16 accumulator tiles = 8 consecutive-by-4 queries per lane)
// Q / dO image: 256-B rows, chunk c of row r at c ^ 2(r & 7) - conflict-free
// for the 16x16x32 row reads and the transposed reads (tests/test_attention_layout.py).
namespace {
__device__ __forceinline__ int swz16(int row, int ch) {
  return row * 256 + ((ch ^ (2 * (row & 7))) << 4);
}
__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8_t pack2x4(const f32x4_t& lo, const f32x4_t& hi) {
  bf16x8_t o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = static_cast<short>(mxk::f2bf(lo[j]));
    o[4 + j] = static_cast<short>(mxk::f2bf(hi[j]));
  }
  return o;
}
constexpr int NT16 = 512;
}  // namespace

// GQA: one workgroup per (batch, KV head, key block) walks every query head
// of the group, so dK^T / dV^T of its keys accumulate in registers over the
// whole group and are written once, in bf16, straight into dk / dv (token
// strides dk_tok / dv_tok).  Without it, one workgroup per query head writes
// fp32 partials that mxk_attn_bwd_gqa_reduce_kernel sums (4x the grid,
// ~1.1 GB more HBM traffic per Llama-3-8B layer at B = 8).
// DMA: Q / dO slices by LDS-DMA (wave w moves the 1-KiB pieces 2w, 2w + 1 of
// each), as in the dQ kernel; the lse / delta rows stay register-staged.
template <bool CAUSAL, bool GQA = false, bool DMA = false, bool PIPE = false>
__global__ void __launch_bounds__(NT16, 1)
mxk_attn_bwd_dkdv16_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                           const uint16_t* __restrict__ v, const uint16_t* __restrict__ dout,
                           const float* __restrict__ lse, const float* __restrict__ delta,
                           float* __restrict__ dk_p, float* __restrict__ dv_p, int S, int Hq,
                           int Hkv, long q_tok, long k_tok, long v_tok, float scale,
                           uint16_t* __restrict__ dk = nullptr, uint16_t* __restrict__ dv = nullptr,
                           long dk_tok = 0, long dv_tok = 0) {
  __shared__ __attribute__((aligned(16))) char smem[2][2 * BQB * 256];   // [buf][Q | dO]
  __shared__ __attribute__((aligned(16))) float srow[2][2][BQB];       // [buf][-lse/scale | -delta]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c16 = lane & 15;
  const int G = lane >> 4;

  const int nkb = S / BQ;
  int bh, kb;
  {
    int qbi;
    map_block(blockIdx.x, gridDim.x / nkb, nkb, CAUSAL, &bh, &qbi);
    kb = CAUSAL ? nkb - 1 - qbi : qbi;
  }
  const int grp = Hq / Hkv;
  const int b = GQA ? bh / Hkv : bh / Hq;
  const int hq0 = GQA ? (bh % Hkv) * grp : bh % Hq;
  const int hkv = GQA ? bh % Hkv : hq0 / grp;
  const int k0 = kb * BQ;
  const int kw0 = k0 + wave * 16;
  const int mykey = kw0 + c16;
  const uint16_t* kb_ptr = k + static_cast<long>(b) * S * k_tok + static_cast<long>(hkv) * D;
  const uint16_t* vb_ptr = v + static_cast<long>(b) * S * v_tok + static_cast<long>(hkv) * D;

  // B operands of S / dP: lane holds K[mykey][32 s + 8 G .. +7]
  bf16x8_t kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8_t*>(kb_ptr + static_cast<long>(mykey) * k_tok + 32 * s + 8 * G);
    vf[s] = *reinterpret_cast<const bf16x8_t*>(vb_ptr + static_cast<long>(mykey) * v_tok + 32 * s + 8 * G);
  }
  if constexpr (DMA) {
    // wait for the K / V fragments here, before the loops: a compiler wait
    // at their first use inside the slice loop would also wait for the
    // untracked DMA of the next slice
#pragma unroll
    for (int s = 0; s < 4; ++s) asm volatile("" ::"v"(kf[s]), "v"(vf[s]));
  }
  const float c = scale * 1.4426950408889634f;
  const float inv_c = 1.f / c;

  f32x4_t dka[8], dva[8];
#pragma unroll
  for (int db = 0; db < 8; ++db) {
    dka[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    dva[db] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  // transposed-read lane constants: row 4G + (i >> 2), column block 4 (i & 3)
  const int tr_row = 4 * G + (c16 >> 2);
  const int tr_chb = (c16 & 3) >> 1;
  const int tr_byte = 8 * (c16 & 1);
  const int q_begin = CAUSAL ? k0 : 0;
  const int nsl = (S - q_begin) / BQB;
  // Work items i = (query slice t, head gq of the group), head-outer, slices
  // ascending from the diagonal; pipelined across head boundaries.  (A
  // slice-outer walk from the last slice down, heads inner, which keeps the
  // key blocks of a group in lockstep on the same Q / dO slice, measured
  // neutral: 1.2417 vs 1.2468 ms per Llama-3-8B layer, profiles/r2_attention.)
  const int ngq = GQA ? grp : 1;
  const int niter = nsl * ngq;
  auto item = [&](int i, int* t, int* gq) {
    *gq = i / nsl;
    *t = i - *gq * nsl;
  };
  const uint16_t* qg_ptr = q + static_cast<long>(b) * S * q_tok + static_cast<long>(hq0) * D;
  const uint16_t* dog_ptr = dout + static_cast<long>(b) * S * Hq * D + static_cast<long>(hq0) * D;
  const float* lse_g = lse + (static_cast<long>(b) * Hq + hq0) * S;
  const float* dl_g = delta + (static_cast<long>(b) * Hq + hq0) * S;
  // loader: 512 threads x 2 chunks per tile (64 rows x 16 chunks)
  const int ld_row = tid >> 4, ld_ch = tid & 15;
  bf16x8_t qst[2], dst[2];
  float rst = 0.f;
  auto load_slice = [&](int i) {
    int t, gq;
    item(i, &t, &gq);
    const long r0 = q_begin + static_cast<long>(t) * BQB + ld_row;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      qst[j] = *reinterpret_cast<const bf16x8_t*>(qg_ptr + (r0 + 32 * j) * q_tok + gq * D + ld_ch * 8);
      dst[j] = *reinterpret_cast<const bf16x8_t*>(dog_ptr + (r0 + 32 * j) * Hq * D + gq * D + ld_ch * 8);
    }
    if (tid < 2 * BQB) {
      const long qi = q_begin + static_cast<long>(t) * BQB + (tid & (BQB - 1));
      rst = tid < BQB ? -lse_g[gq * S + qi] * 1.4426950408889634f * inv_c : -dl_g[gq * S + qi];
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int off = swz16(ld_row + 32 * j, ld_ch);
      *reinterpret_cast<bf16x8_t*>(smem[buf] + off) = qst[j];
      *reinterpret_cast<bf16x8_t*>(smem[buf] + BQB * 256 + off) = dst[j];
    }
    if (tid < 2 * BQB) srow[buf][tid / BQB][tid & (BQB - 1)] = rst;
  };
  // raw load at the top, arithmetic at the store: math right after the load
  // would put a vmcnt(0) there, which also waits for the slice DMA just issued
  auto load_row = [&](int i) {
    if (tid < 2 * BQB) {
      int t, gq;
      item(i, &t, &gq);
      const long qi = q_begin + static_cast<long>(t) * BQB + (tid & (BQB - 1));
      rst = (tid < BQB ? lse_g : dl_g)[gq * S + qi];
    }
  };
  auto store_row = [&](int buf) {
    if (tid < 2 * BQB)
      srow[buf][tid / BQB][tid & (BQB - 1)] = tid < BQB ? -rst * 1.4426950408889634f * inv_c : -rst;
  };
  mxk::u32x4 rq{}, rd{};
  uint32_t qvo[2] = {}, dvo[2] = {};
  const uint32_t sm32 = mxk::lds_addr32(&smem[0][0]);
  if constexpr (DMA) {
    // base at the group's first head; head gq is + 2 D gq bytes of soffset
    rq = mxk::make_rsrc(qg_ptr, static_cast<unsigned>(S * q_tok * 2));
    rd = mxk::make_rsrc(dog_ptr, static_cast<unsigned>(static_cast<long>(S) * Hq * D * 2));
    // lane i lands at row 4g + (i >> 4), slot i & 15 = chunk ^ 2 (row & 7)
    const int prow = lane >> 4, pslot = lane & 15;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int r = 4 * (2 * wave + p) + prow;
      const int ch = pslot ^ (2 * (r & 7));
      qvo[p] = static_cast<uint32_t>(r * q_tok * 2 + ch * 16);
      dvo[p] = static_cast<uint32_t>(r * Hq * D * 2 + ch * 16);
    }
  }
  auto issue = [&](int i, int buf) {
    int t, gq;
    item(i, &t, &gq);
    const long row0 = q_begin + static_cast<long>(t) * BQB;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t d = sm32 + buf * (2 * BQB * 256) + (2 * wave + p) * 1024;
      mxk::dma16m(rq, d, qvo[p], static_cast<uint32_t>(row0 * q_tok * 2 + gq * D * 2));
      mxk::dma16m(rd, d + BQB * 256, dvo[p], static_cast<uint32_t>(row0 * Hq * D * 2 + gq * D * 2));
    }
  };
  if constexpr (DMA) {
    issue(0, 0);
    load_row(0);
    vm_wait0();
    store_row(0);
  } else {
    load_slice(0);
    store_slice(0);
  }
  __syncthreads();

  for (int i = 0; i < niter; ++i) {
    const int buf = i & 1;
    if (i + 1 < niter) {
      if constexpr (DMA) {
        issue(i + 1, buf ^ 1);   // buf ^ 1 last read in item i - 1 (barrier-certified)
        load_row(i + 1);
      } else {
        load_slice(i + 1);
      }
    }
    int t, gq_unused;
    item(i, &t, &gq_unused);
    const int qs0 = q_begin + t * BQB;
    if (!CAUSAL || qs0 + BQB - 1 >= kw0) {
      const char* qt = smem[buf];
      const char* dt = smem[buf] + BQB * 256;
      const bool diag = CAUSAL && qs0 < kw0 + 15;
      if constexpr (PIPE) {
        // Explicitly software-pipelined: every LDS operand is read one MFMA
        // group ahead of its use, and sched_barrier fences keep the compiler
        // from re-serialising read -> lgkmcnt(0) -> MFMA per instruction
        // (what it emits for the plain loop below: 64 waits per slice, each
        // exposing a full LDS latency).  The waitcnt pass then counts
        // lgkmcnt down through each group.
        bf16x8_t qa[8], da[8];          // S / dP A operands, [2 s + h]
        float4 l4[2], d4[2];            // -lse / -delta rows of the two halves
        auto read_a = [&](int ks) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int qr = 32 * ks + 16 * h + 4 * G;
            l4[h] = *reinterpret_cast<const float4*>(&srow[buf][0][qr]);
            d4[h] = *reinterpret_cast<const float4*>(&srow[buf][1][qr]);
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int row = 32 * ks + 16 * h + c16;
              qa[2 * s + h] = *reinterpret_cast<const bf16x8_t*>(qt + swz16(row, 4 * s + G));
              da[2 * s + h] = *reinterpret_cast<const bf16x8_t*>(dt + swz16(row, 4 * s + G));
            }
          }
        };
        auto read_b = [&](int ks, int db, bf16x8_t* ao, bf16x8_t* aq) {
          const int row = 32 * ks + tr_row;
          const int ch = 2 * db + tr_chb;
          *ao = cat8(lds_tr_b64(dt + swz16(row, ch) + tr_byte),
                     lds_tr_b64(dt + swz16(row + 16, ch) + tr_byte));
          *aq = cat8(lds_tr_b64(qt + swz16(row, ch) + tr_byte),
                     lds_tr_b64(qt + swz16(row + 16, ch) + tr_byte));
        };
        read_a(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          __builtin_amdgcn_sched_barrier(0);
          f32x4_t st[2], pt[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            st[h] = f32x4_t{l4[h].x, l4[h].y, l4[h].z, l4[h].w};
            pt[h] = f32x4_t{d4[h].x, d4[h].y, d4[h].z, d4[h].w};
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              st[h] = mfma16(qa[2 * s + h], kf[s], st[h]);
              pt[h] = mfma16(da[2 * s + h], vf[s], pt[h]);
            }
          }
          // first half of the dV / dK operands in flight under the exp
          bf16x8_t ob[8], qb[8];
#pragma unroll
          for (int db = 0; db < 4; ++db) read_b(ks, db, &ob[db], &qb[db]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              const f32x2_t x = f32x2_t{st[h][r], st[h][r + 1]} * f32x2_t{c, c};
              st[h][r] = fexp2(x[0]);   // P
              st[h][r + 1] = fexp2(x[1]);
            }
          if (diag) {   // wave-uniform: only diagonal slices pay for the mask
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (mykey > qs0 + 32 * ks + 16 * h + 4 * G + r) st[h][r] = 0.f;
          }
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              const f32x2_t d = f32x2_t{pt[h][r], pt[h][r + 1]} * f32x2_t{st[h][r], st[h][r + 1]};
              pt[h][r] = d[0];   // dS
              pt[h][r + 1] = d[1];
            }
          const bf16x8_t pf = pack2x4(st[0], st[1]);
          const bf16x8_t sf = pack2x4(pt[0], pt[1]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int db = 0; db < 4; ++db) {
            dva[db] = mfma16(ob[db], pf, dva[db]);
            dka[db] = mfma16(qb[db], sf, dka[db]);
            read_b(ks, db + 4, &ob[db + 4], &qb[db + 4]);
            __builtin_amdgcn_sched_barrier(0);
          }
          if (ks == 0) read_a(1);       // next half's S / dP operands under the last MFMAs
#pragma unroll
          for (int db = 4; db < 8; ++db) {
            dva[db] = mfma16(ob[db], pf, dva[db]);
            dka[db] = mfma16(qb[db], sf, dka[db]);
          }
        }
      } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        f32x4_t st[2], pt[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int qr = 32 * ks + 16 * h + 4 * G;
          const float4 l4 = *reinterpret_cast<const float4*>(&srow[buf][0][qr]);
          const float4 d4 = *reinterpret_cast<const float4*>(&srow[buf][1][qr]);
          st[h] = f32x4_t{l4.x, l4.y, l4.z, l4.w};
          pt[h] = f32x4_t{d4.x, d4.y, d4.z, d4.w};
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = 32 * ks + 16 * h + c16;
            st[h] = mfma16(*reinterpret_cast<const bf16x8_t*>(qt + swz16(row, 4 * s + G)), kf[s], st[h]);
            pt[h] = mfma16(*reinterpret_cast<const bf16x8_t*>(dt + swz16(row, 4 * s + G)), vf[s], pt[h]);
          }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float e = fexp2(st[h][r] * c);
            if (diag && mykey > qs0 + 32 * ks + 16 * h + 4 * G + r) e = 0.f;
            st[h][r] = e;                  // P
            pt[h][r] = e * pt[h][r];       // dS
          }
        }
        const bf16x8_t pf = pack2x4(st[0], st[1]);
        const bf16x8_t sf = pack2x4(pt[0], pt[1]);
#pragma unroll
        for (int db = 0; db < 8; ++db) {
          const int row = 32 * ks + tr_row;
          const int ch = 2 * db + tr_chb;
          const bf16x8_t ao = cat8(lds_tr_b64(dt + swz16(row, ch) + tr_byte),
                                   lds_tr_b64(dt + swz16(row + 16, ch) + tr_byte));
          const bf16x8_t aq = cat8(lds_tr_b64(qt + swz16(row, ch) + tr_byte),
                                   lds_tr_b64(qt + swz16(row + 16, ch) + tr_byte));
          dva[db] = mfma16(ao, pf, dva[db]);
          dka[db] = mfma16(aq, sf, dka[db]);
        }
      }
      }
    }
    if constexpr (DMA) {
      vm_wait0();   // own pieces of item i+1
      if (i + 1 < niter) store_row(buf ^ 1);
    } else {
      if (i + 1 < niter) store_slice(buf ^ 1);
    }
    __syncthreads();
  }
  // lane = key, registers r: d = 16 db + 4 G + r
  if constexpr (GQA) {
    uint16_t* dkr = dk + (static_cast<long>(b) * S + mykey) * dk_tok + static_cast<long>(hkv) * D;
    uint16_t* dvr = dv + (static_cast<long>(b) * S + mykey) * dv_tok + static_cast<long>(hkv) * D;
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const int d = 16 * db + 4 * G;
      uint2 pk;
      pk.x = mxk::pack2bf(dka[db][0] * scale, dka[db][1] * scale);
      pk.y = mxk::pack2bf(dka[db][2] * scale, dka[db][3] * scale);
      *reinterpret_cast<uint2*>(dkr + d) = pk;
      pk.x = mxk::pack2bf(dva[db][0], dva[db][1]);
      pk.y = mxk::pack2bf(dva[db][2], dva[db][3]);
      *reinterpret_cast<uint2*>(dvr + d) = pk;
    }
  } else {
    const long prow = ((static_cast<long>(b) * S + mykey) * Hq + hq0) * D;
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const int d = 16 * db + 4 * G;
      *reinterpret_cast<float4*>(dk_p + prow + d) =
          make_float4(dka[db][0] * scale, dka[db][1] * scale, dka[db][2] * scale,
                      dka[db][3] * scale);
      *reinterpret_cast<float4*>(dv_p + prow + d) =
          make_float4(dva[db][0], dva[db][1], dva[db][2], dva[db][3]);
    }
  }
}

// dk[b][s][hkv][:] = sum over the group's q-heads of dk_p[b][s][hq][:] (bf16 out)
__global__ void __launch_bounds__(256)
mxk_attn_bwd_gqa_reduce_kernel(const float* __restrict__ dk_p, const float* __restrict__ dv_p,
                               uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, long n_out,
                               int Hq, int Hkv, long dk_tok, long dv_tok) {
  const long i = (static_cast<long>(blockIdx.x) * 256 + threadIdx.x) * 4;   // 4 dims per thread
  if (i >= n_out) return;
  const int grp = Hq / Hkv;
  const int d = static_cast<int>(i % D);
  const long t = i / D;               // (b*S + s)*Hkv + hkv
  const int hkv = static_cast<int>(t % Hkv);
  const long bs = t / Hkv;
  float4 ak = make_float4(0.f, 0.f, 0.f, 0.f), av = ak;
  for (int gq = 0; gq < grp; ++gq) {
    const long src = (bs * Hq + hkv * grp + gq) * D + d;
    const float4 x = *reinterpret_cast<const float4*>(dk_p + src);
    const float4 y = *reinterpret_cast<const float4*>(dv_p + src);
    ak.x += x.x; ak.y += x.y; ak.z += x.z; ak.w += x.w;
    av.x += y.x; av.y += y.y; av.z += y.z; av.w += y.w;
  }
  uint2 pk;
  pk.x = mxk::pack2bf(ak.x, ak.y);
  pk.y = mxk::pack2bf(ak.z, ak.w);
  *reinterpret_cast<uint2*>(dk + bs * dk_tok + hkv * D + d) = pk;
  pk.x = mxk::pack2bf(av.x, av.y);
  pk.y = mxk::pack2bf(av.z, av.w);
  *reinterpret_cast<uint2*>(dv + bs * dv_tok + hkv * D + d) = pk;
}

// Workspace: delta [B*Hq*S] fp32 (+ dk/dv partials 2 x [B*S*Hq*128] fp32 for
// variant 0, the per-query-head dK/dV kernel).
MXK_API long mxk_attn_bwd_workspace_variant(int B, int S, int Hq, int variant) {
  const long rows = static_cast<long>(B) * Hq * S;
  if (variant == 6 || variant == 9) return rows * 8;   // {-lse/scale, -delta} row pairs
  if (variant == 7 || variant == 8) return mxk_attn_bwd_onepass_workspace(B, S, Hq, variant == 8);
  return rows * 4 + (variant == 0 ? 2 * rows * D * 4 : 0);
}
// Backward variant 9 with the rotary-embedding backward fused into the dQ
// and dK stores: q / k are the ROTATED projections the forward ran on, and
// dq / dk come out as gradients of the un-rotated ones (rcos / rsin: the
// forward's [S][D/2] fp32 tables), so the fused-QKV projection's backward
// takes d(QKV) straight from here (dq / dk / dv at token strides, e.g.
// slices of one buffer).  Workspace: mxk_attn_bwd_workspace_variant(.., 9).
// hipErrorInvalidValue when variant 9 does not take the layout (the caller
// then runs mxk_attn_bwd_variant and the stand-alone RoPE pass).
MXK_API int mxk_attn_bwd_rope(const void* q, const void* k, const void* v, const void* o,
                              const void* dout, const float* lse, void* dq, void* dk, void* dv,
                              void* workspace, int B, int S, int Hq, int Hkv, int head_dim,
                              long q_tok, long k_tok, long v_tok, long dq_tok, long dk_tok,
                              long dv_tok, const float* rcos, const float* rsin, float scale,
                              int causal, hipStream_t stream) {
  if (head_dim != D || B < 1 || S < 256 || S % 256 || Hkv < 1 || Hq % Hkv || (Hq / Hkv) % 4 ||
      !workspace || !rcos || !rsin ||
      static_cast<long>(S) * (q_tok > static_cast<long>(Hq) * D ? q_tok : Hq * D) * 2 >= (1L << 32))
    return static_cast<int>(hipErrorInvalidValue);
  float* rowc = static_cast<float*>(workspace);
  const int st = mxk_attn_bwd_dq256_rope(q, k, v, o, dout, lse, dq, rowc, B, S, Hq, Hkv, q_tok,
                                         k_tok, v_tok, dq_tok, rcos, rsin, scale, causal, stream);
  if (st) return st;
  return mxk_attn_bwd_dkdv256_rope(q, k, v, dout, rowc, dk, dv, B, S, Hq, Hkv, q_tok, k_tok, v_tok,
                                   dk_tok, dv_tok, rcos, rsin, scale, causal, stream);
}
MXK_API long mxk_attn_bwd_workspace(int B, int S, int Hq) {
  return mxk_attn_bwd_workspace_variant(B, S, Hq, 0);
}

// variant 1: dK/dV per (batch, KV head, key block) over the whole query-head
// group, bf16 out; 2: variant 1 with LDS-DMA tile loads in the dQ and dK/dV
// kernels (register-staged when a panel exceeds the 32-bit buffer range);
// 3: variant 2 with the explicitly software-pipelined (PIPE) dK/dV and dQ
// bodies, bit-identical to 2 (default; 1.262 -> 1.070 ms per Llama-3-8B
// layer, profiles/r2_attention/); 4: 3 with the dQ loop unrolled by two
// (compile-time LDS buffer), bit-identical and within noise (1.1487 vs
// 1.1525 ms); 0: per query head + fp32 partials + GQA reduce.
MXK_API int mxk_attn_bwd_variant(const void* q, const void* k, const void* v, const void* o,
                                 const void* dout, const float* lse, void* dq, void* dk, void* dv,
                                 void* workspace, int B, int S, int Hq, int Hkv, int head_dim,
                                 long q_tok, long k_tok, long v_tok, long dk_tok, long dv_tok,
                                 float scale, int causal, int variant, hipStream_t stream) {
  if (head_dim != D || B < 1 || S < BQ || S % BQ || Hkv < 1 || Hq % Hkv || q_tok % 8 ||
      k_tok % 8 || v_tok % 8 || dk_tok % 4 || dv_tok % 4 || variant < 0 || variant > 9 ||
      (reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
       reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o) |
       reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dq) |
       reinterpret_cast<uintptr_t>(workspace)) % 16 ||
      (reinterpret_cast<uintptr_t>(dk) | reinterpret_cast<uintptr_t>(dv)) % 8)
    return static_cast<int>(hipErrorInvalidValue);
  const long rows = static_cast<long>(B) * Hq * S;
  float* delta = static_cast<float*>(workspace);
  float* dk_p = variant == 0 ? delta + rows : nullptr;
  float* dv_p = variant == 0 ? dk_p + rows * D : nullptr;
  const auto* Q = static_cast<const uint16_t*>(q);
  const auto* K = static_cast<const uint16_t*>(k);
  const auto* V = static_cast<const uint16_t*>(v);
  const auto* dO = static_cast<const uint16_t*>(dout);
  auto* dK = static_cast<uint16_t*>(dk);
  auto* dV = static_cast<uint16_t*>(dv);
  const int nwg = B * Hq * (S / BQ);
  const long span0 = static_cast<long>(S) * (k_tok > v_tok ? k_tok : v_tok) * 2;
  // the one-pass kernel's own layout limits (32-bit buffer ranges of the Q,
  // K and dQ panels): outside them variants 7 / 8 degrade to variant 5, as
  // variant 6 does, instead of failing
  const bool onepass_ok = S % 256 == 0 && static_cast<long>(S) * q_tok * 2 < (1L << 32) &&
                          static_cast<long>(S) * k_tok * 2 < (1L << 32) &&
                          static_cast<long>(S) * Hq * D * 2 < (1L << 32);
  if ((variant == 7 || variant == 8) && onepass_ok) {
    // one pass (attention_bwd256.hip): dQ by fp32 (7) or packed-bf16 (8)
    // atomics from the 256-key workgroups; not bit-reproducible
    return mxk_attn_bwd_onepass(q, k, v, o, dout, lse, dq, dk, dv, workspace, B, S, Hq, Hkv, q_tok,
                                k_tok, v_tok, dk_tok, dv_tok, scale, causal, variant == 8, stream);
  }
  if (variant == 7 || variant == 8) variant = 5;
  if (variant == 9) {
    // dQ by 4-head x 64-row workgroups, one wave per SIMD (attention_dq256.hip,
    // rowc pairs folded in), then the 256-key dK / dV; a layout either kernel
    // does not take (Hq / Hkv not a multiple of 4, S % 256, 32-bit buffer
    // ranges) runs variant 6
    const long qspan9 = static_cast<long>(S) * (q_tok > static_cast<long>(Hq) * D ? q_tok : Hq * D) * 2;
    if (S % 256 == 0 && (Hq / Hkv) % 4 == 0 && span0 < (1L << 32) && qspan9 < (1L << 32)) {
      float* rowc = static_cast<float*>(workspace);
      const int st = mxk_attn_bwd_dq256(q, k, v, o, dout, lse, dq, rowc, B, S, Hq, Hkv, q_tok, k_tok,
                                        v_tok, scale, causal, stream);
      if (st) return st;
      return mxk_attn_bwd_dkdv256(q, k, v, dout, rowc, dk, dv, B, S, Hq, Hkv, q_tok, k_tok, v_tok,
                                  dk_tok, dv_tok, scale, causal, stream);
    }
    variant = 6;
  }
  if (variant == 6) {
    // dQ with the delta pass folded in, writing {-lse/scale, -delta} rows,
    // then dK / dV with 256 keys per workgroup (attention_bwd256.hip)
    const long qspan6 = static_cast<long>(S) * (q_tok > static_cast<long>(Hq) * D ? q_tok : Hq * D) * 2;
    if (S % 256 == 0 && span0 < (1L << 32) && qspan6 < (1L << 32)) {
      float* rowc = static_cast<float*>(workspace);
      auto* dQ6 = static_cast<uint16_t*>(dq);
      const auto* O6 = static_cast<const uint16_t*>(o);
      if (causal)
        hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<true, true, true, false, true, true>), dim3(nwg),
                           dim3(NT), 0, stream, Q, K, V, dO, lse, nullptr, dQ6, S, Hq, Hkv, q_tok,
                           k_tok, v_tok, scale, O6, rowc);
      else
        hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<false, true, true, false, true, true>),
                           dim3(nwg), dim3(NT), 0, stream, Q, K, V, dO, lse, nullptr, dQ6, S, Hq,
                           Hkv, q_tok, k_tok, v_tok, scale, O6, rowc);
      const int st = static_cast<int>(hipGetLastError());
      if (st) return st;
      return mxk_attn_bwd_dkdv256(q, k, v, dout, rowc, dk, dv, B, S, Hq, Hkv, q_tok, k_tok, v_tok,
                                  dk_tok, dv_tok, scale, causal, stream);
    }
    variant = 5;   // layout the 256-key kernel does not take
  }
  if (variant == 5 && span0 < (1L << 32)) {
    // delta folded into the dQ kernel, which therefore runs first; its
    // read-only `delta` argument is null (FOLD writes delta_w, never reads
    // delta: passing the same buffer as both __restrict__ pointers would be
    // undefined behaviour the day the kernel reads it)
    auto* dQ5 = static_cast<uint16_t*>(dq);
    const auto* O5 = static_cast<const uint16_t*>(o);
    if (causal)
      hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<true, true, true, false, true>), dim3(nwg), dim3(NT),
                         0, stream, Q, K, V, dO, lse, nullptr, dQ5, S, Hq, Hkv, q_tok, k_tok, v_tok,
                         scale, O5, delta);
    else
      hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<false, true, true, false, true>), dim3(nwg),
                         dim3(NT), 0, stream, Q, K, V, dO, lse, nullptr, dQ5, S, Hq, Hkv, q_tok, k_tok,
                         v_tok, scale, O5, delta);
  } else {
    hipLaunchKernelGGL(mxk_attn_bwd_delta_kernel, dim3((rows * 16 + 255) / 256), dim3(256), 0,
                       stream, static_cast<const uint16_t*>(o), dO, delta, S, Hq, rows);
  }
  const int nwg_kv = B * Hkv * (S / BQ);
  const long qspan = static_cast<long>(S) * (q_tok > static_cast<long>(Hq) * D ? q_tok : Hq * D) * 2;
  if (variant >= 3 && causal && qspan < (1L << 32)) {
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<true, true, true, true>), dim3(nwg_kv),
                       dim3(NT16), 0, stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok,
                       k_tok, v_tok, scale, dK, dV, dk_tok, dv_tok);
  } else if (variant >= 3 && qspan < (1L << 32)) {
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<false, true, true, true>), dim3(nwg_kv),
                       dim3(NT16), 0, stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok,
                       k_tok, v_tok, scale, dK, dV, dk_tok, dv_tok);
  } else if (variant == 2 && causal && qspan < (1L << 32)) {
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<true, true, true>), dim3(nwg_kv), dim3(NT16), 0,
                       stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok, k_tok,
                       v_tok, scale, dK, dV, dk_tok, dv_tok);
  } else if (variant >= 2 && qspan < (1L << 32)) {
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<false, true, true>), dim3(nwg_kv), dim3(NT16),
                       0, stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok, k_tok,
                       v_tok, scale, dK, dV, dk_tok, dv_tok);
  } else if (variant >= 1) {
    if (causal)
      hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<true, true>), dim3(nwg_kv), dim3(NT16), 0,
                         stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok, k_tok,
                         v_tok, scale, dK, dV, dk_tok, dv_tok);
    else
      hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<false, true>), dim3(nwg_kv), dim3(NT16), 0,
                         stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok, k_tok,
                         v_tok, scale, dK, dV, dk_tok, dv_tok);
  } else if (causal) {
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<true, false>), dim3(nwg), dim3(NT16), 0, stream,
                       Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok, k_tok, v_tok, scale,
                       nullptr, nullptr, 0L, 0L);
  } else {
    hipLaunchKernelGGL((mxk_attn_bwd_dkdv16_kernel<false, false>), dim3(nwg), dim3(NT16), 0,
                       stream, Q, K, V, dO, lse, delta, dk_p, dv_p, S, Hq, Hkv, q_tok, k_tok,
                       v_tok, scale, nullptr, nullptr, 0L, 0L);
  }
  const long span = static_cast<long>(S) * (k_tok > v_tok ? k_tok : v_tok) * 2;
  const bool dq_dma = variant >= 2 && span < (1L << 32);
  auto* dQ = static_cast<uint16_t*>(dq);
  if (variant == 5 && dq_dma) {
    // dQ already done (with delta) above
  } else if (causal && dq_dma && variant == 4)
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<true, true, true, true>), dim3(nwg), dim3(NT), 0,
                       stream, Q, K, V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else if (causal && dq_dma && variant == 3)
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<true, true, true>), dim3(nwg), dim3(NT), 0, stream,
                       Q, K, V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else if (dq_dma && variant >= 3)
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<false, true, true>), dim3(nwg), dim3(NT), 0, stream,
                       Q, K, V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else if (causal && dq_dma)
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<true, true>), dim3(nwg), dim3(NT), 0, stream, Q, K,
                       V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else if (causal)
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<true, false>), dim3(nwg), dim3(NT), 0, stream, Q, K,
                       V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else if (dq_dma)
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<false, true>), dim3(nwg), dim3(NT), 0, stream, Q, K,
                       V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  else
    hipLaunchKernelGGL((mxk_attn_bwd_dq_kernel<false, false>), dim3(nwg), dim3(NT), 0, stream, Q,
                       K, V, dO, lse, delta, dQ, S, Hq, Hkv, q_tok, k_tok, v_tok, scale);
  if (variant == 0) {
    const long n_out = static_cast<long>(B) * S * Hkv * D;
    hipLaunchKernelGGL(mxk_attn_bwd_gqa_reduce_kernel, dim3((n_out / 4 + 255) / 256), dim3(256), 0,
                       stream, dk_p, dv_p, dK, dV, n_out, Hq, Hkv, dk_tok, dv_tok);
  }
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                         const void* dout, const float* lse, void* dq, void* dk, void* dv,
                         void* workspace, int B, int S, int Hq, int Hkv, int head_dim, long q_tok,
                         long k_tok, long v_tok, long dk_tok, long dv_tok, float scale, int causal,
                         hipStream_t stream) {
  return mxk_attn_bwd_variant(q, k, v, o, dout, lse, dq, dk, dv, workspace, B, S, Hq, Hkv,
                              head_dim, q_tok, k_tok, v_tok, dk_tok, dv_tok, scale, causal, 0,
                              stream);
}
