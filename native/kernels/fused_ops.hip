// Fused memory-bound ops for the Llama-3 DDP training step (BASELINE config 5):
// RMSNorm fwd/bwd, SwiGLU fwd/bwd, rotary embedding fwd/bwd.
//
// All are HBM-bound: every kernel moves bf16 as 16 B per lane (8 elements),
// keeps statistics in fp32, and fuses what torch eager would split into 3-6
// separate elementwise launches (cdna_hip_programming.md Guideline 13, App. B).
#include "mx_common.h"

namespace {

__device__ __forceinline__ void load8(const uint16_t* p, float (&f)[8]) {
  const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = mxk::bf2f(static_cast<uint16_t>(v[e]));
}
__device__ __forceinline__ void store8(uint16_t* p, const float (&f)[8]) {
  uint4 o;
  o.x = mxk::pack2bf(f[0], f[1]);
  o.y = mxk::pack2bf(f[2], f[3]);
  o.z = mxk::pack2bf(f[4], f[5]);
  o.w = mxk::pack2bf(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = o;
}

// Block-wide sum for 256-thread blocks (4 waves): wave shuffle, then LDS.
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = mxk::wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  const float s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

constexpr int kRowThreads = 256;
constexpr int kChunk = kRowThreads * 8;   // elements covered per pass over a row

}  // namespace

// ---------------------------------------------------------------------------
// RMSNorm:  y = x * rstd * w,  rstd = 1/sqrt(mean(x^2) + eps)   (one row/block)
// ---------------------------------------------------------------------------
// With `delta` != nullptr this is the fused residual step of a pre-norm
// transformer: h = x + delta is written to h_out and normalised in the same
// pass (saves a separate add kernel and a re-read of h).
__global__ void __launch_bounds__(kRowThreads)
mxk_rmsnorm_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ delta,
                       const uint16_t* __restrict__ w, uint16_t* __restrict__ h_out,
                       uint16_t* __restrict__ y, float* __restrict__ rstd_out, int H, float eps) {
  __shared__ float red[4];
  const size_t row = blockIdx.x;
  const uint16_t* xr = x + row * H;
  const uint16_t* dr = delta ? delta + row * H : nullptr;
  uint16_t* hr = h_out ? h_out + row * H : nullptr;
  float ss = 0.f;
  for (int c = threadIdx.x * 8; c < H; c += kChunk) {
    float f[8];
    load8(xr + c, f);
    if (dr) {
      float d[8];
      load8(dr + c, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += d[e];
      store8(hr + c, f);
      // normalise the bf16-rounded h, exactly what a separate add would feed
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = mxk::bf2f(mxk::f2bf(f[e]));
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
  }
  const float rstd = rsqrtf(block_sum256(ss, red) / static_cast<float>(H) + eps);
  if (threadIdx.x == 0 && rstd_out) rstd_out[row] = rstd;
  const uint16_t* src = dr ? hr : xr;
  uint16_t* yr = y + row * H;
  for (int c = threadIdx.x * 8; c < H; c += kChunk) {
    float f[8], g[8];
    load8(src + c, f);   // second read hits L1/L2 (row is 2*H bytes)
    load8(w + c, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = f[e] * rstd * g[e];
    store8(yr + c, f);
  }
}

// dx = rstd * (g - x * rstd^2 * mean(g*x)),  g = dy * w.
// dw partials: each block sums dy * x * rstd over its rows into an fp32 slab
// [gridDim.x][H]; mxk_colsum_kernel folds the slab (no float atomics: the sum
// is deterministic and bitwise reproducible).
__global__ void __launch_bounds__(kRowThreads)
mxk_rmsnorm_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                       const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                       const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
                       float* __restrict__ dw_part, int rows, int H, int rows_per_block) {
  __shared__ float red[4];
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  // dw accumulators: thread owns columns c = tid*8 + p*kChunk, p < H/kChunk.
  constexpr int kMaxPass = 8;   // H <= 16384 keeps dw partial sums in registers
  float dwacc[kMaxPass][8];
#pragma unroll
  for (int p = 0; p < kMaxPass; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) dwacc[p][e] = 0.f;

  for (int r = r0; r < r1; ++r) {
    const size_t off = static_cast<size_t>(r) * H;
    const float rs = rstd[r];
    float dot = 0.f;
    for (int c = threadIdx.x * 8; c < H; c += kChunk) {
      float a[8], b[8], g[8];
      load8(dy + off + c, a);
      load8(x + off + c, b);
      load8(w + c, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) dot += a[e] * g[e] * b[e];
    }
    const float mean_gx = block_sum256(dot, red) / static_cast<float>(H);
    int p = 0;
    for (int c = threadIdx.x * 8; c < H; c += kChunk, ++p) {
      float a[8], b[8], g[8], o[8];
      load8(dy + off + c, a);
      load8(x + off + c, b);
      load8(w + c, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = rs * (a[e] * g[e] - b[e] * rs * rs * mean_gx);
      }
      if (dres) {   // fused residual: gradient flowing around the norm
        float rv[8];
        load8(dres + off + c, rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rv[e];
      }
      store8(dx + off + c, o);
#pragma unroll
      for (int q = 0; q < kMaxPass; ++q)
        if (q == p) {
#pragma unroll
          for (int e = 0; e < 8; ++e) dwacc[q][e] += a[e] * b[e] * rs;
        }
    }
  }
  float* slab = dw_part + static_cast<size_t>(blockIdx.x) * H;
  int p = 0;
  for (int c = threadIdx.x * 8; c < H; c += kChunk, ++p) {
#pragma unroll
    for (int q = 0; q < kMaxPass; ++q)
      if (q == p) {
        float4* s4 = reinterpret_cast<float4*>(slab + c);
        s4[0] = make_float4(dwacc[q][0], dwacc[q][1], dwacc[q][2], dwacc[q][3]);
        s4[1] = make_float4(dwacc[q][4], dwacc[q][5], dwacc[q][6], dwacc[q][7]);
      }
  }
}

// Wave-per-row backward for H = 512 * NC (Llama-3-8B: H 4096, NC 8): a wave
// keeps its row of dy / x (/ dres) in registers, so every byte is read once
// (the block-per-row kernel above reads dy and x twice and pays a block-wide
// __syncthreads reduction per row); the row dot product is a wave reduction.
// Lane l owns columns 8l + 512c (c < NC) and accumulates dw for them over
// the wave's rows; the block's 4 waves fold their dw partials through LDS
// into one fp32 slab row per block (then mxk_colsum_kernel as before).
template <int NC>
__global__ void __launch_bounds__(256)
mxk_rmsnorm_bwd_wave_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                            const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                            const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
                            float* __restrict__ dw_part, int rows) {
  constexpr int H = 512 * NC;
  __shared__ float fold[4][H];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wave;
  const int nw = gridDim.x * 4;
  float wf[NC][8], dwacc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    load8(w + 512 * c + 8 * lane, wf[c]);
#pragma unroll
    for (int e = 0; e < 8; ++e) dwacc[c][e] = 0.f;
  }
  for (int r = gw; r < rows; r += nw) {
    const size_t off = static_cast<size_t>(r) * H + 8 * lane;
    const float rs = rstd[r];
    bf16x8_t gy[NC], gx[NC], gr[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      gy[c] = *reinterpret_cast<const bf16x8_t*>(dy + off + 512 * c);
      gx[c] = *reinterpret_cast<const bf16x8_t*>(x + off + 512 * c);
    }
    // the residual gradient is loaded with dy / x, not after the row's
    // reduction, where its latency would sit on the critical path
    if (dres) {
#pragma unroll
      for (int c = 0; c < NC; ++c) gr[c] = *reinterpret_cast<const bf16x8_t*>(dres + off + 512 * c);
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        dot += mxk::bf2f(static_cast<uint16_t>(gy[c][e])) * wf[c][e] *
               mxk::bf2f(static_cast<uint16_t>(gx[c][e]));
    const float k = mxk::wave_sum(dot) * (rs * rs / static_cast<float>(H));
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = mxk::bf2f(static_cast<uint16_t>(gy[c][e]));
        const float b = mxk::bf2f(static_cast<uint16_t>(gx[c][e]));
        o[e] = rs * (a * wf[c][e] - b * k);
        dwacc[c][e] += a * b * rs;
      }
      if (dres) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += mxk::bf2f(static_cast<uint16_t>(gr[c][e]));
      }
      store8(dx + off + 512 * c, o);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) fold[wave][512 * c + 8 * lane + e] = dwacc[c][e];
  __syncthreads();
  float* slab = dw_part + static_cast<size_t>(blockIdx.x) * H;
  for (int i = threadIdx.x; i < H; i += 256)
    slab[i] = (fold[0][i] + fold[1][i]) + (fold[2][i] + fold[3][i]);
}

// out[c] = sum_b part[b][c]  (fp32 in, bf16 or fp32 out).  A block owns 64
// columns; its 4 waves take every 4th slab row (each wave reads 256
// contiguous bytes per row) and fold through LDS in a fixed order.
__global__ void __launch_bounds__(256)
mxk_colsum_kernel(const float* __restrict__ part, int nb, int H, uint16_t* __restrict__ out_bf16,
                  float* __restrict__ out_f32) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  float s = 0.f;
  if (c < H)
    for (int b = g; b < nb; b += 4) s += part[static_cast<size_t>(b) * H + c];
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < H) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (out_bf16) out_bf16[c] = mxk::f2bf(t);
    if (out_f32) out_f32[c] = t;
  }
}

// ---------------------------------------------------------------------------
// SwiGLU on a fused gate|up projection: gu[row] = [g (F) | u (F)],
//   h = silu(g) * u
// bwd: dg = dh * u * s * (1 + g * (1 - s)),  du = dh * g * s,  s = sigmoid(g)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
mxk_swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ h, long rows,
                      int F) {
  const long nvec = rows * (F / 8);
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  const int vpr = F / 8;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const long r = i / vpr;
    const int c = static_cast<int>(i - r * vpr) * 8;
    const uint16_t* base = gu + r * 2L * F;
    float g[8], u[8], o[8];
    load8(base + c, g);
    load8(base + F + c, u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e] / (1.f + __expf(-g[e])) * u[e];
    store8(h + r * F + c, o);
  }
}

__global__ void __launch_bounds__(256)
mxk_swiglu_bwd_kernel(const uint16_t* __restrict__ gu, const uint16_t* __restrict__ dh,
                      uint16_t* __restrict__ dgu, long rows, int F) {
  const long nvec = rows * (F / 8);
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  const int vpr = F / 8;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const long r = i / vpr;
    const int c = static_cast<int>(i - r * vpr) * 8;
    const uint16_t* base = gu + r * 2L * F;
    float g[8], u[8], d[8], dg[8], du[8];
    load8(base + c, g);
    load8(base + F + c, u);
    load8(dh + r * F + c, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = 1.f / (1.f + __expf(-g[e]));
      du[e] = d[e] * g[e] * s;
      dg[e] = d[e] * u[e] * s * (1.f + g[e] * (1.f - s));
    }
    store8(dgu + r * 2L * F + c, dg);
    store8(dgu + r * 2L * F + F + c, du);
  }
}

// ---------------------------------------------------------------------------
// Rotary embedding (Llama "rotate-half" pairing: i <-> i + D/2), in place or
// out of place.  x: [tokens][heads][D] bf16; cos/sin: [S][D/2] fp32 tables
// precomputed on the host (no device trig: App. B element-wise); position of
// token t is pos_offset + t % S.  sign = -1 applies the inverse rotation
// (the backward of the forward rotation).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
mxk_rope_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                const float* __restrict__ cos_t, const float* __restrict__ sin_t, long tokens,
                int heads, int D, int S, float sign, long x_tok, long y_tok) {
  const int half = D / 2;
  const int vph = half / 8;   // 8-pair vectors per head
  const long nvec = tokens * heads * vph;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const long th = i / vph;             // token*heads + head
    const int p0 = static_cast<int>(i - th * vph) * 8;
    const long tok = th / heads;
    const int hd = static_cast<int>(th - tok * heads);
    const int pos = static_cast<int>(tok % S);
    const uint16_t* xr = x + tok * x_tok + static_cast<long>(hd) * D;
    float a[8], b[8], ca[8], sa[8];
    load8(xr + p0, a);
    load8(xr + half + p0, b);
    const float4* c4 = reinterpret_cast<const float4*>(cos_t + static_cast<size_t>(pos) * half + p0);
    const float4* s4 = reinterpret_cast<const float4*>(sin_t + static_cast<size_t>(pos) * half + p0);
    const float4 c0 = c4[0], c1 = c4[1], s0 = s4[0], s1 = s4[1];
    ca[0] = c0.x; ca[1] = c0.y; ca[2] = c0.z; ca[3] = c0.w;
    ca[4] = c1.x; ca[5] = c1.y; ca[6] = c1.z; ca[7] = c1.w;
    sa[0] = s0.x; sa[1] = s0.y; sa[2] = s0.z; sa[3] = s0.w;
    sa[4] = s1.x; sa[5] = s1.y; sa[6] = s1.z; sa[7] = s1.w;
    float oa[8], ob[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) mxk::rope_pair(a[e], b[e], ca[e], sign * sa[e], oa[e], ob[e]);
    uint16_t* yr = y + tok * y_tok + static_cast<long>(hd) * D;
    store8(yr + p0, oa);
    store8(yr + half + p0, ob);
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
namespace {
inline int grid_cap(long work) {
  long g = (work + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}
inline bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }
}  // namespace

MXK_API int mxk_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int rows, int H,
                            float eps, hipStream_t s) {
  if (rows <= 0) return 0;
  if (H % 8 || !aligned16(x) || !aligned16(w) || !aligned16(y))
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_rmsnorm_fwd_kernel, dim3(rows), dim3(kRowThreads), 0, s,
                     static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(nullptr),
                     static_cast<const uint16_t*>(w), static_cast<uint16_t*>(nullptr),
                     static_cast<uint16_t*>(y), rstd, H, eps);
  MXK_RETURN_LAUNCH_STATUS();
}

// h = x + delta; y = rmsnorm(h) * w   (one pass)
MXK_API int mxk_add_rmsnorm_fwd(const void* x, const void* delta, const void* w, void* h, void* y,
                                float* rstd, int rows, int H, float eps, hipStream_t s) {
  if (rows <= 0) return 0;
  if (H % 8 || !aligned16(x) || !aligned16(delta) || !aligned16(w) || !aligned16(h) ||
      !aligned16(y))
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_rmsnorm_fwd_kernel, dim3(rows), dim3(kRowThreads), 0, s,
                     static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(delta),
                     static_cast<const uint16_t*>(w), static_cast<uint16_t*>(h),
                     static_cast<uint16_t*>(y), rstd, H, eps);
  MXK_RETURN_LAUNCH_STATUS();
}

// Workspace size (bytes) the backward needs for its dw slab.
namespace {
// one block per CU keeps the dw slab small (256 x H fp32) while every CU
// works (512 blocks: +15 % time without the residual gradient, -3 % with it)
constexpr int kBwdBlocks = 256;
}

MXK_API long mxk_rmsnorm_bwd_workspace(int rows, int H) {
  const int nb = rows < kBwdBlocks ? rows : kBwdBlocks;
  return static_cast<long>(nb) * H * 4;
}

// dx = rmsnorm_bwd(dy) [+ dres].  dres (nullable) is the gradient that flows
// around the norm through the residual stream (fused add_rmsnorm backward).
MXK_API int mxk_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                            const void* dres, void* dx, void* dw_bf16, float* dw_f32,
                            float* workspace, int rows, int H, hipStream_t s) {
  if (rows <= 0) return 0;
  if (H % 8 || H > 8 * kChunk || !aligned16(dy) || !aligned16(x) || !aligned16(dx) ||
      (dres && !aligned16(dres)))
    return static_cast<int>(hipErrorInvalidValue);
  const int nb = rows < kBwdBlocks ? rows : kBwdBlocks;
  if ((H == 2048 || H == 4096 || H == 8192) && aligned16(w) && rows >= 4 * nb) {
    auto* a = static_cast<const uint16_t*>(dy);
    auto* b = static_cast<const uint16_t*>(x);
    auto* g = static_cast<const uint16_t*>(w);
    auto* d = static_cast<const uint16_t*>(dres);
    auto* o = static_cast<uint16_t*>(dx);
    if (H == 2048)
      hipLaunchKernelGGL(mxk_rmsnorm_bwd_wave_kernel<4>, dim3(nb), dim3(256), 0, s, a, b, g, rstd, d, o, workspace, rows);
    else if (H == 4096)
      hipLaunchKernelGGL(mxk_rmsnorm_bwd_wave_kernel<8>, dim3(nb), dim3(256), 0, s, a, b, g, rstd, d, o, workspace, rows);
    else
      hipLaunchKernelGGL(mxk_rmsnorm_bwd_wave_kernel<16>, dim3(nb), dim3(256), 0, s, a, b, g, rstd, d, o, workspace, rows);
    hipLaunchKernelGGL(mxk_colsum_kernel, dim3((H + 63) / 64), dim3(256), 0, s, workspace, nb, H,
                       static_cast<uint16_t*>(dw_bf16), dw_f32);
    MXK_RETURN_LAUNCH_STATUS();
  }
  const int rpb = (rows + nb - 1) / nb;
  const int nblocks = (rows + rpb - 1) / rpb;
  hipLaunchKernelGGL(mxk_rmsnorm_bwd_kernel, dim3(nblocks), dim3(kRowThreads), 0, s,
                     static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(x),
                     static_cast<const uint16_t*>(w), rstd, static_cast<const uint16_t*>(dres),
                     static_cast<uint16_t*>(dx), workspace, rows, H, rpb);
  hipLaunchKernelGGL(mxk_colsum_kernel, dim3((H + 63) / 64), dim3(256), 0, s, workspace, nblocks,
                     H, static_cast<uint16_t*>(dw_bf16), dw_f32);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_swiglu_fwd(const void* gu, void* h, long rows, int F, hipStream_t s) {
  if (rows <= 0) return 0;
  if (F % 8 || !aligned16(gu) || !aligned16(h)) return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_swiglu_fwd_kernel, dim3(grid_cap(rows * (F / 8))), dim3(256), 0, s,
                     static_cast<const uint16_t*>(gu), static_cast<uint16_t*>(h), rows, F);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_swiglu_bwd(const void* gu, const void* dh, void* dgu, long rows, int F,
                           hipStream_t s) {
  if (rows <= 0) return 0;
  if (F % 8 || !aligned16(gu) || !aligned16(dh) || !aligned16(dgu))
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_swiglu_bwd_kernel, dim3(grid_cap(rows * (F / 8))), dim3(256), 0, s,
                     static_cast<const uint16_t*>(gu), static_cast<const uint16_t*>(dh),
                     static_cast<uint16_t*>(dgu), rows, F);
  MXK_RETURN_LAUNCH_STATUS();
}

// x / y: [tokens][heads][D] rows at token strides x_tok / y_tok (elements),
// e.g. q or k read straight out of the fused QKV projection output, or the
// gradient written straight into its slice of the fused dQKV buffer.
MXK_API int mxk_rope_strided(const void* x, void* y, const float* cos_t, const float* sin_t,
                             long tokens, int heads, int D, int S, float sign, long x_tok,
                             long y_tok, hipStream_t s) {
  if (tokens <= 0) return 0;
  if (D % 16 || x_tok % 8 || y_tok % 8 || x_tok < static_cast<long>(heads) * D ||
      y_tok < static_cast<long>(heads) * D || !aligned16(x) || !aligned16(y) ||
      !aligned16(cos_t) || !aligned16(sin_t))
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_rope_kernel, dim3(grid_cap(tokens * heads * (D / 16))), dim3(256), 0, s,
                     static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), cos_t, sin_t,
                     tokens, heads, D, S, sign, x_tok, y_tok);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_rope(const void* x, void* y, const float* cos_t, const float* sin_t, long tokens,
                     int heads, int D, int S, float sign, hipStream_t s) {
  const long t = static_cast<long>(heads) * D;
  return mxk_rope_strided(x, y, cos_t, sin_t, tokens, heads, D, S, sign, t, t, s);
}
