// Fused softmax cross-entropy over bf16 logits (the Llama-3-8B LM head:
// T = 8192 tokens x V = 128256 vocab per micro-batch of 4).
//
// torch's path materialises fp32 logits ([T, V] x 4 B = 4.2 GB), a
// log-softmax and an fp32 gradient, then casts it back: ~6 passes over
// 2-4 GB per step.  Here:
//   forward : one block per row, one pass: per-thread online (max, sum exp),
//             block fold -> lse; loss = lse - logit[label]   (reads 2 B/elem)
//   backward: dlogit = (exp(logit - lse) - [v == label]) * g, written as bf16
//             IN PLACE over the logits (they are dead after the loss), so the
//             gradient costs no extra buffer                 (read + write)
// Rows whose label is negative (ignore_index) get loss 0 and gradient 0; g is
// a device scalar (grad_output / number of counted rows: no host sync).
#include "mx_common.h"

namespace {
constexpr int XT = 256;

__device__ __forceinline__ void fold_max_sum(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
  m = mn;
}
}  // namespace

__global__ void __launch_bounds__(XT)
mxk_xent_fwd_kernel(const uint16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                    float* __restrict__ loss, float* __restrict__ lse_out, int V, long ld) {
  __shared__ float sm[XT / 64], ss[XT / 64];
  const long row = blockIdx.x;
  const uint16_t* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += XT * 8) {
    const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(x + c);
    float f[8], mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      f[e] = mxk::bf2f(static_cast<uint16_t>(v[e]));
      mx = fmaxf(mx, f[e]);
    }
    const float mn = fmaxf(m, mx);
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(f[e] - mn);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + acc;
    m = mn;
  }
  // wave fold, then the 4 waves through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    fold_max_sum(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { sm[wave] = m; ss[wave] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Sx = ss[0];
#pragma unroll
    for (int w = 1; w < XT / 64; ++w) fold_max_sum(M, Sx, sm[w], ss[w]);
    const float lse = M + __logf(Sx);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    loss[row] = lab < 0 ? 0.f : lse - mxk::bf2f(x[lab]);
  }
}

__global__ void __launch_bounds__(XT)
mxk_xent_bwd_kernel(uint16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                    const float* __restrict__ lse_in, const float* __restrict__ gscale, int V,
                    long ld) {
  const long row = blockIdx.x;
  uint16_t* x = logits + row * ld;
  const int64_t lab = labels[row];
  const float g = lab < 0 ? 0.f : gscale[0];
  const float lse = lse_in[row];
  for (int c = threadIdx.x * 8; c < V; c += XT * 8) {
    bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(x + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float p = __expf(mxk::bf2f(static_cast<uint16_t>(v[e])) - lse);
      if (c + e == lab) p -= 1.f;
      v[e] = static_cast<short>(mxk::f2bf(p * g));
    }
    *reinterpret_cast<bf16x8_t*>(x + c) = v;
  }
}

MXK_API int mxk_xent_fwd(const void* logits, const int64_t* labels, float* loss, float* lse,
                         long rows, int V, long ld, hipStream_t s) {
  if (rows <= 0) return 0;
  if (V % 8 || ld % 8 || reinterpret_cast<uintptr_t>(logits) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_xent_fwd_kernel, dim3(rows), dim3(XT), 0, s,
                     static_cast<const uint16_t*>(logits), labels, loss, lse, V, ld);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_xent_bwd(void* logits, const int64_t* labels, const float* lse,
                         const float* gscale, long rows, int V, long ld, hipStream_t s) {
  if (rows <= 0) return 0;
  if (V % 8 || ld % 8 || reinterpret_cast<uintptr_t>(logits) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_xent_bwd_kernel, dim3(rows), dim3(XT), 0, s,
                     static_cast<uint16_t*>(logits), labels, lse, gscale, V, ld);
  MXK_RETURN_LAUNCH_STATUS();
}
