// Flat-buffer mixed-precision AdamW + global grad-norm for the DDP trainer.
//
// The trainer (mxk8s/parallel/ddp.py + optim.py) keeps every parameter of
// the model as a view into ONE bf16 buffer and every gradient as a view into
// ONE bf16 buffer (that is also what the bucketed RCCL all-reduce works on),
// with fp32 master weights / exp_avg / exp_avg_sq as flat fp32 buffers.  The
// whole optimizer step is then three launches, all device-side (no host sync):
//   1. sumsq partials of the reduced gradient  (deterministic, no atomics)
//   2. one-block fold -> clip coefficient * 1/world in a device scalar
//   3. fused AdamW: reads g (bf16), master/m/v (fp32); writes master/m/v and
//      the bf16 parameter copy — 28 B/param, one pass, HBM-bound.
// Update rule = torch.optim.AdamW (decoupled weight decay):
//   p *= 1 - lr*wd;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
#include "mx_common.h"

namespace {
constexpr int kThreads = 256;
}

__global__ void __launch_bounds__(kThreads)
mxk_sumsq_bf16_kernel(const uint16_t* __restrict__ g, long n, float* __restrict__ partial) {
  __shared__ float red[kThreads / 64];
  float s = 0.f;
  const long nvec = n / 8;
  const long stride = static_cast<long>(gridDim.x) * kThreads;
  for (long i = static_cast<long>(blockIdx.x) * kThreads + threadIdx.x; i < nvec; i += stride) {
    const bf16x8_t v = reinterpret_cast<const bf16x8_t*>(g)[i];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float f = mxk::bf2f(static_cast<uint16_t>(v[e]));
      s += f * f;
    }
  }
  if (blockIdx.x == 0) {
    const long t = nvec * 8 + threadIdx.x;
    if (t < n) {
      const float f = mxk::bf2f(g[t]);
      s += f * f;
    }
  }
  s = mxk::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// out[0] = scale applied to the summed gradient, out[1] = grad norm (of the
// averaged gradient).  Single block, fixed order -> deterministic.
__global__ void __launch_bounds__(kThreads)
mxk_clip_scale_kernel(const float* __restrict__ partial, int nb, float inv_world, float max_norm,
                      float* __restrict__ out) {
  __shared__ float red[kThreads / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += kThreads) s += partial[i];
  float f = static_cast<float>(s);
  f = mxk::wave_sum(f);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = f;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]) * inv_world;
    float clip = 1.f;
    if (max_norm > 0.f && norm > max_norm) clip = max_norm / (norm + 1e-6f);
    out[0] = inv_world * clip;
    out[1] = norm;
  }
}

// Sharded optimizer (ZeRO-1): each rank folds the sum of squares of ITS
// gradient shard into out[0]; the trainer all-reduces that scalar and
// mxk_scale_from_sumsq_kernel turns the global sum into [scale, norm].
__global__ void __launch_bounds__(kThreads)
mxk_fold_sum_kernel(const float* __restrict__ partial, int nb, float* __restrict__ out) {
  __shared__ float red[kThreads / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += kThreads) s += partial[i];
  float f = mxk::wave_sum(static_cast<float>(s));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = f;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

__global__ void mxk_scale_from_sumsq_kernel(const float* __restrict__ sumsq, float inv_world,
                                            float max_norm, float* __restrict__ out) {
  const float norm = sqrtf(sumsq[0]) * inv_world;
  float clip = 1.f;
  if (max_norm > 0.f && norm > max_norm) clip = max_norm / (norm + 1e-6f);
  out[0] = inv_world * clip;
  out[1] = norm;
}

__global__ void __launch_bounds__(kThreads)
mxk_adamw_bf16_kernel(uint16_t* __restrict__ param, float* __restrict__ master,
                      float* __restrict__ m, float* __restrict__ v,
                      const uint16_t* __restrict__ grad, long n, float lr, float b1, float b2,
                      float eps, float wd, float bc1, float bc2_sqrt,
                      const float* __restrict__ scale_ptr) {
  const float gs = scale_ptr ? scale_ptr[0] : 1.f;
  const float step = lr / bc1;
  const float decay = 1.f - lr * wd;
  const long nvec = n / 8;
  const long stride = static_cast<long>(gridDim.x) * kThreads;
  for (long i = static_cast<long>(blockIdx.x) * kThreads + threadIdx.x; i < nvec; i += stride) {
    const bf16x8_t gv = reinterpret_cast<const bf16x8_t*>(grad)[i];
    float4* p4 = reinterpret_cast<float4*>(master) + 2 * i;
    float4* m4 = reinterpret_cast<float4*>(m) + 2 * i;
    float4* v4 = reinterpret_cast<float4*>(v) + 2 * i;
    float p[8], mm[8], vv[8];
    {
      const float4 a = p4[0], b = p4[1], c = m4[0], d = m4[1], e = v4[0], f = v4[1];
      p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w; p[4] = b.x; p[5] = b.y; p[6] = b.z; p[7] = b.w;
      mm[0] = c.x; mm[1] = c.y; mm[2] = c.z; mm[3] = c.w; mm[4] = d.x; mm[5] = d.y; mm[6] = d.z; mm[7] = d.w;
      vv[0] = e.x; vv[1] = e.y; vv[2] = e.z; vv[3] = e.w; vv[4] = f.x; vv[5] = f.y; vv[6] = f.z; vv[7] = f.w;
    }
    bf16x8_t out;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float g = mxk::bf2f(static_cast<uint16_t>(gv[k])) * gs;
      mm[k] = b1 * mm[k] + (1.f - b1) * g;
      vv[k] = b2 * vv[k] + (1.f - b2) * g * g;
      p[k] = p[k] * decay - step * mm[k] / (sqrtf(vv[k]) / bc2_sqrt + eps);
      out[k] = static_cast<short>(mxk::f2bf(p[k]));
    }
    p4[0] = make_float4(p[0], p[1], p[2], p[3]);
    p4[1] = make_float4(p[4], p[5], p[6], p[7]);
    m4[0] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    m4[1] = make_float4(mm[4], mm[5], mm[6], mm[7]);
    v4[0] = make_float4(vv[0], vv[1], vv[2], vv[3]);
    v4[1] = make_float4(vv[4], vv[5], vv[6], vv[7]);
    reinterpret_cast<bf16x8_t*>(param)[i] = out;
  }
  if (blockIdx.x == 0) {   // tail (n % 8)
    const long t = nvec * 8 + threadIdx.x;
    if (t < n) {
      const float g = mxk::bf2f(grad[t]) * gs;
      m[t] = b1 * m[t] + (1.f - b1) * g;
      v[t] = b2 * v[t] + (1.f - b2) * g * g;
      master[t] = master[t] * decay - step * m[t] / (sqrtf(v[t]) / bc2_sqrt + eps);
      param[t] = mxk::f2bf(master[t]);
    }
  }
}

namespace {
inline int grid_for(long nvec) {
  long g = (nvec + kThreads - 1) / kThreads;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}
inline bool a16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }
}  // namespace

// number of fp32 partials mxk_grad_clip_scale needs as workspace
MXK_API int mxk_sumsq_partials(long n) { return grid_for(n / 8); }

MXK_API int mxk_grad_clip_scale(const void* grad, long n, float* partial_ws, float inv_world,
                                float max_norm, float* out2, hipStream_t s) {
  if (n <= 0 || !a16(grad)) return static_cast<int>(hipErrorInvalidValue);
  const int nb = grid_for(n / 8);
  hipLaunchKernelGGL(mxk_sumsq_bf16_kernel, dim3(nb), dim3(kThreads), 0, s,
                     static_cast<const uint16_t*>(grad), n, partial_ws);
  hipLaunchKernelGGL(mxk_clip_scale_kernel, dim3(1), dim3(kThreads), 0, s, partial_ws, nb,
                     inv_world, max_norm, out2);
  MXK_RETURN_LAUNCH_STATUS();
}

// out_sumsq[0] = sum of g^2 over this (shard of the) gradient.
MXK_API int mxk_grad_sumsq(const void* grad, long n, float* partial_ws, float* out_sumsq,
                           hipStream_t s) {
  if (n <= 0 || !a16(grad)) return static_cast<int>(hipErrorInvalidValue);
  const int nb = grid_for(n / 8);
  hipLaunchKernelGGL(mxk_sumsq_bf16_kernel, dim3(nb), dim3(kThreads), 0, s,
                     static_cast<const uint16_t*>(grad), n, partial_ws);
  hipLaunchKernelGGL(mxk_fold_sum_kernel, dim3(1), dim3(kThreads), 0, s, partial_ws, nb, out_sumsq);
  MXK_RETURN_LAUNCH_STATUS();
}

// out2 = [inv_world * clip, norm] from the GLOBAL sum of squares.
MXK_API int mxk_clip_scale_from_sumsq(const float* sumsq, float inv_world, float max_norm,
                                      float* out2, hipStream_t s) {
  hipLaunchKernelGGL(mxk_scale_from_sumsq_kernel, dim3(1), dim3(1), 0, s, sumsq, inv_world,
                     max_norm, out2);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_adamw_bf16(void* param, float* master, float* m, float* v, const void* grad,
                           long n, float lr, float b1, float b2, float eps, float wd, int step,
                           const float* scale_ptr, hipStream_t s) {
  if (n <= 0) return 0;
  if (!a16(param) || !a16(master) || !a16(m) || !a16(v) || !a16(grad) || step < 1)
    return static_cast<int>(hipErrorInvalidValue);
  const float bc1 = 1.f - powf(b1, static_cast<float>(step));
  const float bc2 = 1.f - powf(b2, static_cast<float>(step));
  hipLaunchKernelGGL(mxk_adamw_bf16_kernel, dim3(grid_for(n / 8)), dim3(kThreads), 0, s,
                     static_cast<uint16_t*>(param), master, m, v,
                     static_cast<const uint16_t*>(grad), n, lr, b1, b2, eps, wd, bc1, sqrtf(bc2),
                     scale_ptr);
  MXK_RETURN_LAUNCH_STATUS();
}
