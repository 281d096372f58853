// HIP vector add — the device-plugin smoke test payload (BASELINE config 2).
//
// The reference's "cuda-vector-add" pod never launches a kernel (it runs
// nvidia-smi on a -base image, /root/reference/README.md:303-318).  Ours does:
// C[i] = A[i] + B[i] in fp32 (bit-exact against the host) and bf16.
//
// Memory-bound: 16 B per lane per access (float4 / 8 x bf16), grid-stride,
// 256-thread blocks (4 wave64), grid capped at 256 CUs x 8 blocks.
#include "mx_common.h"

__global__ void __launch_bounds__(256)
mxk_vector_add_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                          float* __restrict__ c, long n) {
  const long nvec = n / 4;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  const float4* a4 = reinterpret_cast<const float4*>(a);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4* c4 = reinterpret_cast<float4*>(c);
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const float4 x = a4[i], y = b4[i];
    c4[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
  // tail (n % 4 elements), handled by the first threads of block 0
  if (blockIdx.x == 0) {
    const long t = nvec * 4 + threadIdx.x;
    if (t < n) c[t] = a[t] + b[t];
  }
}

__global__ void __launch_bounds__(256)
mxk_vector_add_bf16_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                           uint16_t* __restrict__ c, long n) {
  const long nvec = n / 8;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const bf16x8_t x = reinterpret_cast<const bf16x8_t*>(a)[i];
    const bf16x8_t y = reinterpret_cast<const bf16x8_t*>(b)[i];
    bf16x8_t z;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      z[e] = static_cast<short>(mxk::f2bf(mxk::bf2f(static_cast<uint16_t>(x[e])) +
                                          mxk::bf2f(static_cast<uint16_t>(y[e]))));
    reinterpret_cast<bf16x8_t*>(c)[i] = z;
  }
  if (blockIdx.x == 0) {
    const long t = nvec * 8 + threadIdx.x;
    if (t < n) c[t] = mxk::f2bf(mxk::bf2f(a[t]) + mxk::bf2f(b[t]));
  }
}

namespace {
inline int grid_for(long nvec) {
  long g = (nvec + 255) / 256;
  if (g > 2048) g = 2048;   // 256 CUs x 8 blocks, grid-stride the rest
  if (g < 1) g = 1;
  return static_cast<int>(g);
}
}  // namespace

MXK_API int mxk_vector_add_f32(const void* a, const void* b, void* c, long n, hipStream_t s) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
       reinterpret_cast<uintptr_t>(c)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_vector_add_f32_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s,
                     static_cast<const float*>(a), static_cast<const float*>(b),
                     static_cast<float*>(c), n);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API int mxk_vector_add_bf16(const void* a, const void* b, void* c, long n, hipStream_t s) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
       reinterpret_cast<uintptr_t>(c)) % 16)
    return static_cast<int>(hipErrorInvalidValue);
  hipLaunchKernelGGL(mxk_vector_add_bf16_kernel, dim3(grid_for(n / 8)), dim3(256), 0, s,
                     static_cast<const uint16_t*>(a), static_cast<const uint16_t*>(b),
                     static_cast<uint16_t*>(c), n);
  MXK_RETURN_LAUNCH_STATUS();
}

MXK_API const char* mxk_error_string(int err) {
  return hipGetErrorString(static_cast<hipError_t>(err));
}
