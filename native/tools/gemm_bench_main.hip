// mx-gemm-bench: standalone CDNA4 bf16 MFMA GEMM validator (BASELINE config 3).
//
// Runs the hand-written kernel (native/kernels/gemm_bf16.hip) on every GPU
// the pod was allocated (one host thread per GPU), on uniform random [-1, 1)
// bf16 operands, checks it against rocBLAS (bf16 in, fp32 compute) and prints
// per GPU and size:
//   RESULT {"test":"gemm","gpu":0,"M":8192,...,"tflops":...,"rel_err":...,"pass":true}
// Protocol: >= warmup_ms of back-to-back launches, then the median of `iters`
// hipEvent-timed launches (BASELINE.md "Measurement protocol").
//   mx-gemm-bench [--sizes 4096,8192,16384] [--iters 50] [--warmup-ms 2000]
//                 [--devices all|0,1] [--no-ref]
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

extern "C" int mxk_gemm_bf16_tn(const void* A, const void* Bt, void* C, int M, int N, int K, int lda,
                                int ldb, int ldc, hipStream_t stream);

namespace {

std::mutex g_print;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess)                                                           \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

__global__ void fill_uniform_bf16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    uint32_t x = static_cast<uint32_t>(i) * 0x9E3779B1u ^ seed;
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    const float u = (x >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f;   // [-1, 1)
    p[i] = static_cast<uint16_t>(__float_as_uint(u) >> 16);
  }
}

__global__ void diff_norms(const uint16_t* c, const uint16_t* r, size_t n, double* out) {
  double d = 0, s = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const float a = __uint_as_float(uint32_t(c[i]) << 16), b = __uint_as_float(uint32_t(r[i]) << 16);
    d += double(a - b) * (a - b);
    s += double(b) * b;
  }
  atomicAdd(&out[0], d);
  atomicAdd(&out[1], s);
}

// JSON has no inf / NaN
std::string json_num(double v) {
  if (!std::isfinite(v)) return "null";
  char b[32];
  std::snprintf(b, sizeof(b), "%.4g", v);
  return b;
}

// fp32 reference of one 256x256 block of C = A * B^T (row-major, K-contiguous
// operands) at (r0, c0), compared with the kernel's bf16 output: max |diff|
// and max |ref| (atomicMax on the float bits: both are non-negative).
__global__ void spot_check(const uint16_t* A, const uint16_t* B, const uint16_t* C, int n, int r0,
                           int c0, unsigned* max_err, unsigned* max_ref) {
  const int r = r0 + blockIdx.x, c = c0 + threadIdx.x;
  const uint16_t* a = A + size_t(r) * n;
  const uint16_t* b = B + size_t(c) * n;
  float acc = 0.f;
  for (int k = 0; k < n; ++k)
    acc = fmaf(__uint_as_float(uint32_t(a[k]) << 16), __uint_as_float(uint32_t(b[k]) << 16), acc);
  const float got = __uint_as_float(uint32_t(C[size_t(r) * n + c]) << 16);
  const float err = fabsf(got - acc);
  atomicMax(max_err, __float_as_uint(err == err ? err : INFINITY));   // NaN -> inf
  atomicMax(max_ref, __float_as_uint(fabsf(acc)));
}

struct Opts {
  std::vector<int> sizes{4096, 8192, 16384};
  int iters = 50;
  int warmup_ms = 2000;
  bool ref = true;
  std::vector<int> devices;
};

bool run_device(int dev, const Opts& o) {
  bool all_ok = true;
  if (hipSetDevice(dev) != hipSuccess) return false;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  rocblas_handle rb = nullptr;
  if (o.ref) {
    rocblas_create_handle(&rb);
    rocblas_set_stream(rb, st);
  }
  for (int n : o.sizes) {
    const size_t elems = size_t(n) * n;
    uint16_t *A, *B, *C, *R = nullptr;
    double* nrm;
    if (hipMalloc(&A, elems * 2) || hipMalloc(&B, elems * 2) || hipMalloc(&C, elems * 2) ||
        hipMalloc(&nrm, 16)) {
      std::lock_guard<std::mutex> lk(g_print);
      std::printf("RESULT {\"test\":\"gemm\",\"gpu\":%d,\"M\":%d,\"pass\":false,\"error\":\"alloc\"}\n", dev, n);
      all_ok = false;
      continue;
    }
    hipLaunchKernelGGL(fill_uniform_bf16, dim3(2048), dim3(256), 0, st, A, elems, 0x1234u + dev);
    hipLaunchKernelGGL(fill_uniform_bf16, dim3(2048), dim3(256), 0, st, B, elems, 0x9876u + dev);
    double rel = -1;
    std::string err_msg;
    // poison C first: a launch that silently did nothing cannot pass
    CK(hipMemsetAsync(C, 0xff, elems * 2, st));
    const char* skip = std::getenv("MXK_GEMM_BENCH_SKIP_KERNEL");   // fault-injection hook
    int launch_st = 0;
    if (!(skip && *skip == '1')) launch_st = mxk_gemm_bf16_tn(A, B, C, n, n, n, n, n, n, st);
    const hipError_t le = hipGetLastError();
    if (launch_st != 0 || le != hipSuccess)
      err_msg = std::string("kernel launch failed: ") +
                hipGetErrorString(launch_st ? static_cast<hipError_t>(launch_st) : le);
    // fp32 spot check of a random 256x256 block
    unsigned* dmax = nullptr;
    unsigned hmax[2] = {0, 0};
    CK(hipMalloc(&dmax, 8));
    CK(hipMemsetAsync(dmax, 0, 8, st));
    const uint32_t h32 = (0x9E3779B1u * uint32_t(n)) ^ (0x85EBCA6Bu * uint32_t(dev + 1));
    const int blocks = n / 256;
    const int r0 = int(h32 % uint32_t(blocks)) * 256, c0 = int((h32 >> 16) % uint32_t(blocks)) * 256;
    hipLaunchKernelGGL(spot_check, dim3(256), dim3(256), 0, st, A, B, C, n, r0, c0, dmax, dmax + 1);
    CK(hipGetLastError());
    CK(hipMemcpyAsync(hmax, dmax, 8, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    CK(hipFree(dmax));
    float max_abs_err, max_ref;
    std::memcpy(&max_abs_err, &hmax[0], 4);
    std::memcpy(&max_ref, &hmax[1], 4);
    const float spot_tol = 0.0078125f * max_ref;   // 2^-7 max|ref|: bf16 output rounding is 2^-8
    const bool spot_ok = max_ref > 0.f && max_abs_err <= spot_tol;
    if (err_msg.empty() && !spot_ok)
      err_msg = max_ref > 0.f ? "fp32 spot check failed" : "fp32 spot check: reference block is zero";
    if (o.ref) {
      CK(hipMalloc(&R, elems * 2));
      const float alpha = 1.f, beta = 0.f;
      // row-major C = A * B^T  ==  column-major C^T = B * A^T  (B^T stored = B row-major)
      const rocblas_status rs = rocblas_gemm_ex(rb, rocblas_operation_transpose, rocblas_operation_none, n, n, n, &alpha,
                      B, rocblas_datatype_bf16_r, n, A, rocblas_datatype_bf16_r, n, &beta, R,
                      rocblas_datatype_bf16_r, n, R, rocblas_datatype_bf16_r, n,
                      rocblas_datatype_f32_r, rocblas_gemm_algo_standard, 0, 0);
      if (rs != rocblas_status_success) {
        std::lock_guard<std::mutex> lk(g_print);
        std::fprintf(stderr, "rocblas_gemm_ex failed: %s\n", rocblas_status_to_string(rs));
        all_ok = false;
      }
      CK(hipMemsetAsync(nrm, 0, 16, st));
      hipLaunchKernelGGL(diff_norms, dim3(1024), dim3(256), 0, st, C, R, elems, nrm);
      double h[2];
      CK(hipMemcpyAsync(h, nrm, 16, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      if (!(h[1] > 0.0)) {
        if (err_msg.empty()) err_msg = "rocBLAS reference norm is 0 (reference did not run)";
        rel = -1;
      } else {
        rel = std::sqrt(h[0] / h[1]);
        if (!(rel == rel) && err_msg.empty()) err_msg = "NaN in the output";
      }
      CK(hipFree(R));
    }
    // warm-up: clocks settle under load on random data
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float spent = 0;
    roctxRangePushA("gemm.warmup");
    while (spent < o.warmup_ms) {
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < 10; ++i) mxk_gemm_bf16_tn(A, B, C, n, n, n, n, n, n, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      spent += ms;
    }
    roctxRangePop();
    std::vector<float> t(o.iters);
    roctxRangePushA("gemm.timed");
    for (int i = 0; i < o.iters; ++i) {
      CK(hipEventRecord(e0, st));
      mxk_gemm_bf16_tn(A, B, C, n, n, n, n, n, n, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t[i], e0, e1));
    }
    roctxRangePop();
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2] * 1e-3;
    const double tflops = 2.0 * n * double(n) * n / med / 1e12;
    const bool pass = err_msg.empty() && (!o.ref || (rel >= 0 && rel < 1e-2));
    all_ok &= pass;
    {
      std::lock_guard<std::mutex> lk(g_print);
      std::printf("RESULT {\"test\":\"gemm\",\"gpu\":%d,\"M\":%d,\"N\":%d,\"K\":%d,\"dtype\":\"bf16\","
                  "\"median_ms\":%.4f,\"min_ms\":%.4f,\"tflops\":%.1f,\"rel_err_vs_rocblas\":%s,"
                  "\"spot_block\":[%d,%d],\"max_abs_err\":%s,\"spot_tolerance\":%.4g,"
                  "\"pass\":%s%s%s%s}\n",
                  dev, n, n, n, med * 1e3, t[0], tflops, json_num(rel).c_str(), r0, c0, json_num(max_abs_err).c_str(),
                  spot_tol,
                  pass ? "true" : "false", err_msg.empty() ? "" : ",\"error\":\"",
                  err_msg.c_str(), err_msg.empty() ? "" : "\"");
      std::fflush(stdout);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(nrm));
  }
  if (rb) rocblas_destroy_handle(rb);
  CK(hipStreamDestroy(st));
  return all_ok;
}

std::vector<int> parse_list(const char* s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string x;
  while (std::getline(ss, x, ',')) if (!x.empty()) v.push_back(std::atoi(x.c_str()));
  return v;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  bool all = true;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--sizes") && i + 1 < argc) o.sizes = parse_list(argv[++i]);
    else if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) o.iters = std::max(1, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--warmup-ms") && i + 1 < argc) o.warmup_ms = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--no-ref")) o.ref = false;
    else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) {
      const char* v = argv[++i];
      if (std::strcmp(v, "all")) { o.devices = parse_list(v); all = false; }
    } else { std::fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
  }
  for (int n : o.sizes)
    if (n <= 0 || n % 256) { std::fprintf(stderr, "sizes must be positive multiples of 256\n"); return 2; }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    std::printf("RESULT {\"test\":\"gemm\",\"pass\":false,\"error\":\"no GPU visible\"}\n");
    return 1;
  }
  if (all) for (int d = 0; d < count; ++d) o.devices.push_back(d);
  std::atomic<bool> ok{true};
  std::vector<std::thread> th;
  for (int d : o.devices) th.emplace_back([&, d] { if (!run_device(d, o)) ok = false; });
  for (auto& t : th) t.join();
  return ok ? 0 : 1;
}
