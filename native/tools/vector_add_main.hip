// mx-vector-add: the hip-vector-add pod payload (BASELINE config 2).
//
// Unlike the reference's "cuda-vector-add" pod, which only runs nvidia-smi
// (/root/reference/README.md:303-318), this launches a real kernel on the GPU
// the device plugin allocated, checks the result bit-exactly against the host
// and prints one machine-readable line:
//   RESULT {"test":"vectoradd","pass":true,...}
// Exit status 0 iff the check passed.
//   mx-vector-add [--n 50000] [--check] [--device 0] [--bw-mib 1024]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

extern "C" int mxk_vector_add_f32(const void* a, const void* b, void* c, long n, hipStream_t s);

#define HIP_OK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("RESULT {\"test\":\"vectoradd\",\"pass\":false,\"error\":\"%s at %s:%d\"}\n", \
                  hipGetErrorString(e_), __FILE__, __LINE__);                       \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

int main(int argc, char** argv) {
  long n = 50000;   // the CUDA-samples vectorAdd default the operator validator uses
  int dev = 0;
  long bw_mib = 1024;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--n") && i + 1 < argc) n = std::atol(argv[++i]);
    else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) dev = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--bw-mib") && i + 1 < argc) bw_mib = std::atol(argv[++i]);
    else if (!std::strcmp(argv[i], "--check")) {}
    else { std::fprintf(stderr, "usage: %s [--n N] [--device D] [--bw-mib M]\n", argv[0]); return 2; }
  }
  int count = 0;
  HIP_OK(hipGetDeviceCount(&count));
  if (count == 0) {
    std::printf("RESULT {\"test\":\"vectoradd\",\"pass\":false,\"error\":\"no GPU visible\"}\n");
    return 1;
  }
  HIP_OK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, dev));

  std::vector<float> a(n), b(n), c(n);
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (long i = 0; i < n; ++i) { a[i] = U(rng); b[i] = U(rng); }
  float *da, *db, *dc;
  HIP_OK(hipMalloc(&da, n * sizeof(float)));
  HIP_OK(hipMalloc(&db, n * sizeof(float)));
  HIP_OK(hipMalloc(&dc, n * sizeof(float)));
  HIP_OK(hipMemcpy(da, a.data(), n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(db, b.data(), n * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(static_cast<hipError_t>(mxk_vector_add_f32(da, db, dc, n, nullptr)));
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(c.data(), dc, n * sizeof(float), hipMemcpyDeviceToHost));
  long mismatches = 0;
  for (long i = 0; i < n; ++i)
    if (c[i] != a[i] + b[i]) ++mismatches;   // bit-exact: same IEEE add on both sides

  // bandwidth on a large buffer (3 x bw_mib MiB moved per launch)
  double gbps = 0;
  if (bw_mib > 0) {
    const long m = bw_mib * (1L << 20) / 4;
    float *x, *y, *z;
    HIP_OK(hipMalloc(&x, m * 4));
    HIP_OK(hipMalloc(&y, m * 4));
    HIP_OK(hipMalloc(&z, m * 4));
    HIP_OK(hipMemset(x, 0, m * 4));
    HIP_OK(hipMemset(y, 0, m * 4));
    for (int w = 0; w < 3; ++w) HIP_OK(static_cast<hipError_t>(mxk_vector_add_f32(x, y, z, m, nullptr)));
    hipEvent_t s, e;
    HIP_OK(hipEventCreate(&s));
    HIP_OK(hipEventCreate(&e));
    const int iters = 20;
    HIP_OK(hipEventRecord(s, nullptr));
    for (int it = 0; it < iters; ++it) HIP_OK(static_cast<hipError_t>(mxk_vector_add_f32(x, y, z, m, nullptr)));
    HIP_OK(hipEventRecord(e, nullptr));
    HIP_OK(hipEventSynchronize(e));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, s, e));
    gbps = 3.0 * m * 4 * iters / (ms * 1e-3) / 1e9;
    HIP_OK(hipFree(x));
    HIP_OK(hipFree(y));
    HIP_OK(hipFree(z));
  }
  HIP_OK(hipFree(da));
  HIP_OK(hipFree(db));
  HIP_OK(hipFree(dc));
  const bool pass = mismatches == 0;
  std::printf("RESULT {\"test\":\"vectoradd\",\"pass\":%s,\"n\":%ld,\"mismatches\":%ld,"
              "\"device\":%d,\"visible_gpus\":%d,\"arch\":\"%s\",\"cus\":%d,"
              "\"hbm_bytes\":%zu,\"stream_GBps\":%.1f}\n",
              pass ? "true" : "false", n, mismatches, dev, count, prop.gcnArchName,
              prop.multiProcessorCount, prop.totalGlobalMem, gbps);
  return pass ? 0 : 1;
}
