// mx-vector-add: the hip-vector-add pod payload (BASELINE config 2).
//
// Unlike the reference's "cuda-vector-add" pod, which only runs nvidia-smi
// (/root/reference/README.md:303-318), this launches a real kernel on the GPU
// the device plugin allocated, checks the result bit-exactly against the host
// and prints one machine-readable line:
//   RESULT {"test":"vectoradd","pass":true,...}
// Exit status 0 iff the check passed.
//
// Device isolation (BASELINE.md:37, "pod sees exactly 1 gfx950 agent"): the
// pod must see exactly the GPUs its amd.com/gpu limit allocated and nothing
// else.  The expected set comes from the flags or, by default, from the
// environment the device plugin's Allocate sets (AMD_GPU_DEVICE_IDS,
// AMD_GPU_ARCH, AMD_GPU_BDFS, AMD_GPU_RENDER_NODES).  A CDI spec that injects
// every render node, or a plugin that hands out the wrong minor, fails here.
//   mx-vector-add [--n 50000] [--check] [--device 0] [--bw-mib 1024]
//                 [--expect-gpus N] [--expect-arch gfx950]
#include <dirent.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <sstream>
#include <string>
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

namespace {

std::vector<std::string> split_csv(const char* s) {
  std::vector<std::string> out;
  if (!s) return out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, ','))
    if (!item.empty()) out.push_back(item);
  return out;
}

// "0000:05:00.0#3" (a compute partition of that device) -> "0000:05:00.0"
std::string norm_bdf(std::string b) {
  b = b.substr(0, b.find('#'));
  for (auto& c : b) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return b;
}

std::string json_list(const std::set<std::string>& v) {
  std::string o = "[";
  for (const auto& x : v) o += (o.size() > 1 ? ",\"" : "\"") + x + "\"";
  return o + "]";
}

// /dev/dri/renderD* visible in this mount namespace
std::set<std::string> render_nodes() {
  std::set<std::string> out;
  if (DIR* d = opendir("/dev/dri")) {
    while (dirent* e = readdir(d))
      if (!std::strncmp(e->d_name, "renderD", 7)) out.insert(std::string("/dev/dri/") + e->d_name);
    closedir(d);
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  long n = 50000;   // the CUDA-samples vectorAdd default the operator validator uses
  int dev = 0;
  long bw_mib = 1024;
  // expected allocation: flags override the Allocate environment
  const auto env_ids = split_csv(std::getenv("AMD_GPU_DEVICE_IDS"));
  int expect_gpus = env_ids.empty() ? -1 : static_cast<int>(std::set<std::string>(env_ids.begin(), env_ids.end()).size());
  std::string expect_arch = std::getenv("AMD_GPU_ARCH") ? std::getenv("AMD_GPU_ARCH") : "";
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--n") && i + 1 < argc) n = std::atol(argv[++i]);
    else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) dev = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--bw-mib") && i + 1 < argc) bw_mib = std::atol(argv[++i]);
    else if (!std::strcmp(argv[i], "--expect-gpus") && i + 1 < argc) expect_gpus = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--expect-arch") && i + 1 < argc) expect_arch = argv[++i];
    else if (!std::strcmp(argv[i], "--check")) {}
    else {
      std::fprintf(stderr, "usage: %s [--n N] [--device D] [--bw-mib M] [--expect-gpus N] "
                   "[--expect-arch gfx950]\n", argv[0]);
      return 2;
    }
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
  // ---- isolation: exactly the allocated GPUs, of the expected arch ----
  std::string arch = prop.gcnArchName;
  arch = arch.substr(0, arch.find(':'));   // "gfx950:sramecc+:xnack-" -> "gfx950"
  std::set<std::string> bdfs;
  for (int d = 0; d < count; ++d) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), d) == hipSuccess) bdfs.insert(norm_bdf(bus));
  }
  std::set<std::string> want_bdfs;
  for (const auto& bdf : split_csv(std::getenv("AMD_GPU_BDFS"))) want_bdfs.insert(norm_bdf(bdf));
  const auto nodes = render_nodes();
  std::set<std::string> want_nodes;
  for (const auto& r : split_csv(std::getenv("AMD_GPU_RENDER_NODES"))) want_nodes.insert(r);
  const bool gpus_ok = expect_gpus < 0 || count == expect_gpus;
  const bool arch_ok = expect_arch.empty() || arch == expect_arch;
  // BDFs: partitions of one device share a BDF, so compare the sets
  const bool bdf_ok = want_bdfs.empty() || bdfs == want_bdfs;
  // render nodes: checked when /dev/dri is mounted the way CDI / DeviceSpecs
  // inject it (one node per allocated GPU or partition)
  const bool render_ok = want_nodes.empty() || nodes == want_nodes;
  const bool isolated = gpus_ok && arch_ok && bdf_ok && render_ok;

  const bool pass = mismatches == 0 && isolated;
  std::printf("RESULT {\"test\":\"vectoradd\",\"pass\":%s,\"n\":%ld,\"mismatches\":%ld,"
              "\"device\":%d,\"visible_gpus\":%d,\"expected_gpus\":%d,\"arch\":\"%s\","
              "\"expected_arch\":\"%s\",\"bdfs\":%s,\"expected_bdfs\":%s,"
              "\"render_nodes\":%s,\"expected_render_nodes\":%s,"
              "\"isolation\":{\"gpus\":%s,\"arch\":%s,\"bdf\":%s,\"render\":%s},"
              "\"cus\":%d,\"hbm_bytes\":%zu,\"stream_GBps\":%.1f}\n",
              pass ? "true" : "false", n, mismatches, dev, count, expect_gpus, arch.c_str(),
              expect_arch.c_str(), json_list(bdfs).c_str(), json_list(want_bdfs).c_str(),
              json_list(nodes).c_str(), json_list(want_nodes).c_str(), gpus_ok ? "true" : "false",
              arch_ok ? "true" : "false", bdf_ok ? "true" : "false", render_ok ? "true" : "false",
              prop.multiProcessorCount, prop.totalGlobalMem, gbps);
  return pass ? 0 : 1;
}
