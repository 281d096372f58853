// mx-allreduce-perf: RCCL all-reduce bus-bandwidth sweep over xGMI (BASELINE config 4).
//
// No rccl-tests binary ships in the image, so this is a from-scratch
// equivalent of `all_reduce_perf -b 8 -e 8G -f 2 -g N`:
//   * single process, N GPUs (ncclCommInitAll over the allocated devices),
//     one ncclGroupStart/End per iteration, out-of-place sum;
//   * or one process per GPU (RANK / WORLD_SIZE / LOCAL_RANK from torchrun;
//     the ncclUniqueId travels through --id-file);
//   * --scaling 1,2,4,8 repeats the sweep on the first n GPUs for each n
//     (the 1/2/4/8 curve of the north star).
// algbw = bytes / t; busbw = algbw * 2 (n-1) / n (n = 1: busbw = 0 by definition).
// Each rank sends (rank+1); the result must be n(n+1)/2 everywhere sampled.
//
//   mx-allreduce-perf [-b 8] [-e 8G] [-f 2] [-g N] [--scaling 1,2,4,8]
//                     [--dtype float|bf16] [--iters 20] [--warmup 5] [--id-file F]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

#define CHECK_HIP(x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)
#define CHECK_NCCL(x)                                                             \
  do {                                                                            \
    ncclResult_t r_ = (x);                                                        \
    if (r_ != ncclSuccess) {                                                      \
      std::fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

size_t parse_size(const char* s) {
  char* end = nullptr;
  double v = std::strtod(s, &end);
  switch (end && *end ? *end : ' ') {
    case 'K': case 'k': v *= 1024.0; break;
    case 'M': case 'm': v *= 1024.0 * 1024.0; break;
    case 'G': case 'g': v *= 1024.0 * 1024.0 * 1024.0; break;
    default: break;
  }
  return static_cast<size_t>(v);
}

std::vector<int> parse_list(const char* s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string x;
  while (std::getline(ss, x, ',')) if (!x.empty()) v.push_back(std::atoi(x.c_str()));
  return v;
}

__global__ void fill_value(void* p, size_t n, float v, int is_bf16) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    if (is_bf16) static_cast<uint16_t*>(p)[i] = static_cast<uint16_t>(__float_as_uint(v) >> 16);
    else static_cast<float*>(p)[i] = v;
  }
}

struct Opts {
  size_t minb = 8, maxb = size_t(1) << 33;
  int factor = 2;
  int ngpus = -1;
  std::vector<int> scaling;
  bool bf16 = false;
  int iters = 20, warmup = 5;
  std::string id_file;
};

float read_elem(const void* dptr, size_t idx, bool bf16) {
  if (bf16) {
    uint16_t h = 0;
    CHECK_HIP(hipMemcpy(&h, static_cast<const uint16_t*>(dptr) + idx, 2, hipMemcpyDeviceToHost));
    uint32_t u = uint32_t(h) << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
  }
  float f = 0;
  CHECK_HIP(hipMemcpy(&f, static_cast<const float*>(dptr) + idx, 4, hipMemcpyDeviceToHost));
  return f;
}

int iters_for(size_t bytes, int base) {
  // keep a point under ~1 s: large messages need fewer iterations
  if (bytes >= (size_t(1) << 31)) return std::max(3, base / 4);
  if (bytes >= (size_t(1) << 29)) return std::max(5, base / 2);
  return base;
}

// -------------------------------------------------------------------------
// single process, n GPUs
// -------------------------------------------------------------------------
bool sweep_single(const Opts& o, int n, double* peak_busbw) {
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  CHECK_NCCL(ncclCommInitAll(comms.data(), n, devs.data()));
  const size_t esz = o.bf16 ? 2 : 4;
  const ncclDataType_t dt = o.bf16 ? ncclBfloat16 : ncclFloat;
  std::vector<void*> sb(n), rb(n);
  std::vector<hipStream_t> st(n);
  for (int g = 0; g < n; ++g) {
    CHECK_HIP(hipSetDevice(g));
    CHECK_HIP(hipStreamCreateWithFlags(&st[g], hipStreamNonBlocking));
    CHECK_HIP(hipMalloc(&sb[g], o.maxb));
    CHECK_HIP(hipMalloc(&rb[g], o.maxb));
    hipLaunchKernelGGL(fill_value, dim3(2048), dim3(256), 0, st[g], sb[g], o.maxb / esz,
                       float(g + 1), int(o.bf16));
  }
  for (int g = 0; g < n; ++g) { CHECK_HIP(hipSetDevice(g)); CHECK_HIP(hipStreamSynchronize(st[g])); }
  const float expect = n * (n + 1) / 2.0f;
  bool ok = true;
  std::printf("# n=%d  %14s %12s %8s %12s %12s %12s %6s\n", n, "bytes", "count", "type",
              "time(us)", "algbw(GB/s)", "busbw(GB/s)", "check");
  for (size_t bytes = o.minb; bytes <= o.maxb; bytes *= o.factor) {
    const size_t count = std::max<size_t>(1, bytes / esz);
    auto launch = [&]() {
      CHECK_NCCL(ncclGroupStart());
      for (int g = 0; g < n; ++g)
        CHECK_NCCL(ncclAllReduce(sb[g], rb[g], count, dt, ncclSum, comms[g], st[g]));
      CHECK_NCCL(ncclGroupEnd());
    };
    auto sync = [&]() {
      for (int g = 0; g < n; ++g) { CHECK_HIP(hipSetDevice(g)); CHECK_HIP(hipStreamSynchronize(st[g])); }
    };
    for (int w = 0; w < o.warmup; ++w) launch();
    sync();
    const int it = iters_for(bytes, o.iters);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < it; ++i) launch();
    sync();
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / it;
    const double algbw = double(count * esz) / t / 1e9;
    const double busbw = n > 1 ? algbw * 2.0 * (n - 1) / n : 0.0;
    bool good = true;
    for (int g = 0; g < n; ++g) {
      CHECK_HIP(hipSetDevice(g));
      good &= read_elem(rb[g], 0, o.bf16) == expect && read_elem(rb[g], count - 1, o.bf16) == expect;
    }
    ok &= good;
    *peak_busbw = std::max(*peak_busbw, busbw);
    std::printf("  n=%d  %14zu %12zu %8s %12.2f %12.2f %12.2f %6s\n", n, count * esz, count,
                o.bf16 ? "bf16" : "float", t * 1e6, algbw, busbw, good ? "ok" : "FAIL");
    std::printf("RESULT {\"test\":\"allreduce\",\"ngpus\":%d,\"bytes\":%zu,\"dtype\":\"%s\","
                "\"op\":\"sum\",\"time_us\":%.3f,\"algbw_GBps\":%.3f,\"busbw_GBps\":%.3f,\"pass\":%s}\n",
                n, count * esz, o.bf16 ? "bf16" : "float", t * 1e6, algbw, busbw,
                good ? "true" : "false");
    std::fflush(stdout);
    if (bytes > o.maxb / o.factor) break;
  }
  for (int g = 0; g < n; ++g) {
    CHECK_HIP(hipSetDevice(g));
    CHECK_HIP(hipFree(sb[g]));
    CHECK_HIP(hipFree(rb[g]));
    CHECK_HIP(hipStreamDestroy(st[g]));
    CHECK_NCCL(ncclCommDestroy(comms[g]));
  }
  return ok;
}

// -------------------------------------------------------------------------
// one process per GPU (torchrun env); unique id through a shared file
// -------------------------------------------------------------------------
bool sweep_multiproc(const Opts& o, int rank, int world, int local) {
  ncclUniqueId id;
  if (o.id_file.empty()) {
    std::fprintf(stderr, "--id-file is required with WORLD_SIZE > 1\n");
    return false;
  }
  if (rank == 0) {
    CHECK_NCCL(ncclGetUniqueId(&id));
    const std::string tmp = o.id_file + ".tmp";
    std::ofstream(tmp, std::ios::binary).write(reinterpret_cast<const char*>(&id), sizeof(id));
    std::rename(tmp.c_str(), o.id_file.c_str());
  } else {
    for (int i = 0;; ++i) {
      std::ifstream f(o.id_file, std::ios::binary);
      if (f && f.read(reinterpret_cast<char*>(&id), sizeof(id))) break;
      if (i > 6000) { std::fprintf(stderr, "timed out waiting for %s\n", o.id_file.c_str()); return false; }
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  CHECK_HIP(hipSetDevice(local));
  ncclComm_t comm;
  CHECK_NCCL(ncclCommInitRank(&comm, world, id, rank));
  const size_t esz = o.bf16 ? 2 : 4;
  const ncclDataType_t dt = o.bf16 ? ncclBfloat16 : ncclFloat;
  void *sb, *rb;
  hipStream_t st;
  CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CHECK_HIP(hipMalloc(&sb, o.maxb));
  CHECK_HIP(hipMalloc(&rb, o.maxb));
  hipLaunchKernelGGL(fill_value, dim3(2048), dim3(256), 0, st, sb, o.maxb / esz, float(rank + 1),
                     int(o.bf16));
  CHECK_HIP(hipStreamSynchronize(st));
  const float expect = world * (world + 1) / 2.0f;
  bool ok = true;
  for (size_t bytes = o.minb; bytes <= o.maxb; bytes *= o.factor) {
    const size_t count = std::max<size_t>(1, bytes / esz);
    for (int w = 0; w < o.warmup; ++w) CHECK_NCCL(ncclAllReduce(sb, rb, count, dt, ncclSum, comm, st));
    CHECK_HIP(hipStreamSynchronize(st));
    const int it = iters_for(bytes, o.iters);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < it; ++i) CHECK_NCCL(ncclAllReduce(sb, rb, count, dt, ncclSum, comm, st));
    CHECK_HIP(hipStreamSynchronize(st));
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / it;
    const bool good = read_elem(rb, 0, o.bf16) == expect && read_elem(rb, count - 1, o.bf16) == expect;
    ok &= good;
    if (rank == 0) {
      const double algbw = double(count * esz) / t / 1e9;
      const double busbw = world > 1 ? algbw * 2.0 * (world - 1) / world : 0.0;
      std::printf("RESULT {\"test\":\"allreduce\",\"ngpus\":%d,\"mode\":\"multiproc\",\"bytes\":%zu,"
                  "\"dtype\":\"%s\",\"op\":\"sum\",\"time_us\":%.3f,\"algbw_GBps\":%.3f,"
                  "\"busbw_GBps\":%.3f,\"pass\":%s}\n",
                  world, count * esz, o.bf16 ? "bf16" : "float", t * 1e6, algbw, busbw,
                  good ? "true" : "false");
      std::fflush(stdout);
    }
    if (bytes > o.maxb / o.factor) break;
  }
  CHECK_HIP(hipFree(sb));
  CHECK_HIP(hipFree(rb));
  CHECK_NCCL(ncclCommDestroy(comm));
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-b") && i + 1 < argc) o.minb = parse_size(argv[++i]);
    else if (!std::strcmp(argv[i], "-e") && i + 1 < argc) o.maxb = parse_size(argv[++i]);
    else if (!std::strcmp(argv[i], "-f") && i + 1 < argc) o.factor = std::max(2, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "-g") && i + 1 < argc) o.ngpus = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--scaling") && i + 1 < argc) o.scaling = parse_list(argv[++i]);
    else if (!std::strcmp(argv[i], "--dtype") && i + 1 < argc) o.bf16 = !std::strcmp(argv[++i], "bf16");
    else if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) o.iters = std::max(1, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--warmup") && i + 1 < argc) o.warmup = std::max(0, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--id-file") && i + 1 < argc) o.id_file = argv[++i];
    else { std::fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
  }
  if (o.minb < 1 || o.maxb < o.minb) { std::fprintf(stderr, "bad size range\n"); return 2; }
  const char* ws = std::getenv("WORLD_SIZE");
  const int world = ws ? std::atoi(ws) : 1;
  if (world > 1) {
    const int rank = std::atoi(std::getenv("RANK") ? std::getenv("RANK") : "0");
    const int local = std::atoi(std::getenv("LOCAL_RANK") ? std::getenv("LOCAL_RANK") : "0");
    return sweep_multiproc(o, rank, world, local) ? 0 : 1;
  }
  int count = 0;
  CHECK_HIP(hipGetDeviceCount(&count));
  if (count == 0) {
    std::printf("RESULT {\"test\":\"allreduce\",\"pass\":false,\"error\":\"no GPU visible\"}\n");
    return 1;
  }
  if (o.scaling.empty()) o.scaling.push_back(o.ngpus > 0 ? o.ngpus : count);
  bool ok = true;
  for (int n : o.scaling) {
    if (n < 1 || n > count) {
      std::printf("RESULT {\"test\":\"allreduce\",\"ngpus\":%d,\"pass\":false,\"skipped\":true,"
                  "\"error\":\"only %d GPU(s) visible\"}\n", n, count);
      continue;
    }
    double peak = 0;
    ok &= sweep_single(o, n, &peak);
    std::printf("RESULT {\"test\":\"allreduce_summary\",\"ngpus\":%d,\"peak_busbw_GBps\":%.3f}\n", n, peak);
  }
  return ok ? 0 : 1;
}
