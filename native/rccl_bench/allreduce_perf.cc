// mx-allreduce-perf: RCCL collective bus-bandwidth sweeps over xGMI (BASELINE
// config 4).
//
// No rccl-tests binary ships in the image, so this is a from-scratch
// equivalent of `all_reduce_perf -b 8 -e 8G -f 2 -g N` (and of the
// reduce_scatter / all_gather / alltoall variants the DP/TP/SP/EP paths use):
//   * single process, N GPUs (ncclCommInitAll over the allocated devices),
//     one ncclGroupStart/End per iteration, out-of-place;
//   * or one process per GPU (RANK / WORLD_SIZE / LOCAL_RANK from torchrun;
//     the ncclUniqueId travels through --id-file);
//   * --scaling 1,2,4,8 repeats the sweep on the first n GPUs for each n
//     (the 1/2/4/8 curve of the north star).
//
// Sizes follow the nccl-tests convention: S = bytes of the LARGER per-rank
// buffer (all-reduce: the buffer; reduce-scatter: the input; all-gather: the
// output; all-to-all: the whole send buffer).  algbw = S / t;
//   busbw = algbw * 2 (n-1)/n   (all-reduce)
//   busbw = algbw * (n-1)/n     (reduce-scatter, all-gather, all-to-all)
// (n = 1: busbw = 0 by definition; the RESULT keeps algbw.)
// Correctness: rank r contributes (r+1) everywhere; sums must equal
// n(n+1)/2, gathered / exchanged chunk j must equal j+1 — checked over the
// WHOLE receive buffer by a device kernel that counts mismatches.
// Multi-process: the ncclUniqueId file carries a per-job nonce
// (MXK_RUN_NONCE, else TORCHELASTIC_RUN_ID:MASTER_PORT); rank 0 deletes any
// old file first and the other ranks ignore a file whose nonce is not theirs,
// so a stale id from an earlier run can neither hang nor mis-wire this one.
// Times are max-reduced over ranks (ncclMax) before they are reported.
//
//   mx-allreduce-perf [-b 8] [-e 8G] [-f 2] [-g N] [--scaling 1,2,4,8]
//                     [--op allreduce|reducescatter|allgather|alltoall|all]
//                     [--dtype float|bf16] [--iters 20] [--warmup 5] [--id-file F]
//                     [--nonce S]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

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

#include <unistd.h>

#include "sweep_plan.h"

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

using mxrb::Op;
using mxrb::Shape;
using mxrb::bus_factor;
using mxrb::op_name;

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
  std::vector<Op> ops{Op::AllReduce};
  bool bf16 = false;
  int iters = 20, warmup = 5;
  std::string id_file;
  std::string nonce;
  size_t esz() const { return bf16 ? 2 : 4; }
  ncclDataType_t dt() const { return bf16 ? ncclBfloat16 : ncclFloat; }
};

// Mismatch count over the whole receive buffer: element i must equal `sum`
// (chunk == 0: reductions) or (i / chunk) + 1 (gather / all-to-all).
__global__ void count_mismatch(const void* p, size_t n, size_t chunk, float sum, int is_bf16,
                               unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const float want = chunk ? float(i / chunk + 1) : sum;
    const float got = is_bf16 ? __uint_as_float(uint32_t(static_cast<const uint16_t*>(p)[i]) << 16)
                              : static_cast<const float*>(p)[i];
    local += got != want;
  }
  if (local) atomicAdd(bad, local);
}

unsigned long long mismatches(Op op, const void* rb, size_t recv, size_t count, int n, bool bf16,
                              hipStream_t st) {
  unsigned long long* d = nullptr;
  unsigned long long h = 0;
  CHECK_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(h), st));
  CHECK_HIP(hipMemsetAsync(d, 0, sizeof(h), st));
  const mxrb::CheckParams c = mxrb::check_params(op, Shape{count, 0, recv}, n);
  hipLaunchKernelGGL(count_mismatch, dim3(1024), dim3(256), 0, st, rb, recv, c.chunk, c.sum,
                     int(bf16), d);
  CHECK_HIP(hipGetLastError());
  CHECK_HIP(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipFreeAsync(d, st));
  CHECK_HIP(hipStreamSynchronize(st));
  return h;
}

void issue(Op op, const void* sb, void* rb, const Shape& s, ncclDataType_t dt, ncclComm_t comm,
           hipStream_t st) {
  switch (op) {
    case Op::AllReduce: CHECK_NCCL(ncclAllReduce(sb, rb, s.count, dt, ncclSum, comm, st)); break;
    case Op::ReduceScatter: CHECK_NCCL(ncclReduceScatter(sb, rb, s.count, dt, ncclSum, comm, st)); break;
    case Op::AllGather: CHECK_NCCL(ncclAllGather(sb, rb, s.count, dt, comm, st)); break;
    default: CHECK_NCCL(ncclAllToAll(sb, rb, s.count, dt, comm, st)); break;
  }
}

// Whole-buffer correctness check of one rank's receive buffer.
bool check_recv(Op op, const void* rb, const Shape& s, int n, bool bf16, hipStream_t st) {
  return mismatches(op, rb, s.recv, s.count, n, bf16, st) == 0;
}

void print_point(Op op, int n, const char* mode, size_t bytes, const Opts& o, double t, bool good) {
  const double algbw = double(bytes) / t / 1e9;
  const double busbw = algbw * bus_factor(op, n);
  std::printf("  %-13s n=%d %14zu %8s %12.2f %12.2f %12.2f %6s\n", op_name(op), n, bytes,
              o.bf16 ? "bf16" : "float", t * 1e6, algbw, busbw, good ? "ok" : "FAIL");
  std::printf("RESULT {\"test\":\"%s\",\"ngpus\":%d,\"mode\":\"%s\",\"bytes\":%zu,\"dtype\":\"%s\","
              "\"op\":\"%s\",\"time_us\":%.3f,\"algbw_GBps\":%.3f,\"busbw_GBps\":%.3f,\"pass\":%s}\n",
              op_name(op), n, mode, bytes, o.bf16 ? "bf16" : "float",
              op == Op::AllToAll || op == Op::AllGather ? "copy" : "sum", t * 1e6, algbw, busbw,
              good ? "true" : "false");
  std::fflush(stdout);
}

// -------------------------------------------------------------------------
// single process, n GPUs
// -------------------------------------------------------------------------
bool sweep_single(const Opts& o, Op op, int n, double* peak_busbw) {
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  CHECK_NCCL(ncclCommInitAll(comms.data(), n, devs.data()));
  const size_t esz = o.esz();
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
  bool ok = true;
  std::printf("# %s n=%d  %14s %8s %12s %12s %12s %6s\n", op_name(op), n, "bytes", "type",
              "time(us)", "algbw(GB/s)", "busbw(GB/s)", "check");
  for (const mxrb::Point& pt : mxrb::sweep_points(op, o.minb, o.maxb, o.factor, esz, n, o.iters)) {
    const Shape& s = pt.shape;
    auto launch = [&]() {
      CHECK_NCCL(ncclGroupStart());
      for (int g = 0; g < n; ++g) issue(op, sb[g], rb[g], s, o.dt(), comms[g], st[g]);
      CHECK_NCCL(ncclGroupEnd());
    };
    auto sync = [&]() {
      for (int g = 0; g < n; ++g) { CHECK_HIP(hipSetDevice(g)); CHECK_HIP(hipStreamSynchronize(st[g])); }
    };
    for (int w = 0; w < o.warmup; ++w) launch();
    sync();
    const int it = pt.iters;
    roctxRangePushA(op_name(op));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < it; ++i) launch();
    sync();
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / it;
    roctxRangePop();
    bool good = true;
    for (int g = 0; g < n; ++g) {
      CHECK_HIP(hipSetDevice(g));
      good &= check_recv(op, rb[g], s, n, o.bf16, st[g]);
    }
    ok &= good;
    const size_t sbytes = pt.reported;
    *peak_busbw = std::max(*peak_busbw, double(sbytes) / t / 1e9 * bus_factor(op, n));
    print_point(op, n, "single", sbytes, o, t, good);
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
// Per-job nonce that binds the id file to this launch.
std::string run_nonce() {
  if (const char* n = std::getenv("MXK_RUN_NONCE")) return n;
  const char* run = std::getenv("TORCHELASTIC_RUN_ID");
  const char* port = std::getenv("MASTER_PORT");
  if (!run && !port) return "";
  return std::string(run ? run : "") + ":" + (port ? port : "");
}

constexpr char kIdMagic[8] = {'M', 'X', 'K', 'N', 'C', 'C', 'L', '1'};

// Rank 0 publishes (magic, nonce, id) atomically after removing any old file;
// the other ranks wait for a file whose magic and nonce match.
bool exchange_id(const std::string& path, const std::string& nonce, int rank, ncclUniqueId* id) {
  if (rank == 0) {
    std::remove(path.c_str());
    CHECK_NCCL(ncclGetUniqueId(id));
    const std::string tmp = path + ".tmp." + std::to_string(::getpid());
    {
      std::ofstream f(tmp, std::ios::binary);
      const uint32_t len = static_cast<uint32_t>(nonce.size());
      f.write(kIdMagic, sizeof(kIdMagic));
      f.write(reinterpret_cast<const char*>(&len), sizeof(len));
      f.write(nonce.data(), len);
      f.write(reinterpret_cast<const char*>(id), sizeof(*id));
      if (!f) return false;
    }
    return std::rename(tmp.c_str(), path.c_str()) == 0;
  }
  const char* ws = std::getenv("MXK_ID_WAIT_S");
  const int polls = (ws ? std::max(1, std::atoi(ws)) : 60) * 100;
  for (int i = 0; i <= polls; ++i) {   // 10 ms polls
    std::ifstream f(path, std::ios::binary);
    char magic[8];
    uint32_t len = 0;
    if (f && f.read(magic, 8) && !std::memcmp(magic, kIdMagic, 8) &&
        f.read(reinterpret_cast<char*>(&len), sizeof(len)) && len < 4096) {
      std::string got(len, '\0');
      if (f.read(&got[0], len) && got == nonce &&
          f.read(reinterpret_cast<char*>(id), sizeof(*id)))
        return true;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  std::fprintf(stderr, "rank %d: timed out waiting for %s with nonce '%s'\n", rank, path.c_str(),
               nonce.c_str());
  return false;
}

// Slowest rank's time (every rank gets it).
double max_over_ranks(double t, ncclComm_t comm, hipStream_t st) {
  double* d = nullptr;
  CHECK_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(double), st));
  CHECK_HIP(hipMemcpyAsync(d, &t, sizeof(double), hipMemcpyHostToDevice, st));
  CHECK_NCCL(ncclAllReduce(d, d, 1, ncclFloat64, ncclMax, comm, st));
  CHECK_HIP(hipMemcpyAsync(&t, d, sizeof(double), hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipFreeAsync(d, st));
  CHECK_HIP(hipStreamSynchronize(st));
  return t;
}

bool sweep_multiproc(const Opts& o, int rank, int world, int local) {
  ncclUniqueId id;
  if (o.id_file.empty()) {
    std::fprintf(stderr, "--id-file is required with WORLD_SIZE > 1\n");
    return false;
  }
  const std::string nonce = o.nonce.empty() ? run_nonce() : o.nonce;
  if (nonce.empty()) {
    std::fprintf(stderr, "no job nonce: set MXK_RUN_NONCE (or run under torchrun) or --nonce\n");
    return false;
  }
  if (!exchange_id(o.id_file, nonce, rank, &id)) return false;
  CHECK_HIP(hipSetDevice(local));
  ncclComm_t comm;
  CHECK_NCCL(ncclCommInitRank(&comm, world, id, rank));
  const size_t esz = o.esz();
  void *sb, *rb;
  hipStream_t st;
  CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CHECK_HIP(hipMalloc(&sb, o.maxb));
  CHECK_HIP(hipMalloc(&rb, o.maxb));
  hipLaunchKernelGGL(fill_value, dim3(2048), dim3(256), 0, st, sb, o.maxb / esz, float(rank + 1),
                     int(o.bf16));
  CHECK_HIP(hipStreamSynchronize(st));
  bool ok = true;
  for (Op op : o.ops) {
    double peak = 0;
    for (const mxrb::Point& pt : mxrb::sweep_points(op, o.minb, o.maxb, o.factor, esz, world,
                                                   o.iters)) {
      const Shape& s = pt.shape;
      for (int w = 0; w < o.warmup; ++w) issue(op, sb, rb, s, o.dt(), comm, st);
      CHECK_HIP(hipStreamSynchronize(st));
      const int it = pt.iters;
      roctxRangePushA(op_name(op));
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < it; ++i) issue(op, sb, rb, s, o.dt(), comm, st);
      CHECK_HIP(hipStreamSynchronize(st));
      double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / it;
      roctxRangePop();
      t = max_over_ranks(t, comm, st);
      unsigned long long bad = mismatches(op, rb, s.recv, s.count, world, o.bf16, st);
      // every rank's verdict: total mismatches over the job
      {
        unsigned long long* d = nullptr;
        CHECK_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(bad), st));
        CHECK_HIP(hipMemcpyAsync(d, &bad, sizeof(bad), hipMemcpyHostToDevice, st));
        CHECK_NCCL(ncclAllReduce(d, d, 1, ncclUint64, ncclSum, comm, st));
        CHECK_HIP(hipMemcpyAsync(&bad, d, sizeof(bad), hipMemcpyDeviceToHost, st));
        CHECK_HIP(hipFreeAsync(d, st));
        CHECK_HIP(hipStreamSynchronize(st));
      }
      const bool good = bad == 0;
      ok &= good;
      const size_t sbytes = pt.reported;
      peak = std::max(peak, double(sbytes) / t / 1e9 * bus_factor(op, world));
      if (rank == 0) print_point(op, world, "multiproc", sbytes, o, t, good);
    }
    if (rank == 0)
      std::printf("RESULT {\"test\":\"%s_summary\",\"ngpus\":%d,\"peak_busbw_GBps\":%.3f}\n",
                  op_name(op), world, peak);
  }
  CHECK_HIP(hipFree(sb));
  CHECK_HIP(hipFree(rb));
  CHECK_NCCL(ncclCommDestroy(comm));
  if (rank == 0) std::remove(o.id_file.c_str());
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-b") && i + 1 < argc) o.minb = mxrb::parse_size(argv[++i]);
    else if (!std::strcmp(argv[i], "-e") && i + 1 < argc) o.maxb = mxrb::parse_size(argv[++i]);
    else if (!std::strcmp(argv[i], "-f") && i + 1 < argc) o.factor = std::max(2, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "-g") && i + 1 < argc) o.ngpus = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--scaling") && i + 1 < argc) o.scaling = mxrb::parse_list(argv[++i]);
    else if (!std::strcmp(argv[i], "--dtype") && i + 1 < argc) o.bf16 = !std::strcmp(argv[++i], "bf16");
    else if (!std::strcmp(argv[i], "--iters") && i + 1 < argc) o.iters = std::max(1, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--warmup") && i + 1 < argc) o.warmup = std::max(0, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--id-file") && i + 1 < argc) o.id_file = argv[++i];
    else if (!std::strcmp(argv[i], "--nonce") && i + 1 < argc) o.nonce = argv[++i];
    else if (!std::strcmp(argv[i], "--op") && i + 1 < argc) {
      if (!mxrb::parse_ops(argv[++i], &o.ops)) { std::fprintf(stderr, "bad --op %s\n", argv[i]); return 2; }
    } else { std::fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
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
  for (Op op : o.ops) {
    for (int n : o.scaling) {
      if (n < 1 || n > count) {
        std::printf("RESULT {\"test\":\"%s\",\"ngpus\":%d,\"pass\":false,\"skipped\":true,"
                    "\"error\":\"only %d GPU(s) visible\"}\n", op_name(op), n, count);
        continue;
      }
      double peak = 0;
      ok &= sweep_single(o, op, n, &peak);
      std::printf("RESULT {\"test\":\"%s_summary\",\"ngpus\":%d,\"peak_busbw_GBps\":%.3f}\n",
                  op_name(op), n, peak);
    }
  }
  return ok ? 0 : 1;
}
