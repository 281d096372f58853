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
// n(n+1)/2, gathered / exchanged chunk j must equal j+1.
//
//   mx-allreduce-perf [-b 8] [-e 8G] [-f 2] [-g N] [--scaling 1,2,4,8]
//                     [--op allreduce|reducescatter|allgather|alltoall|all]
//                     [--dtype float|bf16] [--iters 20] [--warmup 5] [--id-file F]
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

enum class Op { AllReduce, ReduceScatter, AllGather, AllToAll };

const char* op_name(Op op) {
  switch (op) {
    case Op::AllReduce: return "allreduce";
    case Op::ReduceScatter: return "reducescatter";
    case Op::AllGather: return "allgather";
    default: return "alltoall";
  }
}

double bus_factor(Op op, int n) {
  if (n <= 1) return 0.0;
  return op == Op::AllReduce ? 2.0 * (n - 1) / n : double(n - 1) / n;
}

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
  std::vector<Op> ops{Op::AllReduce};
  bool bf16 = false;
  int iters = 20, warmup = 5;
  std::string id_file;
  size_t esz() const { return bf16 ? 2 : 4; }
  ncclDataType_t dt() const { return bf16 ? ncclBfloat16 : ncclFloat; }
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

// Element counts of one sweep point: `chunk` = per-peer block, send/recv =
// per-rank buffer elements; `count` is what the RCCL call takes.
struct Shape {
  size_t count, send, recv;
};

Shape shape_for(Op op, size_t bytes, size_t esz, int n) {
  size_t elems = std::max<size_t>(1, bytes / esz);
  if (op == Op::AllReduce) return {elems, elems, elems};
  const size_t chunk = std::max<size_t>(1, elems / n);
  switch (op) {
    case Op::ReduceScatter: return {chunk, chunk * n, chunk};
    case Op::AllGather: return {chunk, chunk, chunk * n};
    default: return {chunk, chunk * n, chunk * n};   // all-to-all: count per pair
  }
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

// Sampled correctness check of one rank's receive buffer.
bool check_recv(Op op, const void* rb, const Shape& s, int n, bool bf16) {
  const float sum = n * (n + 1) / 2.0f;
  if (op == Op::AllReduce || op == Op::ReduceScatter)
    return read_elem(rb, 0, bf16) == sum && read_elem(rb, s.recv - 1, bf16) == sum;
  for (int j = 0; j < n; ++j) {   // chunk j came from rank j, which sent (j+1)
    if (read_elem(rb, j * s.count, bf16) != float(j + 1)) return false;
    if (read_elem(rb, j * s.count + s.count - 1, bf16) != float(j + 1)) return false;
  }
  return true;
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
  for (size_t bytes = o.minb; bytes <= o.maxb; bytes *= o.factor) {
    const Shape s = shape_for(op, bytes, esz, n);
    if (std::max(s.send, s.recv) * esz > o.maxb) continue;   // tiny sizes x many ranks
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
    const int it = iters_for(bytes, o.iters);
    roctxRangePushA(op_name(op));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < it; ++i) launch();
    sync();
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / it;
    roctxRangePop();
    bool good = true;
    for (int g = 0; g < n; ++g) {
      CHECK_HIP(hipSetDevice(g));
      good &= check_recv(op, rb[g], s, n, o.bf16);
    }
    ok &= good;
    const size_t sbytes = std::max(s.send, s.recv) * esz;
    *peak_busbw = std::max(*peak_busbw, double(sbytes) / t / 1e9 * bus_factor(op, n));
    print_point(op, n, "single", sbytes, o, t, good);
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
    for (size_t bytes = o.minb; bytes <= o.maxb; bytes *= o.factor) {
      const Shape s = shape_for(op, bytes, esz, world);
      if (std::max(s.send, s.recv) * esz > o.maxb) continue;
      for (int w = 0; w < o.warmup; ++w) issue(op, sb, rb, s, o.dt(), comm, st);
      CHECK_HIP(hipStreamSynchronize(st));
      const int it = iters_for(bytes, o.iters);
      roctxRangePushA(op_name(op));
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < it; ++i) issue(op, sb, rb, s, o.dt(), comm, st);
      CHECK_HIP(hipStreamSynchronize(st));
      const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / it;
      roctxRangePop();
      const bool good = check_recv(op, rb, s, world, o.bf16);
      ok &= good;
      const size_t sbytes = std::max(s.send, s.recv) * esz;
      peak = std::max(peak, double(sbytes) / t / 1e9 * bus_factor(op, world));
      if (rank == 0) print_point(op, world, "multiproc", sbytes, o, t, good);
      if (bytes > o.maxb / o.factor) break;
    }
    if (rank == 0)
      std::printf("RESULT {\"test\":\"%s_summary\",\"ngpus\":%d,\"peak_busbw_GBps\":%.3f}\n",
                  op_name(op), world, peak);
  }
  CHECK_HIP(hipFree(sb));
  CHECK_HIP(hipFree(rb));
  CHECK_NCCL(ncclCommDestroy(comm));
  return ok;
}

bool parse_ops(const char* s, std::vector<Op>* out) {
  out->clear();
  std::stringstream ss(s);
  std::string x;
  while (std::getline(ss, x, ',')) {
    if (x == "all") {
      *out = {Op::AllReduce, Op::ReduceScatter, Op::AllGather, Op::AllToAll};
      return true;
    }
    if (x == "allreduce") out->push_back(Op::AllReduce);
    else if (x == "reducescatter") out->push_back(Op::ReduceScatter);
    else if (x == "allgather") out->push_back(Op::AllGather);
    else if (x == "alltoall") out->push_back(Op::AllToAll);
    else return false;
  }
  return !out->empty();
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
    else if (!std::strcmp(argv[i], "--op") && i + 1 < argc) {
      if (!parse_ops(argv[++i], &o.ops)) { std::fprintf(stderr, "bad --op %s\n", argv[i]); return 2; }
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
