// Host-only sweep logic of mx-allreduce-perf (allreduce_perf.cc): which
// message sizes a sweep visits, the element counts each collective takes at
// n ranks, the nccl-tests bus-bandwidth factor, the per-size iteration count
// and the parameters of the whole-buffer correctness check.  Kept free of HIP
// and RCCL so that the CPU test tier compiles it with g++ and checks every op
// at n = 1, 2, 4, 8 (tests/test_rccl_bench_cpu.py) before an 8-GPU node ever
// runs it.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

namespace mxrb {

enum class Op { AllReduce, ReduceScatter, AllGather, AllToAll };

inline const char* op_name(Op op) {
  switch (op) {
    case Op::AllReduce: return "allreduce";
    case Op::ReduceScatter: return "reducescatter";
    case Op::AllGather: return "allgather";
    default: return "alltoall";
  }
}

// busbw = algbw * factor (nccl-tests): 2(n-1)/n for all-reduce, (n-1)/n for
// the others; 0 at n = 1 (nothing crosses a link).
inline double bus_factor(Op op, int n) {
  if (n <= 1) return 0.0;
  return op == Op::AllReduce ? 2.0 * (n - 1) / n : double(n - 1) / n;
}

inline size_t parse_size(const char* s) {
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

inline std::vector<int> parse_list(const char* s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string x;
  while (std::getline(ss, x, ',')) if (!x.empty()) v.push_back(std::atoi(x.c_str()));
  return v;
}

inline bool parse_ops(const char* s, std::vector<Op>* out) {
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

// keep a point under ~1 s: large messages need fewer iterations
inline int iters_for(size_t bytes, int base) {
  if (bytes >= (size_t(1) << 31)) return std::max(3, base / 4);
  if (bytes >= (size_t(1) << 29)) return std::max(5, base / 2);
  return base;
}

// Element counts of one sweep point: `count` is what the RCCL call takes
// (all-reduce: the buffer; reduce-scatter / all-gather: the per-rank block;
// all-to-all: the block per pair), send / recv the per-rank buffers.
struct Shape {
  size_t count, send, recv;
};

inline Shape shape_for(Op op, size_t bytes, size_t esz, int n) {
  const size_t elems = std::max<size_t>(1, bytes / esz);
  if (op == Op::AllReduce) return {elems, elems, elems};
  const size_t chunk = std::max<size_t>(1, elems / n);
  switch (op) {
    case Op::ReduceScatter: return {chunk, chunk * n, chunk};
    case Op::AllGather: return {chunk, chunk, chunk * n};
    default: return {chunk, chunk * n, chunk * n};
  }
}

// The reported size of a point: the LARGER per-rank buffer (nccl-tests).
inline size_t point_bytes(const Shape& s, size_t esz) { return std::max(s.send, s.recv) * esz; }

struct Point {
  size_t bytes;     // the sweep's nominal size
  Shape shape;
  size_t reported;  // point_bytes
  int iters;
};

// The points a sweep visits: bytes = minb, minb*f, ... <= maxb (no overflow
// past maxb), skipping shapes whose buffers would not fit maxb (tiny sizes
// times many ranks).
inline std::vector<Point> sweep_points(Op op, size_t minb, size_t maxb, int factor, size_t esz,
                                       int n, int iters) {
  std::vector<Point> out;
  if (minb < 1 || maxb < minb || factor < 2 || n < 1) return out;
  for (size_t bytes = minb; bytes <= maxb; bytes *= factor) {
    const Shape s = shape_for(op, bytes, esz, n);
    if (point_bytes(s, esz) <= maxb) out.push_back({bytes, s, point_bytes(s, esz), iters_for(bytes, iters)});
    if (bytes > maxb / factor) break;
  }
  return out;
}

// Whole-buffer correctness check: rank r's send buffer holds r + 1 in every
// element; receive element i must equal `sum` = n(n+1)/2 when `chunk` is 0
// (all-reduce, reduce-scatter) or (i / chunk) + 1 (all-gather: block j came
// from rank j; all-to-all: block j is rank j's block for this rank).
struct CheckParams {
  size_t chunk;
  float sum;
};

inline CheckParams check_params(Op op, const Shape& s, int n) {
  const size_t chunk = (op == Op::AllReduce || op == Op::ReduceScatter) ? 0 : s.count;
  return {chunk, n * (n + 1) / 2.0f};
}

// The value the device check kernel expects at receive element i.
inline float expected_at(const CheckParams& c, size_t i) {
  return c.chunk ? float(i / c.chunk + 1) : c.sum;
}

// bf16 encode / decode as the bench's fill and check kernels do (truncation
// of exact small integers: exact for every value the check uses).
inline uint16_t bf16_bits(float v) {
  uint32_t u;
  static_assert(sizeof(u) == sizeof(v), "");
  __builtin_memcpy(&u, &v, 4);
  return static_cast<uint16_t>(u >> 16);
}
inline float bf16_value(uint16_t b) {
  const uint32_t u = uint32_t(b) << 16;
  float v;
  __builtin_memcpy(&v, &u, 4);
  return v;
}

}  // namespace mxrb
