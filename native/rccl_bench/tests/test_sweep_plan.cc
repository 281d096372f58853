// Host test of mx-allreduce-perf's sweep logic (sweep_plan.h): every op at
// n = 1, 2, 4, 8 and both dtypes.  The collectives themselves are simulated
// on the host from their definitions (rank r sends r + 1 everywhere), so the
// shapes, the reported sizes, the bus factors and the mismatch check's
// chunking are pinned without a GPU.  Built and run by
// tests/test_rccl_bench_cpu.py.
#include <cmath>
#include <cstdio>
#include <vector>

#include "../sweep_plan.h"

using namespace mxrb;

static int failures = 0;
#define EXPECT(c)                                                               \
  do {                                                                          \
    if (!(c)) {                                                                 \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);         \
      ++failures;                                                               \
    }                                                                           \
  } while (0)

// receive buffer of rank `me` after op, from the collective's definition
static std::vector<float> simulate(Op op, const Shape& s, int n, int me) {
  std::vector<float> out(s.recv);
  auto send_val = [](int r) { return float(r + 1); };
  switch (op) {
    case Op::AllReduce:
    case Op::ReduceScatter: {
      float sum = 0;
      for (int r = 0; r < n; ++r) sum += send_val(r);
      for (auto& x : out) x = sum;
      break;
    }
    case Op::AllGather:      // block j = rank j's send buffer
      for (int j = 0; j < n; ++j)
        for (size_t e = 0; e < s.count; ++e) out[j * s.count + e] = send_val(j);
      break;
    default:                 // all-to-all: block j = rank j's block `me`
      for (int j = 0; j < n; ++j)
        for (size_t e = 0; e < s.count; ++e) out[j * s.count + e] = send_val(j);
      break;
  }
  (void)me;
  return out;
}

static size_t mismatches(const std::vector<float>& recv, const CheckParams& c, bool bf16) {
  size_t bad = 0;
  for (size_t i = 0; i < recv.size(); ++i) {
    const float got = bf16 ? bf16_value(bf16_bits(recv[i])) : recv[i];
    bad += got != expected_at(c, i);
  }
  return bad;
}

int main() {
  const Op ops[] = {Op::AllReduce, Op::ReduceScatter, Op::AllGather, Op::AllToAll};
  const size_t minb = 8, maxb = size_t(8) << 30;
  for (Op op : ops) {
    for (int n : {1, 2, 4, 8}) {
      // bus factors (nccl-tests)
      const double bf = bus_factor(op, n);
      if (n == 1) EXPECT(bf == 0.0);
      else if (op == Op::AllReduce) EXPECT(std::fabs(bf - 2.0 * (n - 1) / n) < 1e-12);
      else EXPECT(std::fabs(bf - double(n - 1) / n) < 1e-12);
      for (size_t esz : {size_t(2), size_t(4)}) {
        const bool bf16 = esz == 2;
        const auto pts = sweep_points(op, minb, maxb, 2, esz, n, 20);
        EXPECT(!pts.empty() && pts.size() <= 31);
        size_t prev = 0;
        for (const Point& p : pts) {
          const Shape& s = p.shape;
          EXPECT(p.bytes >= minb && p.bytes <= maxb && p.bytes > prev);
          prev = p.bytes;
          EXPECT(s.count >= 1);
          EXPECT(p.reported == std::max(s.send, s.recv) * esz && p.reported <= maxb);
          switch (op) {
            case Op::AllReduce: EXPECT(s.send == s.count && s.recv == s.count); break;
            case Op::ReduceScatter: EXPECT(s.send == s.count * n && s.recv == s.count); break;
            case Op::AllGather: EXPECT(s.send == s.count && s.recv == s.count * n); break;
            default: EXPECT(s.send == s.count * n && s.recv == s.count * n); break;
          }
          // the reported size is the nominal size whenever it divides evenly
          if (p.bytes / esz >= size_t(n) && (p.bytes / esz) % n == 0)
            EXPECT(p.reported == p.bytes);
          EXPECT(p.iters == iters_for(p.bytes, 20));
          EXPECT(p.iters >= 3 && p.iters <= 20);
          // simulated collective + the bench's whole-buffer check (small points)
          if (p.reported <= 4096) {
            const CheckParams c = check_params(op, s, n);
            for (int me = 0; me < n; ++me) {
              auto recv = simulate(op, s, n, me);
              EXPECT(mismatches(recv, c, bf16) == 0);
              recv[recv.size() - 1] += 1.f;        // one corrupted element is caught
              EXPECT(mismatches(recv, c, bf16) == 1);
              if (c.chunk && n > 1) {              // blocks swapped: every element of both
                auto r2 = simulate(op, s, n, me);
                for (size_t e = 0; e < s.count; ++e) std::swap(r2[e], r2[s.count + e]);
                EXPECT(mismatches(r2, c, bf16) == 2 * s.count);
              }
            }
          }
        }
        // the full protocol size list for the all-reduce: 8 B .. 8 GiB, 31 points
        if (op == Op::AllReduce) {
          EXPECT(pts.size() == 31);
          EXPECT(pts.front().bytes == 8 && pts.back().bytes == maxb);
          EXPECT(pts.back().iters == 5);           // 8 GiB: max(3, 20 / 4)
        }
      }
    }
  }
  // a range reaching the top of size_t terminates (no overflow wrap)
  EXPECT(sweep_points(Op::AllReduce, 8, ~size_t(0), 2, 4, 8, 20).size() <= 64);
  EXPECT(sweep_points(Op::AllReduce, 16, 8, 2, 4, 8, 20).empty());
  // parsing
  EXPECT(parse_size("8G") == (size_t(8) << 30) && parse_size("64k") == 65536);
  std::vector<Op> v;
  EXPECT(parse_ops("all", &v) && v.size() == 4);
  EXPECT(parse_ops("allgather,alltoall", &v) && v.size() == 2 && v[1] == Op::AllToAll);
  EXPECT(!parse_ops("bogus", &v));
  EXPECT(parse_list("1,2,4,8").size() == 4);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("PASS sweep_plan\n");
  return 0;
}
