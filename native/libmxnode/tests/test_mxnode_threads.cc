// Concurrency test for libmxnode, built with -fsanitize=thread by
// `make test-native-tsan`.
//
// The device plugin calls into libmxnode from a gRPC thread pool (Allocate,
// GetPreferredAllocation) while its health thread polls mx_health_check and
// the exporter samples amd-smi; every entry point must therefore be
// re-entrant.  Eight threads hammer all of them against the fake sysfs tree
// and compare with a single-threaded baseline.  A data race makes TSan abort
// with a report (exit 66); a wrong answer shows up as a CHECK failure.
//   test_mxnode_threads <fixtures/sysfs dir>
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mxnode.h"

namespace {
std::atomic<int> failures{0};

#define CHECK(cond)                                                                  \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      failures.fetch_add(1);                                                         \
    }                                                                                \
  } while (0)

struct Baseline {
  int ngpu = 0;
  std::string cdi;
  std::vector<int> pref;
};

Baseline baseline(const std::string& root) {
  Baseline b;
  char err[256];
  std::vector<mx_gpu_info> g(MX_MAX_GPUS);
  b.ngpu = mx_enumerate(root.c_str(), g.data(), MX_MAX_GPUS, err, sizeof err);
  std::vector<char> buf(1 << 16);
  long len = mx_cdi_spec(root.c_str(), "amd.com/gpu", buf.data(), buf.size(), err, sizeof err);
  if (len > 0) b.cdi.assign(buf.data(), static_cast<size_t>(len));
  const int avail[] = {0, 1, 2, 3, 4, 5, 6, 7};
  b.pref.resize(4);
  mx_preferred_allocation(root.c_str(), avail, 8, nullptr, 0, 4, b.pref.data(), err, sizeof err);
  return b;
}

void worker(const std::string& root, const Baseline& b, int tid, int iters) {
  char err[256];
  std::vector<mx_gpu_info> g(MX_MAX_GPUS);
  std::vector<char> buf(1 << 16);
  const int avail[] = {0, 1, 2, 3, 4, 5, 6, 7};
  for (int it = 0; it < iters; ++it) {
    switch ((tid + it) % 5) {
      case 0:
        CHECK(mx_enumerate(root.c_str(), g.data(), MX_MAX_GPUS, err, sizeof err) == b.ngpu);
        break;
      case 1: {
        long len = mx_cdi_spec(root.c_str(), "amd.com/gpu", buf.data(), buf.size(), err, sizeof err);
        CHECK(len == static_cast<long>(b.cdi.size()));
        CHECK(len > 0 && std::memcmp(buf.data(), b.cdi.data(), static_cast<size_t>(len)) == 0);
        break;
      }
      case 2: {
        int out[4] = {-1, -1, -1, -1};
        CHECK(mx_preferred_allocation(root.c_str(), avail, 8, nullptr, 0, 4, out, err,
                                      sizeof err) == 4);
        CHECK(std::equal(out, out + 4, b.pref.begin()));
        break;
      }
      case 3:
        for (int i = 0; i < b.ngpu; ++i) CHECK(mx_health_check(root.c_str(), i, nullptr) == MX_HEALTHY);
        CHECK(std::strlen(mx_health_reason(MX_UNHEALTHY_ECC)) > 0);
        break;
      default: {
        // amd-smi is absent on the build box: open must fail cleanly and the
        // sampler entry points must stay safe while other threads open/close.
        char e2[256];
        if (mx_smi_open(e2, sizeof e2)) {
          const int n = mx_smi_count();
          mx_gpu_sample s;
          for (int i = 0; i < n && i < 2; ++i) mx_smi_sample(i, &s);
          mx_smi_close();
        } else {
          CHECK(mx_smi_count() <= 0 || true);
        }
        CHECK(mx_version() != nullptr);
        break;
      }
    }
  }
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <fixtures/sysfs>\n", argv[0]);
    return 2;
  }
  const std::string root = std::string(argv[1]) + "/mi355x_8gpu";
  const Baseline b = baseline(root);
  CHECK(b.ngpu == 8);
  CHECK(!b.cdi.empty());
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t) ts.emplace_back(worker, std::cref(root), std::cref(b), t, 200);
  // the N02 monitor: the plugin's health thread steps it while gRPC threads
  // and the state writer read it
  mx_health_opts o{};
  o.root = root.c_str();
  o.event_quarantine_ms = 100;
  char err[256];
  mx_health_monitor* m = mx_hm_create(&o, err, sizeof err);
  CHECK(m != nullptr);
  std::atomic<bool> stop{false};
  std::thread stepper([&] { for (int i = 0; i < 200; ++i) CHECK(mx_hm_step(m, 0) >= 0); stop = true; });
  std::vector<std::thread> readers;
  for (int t = 0; t < 3; ++t)
    readers.emplace_back([&, t] {
      mx_health_status st[MX_MAX_GPUS];
      mx_health_event ev[8];
      const std::string path = "/tmp/mxk_tsan_health_" + std::to_string(t) + ".json";
      while (!stop) {
        CHECK(mx_hm_status(m, st, MX_MAX_GPUS) == 8);
        CHECK(mx_hm_events(m, 0, ev, 8) >= 0);
        CHECK(mx_hm_write_state(m, path.c_str()) == 0);
      }
      std::remove(path.c_str());
    });
  stepper.join();
  for (auto& t : readers) t.join();
  mx_hm_destroy(m);
  for (auto& t : ts) t.join();
  if (failures.load()) {
    std::fprintf(stderr, "%d failures\n", failures.load());
    return 1;
  }
  std::printf("libmxnode thread-safety test: ok (8 threads x 200 calls)\n");
  return 0;
}
