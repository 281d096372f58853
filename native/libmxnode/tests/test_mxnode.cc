// Host unit tests for libmxnode over the fake sysfs fixtures.
// Built with -fsanitize=address,undefined by `make test-native`.
//   test_mxnode <fixtures/sysfs dir>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "mxnode.h"

static int failures = 0;
#define CHECK(cond)                                                              \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                                \
    }                                                                            \
  } while (0)

static void test_enumerate(const std::string& fx) {
  char err[256];
  std::vector<mx_gpu_info> g(MX_MAX_GPUS);
  int n = mx_enumerate((fx + "/mi355x_8gpu").c_str(), g.data(), MX_MAX_GPUS, err, sizeof err);
  CHECK(n == 8);
  for (int i = 0; i < n; ++i) {
    CHECK(g[i].index == i);
    CHECK(std::strcmp(g[i].gfx_arch, "gfx950") == 0);
    CHECK(g[i].cu_count == 256);
    CHECK(g[i].drm_render_minor == 128 + i);
    CHECK(g[i].numa_node == (i < 4 ? 0 : 1));
    CHECK(g[i].num_xgmi_links == 7);
    CHECK(std::strcmp(g[i].product, "MI355X") == 0);
    CHECK(g[i].vram_bytes == 309220868096ull);
  }
  CHECK(std::strcmp(g[0].pci_bdf, "0000:05:00.0") == 0);
  n = mx_enumerate((fx + "/mixed_nonamd").c_str(), g.data(), MX_MAX_GPUS, err, sizeof err);
  CHECK(n == 1);
  n = mx_enumerate((fx + "/no_driver").c_str(), g.data(), MX_MAX_GPUS, err, sizeof err);
  CHECK(n == -1);
  CHECK(std::strstr(err, "KFD") != nullptr);
  // count-only call with a tiny buffer must not overflow
  n = mx_enumerate((fx + "/mi355x_8gpu").c_str(), g.data(), 2, err, sizeof err);
  CHECK(n == 8);
}

static void test_links(const std::string& fx) {
  char err[256];
  std::vector<mx_link> l(MX_MAX_GPUS * MX_MAX_LINKS);
  int n = mx_links((fx + "/mi355x_8gpu").c_str(), l.data(), static_cast<int>(l.size()), err, sizeof err);
  CHECK(n == 8 * 8);   // 1 PCIe + 7 xGMI per GPU
  int xgmi = 0;
  for (int i = 0; i < n; ++i)
    if (l[i].type == 11) {
      ++xgmi;
      CHECK(l[i].to_index >= 0 && l[i].to_index < 8 && l[i].to_index != l[i].from_index);
    }
  CHECK(xgmi == 56);
}

static void test_cdi(const std::string& fx) {
  char err[256];
  long need = mx_cdi_spec((fx + "/mi355x_8gpu").c_str(), "amd.com/gpu", nullptr, 0, err, sizeof err);
  CHECK(need > 0);
  std::vector<char> buf(need + 1);
  long got = mx_cdi_spec((fx + "/mi355x_8gpu").c_str(), "amd.com/gpu", buf.data(), buf.size(), err, sizeof err);
  CHECK(got == need);
  std::string s(buf.data());
  CHECK(s.find("\"cdiVersion\":\"0.6.0\"") != std::string::npos);
  CHECK(s.find("/dev/kfd") != std::string::npos);
  CHECK(s.find("/dev/dri/renderD135") != std::string::npos);
  CHECK(s.find("\"name\":\"all\"") != std::string::npos);
  // truncation is reported, not overflowed
  char small[16];
  long t = mx_cdi_spec((fx + "/mi355x_8gpu").c_str(), "amd.com/gpu", small, sizeof small, err, sizeof err);
  CHECK(t == need);
  CHECK(std::strlen(small) == sizeof(small) - 1);
}

static void test_alloc(const std::string& fx) {
  char err[256];
  const std::string r = fx + "/mi355x_8gpu";
  int avail[8] = {0, 1, 2, 3, 4, 5, 6, 7};
  int out[8];
  // 4 GPUs: one NUMA node, lowest indices
  CHECK(mx_preferred_allocation(r.c_str(), avail, 8, nullptr, 0, 4, out, err, sizeof err) == 4);
  CHECK(out[0] == 0 && out[1] == 1 && out[2] == 2 && out[3] == 3);
  // must include 5 -> stay on NUMA node 1
  int must[1] = {5};
  CHECK(mx_preferred_allocation(r.c_str(), avail, 8, must, 1, 2, out, err, sizeof err) == 2);
  CHECK(out[0] == 4 && out[1] == 5);
  // available split across sockets: prefer the socket that can host all 3
  int av2[5] = {0, 4, 5, 6, 1};
  CHECK(mx_preferred_allocation(r.c_str(), av2, 5, nullptr, 0, 3, out, err, sizeof err) == 3);
  CHECK(out[0] == 4 && out[1] == 5 && out[2] == 6);
  // invalid: size > available, must not in available
  CHECK(mx_preferred_allocation(r.c_str(), avail, 8, nullptr, 0, 9, out, err, sizeof err) == -1);
  int bad[1] = {9};
  CHECK(mx_preferred_allocation(r.c_str(), avail, 8, bad, 1, 2, out, err, sizeof err) == -1);
  // all 8
  CHECK(mx_preferred_allocation(r.c_str(), avail, 8, nullptr, 0, 8, out, err, sizeof err) == 8);
  for (int i = 0; i < 8; ++i) CHECK(out[i] == i);
}

static void test_health(const std::string& fx) {
  const std::string ok = fx + "/mi355x_8gpu", miss = fx + "/missing_render";
  CHECK(mx_health_check(ok.c_str(), 3, nullptr) == MX_HEALTHY);
  CHECK(mx_health_check(miss.c_str(), 3, nullptr) == MX_UNHEALTHY_NO_RENDER_NODE);
  CHECK(mx_health_check(miss.c_str(), 2, nullptr) == MX_HEALTHY);
  CHECK(mx_health_check(ok.c_str(), 8, nullptr) == MX_UNHEALTHY_NO_KFD_NODE);
  const char* ff = "/tmp/mxnode_fault_test.txt";
  { std::ofstream f(ff); f << "# drill\n5\n"; }
  CHECK(mx_health_check(ok.c_str(), 5, ff) == MX_UNHEALTHY_FAULT_INJECTED);
  CHECK(mx_health_check(ok.c_str(), 4, ff) == MX_HEALTHY);
  { std::ofstream f(ff); f << "all\n"; }
  CHECK(mx_health_check(ok.c_str(), 0, ff) == MX_UNHEALTHY_FAULT_INJECTED);
  std::remove(ff);
  CHECK(std::strcmp(mx_health_reason(MX_UNHEALTHY_NO_RENDER_NODE), "render node missing") == 0);
}

static void test_monitor(const std::string& fx) {
  const std::string root = fx + "/mi355x_8gpu";
  char tmpl[] = "/tmp/mxhmXXXXXX";
  const std::string dir = mkdtemp(tmpl) ? tmpl : "/tmp";
  const std::string fault = dir + "/faults";
  { FILE* f = std::fopen(fault.c_str(), "w"); std::fclose(f); }
  mx_health_opts o{};
  o.root = root.c_str();
  o.fault_file = fault.c_str();
  o.state_dir = dir.c_str();
  o.event_quarantine_ms = 1000;
  o.ecc_quarantine_ms = 0;
  o.use_smi = 0;
  char err[256] = {0};
  mx_health_monitor* m = mx_hm_create(&o, err, sizeof err);
  CHECK(m != nullptr);
  if (!m) return;
  CHECK(mx_hm_smi_active(m) == 0);
  CHECK(mx_hm_step(m, 0) == 0);
  mx_health_status st[MX_MAX_GPUS];
  CHECK(mx_hm_status(m, st, MX_MAX_GPUS) == 8);
  for (int i = 0; i < 8; ++i) CHECK(st[i].code == MX_HEALTHY && st[i].smi_index == -1);
  { FILE* f = std::fopen(fault.c_str(), "w"); std::fputs("6\n", f); std::fclose(f); }
  CHECK(mx_hm_step(m, 0) == 1);
  mx_hm_status(m, st, MX_MAX_GPUS);
  CHECK(st[6].code == MX_UNHEALTHY_FAULT_INJECTED && st[5].code == MX_HEALTHY);
  mx_health_event ev[16];
  const int ne = mx_hm_events(m, 0, ev, 16);
  CHECK(ne == 1 && ev[0].kind == MX_EVT_HEALTH_CHANGE && ev[0].index == 6 &&
        ev[0].value == MX_UNHEALTHY_FAULT_INJECTED);
  CHECK(mx_hm_events(m, ev[0].seq, ev, 16) == 0);
  const std::string state = dir + "/health.json";
  CHECK(mx_hm_write_state(m, state.c_str()) == 0);
  std::string text;
  { FILE* f = std::fopen(state.c_str(), "r"); char b[8192]; size_t k = std::fread(b, 1, sizeof b, f); std::fclose(f); text.assign(b, k); }
  CHECK(text.find("\"index\":6,\"bdf\":\"0000:e5:00.0\"") != std::string::npos);
  CHECK(text.find("\"reason\":\"fault injected\"") != std::string::npos);
  { FILE* f = std::fopen(fault.c_str(), "w"); std::fclose(f); }
  CHECK(mx_hm_step(m, 0) == 1);
  mx_hm_status(m, st, MX_MAX_GPUS);
  CHECK(st[6].code == MX_HEALTHY);
  mx_hm_destroy(m);
  CHECK(mx_hm_create(nullptr, err, sizeof err) == nullptr);
}

int main(int argc, char** argv) {
  const std::string fx = argc > 1 ? argv[1] : "tests/fixtures/sysfs";
  test_enumerate(fx);
  test_links(fx);
  test_cdi(fx);
  test_alloc(fx);
  test_health(fx);
  test_monitor(fx);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("libmxnode tests passed (%s)\n", mx_version());
  return 0;
}
