// Scriptable fake libamd_smi.so for the CPU test tier (SURVEY.md §4.2 "Fake
// amd-smi backend").  libmxnode dlopen()s amd-smi by name, so pointing
// MXK8S_AMDSMI_LIB at this library runs the REAL smi.cc / health.cc code
// paths against GPU state a test writes into files:
//
//   $MXK8S_FAKE_AMDSMI_DIR/gpus    one GPU per line, whitespace-separated
//                                  key=value pairs (re-read on every call):
//       bdf=0000:05:00.0 gfx=37 umc=12 vram_used=<B> vram_total=<B>
//       temp_edge=41 temp_hotspot=55 temp_mem=48 power=612 power_limit=1400
//       sclk=2100 mclk=1300 ecc_ce=0 ecc_ue=0 energy=<uJ>
//       xgmi_status=1,1,1,1,1,1,0      (per link: 0 down, 1 up, 2 disabled)
//       xgmi_read_kb=10,20,...         (per link cumulative KB)
//       xgmi_write_kb=...  xgmi_bitrate=32  xgmi_maxbw=64
//   $MXK8S_FAKE_AMDSMI_DIR/events  appended lines "<gpu> <event-code> <message>";
//                                  each line is delivered once, in order
//   $MXK8S_FAKE_AMDSMI_DIR/procs   lines "<gpu> <pid> <name> <vram-bytes> [container]"
//   $MXK8S_FAKE_AMDSMI_DIR/fail    if present: amdsmi_init fails
//
// Link peers are the other GPUs of the file in order (a full xGMI mesh).
// partition=<k> puts k in the BDF id's bits 31:28 (compute partitions share
// the device's BDF).  Like the real library, amdsmi_init takes the handle
// list: the number of GPUs is fixed until the next init, and a handle from an
// earlier init is invalid (AMDSMI_STATUS_INVAL) — so a partition change that
// rewrites the gpus file (8 -> 64 lines) is only seen after a re-init.
#include <amd_smi/amdsmi.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <chrono>
#include <vector>

namespace {

std::mutex g_mu;
std::atomic<bool> g_init{false};
size_t g_events_consumed = 0;
std::atomic<uint32_t> g_gen{0};     // bumped by every amdsmi_init
std::atomic<uint32_t> g_count{0};   // GPUs enumerated at the last init

std::string dir() {
  const char* d = std::getenv("MXK8S_FAKE_AMDSMI_DIR");
  return d ? d : "";
}

std::vector<std::string> lines_of(const std::string& path) {
  std::vector<std::string> out;
  std::ifstream f(path);
  std::string l;
  while (std::getline(f, l)) {
    if (l.empty() || l[0] == '#') continue;
    out.push_back(l);
  }
  return out;
}

using Gpu = std::map<std::string, std::string>;

std::vector<Gpu> gpus() {
  std::vector<Gpu> out;
  for (const auto& l : lines_of(dir() + "/gpus")) {
    Gpu g;
    std::istringstream in(l);
    std::string kv;
    while (in >> kv) {
      const auto eq = kv.find('=');
      if (eq != std::string::npos) g[kv.substr(0, eq)] = kv.substr(eq + 1);
    }
    out.push_back(g);
  }
  return out;
}

uint64_t num(const Gpu& g, const char* k, uint64_t dflt = 0) {
  auto it = g.find(k);
  return it == g.end() ? dflt : std::strtoull(it->second.c_str(), nullptr, 0);
}

std::vector<uint64_t> list(const Gpu& g, const char* k) {
  std::vector<uint64_t> out;
  auto it = g.find(k);
  if (it == g.end()) return out;
  std::istringstream in(it->second);
  std::string tok;
  while (std::getline(in, tok, ',')) out.push_back(std::strtoull(tok.c_str(), nullptr, 0));
  return out;
}

// handle = (void*)(generation << 20 | (index + 1)); -1 for a stale or unknown one
int idx(amdsmi_processor_handle h) {
  const uintptr_t v = reinterpret_cast<uintptr_t>(h);
  if (!g_init || (v >> 20) != g_gen) return -1;
  const int i = static_cast<int>(v & 0xfffff) - 1;
  return i < static_cast<int>(g_count.load()) ? i : -1;
}
amdsmi_processor_handle handle(int i) {
  return reinterpret_cast<amdsmi_processor_handle>((uintptr_t(g_gen.load()) << 20) |
                                                   uintptr_t(i + 1));
}

bool get(amdsmi_processor_handle h, Gpu* out) {
  auto gs = gpus();
  const int i = idx(h);
  if (i < 0 || i >= static_cast<int>(gs.size())) return false;
  *out = gs[i];
  return true;
}

void parse_bdf(const std::string& s, unsigned* dom, unsigned* bus, unsigned* dev, unsigned* fn) {
  *dom = *bus = *dev = *fn = 0;
  std::sscanf(s.c_str(), "%x:%x:%x.%x", dom, bus, dev, fn);
}

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::ifstream fail(dir() + "/fail");
  if (fail.good()) return AMDSMI_STATUS_INIT_ERROR;
  g_init = true;
  ++g_gen;
  g_count = static_cast<uint32_t>(gpus().size());
  g_events_consumed = lines_of(dir() + "/events").size();   // only events after init
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_init = false;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* socks) {
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  if (socks && *count >= 1) socks[0] = reinterpret_cast<amdsmi_socket_handle>(uintptr_t(1));
  *count = 1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle, uint32_t* count,
                                             amdsmi_processor_handle* ps) {
  if (!g_init) return AMDSMI_STATUS_NOT_INIT;
  const uint32_t n = g_count.load();
  if (ps)
    for (uint32_t i = 0; i < n && i < *count; ++i) ps[i] = handle(static_cast<int>(i));
  *count = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle, processor_type_t* t) {
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bdf_id(amdsmi_processor_handle h, uint64_t* id) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  unsigned dom, bus, dev, fn;
  parse_bdf(g["bdf"], &dom, &bus, &dev, &fn);
  *id = (uint64_t(dom) << 32) | (uint64_t(num(g, "partition") & 0xf) << 28) |
        (uint64_t(bus) << 8) | (uint64_t(dev) << 3) | fn;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_activity(amdsmi_processor_handle h, amdsmi_engine_usage_t* u) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  std::memset(u, 0, sizeof(*u));
  u->gfx_activity = static_cast<uint32_t>(num(g, "gfx"));
  u->umc_activity = static_cast<uint32_t>(num(g, "umc"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_usage(amdsmi_processor_handle h, amdsmi_memory_type_t,
                                            uint64_t* used) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  *used = num(g, "vram_used");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t,
                                            uint64_t* total) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  *total = num(g, "vram_total", 309237645312ull);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_temp_metric(amdsmi_processor_handle h, amdsmi_temperature_type_t type,
                                       amdsmi_temperature_metric_t, int64_t* t) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  const char* key = type == AMDSMI_TEMPERATURE_TYPE_EDGE      ? "temp_edge"
                    : type == AMDSMI_TEMPERATURE_TYPE_HOTSPOT ? "temp_hotspot"
                    : type == AMDSMI_TEMPERATURE_TYPE_VRAM    ? "temp_mem"
                                                              : "";
  if (!g.count(key)) return AMDSMI_STATUS_NOT_SUPPORTED;
  *t = static_cast<int64_t>(num(g, key));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_power_info(amdsmi_processor_handle h, amdsmi_power_info_t* p) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  std::memset(p, 0, sizeof(*p));
  p->current_socket_power = static_cast<uint32_t>(num(g, "power"));
  p->power_limit = static_cast<uint32_t>(num(g, "power_limit", 1400));
  return AMDSMI_STATUS_SUCCESS;
}

// energy=<uJ> (absent: unsupported); the real library reports counts of
// ~15.3 uJ, so the fake uses the same resolution
amdsmi_status_t amdsmi_get_energy_count(amdsmi_processor_handle h, uint64_t* acc, float* res,
                                        uint64_t* ts) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  const uint64_t uj = num(g, "energy", ~0ull);
  if (uj == ~0ull) return AMDSMI_STATUS_NOT_SUPPORTED;
  *res = 15.259f;
  *acc = static_cast<uint64_t>(static_cast<double>(uj) / 15.259);
  *ts = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_clock_info(amdsmi_processor_handle h, amdsmi_clk_type_t type,
                                      amdsmi_clk_info_t* c) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  std::memset(c, 0, sizeof(*c));
  c->clk = static_cast<uint32_t>(num(g, type == AMDSMI_CLK_TYPE_MEM ? "mclk" : "sclk"));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h, amdsmi_error_count_t* e) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  std::memset(e, 0, sizeof(*e));
  e->correctable_count = num(g, "ecc_ce");
  e->uncorrectable_count = num(g, "ecc_ue");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle h, uint32_t* max,
                                            amdsmi_proc_info_t* list) {
  const int i = idx(h);
  uint32_t n = 0;
  for (const auto& l : lines_of(dir() + "/procs")) {
    std::istringstream in(l);
    int gi = -1;
    unsigned pid = 0;
    std::string name, container;
    unsigned long long vram = 0;
    if (!(in >> gi >> pid >> name >> vram) || gi != i) continue;
    in >> container;
    if (list && n < *max) {
      amdsmi_proc_info_t& p = list[n];
      std::memset(&p, 0, sizeof(p));
      std::snprintf(p.name, sizeof(p.name), "%s", name.c_str());
      std::snprintf(p.container_name, sizeof(p.container_name), "%s", container.c_str());
      p.pid = pid;
      p.mem = vram;
      p.memory_usage.vram_mem = vram;
    }
    ++n;
  }
  if (list && n > *max) {
    *max = n;
    return AMDSMI_STATUS_OUT_OF_RESOURCES;
  }
  *max = n;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_driver_info(amdsmi_processor_handle, amdsmi_driver_info_t* d) {
  std::memset(d, 0, sizeof(*d));
  std::snprintf(d->driver_version, sizeof(d->driver_version), "fake-6.14.14");
  std::snprintf(d->driver_name, sizeof(d->driver_name), "amdgpu");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle h,
                                                amdsmi_xgmi_link_status_t* s) {
  Gpu g;
  if (!get(h, &g)) return AMDSMI_STATUS_INVAL;
  const auto st = list(g, "xgmi_status");
  if (st.empty()) return AMDSMI_STATUS_NOT_SUPPORTED;
  std::memset(s, 0, sizeof(*s));
  s->total_links = static_cast<uint32_t>(std::min<size_t>(st.size(), AMDSMI_MAX_NUM_XGMI_LINKS));
  for (uint32_t k = 0; k < s->total_links; ++k)
    s->status[k] = static_cast<amdsmi_xgmi_link_status_type_t>(st[k]);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_link_metrics(amdsmi_processor_handle h, amdsmi_link_metrics_t* m) {
  auto gs = gpus();
  const int i = idx(h);
  if (i < 0 || i >= static_cast<int>(gs.size())) return AMDSMI_STATUS_INVAL;
  const Gpu& g = gs[i];
  const auto rd = list(g, "xgmi_read_kb"), wr = list(g, "xgmi_write_kb");
  if (rd.empty() && wr.empty()) return AMDSMI_STATUS_NOT_SUPPORTED;
  std::memset(m, 0, sizeof(*m));
  uint32_t k = 0;
  for (int p = 0; p < static_cast<int>(gs.size()); ++p) {
    if (p == i) continue;
    auto& L = m->links[k];
    unsigned dom, bus, dev, fn;
    parse_bdf(gs[p].at("bdf"), &dom, &bus, &dev, &fn);
    L.bdf.domain_number = dom;
    L.bdf.bus_number = bus;
    L.bdf.device_number = dev;
    L.bdf.function_number = fn;
    L.bit_rate = static_cast<uint32_t>(num(g, "xgmi_bitrate", 32));
    L.max_bandwidth = static_cast<uint32_t>(num(g, "xgmi_maxbw", 64));
    L.link_type = AMDSMI_LINK_TYPE_XGMI;
    L.read = k < rd.size() ? rd[k] : 0;
    L.write = k < wr.size() ? wr[k] : 0;
    ++k;
  }
  m->num_links = k;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_init_gpu_event_notification(amdsmi_processor_handle) {
  return g_init ? AMDSMI_STATUS_SUCCESS : AMDSMI_STATUS_NOT_INIT;
}

amdsmi_status_t amdsmi_set_gpu_event_notification_mask(amdsmi_processor_handle, uint64_t) {
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_event_notification(int timeout_ms, uint32_t* num_elem,
                                                  amdsmi_evt_notification_data_t* data) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (true) {
    {
      std::lock_guard<std::mutex> lk(g_mu);
      const auto ev = lines_of(dir() + "/events");
      uint32_t n = 0;
      while (g_events_consumed < ev.size() && n < *num_elem) {
        std::istringstream in(ev[g_events_consumed++]);
        int gi = 0, code = 0;
        in >> gi >> code;
        std::string msg;
        std::getline(in, msg);
        std::memset(&data[n], 0, sizeof(data[n]));
        data[n].processor_handle = handle(gi);
        data[n].event = static_cast<amdsmi_evt_notification_type_t>(code);
        std::snprintf(data[n].message, sizeof(data[n].message), "%s", msg.c_str());
        ++n;
      }
      if (n > 0) {
        *num_elem = n;
        return AMDSMI_STATUS_SUCCESS;
      }
    }
    if (std::chrono::steady_clock::now() >= deadline) {
      *num_elem = 0;
      return AMDSMI_STATUS_NO_DATA;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

amdsmi_status_t amdsmi_stop_gpu_event_notification(amdsmi_processor_handle) {
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"
