// N02 (event part) + N06-core: amd-smi backed health events and metrics.
//
// amd-smi (/opt/rocm/lib/libamd_smi.so) is dlopen'ed at run time, so the
// library builds and its sysfs parts run on hosts without ROCm; the types come
// from the installed header.  Replaces the DCGM sampling behind the reference
// stack's dcgm-exporter [ext, R26f] and the NVML Xid watch [ext, R26d].
#include <amd_smi/amdsmi.h>
#include <dlfcn.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

namespace {

#define MX_SMI_FN(name) decltype(&::name) name = nullptr

struct SmiApi {
  void* handle = nullptr;
  MX_SMI_FN(amdsmi_init);
  MX_SMI_FN(amdsmi_shut_down);
  MX_SMI_FN(amdsmi_get_socket_handles);
  MX_SMI_FN(amdsmi_get_processor_handles);
  MX_SMI_FN(amdsmi_get_processor_type);
  MX_SMI_FN(amdsmi_get_gpu_bdf_id);
  MX_SMI_FN(amdsmi_get_gpu_activity);
  MX_SMI_FN(amdsmi_get_gpu_memory_usage);
  MX_SMI_FN(amdsmi_get_gpu_memory_total);
  MX_SMI_FN(amdsmi_get_temp_metric);
  MX_SMI_FN(amdsmi_get_power_info);
  MX_SMI_FN(amdsmi_get_clock_info);
  MX_SMI_FN(amdsmi_get_gpu_total_ecc_count);
  MX_SMI_FN(amdsmi_get_gpu_process_list);
  MX_SMI_FN(amdsmi_get_gpu_driver_info);
  MX_SMI_FN(amdsmi_init_gpu_event_notification);
  MX_SMI_FN(amdsmi_set_gpu_event_notification_mask);
  MX_SMI_FN(amdsmi_get_gpu_event_notification);
  MX_SMI_FN(amdsmi_stop_gpu_event_notification);
  MX_SMI_FN(amdsmi_get_gpu_xgmi_link_status);
  MX_SMI_FN(amdsmi_get_link_metrics);
  MX_SMI_FN(amdsmi_get_energy_count);
  std::vector<amdsmi_processor_handle> gpus;
  bool events_on = false;
  std::string driver_version;
};

// g_mu guards g_api and every amd-smi call except the blocking event wait;
// g_life orders the session's lifetime against that wait: (re)init and
// shutdown take it exclusively, mx_smi_wait_events holds it shared across the
// blocking amdsmi_get_gpu_event_notification.  Lock order: g_life, then g_mu.
std::mutex g_mu;
std::shared_mutex g_life;
SmiApi* g_api = nullptr;
int g_refs = 0;            // mx_smi_open calls not yet matched by mx_smi_close
uint64_t g_gen = 0;        // bumped by every amdsmi_init (open or re-init)

template <typename F>
bool bind(void* h, const char* name, F* slot) {
  *slot = reinterpret_cast<F>(dlsym(h, name));
  return *slot != nullptr;
}

void fmt_bdf(uint64_t bdf, char* out, size_t n) {
  // amd-smi BDF id: domain[63:32] bus[15:8] device[7:3] function[2:0]
  std::snprintf(out, n, "%04llx:%02llx:%02llx.%llx",
                static_cast<unsigned long long>((bdf >> 32) & 0xffff),
                static_cast<unsigned long long>((bdf >> 8) & 0xff),
                static_cast<unsigned long long>((bdf >> 3) & 0x1f),
                static_cast<unsigned long long>(bdf & 0x7));
}

// amdsmi_init + enumeration of the GPU processor handles.  amd-smi takes its
// handle list at init: after a compute-partition change (SPX -> CPX) or a
// driver reload only a fresh init sees the new partitions.
bool init_session(SmiApi* api, std::string* why) {
  api->gpus.clear();
  api->events_on = false;
  api->driver_version.clear();
  amdsmi_status_t st = api->amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    *why = "amdsmi_init failed: status " + std::to_string(st);
    return false;
  }
  uint32_t nsock = 0;
  api->amdsmi_get_socket_handles(&nsock, nullptr);
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (nsock) api->amdsmi_get_socket_handles(&nsock, socks.data());
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    api->amdsmi_get_processor_handles(socks[s], &np, nullptr);
    std::vector<amdsmi_processor_handle> ps(np);
    if (np) api->amdsmi_get_processor_handles(socks[s], &np, ps.data());
    for (uint32_t p = 0; p < np; ++p) {
      processor_type_t t;
      if (api->amdsmi_get_processor_type(ps[p], &t) == AMDSMI_STATUS_SUCCESS &&
          t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
        api->gpus.push_back(ps[p]);
    }
  }
  if (!api->gpus.empty()) {
    amdsmi_driver_info_t di;
    std::memset(&di, 0, sizeof(di));
    if (api->amdsmi_get_gpu_driver_info(api->gpus[0], &di) == AMDSMI_STATUS_SUCCESS)
      api->driver_version = di.driver_version;
  }
  ++g_gen;
  return true;
}

void end_session(SmiApi* api) {
  if (api->events_on && api->amdsmi_stop_gpu_event_notification)
    for (auto h : api->gpus) api->amdsmi_stop_gpu_event_notification(h);
  api->events_on = false;
  api->gpus.clear();
  api->amdsmi_shut_down();
}

void destroy_locked() {
  end_session(g_api);
  dlclose(g_api->handle);
  delete g_api;
  g_api = nullptr;
  g_refs = 0;
}

}  // namespace

// Reference-counted: every user (health monitor, exporter, labeller) opens
// and closes its own reference on the one per-process session.
extern "C" int mx_smi_open(char* err, size_t errlen) {
  std::unique_lock<std::shared_mutex> life(g_life);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api) {
    ++g_refs;
    return 1;
  }
  const char* env = std::getenv("MXK8S_AMDSMI_LIB");
  const char* candidates[] = {env, "libamd_smi.so", "/opt/rocm/lib/libamd_smi.so"};
  void* h = nullptr;
  for (const char* c : candidates) {
    if (!c || !*c) continue;
    h = dlopen(c, RTLD_NOW | RTLD_LOCAL);
    if (h) break;
  }
  if (!h) {
    mx::set_err(err, errlen, std::string("cannot load libamd_smi.so: ") + dlerror());
    return 0;
  }
  auto* api = new SmiApi();
  api->handle = h;
  bool ok = true;
#define B(name) ok &= bind(h, #name, &api->name)
  B(amdsmi_init); B(amdsmi_shut_down); B(amdsmi_get_socket_handles);
  B(amdsmi_get_processor_handles); B(amdsmi_get_processor_type); B(amdsmi_get_gpu_bdf_id);
  B(amdsmi_get_gpu_activity); B(amdsmi_get_gpu_memory_usage); B(amdsmi_get_gpu_memory_total);
  B(amdsmi_get_temp_metric); B(amdsmi_get_power_info); B(amdsmi_get_clock_info);
  B(amdsmi_get_gpu_total_ecc_count); B(amdsmi_get_gpu_process_list);
  B(amdsmi_get_gpu_driver_info);
#undef B
  // event API is optional
  bind(h, "amdsmi_init_gpu_event_notification", &api->amdsmi_init_gpu_event_notification);
  bind(h, "amdsmi_set_gpu_event_notification_mask", &api->amdsmi_set_gpu_event_notification_mask);
  bind(h, "amdsmi_get_gpu_event_notification", &api->amdsmi_get_gpu_event_notification);
  bind(h, "amdsmi_stop_gpu_event_notification", &api->amdsmi_stop_gpu_event_notification);
  // xGMI link state / traffic: optional too (guest / older amd-smi)
  bind(h, "amdsmi_get_gpu_xgmi_link_status", &api->amdsmi_get_gpu_xgmi_link_status);
  bind(h, "amdsmi_get_link_metrics", &api->amdsmi_get_link_metrics);
  // energy accumulator: optional (dcgm-exporter's total-energy counterpart)
  bind(h, "amdsmi_get_energy_count", &api->amdsmi_get_energy_count);
  if (!ok) {
    mx::set_err(err, errlen, "libamd_smi.so lacks required symbols");
    dlclose(h);
    delete api;
    return 0;
  }
  std::string why;
  if (!init_session(api, &why)) {
    mx::set_err(err, errlen, why);
    dlclose(h);
    delete api;
    return 0;
  }
  g_api = api;
  g_refs = 1;
  return 1;
}

// Releases one reference; the session ends with the last one.
extern "C" void mx_smi_close(void) {
  std::unique_lock<std::shared_mutex> life(g_life);
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_api) return;
  if (--g_refs > 0) return;
  destroy_locked();
}

// Ends the session whatever the reference count (process teardown, tests).
extern "C" void mx_smi_reset(void) {
  std::unique_lock<std::shared_mutex> life(g_life);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api) destroy_locked();
}

// amdsmi_shut_down + amdsmi_init on the open session: a new handle list (and
// generation).  Every index from before is void; users re-match by BDF +
// partition when mx_smi_generation() changes.  Waits for a blocked
// mx_smi_wait_events to return.  0 (msg in err) if amd-smi is not open or the
// init failed (the session then has no GPUs until the next re-init).
extern "C" int mx_smi_reinit(char* err, size_t errlen) {
  std::unique_lock<std::shared_mutex> life(g_life);
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_api) {
    mx::set_err(err, errlen, "amd-smi is not open");
    return 0;
  }
  end_session(g_api);
  std::string why;
  if (!init_session(g_api, &why)) {
    ++g_gen;
    mx::set_err(err, errlen, why);
    return 0;
  }
  return 1;
}

extern "C" uint64_t mx_smi_generation(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_api ? g_gen : 0;
}

extern "C" int mx_smi_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_api ? static_cast<int>(g_api->gpus.size()) : -1;
}

extern "C" const char* mx_smi_driver_version(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_api ? g_api->driver_version.c_str() : "";
}

extern "C" int mx_smi_sample(int i, mx_gpu_sample* o) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::memset(o, 0, sizeof(*o));
  o->index = i;
  o->temp_edge_mc = o->temp_hotspot_mc = o->temp_mem_mc = INT64_MIN;
  o->energy_j = -1.0;
  if (!g_api || i < 0 || i >= static_cast<int>(g_api->gpus.size())) return 0;
  SmiApi& a = *g_api;
  amdsmi_processor_handle h = a.gpus[i];
  uint64_t bdf = 0;
  if (a.amdsmi_get_gpu_bdf_id(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
    fmt_bdf(bdf, o->bdf, sizeof(o->bdf));
    o->partition_id = static_cast<int>((bdf >> 28) & 0xf);
  }
  amdsmi_engine_usage_t u;
  std::memset(&u, 0, sizeof(u));
  if (a.amdsmi_get_gpu_activity(h, &u) == AMDSMI_STATUS_SUCCESS) {
    o->gfx_activity_pct = u.gfx_activity;
    o->umc_activity_pct = u.umc_activity;
  }
  a.amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &o->vram_used_bytes);
  a.amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &o->vram_total_bytes);
  int64_t t = 0;
  if (a.amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_EDGE, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
    o->temp_edge_mc = t * 1000;
  if (a.amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
    o->temp_hotspot_mc = t * 1000;
  if (a.amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_VRAM, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
    o->temp_mem_mc = t * 1000;
  amdsmi_power_info_t p;
  std::memset(&p, 0, sizeof(p));
  if (a.amdsmi_get_power_info(h, &p) == AMDSMI_STATUS_SUCCESS) {
    o->power_w = p.current_socket_power ? p.current_socket_power
                                        : (p.socket_power ? p.socket_power : p.average_socket_power);
    // ROCm 7.2 amd-smi reports power_limit in microwatts on MI355X (1.4e9 = 1400 W)
    o->power_limit_w = p.power_limit > 100000u ? p.power_limit / 1000000u : p.power_limit;
  }
  if (a.amdsmi_get_energy_count) {
    uint64_t acc = 0, ts = 0;
    float res = 0.f;   // microjoules per count
    if (a.amdsmi_get_energy_count(h, &acc, &res, &ts) == AMDSMI_STATUS_SUCCESS && res > 0.f)
      o->energy_j = static_cast<double>(acc) * res * 1e-6;
  }
  amdsmi_clk_info_t c;
  std::memset(&c, 0, sizeof(c));
  if (a.amdsmi_get_clock_info(h, AMDSMI_CLK_TYPE_SYS, &c) == AMDSMI_STATUS_SUCCESS) o->sclk_mhz = c.clk;
  std::memset(&c, 0, sizeof(c));
  if (a.amdsmi_get_clock_info(h, AMDSMI_CLK_TYPE_MEM, &c) == AMDSMI_STATUS_SUCCESS) o->mclk_mhz = c.clk;
  amdsmi_error_count_t e;
  std::memset(&e, 0, sizeof(e));
  if (a.amdsmi_get_gpu_total_ecc_count(h, &e) == AMDSMI_STATUS_SUCCESS) {
    o->ecc_correctable = e.correctable_count;
    o->ecc_uncorrectable = e.uncorrectable_count;
  }
  uint32_t np = 0;
  if (a.amdsmi_get_gpu_process_list(h, &np, nullptr) == AMDSMI_STATUS_SUCCESS) o->num_processes = np;
  o->valid = 1;
  return 1;
}

// Accumulated RAS counts of GPU i only (the health monitor's per-pass probe).
extern "C" int mx_smi_ecc(int i, uint64_t* correctable, uint64_t* uncorrectable) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_api || i < 0 || i >= static_cast<int>(g_api->gpus.size())) return 0;
  amdsmi_error_count_t e;
  std::memset(&e, 0, sizeof(e));
  if (g_api->amdsmi_get_gpu_total_ecc_count(g_api->gpus[i], &e) != AMDSMI_STATUS_SUCCESS) return 0;
  *correctable = e.correctable_count;
  *uncorrectable = e.uncorrectable_count;
  return 1;
}

extern "C" int mx_smi_wait_events(int timeout_ms, int* gpu_out, int* event_out, int max) {
  std::shared_lock<std::shared_mutex> life(g_life);   // no re-init / shutdown under the wait
  SmiApi* a;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    a = g_api;
    if (!a || !a->amdsmi_get_gpu_event_notification) return -1;
    if (!a->events_on) {
      const uint64_t mask = (1ull << (AMDSMI_EVT_NOTIF_GPU_PRE_RESET - 1)) |
                            (1ull << (AMDSMI_EVT_NOTIF_GPU_POST_RESET - 1)) |
                            (1ull << (AMDSMI_EVT_NOTIF_THERMAL_THROTTLE - 1)) |
                            (1ull << (AMDSMI_EVT_NOTIF_VMFAULT - 1));
      for (auto h : a->gpus) {
        if (a->amdsmi_init_gpu_event_notification(h) != AMDSMI_STATUS_SUCCESS) return -1;
        a->amdsmi_set_gpu_event_notification_mask(h, mask);
      }
      a->events_on = true;
    }
  }
  std::vector<amdsmi_evt_notification_data_t> ev(max > 0 ? max : 1);
  uint32_t n = static_cast<uint32_t>(ev.size());
  amdsmi_status_t st = a->amdsmi_get_gpu_event_notification(timeout_ms, &n, ev.data());
  if (st != AMDSMI_STATUS_SUCCESS) return st == AMDSMI_STATUS_NO_DATA ? 0 : -1;
  std::lock_guard<std::mutex> lk(g_mu);
  int count = 0;
  for (uint32_t k = 0; k < n && count < max; ++k) {
    int gi = -1;
    for (size_t j = 0; j < a->gpus.size(); ++j)
      if (a->gpus[j] == ev[k].processor_handle) gi = static_cast<int>(j);
    gpu_out[count] = gi;
    event_out[count] = static_cast<int>(ev[k].event);
    ++count;
  }
  return count;
}

// xGMI links of GPU i: link state (amdsmi_get_gpu_xgmi_link_status) merged by
// link index with the per-link traffic counters (amdsmi_get_link_metrics).
// Returns the number of links written, 0 if the GPU has none, -1 if amd-smi
// supports neither query on this host.
extern "C" int mx_smi_xgmi_links(int i, mx_xgmi_link_sample* out, int max) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_api || i < 0 || i >= static_cast<int>(g_api->gpus.size()) || max <= 0) return -1;
  SmiApi& a = *g_api;
  amdsmi_processor_handle h = a.gpus[i];
  int nstat = -1, nmet = -1;
  amdsmi_xgmi_link_status_t ls;
  std::memset(&ls, 0, sizeof(ls));
  if (a.amdsmi_get_gpu_xgmi_link_status &&
      a.amdsmi_get_gpu_xgmi_link_status(h, &ls) == AMDSMI_STATUS_SUCCESS)
    nstat = static_cast<int>(std::min<uint32_t>(ls.total_links, AMDSMI_MAX_NUM_XGMI_LINKS));
  static thread_local amdsmi_link_metrics_t lm;   // ~3 KiB: keep it off the stack
  std::memset(&lm, 0, sizeof(lm));
  if (a.amdsmi_get_link_metrics && a.amdsmi_get_link_metrics(h, &lm) == AMDSMI_STATUS_SUCCESS)
    nmet = static_cast<int>(std::min<uint32_t>(lm.num_links, AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK));
  if (nstat < 0 && nmet < 0) return -1;
  const int n = std::min(max, std::max(nstat, nmet));
  for (int k = 0; k < n; ++k) {
    mx_xgmi_link_sample& o = out[k];
    std::memset(&o, 0, sizeof(o));
    o.link = k;
    o.status = k < nstat ? static_cast<int>(ls.status[k]) : -1;
    if (k < nmet) {
      const auto& L = lm.links[k];
      std::snprintf(o.peer_bdf, sizeof(o.peer_bdf), "%04llx:%02llx:%02llx.%llx",
                    static_cast<unsigned long long>(L.bdf.domain_number & 0xffff),
                    static_cast<unsigned long long>(L.bdf.bus_number),
                    static_cast<unsigned long long>(L.bdf.device_number),
                    static_cast<unsigned long long>(L.bdf.function_number));
      o.link_type = static_cast<int>(L.link_type);
      o.bit_rate_gbps = L.bit_rate;
      o.max_bandwidth_gbps = L.max_bandwidth;
      o.read_kb = L.read;
      o.write_kb = L.write;
      o.has_traffic = 1;
    } else {
      o.link_type = -1;
    }
  }
  return n;
}

// Processes holding GPU i (amdsmi_get_gpu_process_list): pid, name, VRAM.
// Returns the count written (<= max), -1 if amd-smi is not open.
extern "C" int mx_smi_processes(int i, mx_proc_sample* out, int max) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_api || i < 0 || i >= static_cast<int>(g_api->gpus.size())) return -1;
  SmiApi& a = *g_api;
  uint32_t n = 0;
  if (a.amdsmi_get_gpu_process_list(a.gpus[i], &n, nullptr) != AMDSMI_STATUS_SUCCESS) return 0;
  if (n == 0 || max <= 0) return 0;
  std::vector<amdsmi_proc_info_t> ps(n);
  uint32_t got = n;
  const amdsmi_status_t st = a.amdsmi_get_gpu_process_list(a.gpus[i], &got, ps.data());
  if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return 0;
  const int cnt = std::min<int>(max, static_cast<int>(std::min<uint32_t>(got, n)));
  for (int k = 0; k < cnt; ++k) {
    mx_proc_sample& o = out[k];
    std::memset(&o, 0, sizeof(o));
    o.pid = ps[k].pid;
    std::snprintf(o.name, sizeof(o.name), "%s", ps[k].name);
    std::snprintf(o.container, sizeof(o.container), "%s", ps[k].container_name);
    o.vram_bytes = ps[k].memory_usage.vram_mem ? ps[k].memory_usage.vram_mem : ps[k].mem;
    o.gtt_bytes = ps[k].memory_usage.gtt_mem;
    o.cu_occupancy = ps[k].cu_occupancy;
  }
  return cnt;
}
