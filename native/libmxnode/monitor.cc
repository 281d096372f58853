// N02: the device plugin's health state machine (the NVML Xid / DBE watch of
// the NVIDIA device plugin the reference installs at README.md:269-271,
// re-designed for amdgpu: KFD/sysfs presence, amd-smi event notifications and
// RAS uncorrectable-ECC counters).  See mxnode.h "N02 health monitor" for the
// policy; the Python plugin only maps verdicts onto ListAndWatch / Allocate.
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

namespace {

int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int64_t unix_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

bool write_atomic(const std::string& path, const std::string& text) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  if (!f) return false;
  const bool ok = std::fwrite(text.data(), 1, text.size(), f) == text.size();
  if (std::fclose(f) != 0 || !ok) {
    std::remove(tmp.c_str());
    return false;
  }
  return std::rename(tmp.c_str(), path.c_str()) == 0;
}

}  // namespace

struct mx_health_monitor {
  struct Gpu {
    mx_gpu_info info;
    int smi_index = -1;
    int code = MX_HEALTHY;
    int64_t event_until = 0;    // monotonic ms
    int64_t ecc_until = 0;
    bool ecc_valid = false;
    bool base_set = false;
    uint64_t ecc_ue = 0, ecc_base = 0;
    uint64_t vm_faults = 0, thermal = 0, resets = 0;
  };
  std::mutex mu;
  std::string root, fault_file, state_dir, boot_id;
  int64_t event_q_ms = 60000, ecc_q_ms = 0;
  bool smi = false;
  uint64_t smi_gen = 0;          // amd-smi session generation the smi_index values belong to
  std::vector<Gpu> gpus;
  std::deque<mx_health_event> log;
  uint64_t seq = 0;

  int by_smi(int smi_index) const {
    for (size_t i = 0; i < gpus.size(); ++i)
      if (gpus[i].smi_index == smi_index) return static_cast<int>(i);
    return -1;
  }

  void event(int index, int kind, int64_t value, const std::string& msg) {
    mx_health_event e;
    std::memset(&e, 0, sizeof(e));
    e.seq = ++seq;
    e.index = index;
    e.kind = kind;
    e.value = value;
    e.unix_ms = unix_ms();
    std::snprintf(e.message, sizeof(e.message), "%s", msg.c_str());
    log.push_back(e);
    while (log.size() > 1024) log.pop_front();
  }

  // amd-smi index of every GPU, matched by BDF (+ partition id: partitions of
  // one device share the BDF).  Returns the number of GPUs left unmatched.
  int match_smi() {
    for (auto& g : gpus) g.smi_index = -1;
    smi_gen = mx_smi_generation();
    const int ns = mx_smi_count();
    for (int k = 0; k < ns; ++k) {
      mx_gpu_sample s;
      mx_smi_sample(k, &s);
      for (auto& g : gpus)
        if (std::strcmp(s.bdf, g.info.pci_bdf) == 0 && s.partition_id == g.info.partition)
          g.smi_index = k;
    }
    int unmatched = 0;
    for (const auto& g : gpus) unmatched += g.smi_index < 0;
    return unmatched;
  }

  std::string baseline_path() const { return state_dir.empty() ? "" : state_dir + "/ecc-baseline"; }

  void load_baseline() {
    const std::string p = baseline_path();
    std::string text;
    if (p.empty() || !mx::read_file(p, &text)) return;
    std::istringstream in(text);
    std::string tag, id;
    if (!(in >> tag >> id) || tag != "boot" || id != boot_id) return;   // a new boot: fresh
    std::string bdf;
    unsigned long long count = 0;
    while (in >> bdf >> count)
      for (auto& g : gpus)
        if (bdf == g.info.pci_bdf) {
          g.ecc_base = count;
          g.base_set = true;
        }
  }

  void save_baseline() const {
    const std::string p = baseline_path();
    if (p.empty()) return;
    std::ostringstream out;
    out << "boot " << boot_id << "\n";
    for (const auto& g : gpus)
      if (g.base_set) out << g.info.pci_bdf << " " << g.ecc_base << "\n";
    ::mkdir(state_dir.c_str(), 0755);
    write_atomic(p, out.str());
  }
};

extern "C" mx_health_monitor* mx_hm_create(const mx_health_opts* o, char* err, size_t errlen) {
  if (!o) {
    mx::set_err(err, errlen, "null options");
    return nullptr;
  }
  auto* m = new mx_health_monitor();
  m->root = o->root ? o->root : "";
  m->fault_file = o->fault_file ? o->fault_file : "";
  m->state_dir = o->state_dir ? o->state_dir : "";
  m->event_q_ms = o->event_quarantine_ms;
  m->ecc_q_ms = o->ecc_quarantine_ms;
  std::string bid;
  mx::read_file(o->boot_id_file && *o->boot_id_file ? o->boot_id_file
                                                    : "/proc/sys/kernel/random/boot_id",
                &bid);
  m->boot_id = mx::trim(bid).empty() ? "unknown" : mx::trim(bid);

  mx_gpu_info infos[MX_MAX_GPUS];
  const int n = mx_enumerate(m->root.c_str(), infos, MX_MAX_GPUS, err, errlen);
  if (n < 0) {
    delete m;
    return nullptr;
  }
  for (int i = 0; i < n; ++i) {
    mx_health_monitor::Gpu g;
    g.info = infos[i];
    m->gpus.push_back(g);
  }
  if (o->use_smi) {
    char serr[256] = {0};
    if (mx_smi_open(serr, sizeof(serr))) {
      m->smi = true;
      // amd-smi enumerates at init: a session opened before a partition change
      // (SPX -> CPX: 8 -> 64 KFD GPUs) or a driver reload holds the old handle
      // list.  KFD and amd-smi disagreeing on the count is that case: re-init
      // and match again (other users of the session re-match on the new
      // generation).
      if (m->match_smi() > 0 && mx_smi_count() != static_cast<int>(m->gpus.size())) {
        if (mx_smi_reinit(serr, sizeof(serr)))
          m->event(-1, MX_EVT_HEALTH_CHANGE, 0, "amd-smi re-initialised: GPU set changed");
        else
          m->event(-1, MX_EVT_HEALTH_CHANGE, 0, std::string("amd-smi re-init failed: ") + serr);
        m->match_smi();
      }
    } else {
      m->event(-1, MX_EVT_HEALTH_CHANGE, 0, std::string("amd-smi unavailable: ") + serr);
    }
  }
  m->load_baseline();
  return m;
}

extern "C" void mx_hm_destroy(mx_health_monitor* m) {
  if (m && m->smi) mx_smi_close();
  delete m;
}

extern "C" int mx_hm_smi_active(mx_health_monitor* m) { return m && m->smi ? 1 : 0; }

extern "C" int mx_hm_step(mx_health_monitor* m, int wait_ms) {
  if (!m) return -1;
  // 0. another user re-initialised amd-smi: every cached index is void
  if (m->smi && mx_smi_generation() != m->smi_gen) {
    std::lock_guard<std::mutex> lk(m->mu);
    m->match_smi();
  }
  // 1. amd-smi events (blocking wait outside the monitor lock)
  int gi[64], ev[64];
  int nev = 0;
  if (m->smi) {
    nev = mx_smi_wait_events(wait_ms, gi, ev, 64);
    if (nev < 0) nev = 0;
  }
  // 2. ECC counters (amd-smi calls, also outside the lock)
  std::vector<std::pair<int, uint64_t>> ecc;   // (gpu, uncorrectable)
  if (m->smi) {
    for (size_t i = 0; i < m->gpus.size(); ++i) {
      uint64_t ce = 0, ue = 0;
      if (m->gpus[i].smi_index >= 0 && mx_smi_ecc(m->gpus[i].smi_index, &ce, &ue))
        ecc.emplace_back(static_cast<int>(i), ue);
    }
  }
  // 3. sysfs checks
  std::vector<int> sysfs(m->gpus.size());
  for (size_t i = 0; i < m->gpus.size(); ++i)
    sysfs[i] = mx_health_check(m->root.c_str(), static_cast<int>(i), m->fault_file.c_str());

  std::lock_guard<std::mutex> lk(m->mu);
  if (m->smi && mx_smi_generation() != m->smi_gen) m->match_smi();   // re-init during the wait
  const int64_t now = mono_ms();
  for (int k = 0; k < nev; ++k) {
    const int i = m->by_smi(gi[k]);
    mx_health_monitor::Gpu* g = i >= 0 ? &m->gpus[i] : nullptr;
    switch (ev[k]) {
      case MX_EVT_VMFAULT:
        if (g) { ++g->vm_faults; g->event_until = now + m->event_q_ms; }
        m->event(i, MX_EVT_VMFAULT, 0, "amd-smi: VM fault");
        break;
      case MX_EVT_GPU_PRE_RESET:
        if (g) { ++g->resets; g->event_until = now + m->event_q_ms; }
        m->event(i, MX_EVT_GPU_PRE_RESET, 0, "amd-smi: GPU pre-reset");
        break;
      case MX_EVT_GPU_POST_RESET:
        m->event(i, MX_EVT_GPU_POST_RESET, 0, "amd-smi: GPU post-reset");
        break;
      case MX_EVT_THERMAL_THROTTLE:
        if (g) ++g->thermal;
        m->event(i, MX_EVT_THERMAL_THROTTLE, g ? static_cast<int64_t>(g->thermal) : 0,
                 "amd-smi: thermal throttle");
        break;
      default:
        m->event(i, ev[k], 0, "amd-smi: event " + std::to_string(ev[k]));
    }
  }
  bool save = false;
  for (const auto& e : ecc) {
    auto& g = m->gpus[e.first];
    g.ecc_valid = true;
    g.ecc_ue = e.second;
    if (!g.base_set) {
      g.ecc_base = e.second;
      g.base_set = true;
      save = true;
      continue;
    }
    if (e.second > g.ecc_base) {
      const bool first = m->ecc_q_ms > 0 || g.code != MX_UNHEALTHY_ECC;
      if (first)
        m->event(e.first, MX_EVT_ECC_UNCORRECTABLE, static_cast<int64_t>(e.second - g.ecc_base),
                 "uncorrectable ECC errors: " + std::to_string(e.second) + " (baseline " +
                     std::to_string(g.ecc_base) + ")");
      if (m->ecc_q_ms > 0) {   // quarantine, then forgive: the new count is the baseline
        g.ecc_until = now + m->ecc_q_ms;
        g.ecc_base = e.second;
        save = true;
      }
    }
  }
  if (save) m->save_baseline();

  int changed = 0;
  for (size_t i = 0; i < m->gpus.size(); ++i) {
    auto& g = m->gpus[i];
    int code = sysfs[i];
    if (code == MX_HEALTHY) {
      const bool ecc_bad = (m->ecc_q_ms <= 0 && g.ecc_valid && g.ecc_ue > g.ecc_base) ||
                           g.ecc_until > now;
      if (ecc_bad) code = MX_UNHEALTHY_ECC;
      else if (g.event_until > now) code = MX_UNHEALTHY_SMI_EVENT;
    }
    if (code != g.code) {
      g.code = code;
      ++changed;
      m->event(static_cast<int>(i), MX_EVT_HEALTH_CHANGE, code, mx_health_reason(code));
    }
  }
  return changed;
}

extern "C" int mx_hm_status(mx_health_monitor* m, mx_health_status* out, int max) {
  if (!m) return -1;
  std::lock_guard<std::mutex> lk(m->mu);
  const int64_t now = mono_ms();
  const int n = std::min<int>(max, static_cast<int>(m->gpus.size()));
  for (int i = 0; i < n; ++i) {
    const auto& g = m->gpus[i];
    mx_health_status& s = out[i];
    std::memset(&s, 0, sizeof(s));
    s.index = i;
    s.code = g.code;
    s.smi_index = g.smi_index;
    s.ecc_valid = g.ecc_valid;
    s.ecc_uncorrectable = g.ecc_ue;
    s.ecc_baseline = g.ecc_base;
    s.vm_faults = g.vm_faults;
    s.thermal_throttles = g.thermal;
    s.resets = g.resets;
    s.quarantine_left_ms = std::max<int64_t>(0, std::max(g.event_until, g.ecc_until) - now);
    std::snprintf(s.bdf, sizeof(s.bdf), "%s", g.info.pci_bdf);
  }
  return n;
}

extern "C" int mx_hm_events(mx_health_monitor* m, uint64_t after, mx_health_event* out, int max) {
  if (!m) return -1;
  std::lock_guard<std::mutex> lk(m->mu);
  int n = 0;
  for (const auto& e : m->log) {
    if (e.seq <= after) continue;
    if (n >= max) break;
    out[n++] = e;
  }
  return n;
}

extern "C" int mx_hm_write_state(mx_health_monitor* m, const char* path) {
  if (!m || !path) return -1;
  std::ostringstream j;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    const int64_t now = mono_ms();
    j << "{\"boot_id\":\"" << mx::json_escape(m->boot_id) << "\",\"unix_ms\":" << unix_ms()
      << ",\"smi\":" << (m->smi ? "true" : "false") << ",\"ecc_policy\":\""
      << (m->ecc_q_ms > 0 ? "quarantine" : "sticky-until-reboot") << "\",\"gpus\":[";
    for (size_t i = 0; i < m->gpus.size(); ++i) {
      const auto& g = m->gpus[i];
      j << (i ? "," : "") << "{\"index\":" << i << ",\"bdf\":\"" << g.info.pci_bdf
        << "\",\"partition\":" << g.info.partition << ",\"uuid\":\"" << g.info.uuid
        << "\",\"healthy\":"
        << (g.code == MX_HEALTHY ? "true" : "false") << ",\"code\":" << g.code
        << ",\"reason\":\"" << mx_health_reason(g.code) << "\",\"ecc_uncorrectable\":"
        << g.ecc_ue << ",\"ecc_baseline\":" << g.ecc_base << ",\"vm_faults\":" << g.vm_faults
        << ",\"thermal_throttles\":" << g.thermal << ",\"resets\":" << g.resets
        << ",\"quarantine_left_ms\":"
        << std::max<int64_t>(0, std::max(g.event_until, g.ecc_until) - now) << "}";
    }
    j << "]}\n";
  }
  return write_atomic(path, j.str()) ? 0 : -1;
}
