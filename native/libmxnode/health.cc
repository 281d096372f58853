// N02 (sysfs part): per-GPU health for the device plugin's ListAndWatch.
//
// The reference's device plugin marks GPUs unhealthy from NVML Xid events
// [ext, R26d].  Here a GPU is unhealthy when:
//   * its KFD topology node disappeared (device lost / driver unbound),
//   * its /dev/dri/renderD<minor> node is gone (hot-unplug, reset in progress),
//   * the fault-injection file names it (tests / drills: one index per line,
//     or "all"),
// and, from the amd-smi event stream (smi.cc), on GPU reset / RAS events.
#include <sstream>
#include <string>

#include "mxnode.h"
#include "util.h"

extern "C" int mx_health_check(const char* root_c, int index, const char* fault_file) {
  const std::string root = root_c ? root_c : "";
  if (fault_file && *fault_file) {
    std::string text;
    if (mx::read_file(fault_file, &text)) {
      std::istringstream in(text);
      std::string line;
      while (std::getline(in, line)) {
        line = mx::trim(line);
        if (line.empty() || line[0] == '#') continue;
        if (line == "all" || line == std::to_string(index)) return MX_UNHEALTHY_FAULT_INJECTED;
      }
    }
  }
  mx_gpu_info gpus[MX_MAX_GPUS];
  const int n = mx_enumerate(root_c, gpus, MX_MAX_GPUS, nullptr, 0);
  if (n < 0 || index < 0 || index >= n) return MX_UNHEALTHY_NO_KFD_NODE;
  const std::string render = mx::rooted(root, "/dev/dri/renderD" + std::to_string(gpus[index].drm_render_minor));
  if (!mx::path_exists(render)) return MX_UNHEALTHY_NO_RENDER_NODE;
  return MX_HEALTHY;
}

extern "C" const char* mx_health_reason(int code) {
  switch (code) {
    case MX_HEALTHY: return "healthy";
    case MX_UNHEALTHY_NO_KFD_NODE: return "kfd topology node missing";
    case MX_UNHEALTHY_NO_RENDER_NODE: return "render node missing";
    case MX_UNHEALTHY_FAULT_INJECTED: return "fault injected";
    case MX_UNHEALTHY_SMI_EVENT: return "amd-smi reset/fault event";
    case MX_UNHEALTHY_ECC: return "uncorrectable ECC errors";
    default: return "unknown";
  }
}
