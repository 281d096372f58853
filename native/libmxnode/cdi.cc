// N03: ROCm CDI spec generator (replaces nvidia-container-toolkit / nvidia-ctk,
// /root/reference/README.md:138-149).
//
// Emits a CDI 0.6.0 spec for kind `amd.com/gpu`:
//   * top-level containerEdits: /dev/kfd (the compute interface every ROCm
//     process needs, shared by all GPUs)
//   * one device per GPU, named by index ("0".."7") AND by uuid ("GPU-<id>"),
//     carrying that GPU's /dev/dri/renderD<minor> (+ /dev/dri/card<N>)
//   * "all" = every GPU's nodes
// No runtime shim, no hooks, no env: the KFD lets a process use exactly the
// GPUs whose render node it can open, so device-node injection alone scopes a
// container to its allocation.
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

namespace {

void node_json(std::ostringstream& o, const std::string& path) {
  o << "{\"path\":\"" << mx::json_escape(path) << "\",\"type\":\"c\",\"permissions\":\"rw\"}";
}

void gpu_nodes(std::ostringstream& o, const mx_gpu_info& g, bool& first) {
  if (!first) o << ",";
  first = false;
  node_json(o, "/dev/dri/renderD" + std::to_string(g.drm_render_minor));
  if (g.drm_card >= 0) {
    o << ",";
    node_json(o, "/dev/dri/card" + std::to_string(g.drm_card));
  }
}

void device_json(std::ostringstream& o, const std::string& name, const mx_gpu_info& g) {
  o << "{\"name\":\"" << mx::json_escape(name) << "\",\"annotations\":{"
    << "\"amd.com/gpu.bdf\":\"" << g.pci_bdf << "\","
    << "\"amd.com/gpu.arch\":\"" << g.gfx_arch << "\"},"
    << "\"containerEdits\":{\"deviceNodes\":[";
  bool first = true;
  gpu_nodes(o, g, first);
  o << "]}}";
}

}  // namespace

extern "C" long mx_cdi_spec(const char* root, const char* kind, char* buf, size_t buflen, char* err,
                            size_t errlen) {
  mx_gpu_info gpus[MX_MAX_GPUS];
  const int n = mx_enumerate(root, gpus, MX_MAX_GPUS, err, errlen);
  if (n < 0) return -1;
  const std::string k = (kind && *kind) ? kind : "amd.com/gpu";
  std::ostringstream o;
  o << "{\"cdiVersion\":\"0.6.0\",\"kind\":\"" << mx::json_escape(k) << "\",";
  o << "\"containerEdits\":{\"deviceNodes\":[";
  node_json(o, "/dev/kfd");
  o << "]},\"devices\":[";
  const int m = n < MX_MAX_GPUS ? n : MX_MAX_GPUS;
  for (int i = 0; i < m; ++i) {
    if (i) o << ",";
    device_json(o, std::to_string(gpus[i].index), gpus[i]);
    o << ",";
    device_json(o, gpus[i].uuid, gpus[i]);
  }
  if (m > 0) {
    o << ",{\"name\":\"all\",\"containerEdits\":{\"deviceNodes\":[";
    bool first = true;
    for (int i = 0; i < m; ++i) gpu_nodes(o, gpus[i], first);
    o << "]}}";
  }
  o << "]}";
  const std::string s = o.str();
  if (buf && buflen) {
    const size_t c = s.size() < buflen - 1 ? s.size() : buflen - 1;
    std::memcpy(buf, s.data(), c);
    buf[c] = 0;
  }
  return static_cast<long>(s.size());
}
