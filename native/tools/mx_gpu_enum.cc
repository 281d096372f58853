// mx-gpu-enum: print the node's AMD GPUs (and xGMI/PCIe links) as JSON.
//   mx-gpu-enum [--root DIR] [--links]
// The C++ counterpart of `nvidia-smi -L` in the reference's driver gate
// (/root/reference/README.md:76-84), reading the KFD topology directly.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

int main(int argc, char** argv) {
  std::string root;
  bool links = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
    else if (!std::strcmp(argv[i], "--links")) links = true;
    else if (!std::strcmp(argv[i], "-h") || !std::strcmp(argv[i], "--help")) {
      std::printf("usage: %s [--root DIR] [--links]\n", argv[0]);
      return 0;
    } else {
      std::fprintf(stderr, "unknown argument %s\n", argv[i]);
      return 2;
    }
  }
  char err[512] = {0};
  std::vector<mx_gpu_info> g(MX_MAX_GPUS);
  int n = mx_enumerate(root.c_str(), g.data(), MX_MAX_GPUS, err, sizeof(err));
  if (n < 0) {
    std::fprintf(stderr, "mx-gpu-enum: %s\n", err);
    return 1;
  }
  std::printf("{\"count\":%d,\"gpus\":[", n);
  for (int i = 0; i < n && i < MX_MAX_GPUS; ++i) {
    const mx_gpu_info& x = g[i];
    std::printf("%s{\"index\":%d,\"kfd_node\":%d,\"gpu_id\":%u,\"arch\":\"%s\",\"gfx_target_version\":%u,"
                "\"product\":\"%s\",\"device_id\":\"0x%04x\",\"bdf\":\"%s\",\"numa_node\":%d,"
                "\"render_minor\":%d,\"card\":%d,\"cu_count\":%u,\"simd_count\":%u,"
                "\"vram_bytes\":%llu,\"max_sclk_mhz\":%u,\"hive_id\":\"0x%llx\","
                "\"xgmi_links\":%d,\"uuid\":\"%s\"}",
                i ? "," : "", x.index, x.kfd_node, x.gpu_id, x.gfx_arch, x.gfx_target_version,
                mx::json_escape(x.product).c_str(), x.device_id, x.pci_bdf, x.numa_node,
                x.drm_render_minor, x.drm_card, x.cu_count, x.simd_count,
                static_cast<unsigned long long>(x.vram_bytes), x.max_engine_clk_mhz,
                static_cast<unsigned long long>(x.hive_id), x.num_xgmi_links, x.uuid);
  }
  std::printf("]");
  if (links) {
    std::vector<mx_link> l(MX_MAX_GPUS * MX_MAX_LINKS);
    int nl = mx_links(root.c_str(), l.data(), static_cast<int>(l.size()), err, sizeof(err));
    std::printf(",\"links\":[");
    for (int i = 0; i < nl; ++i)
      std::printf("%s{\"from\":%d,\"to\":%d,\"type\":\"%s\",\"weight\":%u,\"max_bandwidth_mbps\":%u}",
                  i ? "," : "", l[i].from_index, l[i].to_index,
                  l[i].type == 11 ? "xgmi" : (l[i].type == 2 ? "pcie" : "other"), l[i].weight,
                  l[i].max_bandwidth_mbps);
    std::printf("]");
  }
  std::printf("}\n");
  return 0;
}
