// N01: GPU discovery from the KFD topology in sysfs (no ROCm runtime needed).
//
// /sys/class/kfd/kfd/topology/nodes/<n>/{properties,gpu_id,name,mem_banks,io_links}
// A node is a GPU when simd_count > 0 and gpu_id != 0; GPU index order is
// KFD node order, which is the ROCr/HIP agent enumeration order.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

namespace {

const char* kTopo = "/sys/class/kfd/kfd/topology/nodes";

struct RawNode {
  int kfd_node;
  std::map<std::string, std::string> props;
  uint32_t gpu_id;
};

bool load_nodes(const std::string& root, std::vector<RawNode>* nodes, std::string* err) {
  const std::string dir = mx::rooted(root, kTopo);
  if (!mx::is_dir(dir)) {
    *err = "no KFD topology at " + dir + " (amdgpu driver not loaded?)";
    return false;
  }
  for (const std::string& name : mx::list_dir(dir)) {
    char* end = nullptr;
    long id = std::strtol(name.c_str(), &end, 10);
    if (!end || *end) continue;
    RawNode n;
    n.kfd_node = static_cast<int>(id);
    std::string text;
    if (!mx::read_file(dir + "/" + name + "/properties", &text)) continue;
    n.props = mx::parse_properties(text);
    std::string gid;
    n.gpu_id = 0;
    if (mx::read_file(dir + "/" + name + "/gpu_id", &gid)) n.gpu_id =
        static_cast<uint32_t>(std::strtoul(mx::trim(gid).c_str(), nullptr, 10));
    nodes->push_back(std::move(n));
  }
  std::sort(nodes->begin(), nodes->end(),
            [](const RawNode& a, const RawNode& b) { return a.kfd_node < b.kfd_node; });
  return true;
}

bool is_gpu(const RawNode& n) {
  return mx::prop_u64(n.props, "simd_count") > 0 && n.gpu_id != 0;
}

uint64_t vram_of(const std::string& root, int kfd_node) {
  const std::string dir = mx::rooted(root, kTopo) + "/" + std::to_string(kfd_node) + "/mem_banks";
  uint64_t best = 0;
  for (const std::string& b : mx::list_dir(dir)) {
    std::string text;
    if (!mx::read_file(dir + "/" + b + "/properties", &text)) continue;
    auto p = mx::parse_properties(text);
    const uint64_t heap = mx::prop_u64(p, "heap_type");
    // 1 = HSA_HEAPTYPE_FRAME_BUFFER_PUBLIC, 2 = FRAME_BUFFER_PRIVATE
    if (heap == 1 || heap == 2) best = std::max(best, mx::prop_u64(p, "size_in_bytes"));
  }
  return best;
}

int numa_of(const std::string& root, const std::string& bdf) {
  std::string t;
  if (!mx::read_file(mx::rooted(root, "/sys/bus/pci/devices/" + bdf + "/numa_node"), &t)) return -1;
  return static_cast<int>(std::strtol(mx::trim(t).c_str(), nullptr, 10));
}

int card_of(const std::string& root, const std::string& bdf, int render_minor) {
  for (const std::string& e : mx::list_dir(mx::rooted(root, "/sys/bus/pci/devices/" + bdf + "/drm"))) {
    if (e.rfind("card", 0) == 0) return static_cast<int>(std::strtol(e.c_str() + 4, nullptr, 10));
  }
  // fallback: scan /sys/class/drm/card*/device links for this BDF
  const std::string drm = mx::rooted(root, "/sys/class/drm");
  for (const std::string& e : mx::list_dir(drm)) {
    if (e.rfind("card", 0) != 0 || e.find('-') != std::string::npos) continue;
    std::string target;
    if (mx::read_link(drm + "/" + e + "/device", &target) &&
        target.size() >= bdf.size() && target.compare(target.size() - bdf.size(), bdf.size(), bdf) == 0)
      return static_cast<int>(std::strtol(e.c_str() + 4, nullptr, 10));
  }
  (void)render_minor;
  return -1;
}

void fill_info(const std::string& root, const RawNode& n, int index, mx_gpu_info* g) {
  std::memset(g, 0, sizeof(*g));
  const auto& p = n.props;
  g->index = index;
  g->kfd_node = n.kfd_node;
  g->gpu_id = n.gpu_id;
  g->gfx_target_version = static_cast<uint32_t>(mx::prop_u64(p, "gfx_target_version"));
  std::snprintf(g->gfx_arch, sizeof(g->gfx_arch), "%s", mx::gfx_name(g->gfx_target_version).c_str());
  g->drm_render_minor = static_cast<int>(mx::prop_u64(p, "drm_render_minor", 0));
  g->vendor_id = static_cast<uint32_t>(mx::prop_u64(p, "vendor_id"));
  g->device_id = static_cast<uint32_t>(mx::prop_u64(p, "device_id"));
  g->domain = static_cast<uint32_t>(mx::prop_u64(p, "domain"));
  g->location_id = static_cast<uint32_t>(mx::prop_u64(p, "location_id"));
  std::snprintf(g->pci_bdf, sizeof(g->pci_bdf), "%04x:%02x:%02x.%x", g->domain & 0xffff,
                (g->location_id >> 8) & 0xff, (g->location_id >> 3) & 0x1f, g->location_id & 0x7);
  g->simd_count = static_cast<uint32_t>(mx::prop_u64(p, "simd_count"));
  g->simd_per_cu = static_cast<uint32_t>(mx::prop_u64(p, "simd_per_cu", 4));
  g->cu_count = g->simd_per_cu ? g->simd_count / g->simd_per_cu : 0;
  g->unique_id = mx::prop_u64(p, "unique_id");
  g->hive_id = mx::prop_u64(p, "hive_id");
  g->max_engine_clk_mhz = static_cast<uint32_t>(mx::prop_u64(p, "max_engine_clk_fcompute"));
  g->vram_bytes = vram_of(root, n.kfd_node);
  if (g->vram_bytes == 0) g->vram_bytes = mx::prop_u64(p, "local_mem_size");
  g->numa_node = numa_of(root, g->pci_bdf);
  g->drm_card = card_of(root, g->pci_bdf, g->drm_render_minor);
  std::snprintf(g->product, sizeof(g->product), "%s", mx::product_name(g->device_id).c_str());
  if (g->unique_id)
    std::snprintf(g->uuid, sizeof(g->uuid), "GPU-%016llx",
                  static_cast<unsigned long long>(g->unique_id));
  else
    std::snprintf(g->uuid, sizeof(g->uuid), "GPU-%s", g->pci_bdf);
  // xGMI links
  const std::string ldir = mx::rooted(root, kTopo) + "/" + std::to_string(n.kfd_node) + "/io_links";
  int xg = 0;
  for (const std::string& l : mx::list_dir(ldir)) {
    std::string text;
    if (!mx::read_file(ldir + "/" + l + "/properties", &text)) continue;
    if (mx::prop_u64(mx::parse_properties(text), "type") == 11) ++xg;
  }
  g->num_xgmi_links = xg;
  g->num_xcc = static_cast<uint32_t>(mx::prop_u64(p, "num_xcc", 0));
  g->partition = 0;
  g->partitions = 1;
}

// Partitions of one PCI device (shared domain + location_id): number them in
// render-minor order and make their UUIDs distinct.
void mark_partitions(const std::string& root, mx_gpu_info* g, int n) {
  for (int i = 0; i < n; ++i) {
    int count = 0, rank = 0;
    for (int j = 0; j < n; ++j) {
      if (g[j].domain != g[i].domain || g[j].location_id != g[i].location_id) continue;
      ++count;
      if (g[j].drm_render_minor < g[i].drm_render_minor ||
          (g[j].drm_render_minor == g[i].drm_render_minor && j < i))
        ++rank;
    }
    g[i].partitions = count;
    g[i].partition = rank;
  }
  for (int i = 0; i < n; ++i) {
    if (g[i].partitions <= 1) continue;
    const size_t len = std::strlen(g[i].uuid);
    std::snprintf(g[i].uuid + len, sizeof(g[i].uuid) - len, "-p%d", g[i].partition);
    // each partition has its own DRM card: the PCI device's drm/ directory
    // lists all of them; pair the k-th card with the k-th render node
    std::vector<int> cards, renders;
    for (const std::string& e :
         mx::list_dir(mx::rooted(root, std::string("/sys/bus/pci/devices/") + g[i].pci_bdf + "/drm"))) {
      if (e.rfind("card", 0) == 0) cards.push_back(static_cast<int>(std::strtol(e.c_str() + 4, nullptr, 10)));
      else if (e.rfind("renderD", 0) == 0)
        renders.push_back(static_cast<int>(std::strtol(e.c_str() + 7, nullptr, 10)));
    }
    std::sort(cards.begin(), cards.end());
    std::sort(renders.begin(), renders.end());
    g[i].drm_card = -1;
    if (cards.size() == renders.size())
      for (size_t k = 0; k < renders.size(); ++k)
        if (renders[k] == g[i].drm_render_minor) g[i].drm_card = cards[k];
  }
}

}  // namespace

extern "C" {

const char* mx_version(void) { return "mxnode 0.1.0"; }

int mx_enumerate(const char* root_c, mx_gpu_info* out, int max, char* err, size_t errlen) {
  const std::string root = root_c ? root_c : "";
  std::vector<RawNode> nodes;
  std::string e;
  if (!load_nodes(root, &nodes, &e)) {
    mx::set_err(err, errlen, e);
    return -1;
  }
  std::vector<mx_gpu_info> all;
  for (const RawNode& n : nodes) {
    if (!is_gpu(n)) continue;
    if (mx::prop_u64(n.props, "vendor_id") != 0x1002) continue;   // AMD only
    all.emplace_back();
    fill_info(root, n, static_cast<int>(all.size()) - 1, &all.back());
  }
  mark_partitions(root, all.data(), static_cast<int>(all.size()));
  if (out)
    for (int i = 0; i < static_cast<int>(all.size()) && i < max; ++i) out[i] = all[i];
  return static_cast<int>(all.size());
}

int mx_links(const char* root_c, mx_link* out, int max, char* err, size_t errlen) {
  const std::string root = root_c ? root_c : "";
  std::vector<RawNode> nodes;
  std::string e;
  if (!load_nodes(root, &nodes, &e)) {
    mx::set_err(err, errlen, e);
    return -1;
  }
  std::map<int, int> node_to_index;
  int idx = 0;
  for (const RawNode& n : nodes)
    if (is_gpu(n) && mx::prop_u64(n.props, "vendor_id") == 0x1002) node_to_index[n.kfd_node] = idx++;
  int count = 0;
  for (const auto& kv : node_to_index) {
    const std::string ldir = mx::rooted(root, kTopo) + "/" + std::to_string(kv.first) + "/io_links";
    for (const std::string& l : mx::list_dir(ldir)) {
      std::string text;
      if (!mx::read_file(ldir + "/" + l + "/properties", &text)) continue;
      auto p = mx::parse_properties(text);
      if (count < max && out) {
        mx_link& k = out[count];
        k.from_index = kv.second;
        const int to_node = static_cast<int>(mx::prop_u64(p, "node_to"));
        auto it = node_to_index.find(to_node);
        k.to_index = it == node_to_index.end() ? -1 : it->second;
        k.type = static_cast<int>(mx::prop_u64(p, "type"));
        k.weight = static_cast<uint32_t>(mx::prop_u64(p, "weight"));
        k.min_bandwidth_mbps = static_cast<uint32_t>(mx::prop_u64(p, "min_bandwidth"));
        k.max_bandwidth_mbps = static_cast<uint32_t>(mx::prop_u64(p, "max_bandwidth"));
      }
      ++count;
    }
  }
  return count < max ? count : max;
}

}  // extern "C"
