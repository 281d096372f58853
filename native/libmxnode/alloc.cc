// N04-core: GetPreferredAllocation policy for amd.com/gpu.
//
// MI355X nodes are 8 GPUs in one fully connected xGMI hive split over two
// CPU sockets (NUMA nodes).  RCCL's rings run over point-to-point xGMI links,
// and host staging/IPC prefers the local socket, so for a request of k GPUs:
//   1. every chosen GPU in the same xGMI hive (fewest distinct hives)
//   2. fewest distinct NUMA nodes
//   3. fewest distinct PCI devices: in DPX..CPX compute-partition mode the
//      partitions of one MI355X share its HBM and need no xGMI hop, and
//      packing them leaves whole devices free (the MIG-packing counterpart)
//   4. most xGMI adjacencies inside the set (= most usable ring links)
//   5. lowest indices (stable, deterministic)
// must_include (devices the kubelet already decided on) are always kept.
// Exhaustive over C(avail, k) when that is small (<= 200k sets); greedy
// otherwise.
#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "mxnode.h"
#include "util.h"

namespace {

struct Score {
  int hives, numas, devs, neg_links;
  std::vector<int> ids;
  bool operator<(const Score& o) const {
    if (hives != o.hives) return hives < o.hives;
    if (numas != o.numas) return numas < o.numas;
    if (devs != o.devs) return devs < o.devs;
    if (neg_links != o.neg_links) return neg_links < o.neg_links;
    return ids < o.ids;
  }
};

Score score(const std::vector<int>& ids, const int* numa, const uint64_t* hive, const int* dev,
            const int* adj, int n) {
  std::set<uint64_t> hs;
  std::set<int> ns, ds;
  int links = 0;
  for (size_t a = 0; a < ids.size(); ++a) {
    hs.insert(hive[ids[a]]);
    ns.insert(numa[ids[a]]);
    ds.insert(dev ? dev[ids[a]] : ids[a]);
    for (size_t b = a + 1; b < ids.size(); ++b) links += adj[ids[a] * n + ids[b]] ? 1 : 0;
  }
  Score s{static_cast<int>(hs.size()), static_cast<int>(ns.size()), static_cast<int>(ds.size()),
          -links, ids};
  std::sort(s.ids.begin(), s.ids.end());
  return s;
}

double n_choose_k(int n, int k) {
  double r = 1;
  for (int i = 1; i <= k; ++i) r = r * (n - k + i) / i;
  return r;
}

}  // namespace

namespace {
int preferred(int n, const int* numa, const uint64_t* hive, const int* dev, const int* adj,
              const int* available, int navail, const int* must, int nmust, int size, int* out) {
  if (size <= 0 || size > navail || nmust > size) return -1;
  std::vector<int> avail(available, available + navail);
  std::sort(avail.begin(), avail.end());
  avail.erase(std::unique(avail.begin(), avail.end()), avail.end());
  for (int v : avail)
    if (v < 0 || v >= n) return -1;
  std::vector<int> req(must, must + nmust);
  std::sort(req.begin(), req.end());
  req.erase(std::unique(req.begin(), req.end()), req.end());
  for (int r : req)
    if (!std::binary_search(avail.begin(), avail.end(), r)) return -1;
  std::vector<int> pool;
  for (int v : avail)
    if (!std::binary_search(req.begin(), req.end(), v)) pool.push_back(v);
  const int need = size - static_cast<int>(req.size());
  if (need > static_cast<int>(pool.size())) return -1;

  Score best{1 << 30, 1 << 30, 1 << 30, 0, {}};
  if (n_choose_k(static_cast<int>(pool.size()), need) <= 200000.0) {
    std::vector<int> idx(need);
    for (int i = 0; i < need; ++i) idx[i] = i;
    while (true) {
      std::vector<int> ids = req;
      for (int i : idx) ids.push_back(pool[i]);
      Score s = score(ids, numa, hive, dev, adj, n);
      if (s < best) best = s;
      int i = need - 1;
      while (i >= 0 && idx[i] == static_cast<int>(pool.size()) - need + i) --i;
      if (i < 0) break;
      ++idx[i];
      for (int j = i + 1; j < need; ++j) idx[j] = idx[j - 1] + 1;
    }
  } else {
    std::vector<int> ids = req;
    std::vector<bool> used(pool.size(), false);
    for (int step = 0; step < need; ++step) {
      Score b{1 << 30, 1 << 30, 1 << 30, 0, {}};
      int bi = -1;
      for (size_t i = 0; i < pool.size(); ++i) {
        if (used[i]) continue;
        std::vector<int> t = ids;
        t.push_back(pool[i]);
        Score s = score(t, numa, hive, dev, adj, n);
        if (s < b) { b = s; bi = static_cast<int>(i); }
      }
      used[bi] = true;
      ids.push_back(pool[bi]);
    }
    best = score(ids, numa, hive, dev, adj, n);
  }
  for (int i = 0; i < size; ++i) out[i] = best.ids[i];
  return size;
}
}  // namespace

extern "C" int mx_preferred_allocation_topo(int n, const int* numa, const uint64_t* hive,
                                            const int* adj, const int* available, int navail,
                                            const int* must, int nmust, int size, int* out) {
  return preferred(n, numa, hive, nullptr, adj, available, navail, must, nmust, size, out);
}

extern "C" int mx_preferred_allocation(const char* root, const int* available, int navail,
                                       const int* must, int nmust, int size, int* out, char* err,
                                       size_t errlen) {
  mx_gpu_info gpus[MX_MAX_GPUS];
  const int n = mx_enumerate(root, gpus, MX_MAX_GPUS, err, errlen);
  if (n < 0) return -1;
  std::vector<int> numa(n), dev(n);
  std::vector<uint64_t> hive(n);
  std::vector<int> adj(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i) {
    numa[i] = gpus[i].numa_node;
    hive[i] = gpus[i].hive_id;
    dev[i] = i;   // physical device = the first GPU index with this PCI address
    for (int j = 0; j < i; ++j)
      if (gpus[j].domain == gpus[i].domain && gpus[j].location_id == gpus[i].location_id) {
        dev[i] = j;
        break;
      }
  }
  std::vector<mx_link> links(MX_MAX_GPUS * MX_MAX_LINKS);
  const int nl = mx_links(root, links.data(), static_cast<int>(links.size()), err, errlen);
  for (int i = 0; i < nl; ++i) {
    const mx_link& l = links[i];
    if (l.type == 11 && l.to_index >= 0 && l.from_index < n && l.to_index < n) {
      adj[l.from_index * n + l.to_index] = 1;
      adj[l.to_index * n + l.from_index] = 1;
    }
  }
  const int r = preferred(n, numa.data(), hive.data(), dev.data(), adj.data(), available, navail,
                          must, nmust, size, out);
  if (r < 0) mx::set_err(err, errlen, "invalid allocation request");
  return r;
}
