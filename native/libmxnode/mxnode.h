// libmxnode — MI355X node discovery / CDI / allocation / health / metrics core.
//
// Plain C ABI so the same shared object serves the Python device plugin,
// labeller and exporter (ctypes) and the C++ CLIs (mx-gpu-enum, mx-cdi-gen).
//
// Every host path is taken relative to a caller-supplied ROOT ("" or "/" for
// the real host), so all of it is testable against fake sysfs trees
// (tests/fixtures/sysfs/*) without root, a cluster or a GPU.
//
// Replaces, MI355X-first, the native pieces the reference's runbook pulls in
// through the NVIDIA GPU Operator (/root/reference/README.md:264-272):
// NVML enumeration (device plugin + GFD), libnvidia-container / nvidia-ctk
// (README.md:138-149), NVML Xid health, DCGM sampling.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MX_MAX_GPUS 64
#define MX_MAX_LINKS 64

typedef struct mx_gpu_info {
  int index;                    // 0..n-1, ordered by DRM render minor (HIP order)
  int kfd_node;                 // /sys/class/kfd/kfd/topology/nodes/<kfd_node>
  uint32_t gpu_id;              // KFD gpu_id
  uint32_t gfx_target_version;  // e.g. 90500 for gfx950
  char gfx_arch[16];            // "gfx950"
  int drm_render_minor;         // 128 + i -> /dev/dri/renderD<minor>
  int drm_card;                 // /dev/dri/card<drm_card>, -1 if unknown
  uint32_t vendor_id;           // 0x1002
  uint32_t device_id;           // PCI device id
  uint32_t domain;
  uint32_t location_id;         // bus << 8 | dev << 3 | fn
  char pci_bdf[20];             // "0000:05:00.0"
  int numa_node;                // -1 if unknown
  uint32_t simd_count;
  uint32_t simd_per_cu;
  uint32_t cu_count;
  uint64_t vram_bytes;          // sum of KFD mem_banks (local heap)
  uint64_t unique_id;
  uint64_t hive_id;             // xGMI hive id (0 if none)
  uint32_t max_engine_clk_mhz;
  int num_xgmi_links;
  char product[48];             // "MI355X", from the device-id table
  char uuid[40];                // "GPU-<unique_id hex>" (+ "-p<k>" for a partition)
  // Compute partitioning (SPX/DPX/QPX/CPX): in DPX..CPX mode amdgpu exposes
  // each partition of one PCI device as its own KFD node + render node; they
  // share the BDF.  partition = 0..partitions-1 in render-minor order.
  int partition;
  int partitions;               // KFD nodes sharing this PCI device (1 = SPX)
  uint32_t num_xcc;             // XCDs in this (partition of the) device
} mx_gpu_info;

typedef struct mx_link {
  int from_index;
  int to_index;                 // GPU index of the peer, -1 if the peer is a CPU node
  int type;                     // KFD io_link type: 2 = PCIe, 11 = xGMI
  uint32_t weight;
  uint32_t min_bandwidth_mbps;
  uint32_t max_bandwidth_mbps;
} mx_link;

// Library version string.
const char* mx_version(void);

// Enumerate AMD GPUs under ROOT.  Returns the count (>= 0) or -1 on error
// (message in err).  Fills at most `max` entries.
int mx_enumerate(const char* root, mx_gpu_info* out, int max, char* err, size_t errlen);

// GPU<->GPU and GPU->CPU io_links.  Returns the number of links written.
int mx_links(const char* root, mx_link* out, int max, char* err, size_t errlen);

// Write the CDI spec (JSON, cdiVersion 0.6.0, kind `kind`, e.g. "amd.com/gpu")
// into buf.  Returns the full length needed (excluding NUL) or -1 on error;
// if the return is >= buflen the output was truncated.
long mx_cdi_spec(const char* root, const char* kind, char* buf, size_t buflen, char* err,
                 size_t errlen);

// Preferred allocation (kubelet GetPreferredAllocation):
// choose `size` GPU indices from `available` (must contain all of
// `must_include`), preferring one xGMI hive, then the fewest NUMA nodes, then
// the most xGMI-connected set, then the lowest indices.  Writes `size`
// indices (ascending) into out; returns size or -1.
int mx_preferred_allocation(const char* root, const int* available, int navail,
                            const int* must_include, int nmust, int size, int* out, char* err,
                            size_t errlen);

// Same policy over explicit topology arrays (no sysfs): numa[i], hive[i] and a
// row-major n x n xGMI adjacency matrix for device ids 0..n-1.
int mx_preferred_allocation_topo(int n, const int* numa, const uint64_t* hive,
                                 const int* xgmi_adj, const int* available, int navail,
                                 const int* must_include, int nmust, int size, int* out);

// Health of GPU `index`: 0 = healthy, >0 = reason code (see MX_UNHEALTHY_*).
// Checks: KFD node still present, render node present under ROOT/dev/dri,
// and the optional fault-injection file (one index per line, or "all").
#define MX_HEALTHY 0
#define MX_UNHEALTHY_NO_KFD_NODE 1
#define MX_UNHEALTHY_NO_RENDER_NODE 2
#define MX_UNHEALTHY_FAULT_INJECTED 3
#define MX_UNHEALTHY_SMI_EVENT 4
#define MX_UNHEALTHY_ECC 5
int mx_health_check(const char* root, int index, const char* fault_file);
const char* mx_health_reason(int code);

// ---- N02 health monitor: sysfs checks + amd-smi events + RAS ECC ----------
// One monitor per device plugin.  mx_hm_step() runs one pass: it drains the
// amd-smi event queue (waiting up to wait_ms for the first event), samples the
// uncorrectable ECC count of every GPU, re-runs the sysfs checks and updates
// each GPU's verdict:
//   * sysfs (KFD node / render node gone, fault injected) — while it lasts;
//   * VM fault or GPU pre-reset event  -> MX_UNHEALTHY_SMI_EVENT for
//     event_quarantine_ms after the LAST such event;
//   * uncorrectable ECC above the per-boot baseline -> MX_UNHEALTHY_ECC:
//     sticky until reboot when ecc_quarantine_ms <= 0, otherwise for
//     ecc_quarantine_ms after the increase (the new count becomes the
//     baseline).  The baseline is the first count seen this boot, kept in
//     <state_dir>/ecc-baseline keyed by the kernel boot id, so a plugin
//     restart neither forgets nor forgives an error;
//   * thermal-throttle and post-reset events are counted and logged only.
// All entry points are thread-safe.
#define MX_EVT_VMFAULT 1
#define MX_EVT_THERMAL_THROTTLE 2
#define MX_EVT_GPU_PRE_RESET 3
#define MX_EVT_GPU_POST_RESET 4
#define MX_EVT_ECC_UNCORRECTABLE 100    // value = increase over the baseline
#define MX_EVT_HEALTH_CHANGE 101        // value = new code (MX_HEALTHY / MX_UNHEALTHY_*)

typedef struct mx_health_opts {
  const char* root;                 // sysfs/dev root ("" = host)
  const char* fault_file;           // fault-injection file or NULL
  const char* state_dir;            // ECC baseline directory or NULL (in-memory only)
  const char* boot_id_file;         // NULL = /proc/sys/kernel/random/boot_id
  int event_quarantine_ms;
  int ecc_quarantine_ms;            // <= 0: sticky until reboot
  int use_smi;                      // 0: sysfs checks only
} mx_health_opts;

typedef struct mx_health_status {
  int index;
  int code;                         // MX_HEALTHY or MX_UNHEALTHY_*
  int smi_index;                    // amd-smi index matched by BDF, -1 if none
  int ecc_valid;
  uint64_t ecc_uncorrectable;
  uint64_t ecc_baseline;
  uint64_t vm_faults;
  uint64_t thermal_throttles;
  uint64_t resets;
  int64_t quarantine_left_ms;       // 0 if not quarantined
  char bdf[20];
} mx_health_status;

typedef struct mx_health_event {
  uint64_t seq;                     // 1, 2, ... per monitor
  int index;                        // GPU index (KFD order), -1 unknown
  int kind;                         // MX_EVT_*
  int64_t value;
  int64_t unix_ms;
  char message[96];
} mx_health_event;

typedef struct mx_health_monitor mx_health_monitor;
mx_health_monitor* mx_hm_create(const mx_health_opts* opts, char* err, size_t errlen);
void mx_hm_destroy(mx_health_monitor* m);
// 1 if the amd-smi event/ECC source is live.
int mx_hm_smi_active(mx_health_monitor* m);
// One pass; returns the number of GPUs whose code changed.
int mx_hm_step(mx_health_monitor* m, int wait_ms);
int mx_hm_status(mx_health_monitor* m, mx_health_status* out, int max);
// Events with seq > after_seq (oldest first, the last 1024 are kept).
int mx_hm_events(mx_health_monitor* m, uint64_t after_seq, mx_health_event* out, int max);
// Atomically write the verdicts as JSON (tmp + rename) for the exporter.
int mx_hm_write_state(mx_health_monitor* m, const char* path);

// ---- amd-smi backed sampling (dlopen("libamd_smi.so"); no link dependency) ----
typedef struct mx_gpu_sample {
  int index;
  int valid;                        // 0 if amd-smi could not sample this GPU
  uint32_t gfx_activity_pct;
  uint32_t umc_activity_pct;
  uint64_t vram_used_bytes;
  uint64_t vram_total_bytes;
  int64_t temp_edge_mc;             // milli-degrees C, INT64_MIN if unsupported
  int64_t temp_hotspot_mc;
  int64_t temp_mem_mc;
  uint64_t power_w;
  uint32_t power_limit_w;
  uint32_t sclk_mhz;
  uint32_t mclk_mhz;
  uint64_t ecc_correctable;
  uint64_t ecc_uncorrectable;
  uint32_t num_processes;
  char bdf[20];
  int partition_id;                 // amd-smi BDFID bits 31:28 (0 in SPX mode)
  double energy_j;                  // accumulated energy (J) since driver load, < 0 if unsupported
} mx_gpu_sample;

// 1 if amd-smi could be loaded and initialised, 0 otherwise (msg in err).
// Reference-counted per process: each successful open needs one close.
int mx_smi_open(char* err, size_t errlen);
void mx_smi_close(void);
// End the session whatever the reference count (tests, process teardown).
void mx_smi_reset(void);
// Shut amd-smi down and initialise it again on the open session, so that a
// changed GPU set (compute-partition change, driver reload) gets new handles.
// Every amd-smi index from before is void afterwards; 1 on success.
int mx_smi_reinit(char* err, size_t errlen);
// Changes whenever amd-smi was (re)initialised; 0 if not open.  Users that
// cache amd-smi indices re-match them (by BDF + partition) when it changes.
uint64_t mx_smi_generation(void);
// Number of GPUs amd-smi sees (after mx_smi_open), -1 if not open.
int mx_smi_count(void);
// Sample GPU i (amd-smi enumeration order, matched to BDF by the caller).
int mx_smi_sample(int i, mx_gpu_sample* out);
// RAS error counts of GPU i; 1 on success.
int mx_smi_ecc(int i, uint64_t* correctable, uint64_t* uncorrectable);
// Block up to timeout_ms for amd-smi GPU events (reset / thermal / VM fault).
// Writes up to `max` (gpu_bdf_index, event_code) pairs; returns count or -1.
int mx_smi_wait_events(int timeout_ms, int* gpu_out, int* event_out, int max);
const char* mx_smi_driver_version(void);

// xGMI link state + traffic of GPU i (amd-smi order).  Returns links written,
// -1 if amd-smi supports neither amdsmi_get_gpu_xgmi_link_status nor
// amdsmi_get_link_metrics here.
typedef struct mx_xgmi_link_sample {
  int link;                         // link index
  int status;                       // 0 down, 1 up, 2 disabled, -1 unknown
  int link_type;                    // amdsmi_link_type_t (2 = xGMI), -1 unknown
  int has_traffic;                  // read_kb / write_kb valid
  char peer_bdf[20];
  uint32_t bit_rate_gbps;
  uint32_t max_bandwidth_gbps;
  uint64_t read_kb;                 // cumulative KB received on the link
  uint64_t write_kb;                // cumulative KB sent
} mx_xgmi_link_sample;
int mx_smi_xgmi_links(int i, mx_xgmi_link_sample* out, int max);

// Per-process GPU memory of GPU i (amdsmi_get_gpu_process_list).
typedef struct mx_proc_sample {
  uint32_t pid;
  uint32_t cu_occupancy;
  char name[64];
  char container[64];
  uint64_t vram_bytes;
  uint64_t gtt_bytes;
} mx_proc_sample;
int mx_smi_processes(int i, mx_proc_sample* out, int max);

#ifdef __cplusplus
}
#endif
