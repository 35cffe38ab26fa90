// Node-local AMD GPU topology + partition discovery.
//
// The reference has no topology notion: it derives the GPU count from node capacity
// (pkg/utils/node.go:8-14) and leaves discovery to an external NVIDIA device plugin
// (README.md:9, 30-34). On MI355X the schedulable unit depends on the compute-partition
// mode (SPX/DPX/QPX/CPX: 1/2/4/8 partitions of the 8 XCDs), memory partitioning (NPS1..8),
// the xGMI link graph of the 8 GPUs of a node, NUMA placement and virtualisation
// (SR-IOV).  This reader gets those facts from:
//   1. KFD sysfs  (/sys/class/kfd/kfd/topology/nodes/*/{properties,io_links,mem_banks})
//   2. DRM sysfs  (/sys/class/drm/renderD*/device/{current_compute_partition,...})
//   3. libamd_smi (dlopen'ed, optional) for virtualisation mode, VRAM and link bandwidth.
// Every path can be re-rooted so 8-GPU SPX/CPX fixtures test the same code.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace nanogpu {

struct GpuInfo {
  int kfd_node = -1;
  uint32_t gpu_id = 0;            // KFD gpu_id
  uint32_t render_minor = 0;
  uint64_t location_id = 0;       // PCI BDF as KFD reports it
  uint32_t domain = 0;
  uint64_t unique_id = 0;
  uint64_t hive_id = 0;
  uint32_t gfx_target_version = 0;
  uint32_t vendor_id = 0, device_id = 0;
  int simd_count = 0, simd_per_cu = 0, cus = 0, num_xcc = 0;
  int max_waves_per_simd = 0, wave_front_size = 0;
  int64_t lds_size_kib = 0;
  int64_t vram_bytes = 0;
  int numa = -1;
  std::string compute_partition;          // SPX/DPX/QPX/CPX ("" if unknown)
  std::string memory_partition;           // NPS1/NPS2/NPS4/NPS8
  std::string available_compute_partitions;
  // RAS error counters summed over the amdgpu `ras/*_err_count` blocks (umc = HBM, gfx,
  // sdma, xgmi_wafl, ...): uncorrectable errors make the device unschedulable.
  bool ras_available = false;
  int64_t ras_ue = 0, ras_ce = 0;
  int xgmi_peers = 0;              // xGMI io_links (type 11) to other GPU nodes, visible or not
  int64_t xgmi_min_bw_mbs = 0;     // slowest / fastest of those links (KFD max_bandwidth, MB/s)
  int64_t xgmi_max_bw_mbs = 0;
  int parent = -1;        // physical GPU index within the node (filled by group_partitions)
  int partition = 0;      // partition index within the physical GPU
};

struct LinkInfo {
  int from = -1, to = -1;     // KFD node ids
  int type = 0;               // KFD io_link type, 11 = XGMI, 2 = PCIe
  int weight = 0;
  int64_t min_bw_mbs = 0, max_bw_mbs = 0;
};

struct HostTopology {
  std::vector<GpuInfo> gpus;       // schedulable devices (partitions in DPX..CPX)
  std::vector<LinkInfo> links;     // GPU<->GPU io_links
  int n_physical = 0;
  std::string source;              // "sysfs", "sysfs+amdsmi"
  std::string virtualization;      // BAREMETAL/HOST/GUEST/PASSTHROUGH/UNKNOWN
  std::vector<std::string> warnings;
};

// Reads KFD + DRM sysfs under `root` ("" or "/" for the live system).
HostTopology read_sysfs(const std::string& root);
// Groups partitions of one physical GPU (same PCI domain+location/unique id) and numbers them.
void group_partitions(HostTopology* t);
// Enriches with libamd_smi if it can be loaded and initialised. Returns false otherwise.
bool enrich_amdsmi(HostTopology* t);
// Convenience: read_sysfs + group + (live system only) amdsmi.
HostTopology discover(const std::string& root, bool use_amdsmi);

std::map<std::string, std::string> parse_properties(const std::string& text);
std::string to_json(const HostTopology& t);

}  // namespace nanogpu
