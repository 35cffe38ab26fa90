// KFD/DRM sysfs + libamd_smi topology reader (see topo.h).
#include "nanogpu/topo.h"

#include <dirent.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include <amd_smi/amdsmi.h>

namespace nanogpu {

static std::string read_file(const std::string& p) {
  std::ifstream f(p);
  if (!f) return {};
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static std::string trim(std::string s) {
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ' || s.back() == '\r' || s.back() == '\t'))
    s.pop_back();
  size_t i = 0;
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
  return s.substr(i);
}

static std::vector<std::string> list_dir(const std::string& p) {
  std::vector<std::string> out;
  DIR* d = opendir(p.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    out.emplace_back(e->d_name);
  }
  closedir(d);
  std::sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) {
    // numeric order when both are numbers
    char* ea;
    char* eb;
    long ia = std::strtol(a.c_str(), &ea, 10), ib = std::strtol(b.c_str(), &eb, 10);
    if (*ea == 0 && *eb == 0) return ia < ib;
    return a < b;
  });
  return out;
}

std::map<std::string, std::string> parse_properties(const std::string& text) {
  std::map<std::string, std::string> m;
  std::istringstream is(text);
  std::string line;
  while (std::getline(is, line)) {
    line = trim(line);
    const size_t sp = line.find_first_of(" \t");
    if (sp == std::string::npos) continue;
    m[line.substr(0, sp)] = trim(line.substr(sp + 1));
  }
  return m;
}

static int64_t as_i64(const std::map<std::string, std::string>& m, const char* k, int64_t dflt = 0) {
  auto it = m.find(k);
  if (it == m.end()) return dflt;
  return std::strtoll(it->second.c_str(), nullptr, 10);
}

static uint64_t as_u64(const std::map<std::string, std::string>& m, const char* k) {
  auto it = m.find(k);
  if (it == m.end()) return 0;
  return std::strtoull(it->second.c_str(), nullptr, 10);
}

static std::string join(const std::string& root, const std::string& p) {
  if (root.empty() || root == "/") return p;
  return root + p;
}

HostTopology read_sysfs(const std::string& root) {
  HostTopology t;
  t.source = "sysfs";
  t.virtualization = "UNKNOWN";
  const std::string kfd = join(root, "/sys/class/kfd/kfd/topology/nodes");
  std::map<int, int> kfd_to_gpu;
  for (const std::string& nd : list_dir(kfd)) {
    const std::string base = kfd + "/" + nd;
    auto props = parse_properties(read_file(base + "/properties"));
    if (as_i64(props, "simd_count") <= 0) continue;  // CPU node
    GpuInfo g;
    g.kfd_node = std::atoi(nd.c_str());
    const std::string gid = trim(read_file(base + "/gpu_id"));
    g.gpu_id = static_cast<uint32_t>(std::strtoul(gid.c_str(), nullptr, 10));
    g.render_minor = static_cast<uint32_t>(as_i64(props, "drm_render_minor"));
    g.location_id = as_u64(props, "location_id");
    g.domain = static_cast<uint32_t>(as_i64(props, "domain"));
    g.unique_id = as_u64(props, "unique_id");
    g.hive_id = as_u64(props, "hive_id");
    g.gfx_target_version = static_cast<uint32_t>(as_i64(props, "gfx_target_version"));
    g.vendor_id = static_cast<uint32_t>(as_i64(props, "vendor_id"));
    g.device_id = static_cast<uint32_t>(as_i64(props, "device_id"));
    g.simd_count = static_cast<int>(as_i64(props, "simd_count"));
    g.simd_per_cu = static_cast<int>(as_i64(props, "simd_per_cu", 4));
    g.cus = g.simd_per_cu > 0 ? g.simd_count / g.simd_per_cu : 0;
    g.num_xcc = static_cast<int>(as_i64(props, "num_xcc", 1));
    g.max_waves_per_simd = static_cast<int>(as_i64(props, "max_waves_per_simd"));
    g.wave_front_size = static_cast<int>(as_i64(props, "wave_front_size", 64));
    g.lds_size_kib = as_i64(props, "lds_size_in_kb");
    // VRAM: local memory banks (heap types 1/2 = frame buffer public/private)
    int64_t vram = 0;
    for (const std::string& mb : list_dir(base + "/mem_banks")) {
      auto mp = parse_properties(read_file(base + "/mem_banks/" + mb + "/properties"));
      const int64_t ht = as_i64(mp, "heap_type", -1);
      if (ht == 1 || ht == 2) vram += as_i64(mp, "size_in_bytes");
    }
    g.vram_bytes = vram;
    // DRM side: partition modes, NUMA, VRAM total
    const std::string drm = join(root, "/sys/class/drm/renderD" + std::to_string(g.render_minor) + "/device");
    const std::string vt = trim(read_file(drm + "/mem_info_vram_total"));
    if (!vt.empty()) g.vram_bytes = std::strtoll(vt.c_str(), nullptr, 10);
    g.compute_partition = trim(read_file(drm + "/current_compute_partition"));
    g.memory_partition = trim(read_file(drm + "/current_memory_partition"));
    g.available_compute_partitions = trim(read_file(drm + "/available_compute_partition"));
    const std::string numa = trim(read_file(drm + "/numa_node"));
    if (!numa.empty()) g.numa = std::atoi(numa.c_str());
    // RAS: every "<block>_err_count" file reads "ue: N\nce: M"
    for (const std::string& f : list_dir(drm + "/ras")) {
      if (f.size() <= 10 || f.compare(f.size() - 10, 10, "_err_count") != 0) continue;
      for (const auto& kv : parse_properties(read_file(drm + "/ras/" + f))) {
        std::string k = kv.first;
        if (!k.empty() && k.back() == ':') k.pop_back();
        const int64_t v = std::strtoll(kv.second.c_str(), nullptr, 10);
        if (k == "ue") g.ras_ue += v;
        else if (k == "ce") g.ras_ce += v;
        else continue;
        g.ras_available = true;
      }
    }
    kfd_to_gpu[g.kfd_node] = static_cast<int>(t.gpus.size());
    t.gpus.push_back(g);
  }
  for (size_t gi_idx = 0; gi_idx < t.gpus.size(); ++gi_idx) {
    const GpuInfo g = t.gpus[gi_idx];
    const std::string base = kfd + "/" + std::to_string(g.kfd_node) + "/io_links";
    for (const std::string& l : list_dir(base)) {
      auto lp = parse_properties(read_file(base + "/" + l + "/properties"));
      LinkInfo li;
      li.from = static_cast<int>(as_i64(lp, "node_from", g.kfd_node));
      li.to = static_cast<int>(as_i64(lp, "node_to", -1));
      li.type = static_cast<int>(as_i64(lp, "type"));
      if (li.type == 11) {
        // xGMI peer: counted even when the peer's node is hidden from this container (its
        // KFD properties unreadable), so a 1-GPU view still knows its hive's link fabric.
        GpuInfo& gi = t.gpus[kfd_to_gpu[g.kfd_node]];
        const int64_t bw = as_i64(lp, "max_bandwidth");
        gi.xgmi_peers += 1;
        gi.xgmi_min_bw_mbs = gi.xgmi_peers == 1 ? bw : std::min(gi.xgmi_min_bw_mbs, bw);
        gi.xgmi_max_bw_mbs = std::max(gi.xgmi_max_bw_mbs, bw);
      }
      if (kfd_to_gpu.find(li.to) == kfd_to_gpu.end()) continue;  // GPU<->CPU or hidden peer
      li.weight = static_cast<int>(as_i64(lp, "weight"));
      li.min_bw_mbs = as_i64(lp, "min_bandwidth");
      li.max_bw_mbs = as_i64(lp, "max_bandwidth");
      t.links.push_back(li);
    }
  }
  if (t.gpus.empty()) t.warnings.push_back("no GPU nodes under " + kfd);
  return t;
}

void group_partitions(HostTopology* t) {
  // Partitions of one physical GPU share the PCI domain + location_id (and unique_id when
  // the firmware exposes one); physical GPUs are numbered in KFD order.
  std::vector<std::pair<uint64_t, uint64_t>> keys;
  for (GpuInfo& g : t->gpus) {
    const std::pair<uint64_t, uint64_t> k{(static_cast<uint64_t>(g.domain) << 32) | (g.location_id & ~0x7ULL),
                                          g.unique_id};
    auto it = std::find(keys.begin(), keys.end(), k);
    int parent;
    if (it == keys.end()) {
      parent = static_cast<int>(keys.size());
      keys.push_back(k);
    } else {
      parent = static_cast<int>(it - keys.begin());
    }
    int part = 0;
    for (const GpuInfo& o : t->gpus) {
      if (&o == &g) break;
      if (o.parent == parent) ++part;
    }
    g.parent = parent;
    g.partition = part;
  }
  t->n_physical = static_cast<int>(keys.size());
}

namespace {
struct SmiApi {
  void* h = nullptr;
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) procs = nullptr;
  decltype(&amdsmi_get_gpu_kfd_info) kfd_info = nullptr;
  decltype(&amdsmi_get_gpu_virtualization_mode) virt = nullptr;
  decltype(&amdsmi_get_gpu_memory_total) mem_total = nullptr;
  decltype(&amdsmi_get_gpu_compute_partition) cpart = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition) mpart = nullptr;
  decltype(&amdsmi_get_minmax_bandwidth_between_processors) minmax_bw = nullptr;
  decltype(&amdsmi_topo_get_link_type) link_type = nullptr;
  decltype(&amdsmi_topo_get_numa_node_number) numa = nullptr;
  bool load() {
    for (const char* n : {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"}) {
      h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
#define NG_SYM(field, name) field = reinterpret_cast<decltype(field)>(dlsym(h, name))
    NG_SYM(init, "amdsmi_init");
    NG_SYM(shut_down, "amdsmi_shut_down");
    NG_SYM(sockets, "amdsmi_get_socket_handles");
    NG_SYM(procs, "amdsmi_get_processor_handles");
    NG_SYM(kfd_info, "amdsmi_get_gpu_kfd_info");
    NG_SYM(virt, "amdsmi_get_gpu_virtualization_mode");
    NG_SYM(mem_total, "amdsmi_get_gpu_memory_total");
    NG_SYM(cpart, "amdsmi_get_gpu_compute_partition");
    NG_SYM(mpart, "amdsmi_get_gpu_memory_partition");
    NG_SYM(minmax_bw, "amdsmi_get_minmax_bandwidth_between_processors");
    NG_SYM(link_type, "amdsmi_topo_get_link_type");
    NG_SYM(numa, "amdsmi_topo_get_numa_node_number");
#undef NG_SYM
    return init && shut_down && sockets && procs;
  }
};
const char* virt_name(int v) {
  switch (v) {
    case AMDSMI_VIRTUALIZATION_MODE_BAREMETAL: return "BAREMETAL";
    case AMDSMI_VIRTUALIZATION_MODE_HOST: return "HOST";
    case AMDSMI_VIRTUALIZATION_MODE_GUEST: return "GUEST";
    case AMDSMI_VIRTUALIZATION_MODE_PASSTHROUGH: return "PASSTHROUGH";
    default: return "UNKNOWN";
  }
}
}  // namespace

bool enrich_amdsmi(HostTopology* t) {
  SmiApi api;
  if (!api.load()) {
    t->warnings.push_back("libamd_smi not loadable");
    return false;
  }
  if (api.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) {
    t->warnings.push_back("amdsmi_init failed (amdgpu driver not loaded?)");
    dlclose(api.h);
    return false;
  }
  uint32_t ns = 0;
  std::vector<amdsmi_processor_handle> handles;
  if (api.sockets(&ns, nullptr) == AMDSMI_STATUS_SUCCESS && ns > 0) {
    std::vector<amdsmi_socket_handle> socks(ns);
    api.sockets(&ns, socks.data());
    for (uint32_t s = 0; s < ns; ++s) {
      uint32_t np = 0;
      if (api.procs(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      api.procs(socks[s], &np, ph.data());
      handles.insert(handles.end(), ph.begin(), ph.begin() + np);
    }
  }
  // map amdsmi handles to our GPUs through the KFD node id
  std::vector<int> of_gpu(t->gpus.size(), -1);
  for (size_t h = 0; h < handles.size(); ++h) {
    amdsmi_kfd_info_t ki{};
    if (!api.kfd_info || api.kfd_info(handles[h], &ki) != AMDSMI_STATUS_SUCCESS) continue;
    for (size_t g = 0; g < t->gpus.size(); ++g)
      if (static_cast<uint32_t>(t->gpus[g].kfd_node) == ki.node_id) of_gpu[g] = static_cast<int>(h);
  }
  for (size_t g = 0; g < t->gpus.size(); ++g) {
    if (of_gpu[g] < 0) continue;
    amdsmi_processor_handle ph = handles[of_gpu[g]];
    GpuInfo& gi = t->gpus[g];
    if (api.virt) {
      amdsmi_virtualization_mode_t vm{};
      if (api.virt(ph, &vm) == AMDSMI_STATUS_SUCCESS) t->virtualization = virt_name(vm);
    }
    if (api.mem_total) {
      uint64_t total = 0;
      if (api.mem_total(ph, AMDSMI_MEM_TYPE_VRAM, &total) == AMDSMI_STATUS_SUCCESS && total > 0)
        gi.vram_bytes = static_cast<int64_t>(total);
    }
    char buf[64];
    if (api.cpart && gi.compute_partition.empty() &&
        api.cpart(ph, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      gi.compute_partition = buf;
    if (api.mpart && gi.memory_partition.empty() &&
        api.mpart(ph, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS)
      gi.memory_partition = buf;
    if (api.numa && gi.numa < 0) {
      uint32_t nn = 0;
      if (api.numa(ph, &nn) == AMDSMI_STATUS_SUCCESS) gi.numa = static_cast<int>(nn);
    }
  }
  // fill missing link bandwidth from amdsmi
  if (api.minmax_bw) {
    for (LinkInfo& l : t->links) {
      if (l.max_bw_mbs > 0) continue;
      int gf = -1, gt = -1;
      for (size_t g = 0; g < t->gpus.size(); ++g) {
        if (t->gpus[g].kfd_node == l.from) gf = of_gpu[g];
        if (t->gpus[g].kfd_node == l.to) gt = of_gpu[g];
      }
      if (gf < 0 || gt < 0) continue;
      uint64_t mn = 0, mx = 0;
      if (api.minmax_bw(handles[gf], handles[gt], &mn, &mx) == AMDSMI_STATUS_SUCCESS) {
        l.min_bw_mbs = static_cast<int64_t>(mn);
        l.max_bw_mbs = static_cast<int64_t>(mx);
      }
    }
  }
  api.shut_down();
  dlclose(api.h);
  t->source += "+amdsmi";
  return true;
}

HostTopology discover(const std::string& root, bool use_amdsmi) {
  HostTopology t = read_sysfs(root);
  group_partitions(&t);
  if (use_amdsmi && (root.empty() || root == "/")) enrich_amdsmi(&t);
  return t;
}

static std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += c;
    } else if (static_cast<unsigned char>(c) < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", c);
      o += b;
    } else {
      o += c;
    }
  }
  return o;
}

std::string to_json(const HostTopology& t) {
  std::ostringstream os;
  os << "{\"source\":\"" << esc(t.source) << "\",\"virtualization\":\"" << esc(t.virtualization)
     << "\",\"n_physical\":" << t.n_physical << ",\"gpus\":[";
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    const GpuInfo& g = t.gpus[i];
    if (i) os << ",";
    os << "{\"kfd_node\":" << g.kfd_node << ",\"gpu_id\":" << g.gpu_id
       << ",\"render_minor\":" << g.render_minor << ",\"location_id\":" << g.location_id
       << ",\"domain\":" << g.domain << ",\"unique_id\":" << g.unique_id
       << ",\"hive_id\":" << g.hive_id << ",\"gfx_target_version\":" << g.gfx_target_version
       << ",\"device_id\":" << g.device_id << ",\"simd_count\":" << g.simd_count
       << ",\"cus\":" << g.cus << ",\"num_xcc\":" << g.num_xcc << ",\"vram_bytes\":" << g.vram_bytes
       << ",\"lds_size_kib\":" << g.lds_size_kib << ",\"numa\":" << g.numa
       << ",\"compute_partition\":\"" << esc(g.compute_partition) << "\",\"memory_partition\":\""
       << esc(g.memory_partition) << "\",\"available_compute_partitions\":\""
       << esc(g.available_compute_partitions) << "\",\"ras_available\":" << (g.ras_available ? "true" : "false")
       << ",\"ras_ue\":" << g.ras_ue << ",\"ras_ce\":" << g.ras_ce << ",\"xgmi_peers\":" << g.xgmi_peers
       << ",\"xgmi_min_bw_mbs\":" << g.xgmi_min_bw_mbs << ",\"xgmi_max_bw_mbs\":" << g.xgmi_max_bw_mbs
       << ",\"parent\":" << g.parent
       << ",\"partition\":" << g.partition << "}";
  }
  os << "],\"links\":[";
  for (size_t i = 0; i < t.links.size(); ++i) {
    const LinkInfo& l = t.links[i];
    if (i) os << ",";
    os << "{\"from\":" << l.from << ",\"to\":" << l.to << ",\"type\":" << l.type
       << ",\"weight\":" << l.weight << ",\"min_bw_mbs\":" << l.min_bw_mbs
       << ",\"max_bw_mbs\":" << l.max_bw_mbs << "}";
  }
  os << "],\"warnings\":[";
  for (size_t i = 0; i < t.warnings.size(); ++i) os << (i ? "," : "") << "\"" << esc(t.warnings[i]) << "\"";
  os << "]}";
  return os.str();
}

}  // namespace nanogpu
