// pybind11 module `nanogpu._native`: ledger, policies, frag metrics, topology reader.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <tuple>
#include <unordered_set>
#include <vector>

#include "nanogpu/iotally.h"
#include "nanogpu/alloc.h"
#include "nanogpu/apiserver.h"
#include "nanogpu/frontend.h"
#include "nanogpu/gosort.h"
#include "nanogpu/json.h"
#include "nanogpu/ledger.h"
#include "nanogpu/podwatch.h"
#include "nanogpu/sampler.h"
#include "nanogpu/schedsim.h"
#include "nanogpu/topo.h"

namespace py = pybind11;
using namespace nanogpu;

namespace {

// A pod demand from Python: one (percent, MiB) tuple per container; an item may carry
// `flags` (nanogpu.k8s.podutil.Req: kFlagMemBound). Called with the GIL held.
Demand to_demand(const py::sequence& v) {
  if (v.size() > static_cast<size_t>(kMaxContainers))
    throw py::value_error("too many containers (max " + std::to_string(kMaxContainers) + ")");
  Demand d;
  std::memset(&d, 0, sizeof(d));
  d.n = static_cast<int32_t>(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    const py::handle it = v[i];
    const py::sequence t = py::reinterpret_borrow<py::sequence>(it);
    if (t.size() < 2) throw py::value_error("demand items are (percent, MiB)");
    const int64_t pct = t[0].cast<int64_t>(), mib = t[1].cast<int64_t>();
    if (pct < 0 || mib < 0) throw py::value_error("negative demand");
    if (pct > INT32_MAX) throw py::value_error("percent out of range");
    d.c[i].pct = static_cast<int32_t>(pct);
    d.c[i].mib = mib;
    if (t.size() >= 3) d.c[i].flags = t[2].cast<int32_t>();
    else if (py::hasattr(it, "flags")) d.c[i].flags = it.attr("flags").cast<int32_t>();
  }
  return d;
}

template <class T>
T get(const py::dict& d, const char* k, T dflt) {
  if (!d.contains(k)) return dflt;
  return d[k].cast<T>();
}

Device to_device(const py::dict& d) {
  Device v;
  std::memset(&v, 0, sizeof(v));
  v.pct_total = get<int32_t>(d, "pct_total", kPercentPerDevice);
  v.pct_free = get<int32_t>(d, "pct_free", v.pct_total);
  v.mib_total = get<int64_t>(d, "mib_total", 0);
  v.mib_free = get<int64_t>(d, "mib_free", v.mib_total);
  v.load_usage = get<float>(d, "load_usage", 0.f);
  v.remain_load = get<int16_t>(d, "remain_load", 0);
  v.gpu = get<int16_t>(d, "gpu", 0);
  v.part = get<int16_t>(d, "part", 0);
  v.numa = get<int16_t>(d, "numa", -1);
  v.healthy = get<bool>(d, "healthy", true) ? 1 : 0;
  v.xcds = get<int16_t>(d, "xcds", 0);
  v.cus = get<int32_t>(d, "cus", 0);
  v.pool = get<int16_t>(d, "pool", -1);
  v.mib_share = get<int64_t>(d, "mib_share", 0);
  v.mem_hot = get<bool>(d, "mem_hot", false) ? 1 : 0;
  v.mem_busy = get<int16_t>(d, "mem_busy", 0);
  if (v.pool >= 0 && v.mib_share <= 0) v.mib_share = v.mib_total;
  return v;
}

py::dict from_device(const Device& v) {
  py::dict d;
  d["pct_free"] = v.pct_free;
  d["pct_total"] = v.pct_total;
  d["mib_free"] = v.mib_free;
  d["mib_total"] = v.mib_total;
  d["load_usage"] = v.load_usage;
  d["remain_load"] = v.remain_load;
  d["gpu"] = v.gpu;
  d["part"] = v.part;
  d["numa"] = v.numa;
  d["healthy"] = v.healthy != 0;
  d["xcds"] = v.xcds;
  d["cus"] = v.cus;
  d["pool"] = v.pool;
  d["mib_share"] = v.mib_share;
  d["mem_bound"] = v.mem_bound;
  d["mem_hot"] = v.mem_hot != 0;
  d["mem_busy"] = v.mem_busy;
  return d;
}

std::vector<Device> to_devices(const py::list& l) {
  if (l.size() > static_cast<size_t>(kMaxDevs)) throw py::value_error("too many devices (max 64)");
  std::vector<Device> out;
  out.reserve(l.size());
  for (auto h : l) out.push_back(to_device(h.cast<py::dict>()));
  return out;
}

Topology to_topo(const py::object& o, const std::vector<Device>& devs) {
  Topology t;
  std::memset(&t, 0, sizeof(t));
  for (int i = 0; i < kMaxGpus; ++i) t.numa[i] = -1;
  int n_gpus = 0;
  for (const Device& d : devs) n_gpus = std::max<int>(n_gpus, d.gpu + 1);
  if (!o.is_none()) {
    py::dict d = o.cast<py::dict>();
    n_gpus = std::max<int>(n_gpus, get<int>(d, "n_gpus", 0));
    if (d.contains("numa")) {
      auto v = d["numa"].cast<std::vector<int>>();
      for (size_t i = 0; i < v.size() && i < static_cast<size_t>(kMaxGpus); ++i) t.numa[i] = static_cast<int16_t>(v[i]);
    }
    if (d.contains("link_bw")) {
      auto m = d["link_bw"].cast<std::vector<std::vector<float>>>();
      for (size_t a = 0; a < m.size() && a < static_cast<size_t>(kMaxGpus); ++a)
        for (size_t b = 0; b < m[a].size() && b < static_cast<size_t>(kMaxGpus); ++b)
          t.link_bw[a * kMaxGpus + b] = m[a][b];
    }
  }
  if (n_gpus > kMaxGpus) throw py::value_error("too many physical GPUs (max 16)");
  t.n_gpus = n_gpus;
  return t;
}

py::dict from_topo(const Topology& t) {
  py::dict d;
  d["n_gpus"] = t.n_gpus;
  std::vector<int> numa(t.numa, t.numa + t.n_gpus);
  std::vector<std::vector<float>> bw(t.n_gpus, std::vector<float>(t.n_gpus));
  for (int a = 0; a < t.n_gpus; ++a)
    for (int b = 0; b < t.n_gpus; ++b) bw[a][b] = t.link_bw[a * kMaxGpus + b];
  d["numa"] = numa;
  d["link_bw"] = bw;
  return d;
}

py::list plan_list(const Plan& p) {
  py::list out;
  if (p.n < 0 || p.n > kMaxContainers) return out;
  for (int c = 0; c < p.n; ++c) {
    if (p.off[c] < 0 || p.off[c + 1] > kMaxPlanIdx || p.off[c] > p.off[c + 1]) break;
    py::list idx;
    for (int k = p.off[c]; k < p.off[c + 1]; ++k) idx.append(static_cast<int>(p.idx[k]));
    out.append(idx);
  }
  return out;
}

Plan to_plan(const std::vector<std::vector<int>>& v) {
  Plan p;
  std::memset(&p, 0, sizeof(p));
  if (v.size() > static_cast<size_t>(kMaxContainers)) throw py::value_error("plan too long");
  p.n = static_cast<int32_t>(v.size());
  int pos = 0;
  for (size_t c = 0; c < v.size(); ++c) {
    p.off[c] = static_cast<int16_t>(pos);
    if (v[c].empty()) throw py::value_error("empty plan entry");
    for (int i : v[c]) {
      if (pos >= kMaxPlanIdx) throw py::value_error("plan too long");
      p.idx[pos++] = static_cast<int16_t>(i);
    }
  }
  p.off[p.n] = static_cast<int16_t>(pos);
  return p;
}

std::vector<int> size_list(const SizeSet& s) {
  std::vector<int> out;
  for (int q = 1; q <= kPercentPerDevice; ++q)
    if (s.has(q)) out.push_back(q);
  return out;
}

py::dict frag_dict(const FragStats& s) {
  py::dict d;
  d["pct_free_total"] = s.pct_free_total;
  d["pct_free_partial"] = s.pct_free_partial;
  d["mib_free_total"] = s.mib_free_total;
  d["mib_free_partial"] = s.mib_free_partial;
  d["pct_stranded"] = s.pct_stranded;
  d["devices"] = s.devices;
  d["devices_full_free"] = s.devices_full_free;
  d["devices_used"] = s.devices_used;
  d["frag_pct"] = s.pct_free_total > 0 ? 100.0 * s.pct_free_partial / s.pct_free_total : 0.0;
  d["frag_mib"] = s.mib_free_total > 0 ? 100.0 * s.mib_free_partial / s.mib_free_total : 0.0;
  d["stranded_pct"] = s.pct_free_total > 0 ? 100.0 * s.pct_stranded / s.pct_free_total : 0.0;
  return d;
}

py::dict record_dict(const PodRecord& r) {
  py::dict d;
  d["key"] = r.key;
  d["node"] = r.node;
  d["state"] = r.state == kPodReserved ? "reserved" : r.state == kPodNominated ? "nominated" : "committed";
  d["t_reserved"] = r.t_reserved;
  std::vector<std::pair<int32_t, int64_t>> dem;
  for (int i = 0; i < r.demand.n; ++i) dem.emplace_back(r.demand.c[i].pct, r.demand.c[i].mib);
  d["demand"] = dem;
  d["plan"] = plan_list(r.plan);
  d["owner"] = r.owner;
  return d;
}

}  // namespace


// ------------------------------------------------------------------ slim pod watch decoding
// What the pod informer keeps of a Pod (nanogpu/k8s/informer.py, pods.py, podutil.py):
// metadata identity + labels + the nano-gpu/* annotations, nodeName, each container's name
// and nano-gpu/* limits/requests, and the phase. Everything else of a real Pod (env, volumes,
// probes, managedFields, other annotations) is never read, so it is not turned into Python
// objects: one C++ parse per event instead of json.loads of the whole object.
static py::object jnode(const json::Doc& d, int32_t i) {
  const json::Node& n = d.at(i);
  switch (n.type) {
    case json::Type::kNull: return py::none();
    case json::Type::kBool: return py::bool_(n.b);
    case json::Type::kNum: {
      const std::string_view t = d.str(i);
      if (t.find_first_of(".eE") == std::string_view::npos) {
        try {
          return py::int_(std::stoll(std::string(t)));
        } catch (...) {
        }
      }
      return py::float_(std::stod(std::string(t)));
    }
    case json::Type::kStr: return py::str(std::string(d.str(i)));
    case json::Type::kArr: {
      py::list l;
      for (int32_t c = n.first; c >= 0; c = d.at(c).next) l.append(jnode(d, c));
      return std::move(l);
    }
    case json::Type::kObj: {
      py::dict o;
      for (int32_t c = n.first; c >= 0; c = d.at(c).next) o[py::str(std::string(d.key(c)))] = jnode(d, c);
      return std::move(o);
    }
  }
  return py::none();
}

static bool nanogpu_key(std::string_view k) { return k.rfind("nano-gpu/", 0) == 0; }

static py::dict slim_map(const json::Doc& d, int32_t obj, bool only_ours) {
  py::dict o;
  if (!d.is(obj, json::Type::kObj)) return o;
  for (int32_t c = d.at(obj).first; c >= 0; c = d.at(c).next)
    if (!only_ours || nanogpu_key(d.key(c))) o[py::str(std::string(d.key(c)))] = jnode(d, c);
  return o;
}

static void copy_str(const json::Doc& d, int32_t obj, const char* k, py::dict& out) {
  const int32_t v = d.get(obj, k);
  if (v >= 0 && d.at(v).type != json::Type::kNull) out[k] = jnode(d, v);
}

static py::dict slim_pod(const json::Doc& d, int32_t pod) {
  py::dict out, md, spec, st;
  const int32_t m = d.get(pod, "metadata");
  if (d.is(m, json::Type::kObj)) {
    for (const char* k : {"name", "namespace", "uid", "resourceVersion", "creationTimestamp", "deletionTimestamp"})
      copy_str(d, m, k, md);
    md["labels"] = slim_map(d, d.get(m, "labels"), false);
    md["annotations"] = slim_map(d, d.get(m, "annotations"), true);
  }
  const int32_t sp = d.get(pod, "spec");
  if (d.is(sp, json::Type::kObj)) {
    copy_str(d, sp, "nodeName", spec);
    copy_str(d, sp, "schedulerName", spec);
    for (const char* list : {"containers", "initContainers"}) {
      const int32_t cs = d.get(sp, list);
      if (!d.is(cs, json::Type::kArr)) continue;
      py::list out_cs;
      for (int32_t c = d.at(cs).first; c >= 0; c = d.at(c).next) {
        py::dict oc;
        copy_str(d, c, "name", oc);
        const int32_t res = d.get(c, "resources");
        if (d.is(res, json::Type::kObj)) {
          py::dict ores;
          for (const char* k : {"limits", "requests"}) {
            const int32_t lm = d.get(res, k);
            if (d.is(lm, json::Type::kObj)) ores[k] = slim_map(d, lm, true);
          }
          oc["resources"] = ores;
        }
        out_cs.append(oc);
      }
      spec[list] = out_cs;
    }
  }
  const int32_t s = d.get(pod, "status");
  if (d.is(s, json::Type::kObj)) copy_str(d, s, "phase", st);
  for (const char* k : {"apiVersion", "kind"}) copy_str(d, pod, k, out);
  out["metadata"] = md;
  out["spec"] = spec;
  out["status"] = st;
  return out;
}


// One event line, parsed in full, as the informer's {type, object} (a Pod slimmed).
static py::dict pod_event(json::Doc& d, std::string_view line) {
  if (!d.parse(line) || !d.is(d.root(), json::Type::kObj)) throw py::value_error("bad watch event line");
  const int32_t t = d.get(d.root(), "type");
  const int32_t obj = d.get(d.root(), "object");
  const std::string_view type = d.is(t, json::Type::kStr) ? d.str(t) : std::string_view();
  py::dict ev;
  ev["type"] = py::str(std::string(type));
  const bool plain = type == "ERROR" || type == "BOOKMARK";
  ev["object"] = d.is(obj, json::Type::kObj) ? (plain ? jnode(d, obj) : py::object(slim_pod(d, obj))) : py::dict();
  return ev;
}

// events were dropped after the last one kept: a bookmark carries the resume point
static py::dict bookmark(const std::string& rv) {
  py::dict md, o, ev;
  md["resourceVersion"] = rv;
  o["metadata"] = md;
  ev["type"] = "BOOKMARK";
  ev["object"] = o;
  return ev;
}

// The pod informer's decoder (nanogpu/k8s/informer.py); with a filter (podwatch.h) only what
// the filter keeps is decoded.
static py::list decode_pod_events(const py::bytes& data, PodWatchFilter* f) {
  std::string_view sv = data;
  py::list out;
  size_t p = 0;
  json::Doc d;
  std::string rv, last_rv;   // resourceVersion of dropped events after the last kept one
  while (p < sv.size()) {
    size_t e = sv.find('\n', p);
    if (e == std::string_view::npos) e = sv.size();
    std::string_view line = sv.substr(p, e - p);
    p = e + 1;
    while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.remove_suffix(1);
    if (line.empty()) continue;
    if (f && !filter_pod_event(*f, line, d, &rv)) {
      last_rv = rv;
      continue;
    }
    out.append(pod_event(d, line));
    last_rv.clear();
  }
  if (f && !last_rv.empty()) out.append(bookmark(last_rv));
  return out;
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "nanogpu native core: ledger, placement policies, topology reader";
  m.attr("MAX_DEVS") = kMaxDevs;
  m.attr("MAX_GPUS") = kMaxGpus;
  m.attr("MAX_CONTAINERS") = kMaxContainers;
  m.attr("OK") = static_cast<int>(kOk);
  m.attr("FLAG_MEM_BOUND") = static_cast<int>(kFlagMemBound);
  m.attr("ERR_NO_FIT") = static_cast<int>(kErrNoFit);
  m.attr("ERR_NO_DEVICES") = static_cast<int>(kErrNoDevices);
  m.attr("ERR_BAD_PLAN") = static_cast<int>(kErrBadPlan);
  m.attr("ERR_PLAN_NO_LONGER_FITS") = static_cast<int>(kErrPlanNoLongerFits);
  m.attr("ERR_UNKNOWN_NODE") = static_cast<int>(kErrUnknownNode);
  m.attr("ERR_UNKNOWN_POD") = static_cast<int>(kErrUnknownPod);
  m.attr("ERR_POD_EXISTS") = static_cast<int>(kErrPodExists);
  m.attr("ERR_TABLE_FULL") = static_cast<int>(kErrTableFull);
  m.attr("ERR_BAD_DEMAND") = static_cast<int>(kErrBadDemand);
  m.attr("OK_EXISTING") = static_cast<int>(kOkExisting);
  m.def("err_str", &err_str);

  py::enum_<Policy>(m, "Policy")
      .value("BINPACK", Policy::kBinpack)
      .value("SPREAD", Policy::kSpread)
      .value("RANDOM", Policy::kRandom)
      .value("FIRSTFIT", Policy::kFirstFit);

  py::class_<Options>(m, "Options")
      .def(py::init([](Policy p, bool compat, bool load_aware, float topo_weight, uint64_t seed,
                       const std::vector<int>& request_sizes, bool learn_sizes) {
             Options o;
             o.policy = p;
             o.compat = compat ? 1 : 0;
             o.load_aware = load_aware ? 1 : 0;
             o.topo_weight = topo_weight;
             o.seed = seed;
             o.learn_sizes = learn_sizes ? 1 : 0;
             SizeSet ss;
             for (int q : request_sizes) {
               if (q <= 0 || q > kPercentPerDevice) throw py::value_error("request size must be 1..100");
               ss.add(q);
             }
             o.set_sizes(ss);
             return o;
           }),
           py::arg("policy") = Policy::kBinpack, py::arg("compat") = false,
           py::arg("load_aware") = false, py::arg("topo_weight") = 1.0f, py::arg("seed") = 0,
           py::arg("request_sizes") = std::vector<int>{}, py::arg("learn_sizes") = true)
      .def_property_readonly("request_sizes", [](const Options& o) { return size_list(o.sizes); })
      .def_property_readonly("learn_sizes", [](const Options& o) { return o.learn_sizes != 0; })
      .def_property_readonly("waste", [](const Options& o) {
        return std::vector<int>(o.waste, o.waste + kWasteSlots);
      })
      .def_property_readonly("policy", [](const Options& o) { return o.policy; })
      .def_property_readonly("compat", [](const Options& o) { return o.compat != 0; })
      .def_property_readonly("load_aware", [](const Options& o) { return o.load_aware != 0; })
      .def_property_readonly("topo_weight", [](const Options& o) { return o.topo_weight; })
      .def_property_readonly("seed", [](const Options& o) { return o.seed; })
      .def("__repr__", [](const Options& o) {
        return "Options(policy=" + std::to_string(static_cast<int>(o.policy)) +
               ", compat=" + std::to_string(o.compat) + ", load_aware=" + std::to_string(o.load_aware) + ")";
      });

  // Stateless policy entry points (tests, simulators, the reference oracle diff).
  m.def(
      "choose",
      [](const py::list& devices, const py::sequence& demand,
         const Options& o, const py::object& topo) -> py::tuple {
        auto devs = to_devices(devices);
        Topology t = to_topo(topo, devs);
        Demand d = to_demand(demand);
        Plan p;
        std::memset(&p, 0, sizeof(p));
        int32_t rc;
        {
          py::gil_scoped_release nogil;
          rc = choose(devs.data(), static_cast<int>(devs.size()), &t, d, o, &p);
        }
        if (rc != kOk) return py::make_tuple(rc, py::none(), 0);
        return py::make_tuple(rc, plan_list(p), p.score);
      },
      py::arg("devices"), py::arg("demand"), py::arg("options"), py::arg("topo") = py::none());
  m.def(
      "rate",
      [](const py::list& devices, const py::sequence& demand,
         const Options& o) {
        auto devs = to_devices(devices);
        Demand d = to_demand(demand);
        return rate(devs.data(), static_cast<int>(devs.size()), d, o, nullptr);
      },
      py::arg("devices"), py::arg("demand"), py::arg("options"));
  m.def(
      "apply",
      [](const py::list& devices, const py::sequence& demand,
         const std::vector<std::vector<int>>& plan, bool release) {
        auto devs = to_devices(devices);
        Demand d = to_demand(demand);
        Plan p = to_plan(plan);
        const int32_t rc = release ? unapply(devs.data(), static_cast<int>(devs.size()), d, p)
                                   : apply(devs.data(), static_cast<int>(devs.size()), d, p);
        py::list out;
        for (const Device& v : devs) out.append(from_device(v));
        return py::make_tuple(rc, out);
      },
      py::arg("devices"), py::arg("demand"), py::arg("plan"), py::arg("release") = false);
  m.def(
      "frag",
      [](const py::list& devices, int32_t min_request) {
        auto devs = to_devices(devices);
        FragStats s{};
        frag_accumulate(devs.data(), static_cast<int>(devs.size()), min_request, &s);
        return frag_dict(s);
      },
      py::arg("devices"), py::arg("min_request") = 0);
  m.def("go116_sort_perm", [](const std::vector<int64_t>& keys) {
    // Returns the permutation Go 1.16 sort.Sort leaves for ascending `keys`.
    std::vector<int64_t> k = keys;
    std::vector<int> idx(keys.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = static_cast<int>(i);
    gosort::sort(
        static_cast<int>(k.size()), [&](int i, int j) { return k[i] < k[j]; },
        [&](int i, int j) {
          std::swap(k[i], k[j]);
          std::swap(idx[i], idx[j]);
        });
    return idx;
  });
  m.def("demand_hash", [](const py::sequence& demand) {
    return to_demand(demand).hash();
  });

  py::class_<Ledger, std::shared_ptr<Ledger>>(m, "Ledger")
      .def(py::init<const std::string&, uint32_t, uint32_t, bool>(), py::arg("path") = "",
           py::arg("max_nodes") = 1024, py::arg("max_pods") = 65536, py::arg("create") = true)
      .def_static("region_bytes", &Ledger::region_bytes)
      .def_property_readonly("path", &Ledger::path)
      .def_property_readonly("bytes", &Ledger::bytes)
      .def_property_readonly("n_nodes", &Ledger::n_nodes)
      .def_property_readonly("n_pods", &Ledger::n_pods)
      .def_property_readonly("overflow_records_used", &Ledger::overflow_records_used)
      .def_property_readonly("attached", &Ledger::attached, "processes attached to the region")
      .def("put_pod_info",
           [](Ledger& l, const std::string& key, py::bytes blob) { return l.put_pod_info(key, std::string(blob)); },
           py::arg("key"), py::arg("blob"))
      .def(
          "take_pod_info",
          [](Ledger& l, const std::string& key) -> py::object {
            std::string b;
            if (!l.take_pod_info(key, &b)) return py::none();
            return py::bytes(b);
          },
          py::arg("key"))
      .def_property_readonly("epoch", &Ledger::epoch)
      .def(
          "upsert_node",
          [](Ledger& l, const std::string& name, const py::list& devices, const py::object& topo) {
            auto devs = to_devices(devices);
            Topology t = to_topo(topo, devs);
            const int32_t id = l.upsert_node(name, devs.data(), static_cast<int>(devs.size()), t);
            if (id < 0) throw py::value_error(std::string("upsert_node: ") + err_str(-id));
            return id;
          },
          py::arg("name"), py::arg("devices"), py::arg("topo") = py::none())
      .def_property("serving", &Ledger::serving, &Ledger::set_serving,
                    "shared across workers: whether this replica schedules (leader election)")
      .def_property_readonly("nomination_margin", &Ledger::nomination_margin)
      .def("nomination_counts", [](const Ledger& l) {
        uint64_t m, a, v;
        l.nomination_counts(&m, &a, &v);
        py::dict d;
        d["made"] = m;
        d["adopted"] = a;
        d["moved"] = v;
        return d;
      })
      .def("find_node", &Ledger::find_node)
      .def("node_name", &Ledger::node_name)
      .def("remove_node", &Ledger::remove_node)
      .def("generation", &Ledger::generation)
      .def("snapshot",
           [](const Ledger& l, int32_t id) -> py::object {
             NodeSnapshot s;
             if (!l.snapshot(id, &s)) return py::none();
             py::dict d;
             py::list devs;
             for (int i = 0; i < s.n_devs; ++i) devs.append(from_device(s.devs[i]));
             d["devices"] = devs;
             d["generation"] = s.generation;
             d["topo"] = from_topo(s.topo);
             d["name"] = l.node_name(id);
             return d;
           })
      .def("cached_plans",
           [](const Ledger& l, int32_t id) {
             std::vector<Ledger::CachedPlan> v;
             {
               py::gil_scoped_release nogil;
               v = l.cached_plans(id);
             }
             py::list out;
             for (const auto& c : v) {
               // an entry that does not fit carries no plan (its Plan bytes are not filled in)
               const bool fits = c.rc == kOk || c.rc == kOkExisting;
               out.append(py::make_tuple(c.demand_hash, c.options_hash, c.rc, fits ? plan_list(c.plan) : py::list(),
                                         fits ? c.plan.score : 0));
             }
             return out;
           },
           "Valid plan-cache entries of node `id` in this process: (demand hash, options hash, rc, plan, score).")
      .def(
          "filter",
          [](Ledger& l, const std::vector<int32_t>& ids,
             const py::sequence& demand, const Options& o) {
            Demand d = to_demand(demand);
            std::vector<int32_t> rcs(ids.size());
            {
              py::gil_scoped_release nogil;
              Plan p;
              for (size_t i = 0; i < ids.size(); ++i) rcs[i] = ids[i] < 0 ? kErrUnknownNode : l.assume(ids[i], d, o, &p);
            }
            return rcs;
          },
          "Assume `demand` on every node id; returns one error code per node (0 = fits).")
      .def(
          "score",
          [](Ledger& l, const std::vector<int32_t>& ids,
             const py::sequence& demand, const Options& o) {
            Demand d = to_demand(demand);
            std::vector<int32_t> scores(ids.size());
            {
              py::gil_scoped_release nogil;
              Plan p;
              for (size_t i = 0; i < ids.size(); ++i) {
                const int32_t rc = ids[i] < 0 ? kErrUnknownNode : l.assume(ids[i], d, o, &p);
                scores[i] = rc == kOk ? p.score : 0;  // ScoreMin for unfit nodes (node.go:63-65)
              }
            }
            return scores;
          })
      .def(
          "assume_many",
          [](Ledger& l, const std::vector<int32_t>& ids, const py::sequence& demand, const Options& o) {
            Demand d = to_demand(demand);
            std::vector<int32_t> rcs(ids.size()), scores(ids.size());
            {
              py::gil_scoped_release nogil;
              l.assume_many(ids.data(), static_cast<int>(ids.size()), d, o, rcs.data(), scores.data());
            }
            return py::make_tuple(rcs, scores);
          },
          "The front door's filter / priorities path over node ids (this thread's score memo, memo "
          "entries re-validated against the devices changed since): (error codes, scores).")
      .def("assume",
           [](Ledger& l, int32_t id, const py::sequence& demand,
              const Options& o) -> py::tuple {
             Demand d = to_demand(demand);
             Plan p;
             std::memset(&p, 0, sizeof(p));
             int32_t rc;
             {
               py::gil_scoped_release nogil;
               rc = l.assume(id, d, o, &p);
             }
             if (rc != kOk) return py::make_tuple(rc, py::none(), 0);
             return py::make_tuple(rc, plan_list(p), p.score);
           })
      .def("reserve",
           [](Ledger& l, int32_t id, const std::string& key,
              const py::sequence& demand, const Options& o) -> py::tuple {
             Demand d = to_demand(demand);
             Plan p;
             std::memset(&p, 0, sizeof(p));
             int32_t rc;
             {
               py::gil_scoped_release nogil;
               rc = l.reserve(id, key, d, o, &p);
             }
             if (rc != kOk && rc != kOkExisting) return py::make_tuple(rc, py::none());
             return py::make_tuple(rc, plan_list(p));
           })
      .def("allocate_plan",
           [](Ledger& l, int32_t id, const std::string& key,
              const py::sequence& demand,
              const std::vector<std::vector<int>>& plan, bool committed) {
             Demand d = to_demand(demand);
             Plan p = to_plan(plan);
             py::gil_scoped_release nogil;
             return l.allocate_plan(id, key, d, p, committed);
           },
           py::arg("node"), py::arg("key"), py::arg("demand"), py::arg("plan"),
           py::arg("committed") = true)
      .def("commit", &Ledger::commit, py::call_guard<py::gil_scoped_release>())
      .def("release", &Ledger::release, py::call_guard<py::gil_scoped_release>())
      .def("reserve_wide",
           [](Ledger& l, int32_t id, const std::string& key, const py::sequence& folded,
              const std::vector<std::vector<int>>& fplan, const WidePlan& wide, bool committed) -> py::tuple {
             Demand d = to_demand(folded);
             Plan p = to_plan(fplan);
             WidePlan held;
             int32_t rc;
             {
               py::gil_scoped_release nogil;
               rc = l.reserve_wide(id, key, d, p, wide, committed, &held);
             }
             if (rc == kOkExisting) return py::make_tuple(rc, held.empty() ? py::object(py::none()) : py::cast(held));
             return py::make_tuple(rc, py::none());
           },
           py::arg("node"), py::arg("key"), py::arg("folded"), py::arg("fplan"), py::arg("wide"),
           py::arg("committed") = false,
           "A wide pod: its folded record and its per-container plan, in the shared ledger. (rc, held): "
           "OK; OK_EXISTING with the per-container plan the ledger already holds for the pod on that node "
           "(None if it holds none); or an error")
      .def("wide_plan",
           [](const Ledger& l, const std::string& key) -> py::object {
             WidePlan w;
             if (!l.wide_plan(key, &w)) return py::none();
             return py::cast(w);
           },
           "The per-container plan of wide pod `key` held in the ledger (None: not a wide pod here)")
      .def_property_readonly("wide_records_used", &Ledger::wide_records_used)
      .def("lookup",
           [](const Ledger& l, const std::string& key) -> py::object {
             PodRecord r;
             if (!l.lookup(key, &r)) return py::none();
             return record_dict(r);
           })
      .def(
          "holds_any",
          [](const Ledger& l, const std::vector<std::string>& keys) {
            py::gil_scoped_release nogil;
            for (const std::string& k : keys)
              if (l.holds(k)) return true;
            return false;
          },
          py::arg("keys"), "Whether the ledger holds a record of any of `keys` (one call for many)")
      .def("pods_on",
           [](const Ledger& l, int32_t node) {
             py::list out;
             for (const PodRecord& r : l.pods_on(node)) out.append(record_dict(r));
             return out;
           },
           py::arg("node") = -1)
      .def(
          "fits_without",
          [](const Ledger& l, int32_t id, const std::vector<std::string>& victims, const py::sequence& demand,
             const Options& o) {
            Demand d = to_demand(demand);
            Plan p;
            std::memset(&p, 0, sizeof(p));
            int32_t rc;
            {
              py::gil_scoped_release nogil;
              rc = l.fits_without(id, victims, d, o, &p);
            }
            return py::make_tuple(rc, rc == kOk ? plan_list(p) : py::list());
          },
          py::arg("node"), py::arg("victims"), py::arg("demand"), py::arg("options"),
          "(rc, plan): would `demand` fit on `node` once the victims' shares are released (simulated)")
      .def("expired_reservations", &Ledger::expired_reservations, py::call_guard<py::gil_scoped_release>())
      .def("expired_nominations", &Ledger::expired_nominations, py::call_guard<py::gil_scoped_release>())
      .def("drop_reservation", &Ledger::drop_reservation, py::call_guard<py::gil_scoped_release>())
      .def("drop_committed", &Ledger::drop_committed, py::call_guard<py::gil_scoped_release>())
      .def(
          "reconcile_joined",
          [](Ledger& l, const std::string& joined, double before) {
            py::gil_scoped_release nogil;
            std::vector<std::string_view> v;
            v.reserve(joined.size() / 37 + 1);
            size_t a = 0;
            while (a < joined.size()) {
              size_t b = joined.find('\n', a);
              if (b == std::string::npos) b = joined.size();
              if (b > a) v.emplace_back(joined.data() + a, b - a);
              a = b + 1;
            }
            return l.reconcile_views(v, before);
          },
          py::arg("joined"), py::arg("before"),
          "reconcile() with the listed UIDs as one newline-joined string: one copy across the "
          "binding, the split and the walk without the GIL")
      .def("reconcile", &Ledger::reconcile, py::arg("live"), py::arg("before"),
           py::call_guard<py::gil_scoped_release>(),
           "Relist: release Committed pods recorded before `before` (mono_now) whose key is not in "
           "`live`; returns the keys released")
      .def("drop_nomination", &Ledger::drop_nomination, py::call_guard<py::gil_scoped_release>())
      .def("deferred_nomination_begin", &Ledger::deferred_nomination_begin)
      .def("deferred_nomination_end", &Ledger::deferred_nomination_end)
      .def("wait_deferred_nominations", &Ledger::wait_deferred_nominations, py::arg("max_ns"),
           py::call_guard<py::gil_scoped_release>(),
           "Until every nomination a worker deferred past its answer is made (False: `max_ns` passed).")
      .def(
          "nominate",
          [](Ledger& l, int32_t id, const std::string& key, const py::sequence& demand,
             const Options& o) {
            Demand d = to_demand(demand);
            py::gil_scoped_release nogil;
            return l.nominate(id, key, d, o);
          },
          "tentative reservation for the top-scored node (priorities); adopted by reserve()")
      .def("set_load", &Ledger::set_load)
      .def("set_health", &Ledger::set_health)
      .def("set_mem_hot", &Ledger::set_mem_hot)
      .def("set_mem_busy", &Ledger::set_mem_busy, py::arg("node"), py::arg("dev"), py::arg("percent"))
      .def(
          "set_stream_owner",
          [](Ledger& l, const std::string& uid, bool streaming) { l.set_stream_owner(owner_hash(uid), streaming); },
          py::arg("uid"), py::arg("streaming"))
      .def(
          "is_stream_owner", [](const Ledger& l, const std::string& uid) { return l.is_stream_owner(owner_hash(uid)); },
          py::arg("uid"))
      .def(
          "set_pod_owner",
          [](Ledger& l, const std::string& key, const std::string& owner_uid) {
            return l.set_pod_owner(key, owner_uid.empty() ? 0 : owner_hash(owner_uid));
          },
          py::arg("key"), py::arg("owner_uid"))
      .def(
          "learn_stream_owners",
          [](Ledger& l, bool forget_cool, double reserved_before, int32_t forget_after,
             const std::vector<std::pair<float, float>>& hot_curve) {
            std::pair<int32_t, int32_t> r;
            {
              py::gil_scoped_release nogil;
              r = l.learn_stream_owners(forget_cool, reserved_before, forget_after, hot_curve);
            }
            return r;
          },
          py::arg("forget_cool") = true, py::arg("reserved_before") = 1e300, py::arg("forget_after") = 1,
          py::arg("hot_curve") = std::vector<std::pair<float, float>>{})
      .def_static("owner_hash", [](const std::string& uid) { return owner_hash(uid); })
      .def("frag", [](const Ledger& l, int32_t min_request) { return frag_dict(l.frag(min_request)); },
           py::arg("min_request") = 0)
      .def("learned_sizes", [](const Ledger& l) { return size_list(l.learned_sizes()); },
           "share sizes (percent) the ledger has learned are common (native binpack's waste model)")
      .def("note_request", [](Ledger& l, const py::sequence& demand) { l.note_request(to_demand(demand)); })
      .def("clear_cache", &Ledger::clear_cache)
      .def_property_readonly("cache_size", &Ledger::cache_size);

  m.def(
      "discover_topology",
      [](const std::string& root, bool use_amdsmi) {
        HostTopology t;
        {
          py::gil_scoped_release nogil;
          t = discover(root, use_amdsmi);
        }
        return to_json(t);
      },
      py::arg("root") = "", py::arg("use_amdsmi") = true,
      "Reads KFD/DRM sysfs (+ libamd_smi) and returns the node GPU topology as JSON.");
  m.def("parse_properties", &parse_properties, "KFD `key value` properties text -> dict");
  m.def(
      "quantity_value",
      [](const std::string& s, bool mib) -> py::object {
        int64_t v;
        if (!quantity_value(s, mib, &v)) return py::none();
        return py::int_(v);
      },
      py::arg("text"), py::arg("mib") = false, "Native Quantity.Value() (None when the fast path declines).");
  py::class_<Frontend, std::shared_ptr<Frontend>>(m, "Frontend")
      .def(py::init<std::shared_ptr<Ledger>, const std::string&, int, int>(), py::arg("ledger"),
           py::arg("host") = "0.0.0.0", py::arg("port") = 0, py::arg("threads") = 2)
      .def_property_readonly("port", &Frontend::port)
      .def("notify_fd", &Frontend::notify_fd)
      .def("set_options", &Frontend::set_options, py::arg("options"), py::arg("score_normalize") = false,
           py::arg("nominate") = false, py::arg("decisive") = false, py::arg("lead") = 0,
           "lead: priorities answer the nominated node this many points above every other fitting node "
           "(normalised scores: 10 and 0), so kube-scheduler's own plugins do not move the pod")
      .def("set_serving", &Frontend::set_serving)
      .def("set_busy_poll_us", &Frontend::set_busy_poll_us)
      .def("set_busy_poll_prio_us", &Frontend::set_busy_poll_prio_us)
      .def("set_lazy_labels", &Frontend::set_lazy_labels, py::arg("on"),
           "Evented / inline writer: label PATCH answers read by a later pass of the loop, not woken for.")
      .def("set_fe_send", &Frontend::set_fe_send, py::arg("on"),
           "Evented writer: front-door workers send each bind's requests themselves; the writer "
           "thread reads the answers (KubeWriter::send_from_caller).")
      .def("set_bind_first", &Frontend::set_bind_first)
      .def("set_spin_nap", &Frontend::set_spin_nap)
      .def("set_spin_recv", &Frontend::set_spin_recv)
      .def("set_spin_recv_binds", &Frontend::set_spin_recv_binds)
      .def(
          "set_kube_writer",
          [](Frontend& f, const std::string& host, int port, bool tls, const std::string& token,
             const std::string& token_file, const std::string& ca_file, const std::string& cert_file,
             const std::string& key_file, bool insecure, int threads, int retries, bool record_events,
             bool evented, bool label, double timeout_s, bool inline_io, bool batch_labels, int max_binds) {
            KubeTarget t;
            t.host = host;
            t.port = port;
            t.tls = tls;
            t.token = token;
            t.token_file = token_file;
            t.ca_file = ca_file;
            t.cert_file = cert_file;
            t.key_file = key_file;
            t.insecure = insecure;
            f.set_kube_writer(t, threads, retries, record_events, evented, label, timeout_s, inline_io, batch_labels,
                              max_binds);
          },
          py::arg("host"), py::arg("port"), py::arg("tls") = false, py::arg("token") = "",
          py::arg("token_file") = "", py::arg("ca_file") = "", py::arg("cert_file") = "", py::arg("key_file") = "",
          py::arg("insecure") = false, py::arg("threads") = 32, py::arg("retries") = 3,
          py::arg("record_events") = true, py::arg("evented") = true, py::arg("label") = true,
          py::arg("timeout_s") = 30.0, py::arg("inline_io") = false, py::arg("batch_labels") = false,
          py::arg("max_binds") = 0,
          "Binds whose reservation succeeded natively are finished natively (PATCH + binding + "
          "commit/rollback) on keep-alive connections to kube-apiserver: one epoll thread "
          "(evented) or `threads` blocking threads; `threads` x 8 binds in flight.")
      .def("kube_writer_stats",
           [](const Frontend& f) -> py::object {
             const KubeWriter* w = f.kube_writer();
             if (!w) return py::none();
             py::dict d;
             d["ok"] = w->stats.ok.load();
             d["failed"] = w->stats.failed.load();
             d["rollbacks"] = w->stats.rollbacks.load();
             d["retries"] = w->stats.retries.load();
             d["inflight"] = w->stats.inflight.load();
             d["patch_seconds_total"] = static_cast<double>(w->stats.patch_ns.load()) * 1e-9;
             d["binding_seconds_total"] = static_cast<double>(w->stats.binding_ns.load()) * 1e-9;
             d["label_failures"] = w->stats.label_failures.load();
             d["timeouts"] = w->stats.timeouts.load();
             d["throttled"] = w->stats.throttled.load();
             d["throttle_resends"] = w->stats.throttle_resends.load();
             d["window_cuts"] = w->stats.window_cuts.load();
             d["window"] = w->stats.window.load();
             d["bindings_first"] = w->stats.bindings_first.load();
             return d;
           })
      .def("take",
           [](Frontend& f) {
             std::vector<PyRequest> v;
             {
               py::gil_scoped_release nogil;
               v = f.take();
             }
             py::list out;
             for (auto& r : v) {
               py::object prep = py::none();
               if (r.bind.ok) {
                 const PreparedBind& b = r.bind;
                 py::dict pd;
                 pd["rc"] = b.rc;
                 pd["ns"] = b.ns;
                 pd["name"] = b.name;
                 pd["uid"] = b.uid;
                 pd["node"] = b.node;
                 pd["containers"] = b.containers;
                 pd["plan"] = b.plan;
                 pd["demand"] = b.demand;
                 prep = pd;
               }
               // a prepared bind needs neither its request body nor the cached pod JSON in Python
               const bool bare = r.bind.ok;
               out.append(py::make_tuple(r.id, r.method, r.path, r.query,
                                         bare ? py::bytes() : py::bytes(r.body),
                                         bare ? py::bytes() : py::bytes(r.pod_json), r.t_arrival, prep));
             }
             return out;
           })
      .def("respond",
           [](Frontend& f, uint64_t id, int status, const std::string& ctype, const py::bytes& body, bool notify) {
             std::string b = body;
             f.respond(id, status, ctype, b, notify);   // a short mailbox lock: no GIL round trip
           },
           py::arg("id"), py::arg("status"), py::arg("content_type"), py::arg("body"), py::arg("notify") = true)
      .def("flush", &Frontend::wake_workers, "wake the workers holding responses queued with notify=False")
      .def("stop", &Frontend::stop, py::call_guard<py::gil_scoped_release>())
      .def("pod_cache_size", &Frontend::pod_cache_size)
      .def("take_bind_wall", [](Frontend& f) {
             std::vector<uint64_t> ns = f.take_bind_wall();
             std::vector<double> s(ns.size());
             for (size_t i = 0; i < ns.size(); ++i) s[i] = static_cast<double>(ns[i]) * 1e-9;
             return s;
           },
           "seconds from request read to response written, per bind since the last call")
      .def("bind_samples_waiting", &Frontend::bind_samples_waiting,
           "(bind wall times, bind hop splits) recorded and not yet taken")
      .def("set_bind_hops", &Frontend::set_bind_hops, py::arg("on"),
           "record each native bind's hop split (false: off, or no invariant TSC on this host)")
      .def("take_bind_hops", [](Frontend& f) {
             const std::vector<std::array<uint32_t, kHopSplits>> v = f.take_bind_hops();
             std::vector<std::vector<uint32_t>> out;
             out.reserve(v.size());
             for (const auto& a : v) out.emplace_back(a.begin(), a.end());
             return out;
           },
           "per native bind since the last call, ns of: parse+reserve, hand-off to the writer, wait for the "
           "admission window, build+send, API answer, commit+post, reply")
      .def("stats", [](Frontend& f) {
        auto one = [](const VerbStats& s) {
          py::dict d;
          d["count"] = s.count.load();
          d["errors"] = s.errors.load();
          d["deferred"] = s.deferred.load();
          d["seconds_total"] = static_cast<double>(s.ns_total.load()) * 1e-9;
          d["max_s"] = static_cast<double>(s.max_ns.load()) * 1e-9;
          py::list b;
          for (const auto& x : s.buckets) b.append(x.load());
          d["buckets_8us_pow2"] = b;
          return d;
        };
        py::dict d;
        d["filter"] = one(f.filter_stats);
        d["priorities"] = one(f.prio_stats);
        d["filter_wall"] = one(f.filter_wall_stats);
        d["priorities_wall"] = one(f.prio_wall_stats);
        d["python"] = one(f.py_stats);
        d["bind_reserve"] = one(f.bind_stats);
        d["connections"] = f.connections.load();
        d["requests"] = f.requests.load();
        d["loop_max_s"] = static_cast<double>(f.loop_max_ns.load()) * 1e-9;
        d["spin_hits"] = f.spin_hits.load();
        d["mailbox_wakeups"] = f.mb_wakeups.load();
        d["bind_handoffs"] = f.bind_handoffs.load();
        d["pods_published"] = f.pods_published.load();
        d["handoff_waits"] = f.handoff_waits.load();
        py::list ph;
        for (const auto& x : f.phase_max_ns) ph.append(static_cast<double>(x.load()) * 1e-9);
        d["phase_max_s"] = ph;
        return d;
      })
      .def("verb",
           [](Frontend& f, const py::bytes& body, bool prioritize) {
             const std::string b = body;
             std::string out;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = f.filter_verb(b, prioritize, &out);
             }
             return py::make_tuple(ok, ok ? out : std::string());
           },
           py::arg("body"), py::arg("prioritize"),
           "The native filter / priorities verb on one body: (answered natively, answer JSON).")
      .def("time_verb",
           [](Frontend& f, const py::bytes& body, bool prioritize, int iters) {
             const std::string b = body;
             std::string out;
             bool ok = true;
             double dt;
             {
               py::gil_scoped_release nogil;
               const double t0 = mono_now();
               for (int i = 0; i < iters && ok; ++i) ok = f.filter_verb(b, prioritize, &out);
               dt = mono_now() - t0;
             }
             return py::make_tuple(ok, dt / std::max(1, iters), py::bytes(out));
           },
           py::arg("body"), py::arg("prioritize") = false, py::arg("iters") = 1000,
           "Runs the native verb `iters` times in place (no socket): (ok, seconds per call, last body).")
      .def("reset_max", &Frontend::reset_max, "zero the per-verb and event-loop maxima");
  m.def("mono_now", &mono_now);
  m.def("json_skip", [](const py::bytes& src, bool scalar) { return json::Doc::skip_for_test(std::string(src), scalar); },
        py::arg("src"), py::arg("scalar") = false,
        "The JSON container skipper from offset 0 (AVX2, or the scalar fallback): end offset, -1 = refused.");
  m.def("json_skip_uses_avx2", &json::Doc::skip_uses_avx2, "Whether the JSON skipper runs its AVX2 walk on this host.");
  m.def("io_tally_enable", [](bool on) { g_io.on.store(on, std::memory_order_relaxed); }, py::arg("on"),
        "Switches the per-call-site system-call / phase tally (iotally.h) on or off.");
  m.def("io_tally_reset", []() { g_io.reset(); }, "Zeroes the tally.");
  m.def("io_tally", []() {
    const double r = io_ns_per_tick();
    py::dict out;
    for (int k = 0; k < kIoKinds; ++k) {
      const uint64_t n = g_io.s[k].n.load(std::memory_order_relaxed);
      if (n) out[io_kind_name(k)] = py::make_tuple(n, 1e-9 * r * static_cast<double>(g_io.s[k].ticks.load(std::memory_order_relaxed)));
    }
    return out;
  }, "{kind: (calls, seconds)} since the last reset (kinds with calls only).");
  m.def("sampler_start", &sampler::start, py::arg("hz") = 1000,
        "CPU sampling profiler: SIGPROF every 1/hz s of process CPU time (false: already running).");
  m.def("sampler_stop", []() {
    const std::vector<sampler::Sample> v = sampler::stop();
    py::list out;
    for (const auto& x : v) out.append(py::make_tuple(x.pc, x.caller, x.tid));
    return out;
  }, "Stops the sampler: [(pc, caller pc or 0, tid)] (nanogpu.obs.cpu_profile symbolizes them).");
  m.def("num_feasible_nodes_to_find", &sim::num_feasible_nodes_to_find, py::arg("all_nodes"),
        py::arg("percentage") = 0, "kube-scheduler's numFeasibleNodesToFind (schedsim.h)");
  m.def("presize_fd_table", &presize_fd_table, py::arg("want") = 16384,
        "Grow the process fd table once up front (no RCU-synchronised growth under load).");
  py::class_<sim::Session, std::shared_ptr<sim::Session>>(m, "SchedulerSession")
      .def(py::init<>());
  // a burst's pods converted once (kube-scheduler holds its pods decoded in the informer
  // before a cycle starts): drive_scheduler then takes them without per-run conversion
  struct SimBurst {
    std::vector<sim::SimPod> pods;
  };
  auto to_sim_pods = [](const py::list& pods) {
    std::vector<sim::SimPod> ps(pods.size());
    for (size_t i = 0; i < pods.size(); ++i) {
      // (json, ns, name, uid, need[, cpu_m, mem[, owner]])
      auto t = pods[i].cast<py::tuple>();
      if (t.size() != 5 && t.size() != 7 && t.size() != 8)
        throw py::value_error("pod tuple: (json, ns, name, uid, need[, cpu_m, mem[, owner]])");
      ps[i].json = t[0].cast<std::string>();
      ps[i].ns = t[1].cast<std::string>();
      ps[i].name = t[2].cast<std::string>();
      ps[i].uid = t[3].cast<std::string>();
      ps[i].need = t[4].cast<int64_t>();
      if (t.size() >= 7) {
        ps[i].cpu_m = t[5].cast<int64_t>();
        ps[i].mem = t[6].cast<int64_t>();
      }
      if (t.size() == 8) ps[i].owner = t[7].cast<int32_t>();
    }
    return ps;
  };
  py::class_<SimBurst, std::shared_ptr<SimBurst>>(m, "SimBurst")
      .def(py::init([to_sim_pods](const py::list& pods) {
             auto b = std::make_shared<SimBurst>();
             b->pods = to_sim_pods(pods);
             return b;
           }),
           py::arg("pods"))
      .def("__len__", [](const SimBurst& b) { return b.pods.size(); });
  m.def(
      "drive_scheduler",
      [to_sim_pods](const std::string& host, int port, const py::object& pods,
         const std::vector<std::string>& nodes, const std::vector<int64_t>& capacity, int bind_threads, uint64_t seed,
         int max_attempts, double backoff_s, std::shared_ptr<sim::Session> session, int kube_combine,
         int extender_weight, int sample_nodes, int percentage_of_nodes_to_score, int spread_weight,
         const std::vector<std::tuple<int32_t, int64_t, int64_t, int64_t, int32_t>>& live,
         const std::vector<int>& bind_ports) {
        sim::SimConfig cfg;
        cfg.host = host;
        cfg.port = port;
        cfg.nodes = nodes;
        cfg.capacity = capacity;
        cfg.bind_threads = bind_threads;
        cfg.seed = seed;
        cfg.max_attempts = max_attempts;
        cfg.backoff_s = backoff_s;
        cfg.kube_combine = kube_combine;
        cfg.extender_weight = extender_weight;
        cfg.sample_nodes = sample_nodes;
        cfg.percentage_of_nodes_to_score = percentage_of_nodes_to_score;
        cfg.spread_weight = spread_weight;
        cfg.bind_ports = bind_ports;
        for (const auto& [node, need, cpu, mem, owner] : live) cfg.live.push_back({node, need, cpu, mem, owner});
        if (!capacity.empty() && capacity.size() != nodes.size())
          throw py::value_error("capacity must be empty or one entry per node");
        std::shared_ptr<SimBurst> burst;
        if (py::isinstance<SimBurst>(pods)) {
          burst = pods.cast<std::shared_ptr<SimBurst>>();
        } else {
          burst = std::make_shared<SimBurst>();
          burst->pods = to_sim_pods(pods.cast<py::list>());
        }
        sim::SimResult r;
        {
          py::gil_scoped_release nogil;
          r = sim::drive(cfg, burst->pods, session.get());
        }
        py::dict d;
        d["scheduled"] = r.scheduled;
        d["failed"] = r.failed;
        d["bind_errors"] = r.bind_errors;
        d["unschedulable_attempts"] = r.unschedulable_attempts;
        d["t_first_filter"] = r.t_first_filter;
        d["cycle_max_s"] = r.cycle_max_s;
        d["cycle_sum_s"] = r.cycle_sum_s;
        d["cycle_wire_s"] = r.cycle_wire_s;
        d["t_last_bind"] = r.t_last_bind;
        d["bind_latencies"] = r.bind_latencies;
        d["e2e_latencies"] = r.e2e_latencies;
        d["node_of"] = r.node_of;
        d["last_error"] = r.last_error;
        d["nodes_sent_filter"] = r.nodes_sent_filter;
        d["cycles"] = r.cycles;
        return d;
      },
      py::arg("host"), py::arg("port"), py::arg("pods"), py::arg("nodes"), py::arg("capacity"),
      py::arg("bind_threads") = 256, py::arg("seed") = 0, py::arg("max_attempts") = 8, py::arg("backoff_s") = 0.001,
      py::arg("session") = nullptr, py::arg("kube_combine") = 0, py::arg("extender_weight") = 1,
      py::arg("sample_nodes") = 1, py::arg("percentage_of_nodes_to_score") = 0, py::arg("spread_weight") = 2,
      py::arg("live") = std::vector<std::tuple<int32_t, int64_t, int64_t, int64_t, int32_t>>{},
      py::arg("bind_ports") = std::vector<int>{},
      "kube-scheduler stand-in (native/src/schedsim.cpp): schedule `pods` through the extender at host:port");

  // ------------------------------------------------------------------ native API server
  py::class_<apisrv::Server, std::shared_ptr<apisrv::Server>>(
      m, "ApiServer", "In-memory Kubernetes API server over HTTP (native/src/apiserver.cpp)")
      .def(py::init([](const std::string& host, int port, int threads, size_t history) {
             apisrv::Config c;
             c.host = host;
             c.port = port;
             c.threads = threads;
             c.history = history;
             return std::make_shared<apisrv::Server>(c);
           }),
           py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("threads") = 4,
           py::arg("history") = size_t(200000))
      .def_property_readonly("port", &apisrv::Server::port)
      .def("stop", &apisrv::Server::stop, py::call_guard<py::gil_scoped_release>())
      .def(
          "call",
          [](apisrv::Server& s, const std::string& method, const std::string& target, const std::string& body) {
            std::pair<int, std::string> r;
            {
              py::gil_scoped_release nogil;
              r = s.call(method, target, body);
            }
            return py::make_tuple(r.first, py::bytes(r.second));
          },
          py::arg("method"), py::arg("target"), py::arg("body") = "",
          "One request without a socket: (status, body bytes).")
      .def("create_pods", &apisrv::Server::create_pods, py::arg("pods"), py::arg("threads") = 0,
           py::call_guard<py::gil_scoped_release>(),
           "Creates pods from JSON texts under one lock hold; one status code per pod.")
      .def("delete_pods", &apisrv::Server::delete_pods, py::arg("keys"), py::call_guard<py::gil_scoped_release>(),
           "Deletes (namespace, name) pods; returns how many existed.")
      .def("stats", [](const apisrv::Server& s) { return s.stats_json(); })
      .def("set_latency", &apisrv::Server::set_latency, py::arg("seconds"))
      .def("set_spin", &apisrv::Server::set_spin, py::arg("seconds"),
           "IO threads poll this long after their last event before sleeping (a diagnostic)")
      .def("set_max_mutating_inflight", &apisrv::Server::set_max_mutating_inflight, py::arg("n"),
           "kube-apiserver's --max-mutating-requests-inflight (0: none): mutating requests over it get 429 "
           "with Retry-After: 1")
      .def("compact", &apisrv::Server::compact, py::arg("kind") = "")
      .def("drop_watches", &apisrv::Server::drop_watches, py::arg("kind") = "");

  m.def(
      "decode_pod_watch", [](py::bytes data) { return decode_pod_events(data, nullptr); }, py::arg("data"),
      "Newline-delimited pod watch events -> [{type, object}] with each Pod reduced to the fields the "
      "pod informer reads (identity, labels, nano-gpu/* annotations and resources, nodeName, phase).");

  m.def(
      "decode_pod_list",
      [](py::bytes data) {
        const std::string_view sv = data;
        json::Doc d;
        if (!d.parse(sv) || !d.is(d.root(), json::Type::kObj)) throw py::value_error("bad PodList");
        py::list items;
        const int32_t arr = d.get(d.root(), "items");
        if (d.is(arr, json::Type::kArr))
          for (int32_t c = d.at(arr).first; c >= 0; c = d.at(c).next)
            if (d.is(c, json::Type::kObj)) items.append(slim_pod(d, c));
        std::string rv, cont;
        const int32_t md = d.get(d.root(), "metadata");
        if (d.is(md, json::Type::kObj)) {
          const int32_t r = d.get(md, "resourceVersion"), k = d.get(md, "continue");
          if (d.is(r, json::Type::kStr)) rv = std::string(d.str(r));
          if (d.is(k, json::Type::kStr)) cont = std::string(d.str(k));
        }
        return py::make_tuple(items, rv, cont);
      },
      py::arg("data"),
      "A PodList page -> (pods reduced as decode_pod_watch reduces them, resourceVersion, continue token): "
      "what the pod informer keeps of a LIST, without decoding every field of every pod in Python.");

  py::class_<PodWatchFilter, std::shared_ptr<PodWatchFilter>>(
      m, "PodWatchFilter",
      "decode_pod_watch plus the pod controller's ledger-only work done natively: ADDED/MODIFIED of "
      "pending pods and of bound pods the ledger holds are dropped, DELETED of pods Python never saw "
      "is released from the ledger here and dropped; every event of a pod once handed to Python keeps "
      "going to Python. A trailing BOOKMARK carries the resume resourceVersion of dropped events.")
      .def(py::init([](std::shared_ptr<Ledger> l) {
             auto f = std::make_shared<PodWatchFilter>();
             f->ledger = std::move(l);
             return f;
           }),
           py::arg("ledger"))
      .def("decode", [](PodWatchFilter& f, py::bytes data) { return decode_pod_events(data, &f); }, py::arg("data"))
      .def(
          "reset",
          [](PodWatchFilter& f, const std::vector<std::string>& keys) {
            std::lock_guard<std::mutex> g(f.mu);
            f.forwarded.clear();
            f.forwarded.insert(keys.begin(), keys.end());
          },
          py::arg("keys"), "After a relist: the keys now in the informer's store.")
      .def_property(
          "release_on_terminating",
          [](const PodWatchFilter& f) { return f.release_on_terminating.load(std::memory_order_relaxed); },
          [](PodWatchFilter& f, bool v) { f.release_on_terminating.store(v, std::memory_order_relaxed); })
      .def_property_readonly("released",
                             [](PodWatchFilter& f) {
                               std::lock_guard<std::mutex> g(f.mu);
                               return f.released;
                             })
      .def_property_readonly("dropped",
                             [](PodWatchFilter& f) {
                               std::lock_guard<std::mutex> g(f.mu);
                               return f.dropped;
                             })
      .def_property_readonly("forwarded", [](PodWatchFilter& f) {
        std::lock_guard<std::mutex> g(f.mu);
        return f.forwarded.size();
      });

  py::class_<PodWatchStream>(
      m, "PodWatchStream",
      "A pod watch read by a native thread: the stream's event lines run through a PodWatchFilter "
      "as they arrive and only the kept ones are queued; notify_fd() becomes readable when there "
      "are some, or when the stream ended. take() -> (events, state, status, message): events "
      "decoded as PodWatchFilter.decode does (a trailing BOOKMARK for dropped ones), state 0 "
      "streaming, 1 ended cleanly, 2 HTTP error (status, body), 3 transport failure.")
      .def(py::init([](const std::string& host, int port, bool tls, const std::string& token,
                       const std::string& ca_file, const std::string& cert_file, const std::string& key_file,
                       bool insecure, const std::string& path, std::shared_ptr<PodWatchFilter> filter,
                       int read_timeout_s) {
             KubeTarget t;
             t.host = host;
             t.port = port;
             t.tls = tls;
             t.token = token;
             t.ca_file = ca_file;
             t.cert_file = cert_file;
             t.key_file = key_file;
             t.insecure = insecure;
             return std::make_unique<PodWatchStream>(std::move(t), path, std::move(filter), read_timeout_s);
           }),
           py::arg("host"), py::arg("port"), py::arg("tls"), py::arg("token"), py::arg("ca_file"),
           py::arg("cert_file"), py::arg("key_file"), py::arg("insecure"), py::arg("path"), py::arg("filter"),
           py::arg("read_timeout_s") = 330)
      .def("notify_fd", &PodWatchStream::notify_fd)
      .def("take",
           [](PodWatchStream& s) {
             PodWatchStream::Batch b;
             {
               py::gil_scoped_release nogil;
               b = s.take();
             }
             py::list out;
             json::Doc d;
             for (const auto& l : b.lines) out.append(pod_event(d, l));
             if (!b.last_rv.empty()) out.append(bookmark(b.last_rv));
             return py::make_tuple(out, b.state, b.status, b.message);
           })
      .def("stop", &PodWatchStream::stop, py::call_guard<py::gil_scoped_release>());
}
