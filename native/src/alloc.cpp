// Placement policies: reference-exact (compat) and MI355X-native.
// See alloc.h for the reference parity map.
#include "nanogpu/alloc.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <sstream>

#include "nanogpu/gosort.h"

namespace nanogpu {

const char* err_str(int32_t e) {
  switch (e) {
    case kOk: return "ok";
    case kErrNoFit: return "insufficient gpu resource";
    case kErrNoDevices: return "node has no gpu devices";
    case kErrBadPlan: return "plan does not match node devices";
    case kErrPlanNoLongerFits: return "plan no longer fits node";
    case kErrUnknownNode: return "unknown node";
    case kErrUnknownPod: return "unknown pod";
    case kErrPodExists: return "pod already allocated on another node";
    case kErrTableFull: return "ledger table full";
    case kErrBadDemand: return "invalid demand";
    case kOkExisting: return "already allocated";
    default: return "unknown error";
  }
}

static inline uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

uint64_t Demand::hash() const {
  uint64_t h = 0xcbf29ce484222325ULL ^ static_cast<uint64_t>(n);
  for (int i = 0; i < n; ++i) {
    h = mix64(h ^ static_cast<uint64_t>(static_cast<uint32_t>(c[i].pct)));
    h = mix64(h ^ static_cast<uint64_t>(c[i].mib));
    if (c[i].flags) h = mix64(h ^ (static_cast<uint64_t>(static_cast<uint32_t>(c[i].flags)) << 40));
  }
  return h;
}

uint64_t Options::hash() const {
  uint64_t h = mix64(static_cast<uint64_t>(policy) | (static_cast<uint64_t>(compat) << 8) |
                     (static_cast<uint64_t>(load_aware) << 16));
  uint32_t tw;
  std::memcpy(&tw, &topo_weight, sizeof(tw));
  h = mix64(h ^ tw ^ mix64(seed));
  if (!sizes.empty()) h = mix64(h ^ mix64(sizes.bits[0]) ^ (mix64(sizes.bits[1]) << 1));
  return h;
}

void Options::set_sizes(const SizeSet& s) {
  sizes = s;
  // best[h]: the largest sum of request sizes (with repetition) that fits in h
  int best[kWasteSlots];
  best[0] = 0;
  for (int h = 1; h <= kPercentPerDevice; ++h) {
    best[h] = best[h - 1];
    for (int q = 1; q <= h; ++q)
      if (s.has(q)) best[h] = std::max(best[h], best[h - q] + q);
  }
  for (int h = 0; h <= kPercentPerDevice; ++h)
    waste[h] = s.empty() ? 0 : static_cast<uint8_t>(h - best[h]);
}

// Waste a share placement adds: dead capacity of the hole it leaves minus that of the hole
// it fills (0 when both are fillable, or the hole was already dead).
static inline int waste_delta(const Options& o, int32_t free_before, int32_t pct) {
  if (!o.waste_aware()) return 0;
  const int a = std::clamp(free_before, 0, kPercentPerDevice);
  const int b = std::clamp(free_before - pct, 0, kPercentPerDevice);
  return static_cast<int>(o.waste[b]) - static_cast<int>(o.waste[a]);
}

int devices_needed(const ContainerDemand& c) {
  if (c.pct <= 0) return c.mib > 0 ? 1 : 0;
  if (c.pct <= kPercentPerDevice) return 1;
  return c.pct / kPercentPerDevice;
}

static inline bool hbm_fits(const Device& d, int64_t mib) {
  return mib <= 0 || d.mib_total <= 0 || d.mib_free >= mib;
}

// Adds `delta` MiB to device i's HBM, or to every member of its pool (mirrored state).
static inline void mib_adjust(Device* devs, int n, int i, int64_t delta) {
  if (devs[i].mib_total <= 0 || delta == 0) return;
  const int16_t p = devs[i].pool;
  if (p < 0) {
    devs[i].mib_free += delta;
    return;
  }
  for (int j = 0; j < n; ++j)
    if (devs[j].pool == p) devs[j].mib_free += delta;
}

// HBM a whole-device grant takes: the device's own HBM, or its share of the pool.
static inline int64_t whole_mib(const Device& d) {
  if (d.mib_total <= 0) return 0;
  return d.pool < 0 ? d.mib_total : d.mib_share;
}

// Pool-deduplicated HBM totals of a node (each pool counted once).
static void hbm_totals(const Device* devs, int n, int64_t* total, int64_t* free_) {
  uint64_t seen = 0;
  *total = *free_ = 0;
  for (int i = 0; i < n; ++i) {
    const Device& d = devs[i];
    if (d.mib_total <= 0) continue;
    if (d.pool >= 0) {
      const uint64_t bit = 1ULL << (d.pool & 63);
      if (seen & bit) continue;
      seen |= bit;
    }
    *total += d.mib_total;
    *free_ += d.mib_free;
  }
}

static inline float link_bw(const Topology* t, int a, int b) {
  if (!t || a < 0 || b < 0 || a >= t->n_gpus || b >= t->n_gpus) return 0.f;
  return t->link_bw[a * kMaxGpus + b];
}

static inline int numa_of(const Topology* t, int g) {
  if (!t || g < 0 || g >= t->n_gpus) return -1;
  return t->numa[g];
}

static void plan_init(Plan* p, int n) {
  std::memset(p, 0, sizeof(*p));
  p->n = n;
}

// ---------------------------------------------------------------------------
// compat: reference Binpack/Spread/SampleRater, Go 1.16 ordering
// ---------------------------------------------------------------------------

namespace {

struct SortDev {
  int32_t free;
  int32_t remain;
  int64_t mib_free;
  int64_t mib_total;
  int32_t index;
  int32_t pool;
};

struct SortDem {
  int32_t pct;
  int32_t index;
  int64_t mib;
};

}  // namespace

static int32_t compat_choose(const Device* devs, int n, const Demand& d, const Options& o,
                             Plan* plan) {
  const int C = d.n;
  SortDem sd[kMaxContainers];
  for (int i = 0; i < C; ++i) sd[i] = SortDem{d.c[i].pct, i, d.c[i].mib};
  // Demand.ToSortableGPUs + sort.Sort: key = Percent + 50*RemainLoad, RemainLoad = 0.
  gosort::sort(
      C, [&](int i, int j) { return sd[i].pct < sd[j].pct; },
      [&](int i, int j) { std::swap(sd[i], sd[j]); });

  if (o.policy == Policy::kFirstFit) {
    // SampleRater.Choose (rater.go:29-50), on a copy (fixes D19: the reference debits live GPUs).
    int32_t free[kMaxDevs];
    int64_t mfree[kMaxDevs];
    for (int i = 0; i < n; ++i) {
      free[i] = devs[i].pct_free;
      mfree[i] = devs[i].mib_free;
    }
    plan_init(plan, C);
    int placed = 0;
    for (int c = 0; c < C; ++c) {
      plan->off[c] = static_cast<int16_t>(c);
      plan->idx[c] = kNotNeedGPU;
      if (d.c[c].pct == 0) {
        ++placed;
        continue;
      }
      for (int j = 0; j < n; ++j) {
        if (free[j] >= d.c[c].pct && (d.c[c].mib <= 0 || devs[j].mib_total <= 0 || mfree[j] >= d.c[c].mib)) {
          plan->idx[c] = static_cast<int16_t>(j);
          free[j] -= d.c[c].pct;
          if (devs[j].mib_total > 0) {
            if (devs[j].pool < 0) {
              mfree[j] -= d.c[c].mib;
            } else {
              for (int k = 0; k < n; ++k)
                if (devs[k].pool == devs[j].pool) mfree[k] -= d.c[c].mib;
            }
          }
          ++placed;
          break;
        }
      }
    }
    plan->off[C] = static_cast<int16_t>(C);
    return placed == C ? kOk : kErrNoFit;
  }

  SortDev sg[kMaxDevs];
  for (int i = 0; i < n; ++i)
    sg[i] = SortDev{devs[i].pct_free, devs[i].remain_load, devs[i].mib_free, devs[i].mib_total, i, devs[i].pool};
  auto sg_mib = [&](int i, int64_t mib) {  // pooled members mirror the pool's free HBM
    if (sg[i].mib_total <= 0) return;
    if (sg[i].pool < 0) {
      sg[i].mib_free -= mib;
      return;
    }
    for (int k = 0; k < n; ++k)
      if (sg[k].pool == sg[i].pool) sg[k].mib_free -= mib;
  };
  auto less = [&](int i, int j) {
    return sg[i].free + sg[i].remain * 50 < sg[j].free + sg[j].remain * 50;  // allocate.go:247
  };
  auto swp = [&](int i, int j) { std::swap(sg[i], sg[j]); };

  int indexes[kMaxContainers];
  int cnt = 0;
  const bool spread = o.policy == Policy::kSpread;
  for (int j = C - 1; j >= 0; --j) {
    if (sd[j].pct == 0) {
      indexes[cnt++] = kNotNeedGPU;
      continue;
    }
    gosort::sort(n, less, swp);
    auto fits = [&](int i) {
      return sg[i].free >= sd[j].pct &&
             (sd[j].mib <= 0 || sg[i].mib_total <= 0 || sg[i].mib_free >= sd[j].mib);
    };
    if (!spread) {
      for (int i = 0; i < n; ++i) {
        if (!fits(i)) continue;
        indexes[cnt++] = sg[i].index;
        sg[i].free -= sd[j].pct;
        sg_mib(i, sd[j].mib);
        break;
      }
    } else {
      for (int i = n - 1; i >= 0; --i) {
        if (!fits(i)) continue;
        indexes[cnt++] = sg[i].index;
        sg[i].free -= sd[j].pct;
        sg_mib(i, sd[j].mib);
        break;
      }
    }
  }
  if (cnt != C) return kErrNoFit;
  plan_init(plan, C);
  int result[kMaxContainers];
  for (int j = C - 1; j >= 0; --j) result[sd[j].index] = indexes[C - 1 - j];
  for (int c = 0; c < C; ++c) {
    plan->off[c] = static_cast<int16_t>(c);
    plan->idx[c] = static_cast<int16_t>(result[c]);
  }
  plan->off[C] = static_cast<int16_t>(C);
  return kOk;
}

static int32_t compat_rate(const Device* devs, int n, const Options& o) {
  if (n == 0) return 0;
  double load = 0.0;
  if (o.load_aware)
    for (int i = 0; i < n; ++i) load += devs[i].load_usage;
  const int load_int = static_cast<int>(load) / n;
  if (o.policy == Policy::kBinpack) {
    int64_t sum = 0, used = 0;
    for (int i = 0; i < n; ++i) {
      sum += devs[i].pct_total;
      used += devs[i].pct_total - devs[i].pct_free;
    }
    const double usage = static_cast<double>(used) / static_cast<double>(sum);
    return static_cast<int32_t>(usage * 100) + load_int * 50 - n;
  }
  if (o.policy == Policy::kSpread) {
    int64_t avail = 0;
    int free_cnt = 0;
    for (int i = 0; i < n; ++i) {
      avail += devs[i].pct_free;
      if (devs[i].pct_free == devs[i].pct_total) ++free_cnt;
    }
    return static_cast<int32_t>(100 * free_cnt + avail / 10 - n - load_int);
  }
  return 100;  // SampleRater: ScoreMax
}

// ---------------------------------------------------------------------------
// native policies
// ---------------------------------------------------------------------------

namespace {

struct Work {
  Device dev[kMaxDevs];
  int n;
  int16_t chosen[kMaxPlanIdx];
  int n_chosen;
};

// Affinity of device `i` to the devices already chosen for this pod.
// Binpack wants siblings (same physical GPU) and high-bandwidth neighbours;
// spread wants distinct GPUs that are still well connected (max of the min link).
float affinity(const Work& w, const Topology* t, int i, bool spread) {
  if (w.n_chosen == 0) return 0.f;
  const int gi = w.dev[i].gpu;
  float sum = 0.f, mn = 1e30f;
  int same = 0, same_numa = 0;
  for (int k = 0; k < w.n_chosen; ++k) {
    const int gk = w.dev[w.chosen[k]].gpu;
    if (gk == gi) {
      ++same;
      continue;
    }
    const float bw = link_bw(t, gi, gk);
    sum += bw;
    mn = std::min(mn, bw);
    if (numa_of(t, gi) >= 0 && numa_of(t, gi) == numa_of(t, gk)) ++same_numa;
  }
  if (mn > 1e29f) mn = 0.f;
  if (spread) return (same ? -1000.f * same : 0.f) + mn + 10.f * same_numa;
  return 1000.f * same + sum + 10.f * same_numa;
}

bool share_fits(const Device& d, const ContainerDemand& c) {
  return d.healthy && d.pct_free >= c.pct && hbm_fits(d, c.mib);
}

int pick_share(Work& w, const Topology* t, const ContainerDemand& c, const Options& o,
               uint64_t rnd) {
  const bool spread = o.policy == Policy::kSpread;
  const bool membound = (c.flags & kFlagMemBound) != 0;
  const bool waste = o.policy == Policy::kBinpack && o.waste_aware();
  int best = -1;
  int64_t bk0 = 0, bkw = 0, bk1 = 0, bk2 = 0;
  float bk3 = 0.f;
  int fit_cnt = 0;
  for (int i = 0; i < w.n; ++i) {
    const Device& d = w.dev[i];
    if (!share_fits(d, c)) continue;
    ++fit_cnt;
    if (o.policy == Policy::kRandom) continue;
    if (o.policy == Policy::kFirstFit) return i;
    // binpack: no dead capacity created first, then best fit
    const int64_t kw = waste ? waste_delta(o, d.pct_free, c.pct) : 0;
    int64_t k1 = d.pct_free - c.pct;
    if (o.load_aware) k1 += 50 * d.remain_load;
    int64_t k2 = d.mib_total > 0 && c.mib > 0 ? (d.mib_free - c.mib) * 1000 / d.mib_total : 0;
    const float k3 = o.topo_weight * affinity(w, t, i, spread);
    if (spread) {
      k1 = -k1;  // worst fit: most free first
      k2 = -k2;
    }
    // fewest memory-bound neighbours first, declared or measured
    const int64_t k0 = membound ? d.mem_bound + (d.mem_hot ? 1 : 0) : 0;
    bool better;
    if (best < 0) better = true;
    else if (k0 != bk0) better = k0 < bk0;
    else if (kw != bkw) better = kw < bkw;
    else if (k1 != bk1) better = k1 < bk1;
    else if (k2 != bk2) better = k2 < bk2;
    else better = k3 > bk3;
    if (better) {
      best = i;
      bk0 = k0;
      bkw = kw;
      bk1 = k1;
      bk2 = k2;
      bk3 = k3;
    }
  }
  if (o.policy == Policy::kRandom && fit_cnt > 0) {
    int target = static_cast<int>(rnd % static_cast<uint64_t>(fit_cnt));
    for (int i = 0; i < w.n; ++i) {
      if (!share_fits(w.dev[i], c)) continue;
      if (target-- == 0) return i;
    }
  }
  return best;
}

bool whole_free(const Device& d) {
  return d.healthy && d.pct_free == d.pct_total && d.pct_total > 0 &&
         (d.mib_total <= 0 || (d.pool < 0 ? d.mib_free == d.mib_total : d.mib_free >= d.mib_share));
}

// Set score for whole-device groups (multi-GPU containers: TP/EP groups, RCCL rings).
// Every pair of MI355X GPUs in a node is one xGMI hop, so hop count does not discriminate;
// the score ranks partition siblings, min link bandwidth, NUMA locality, then policy intent.
float group_score(const Work& w, const Topology* t, const int* set, int k, const Options& o) {
  int siblings = 0, numa_mix = 0;
  float min_bw = 1e30f;
  bool any_pair = false;
  for (int a = 0; a < k; ++a)
    for (int b = a + 1; b < k; ++b) {
      const int ga = w.dev[set[a]].gpu, gb = w.dev[set[b]].gpu;
      if (ga == gb) {
        ++siblings;
        continue;
      }
      any_pair = true;
      min_bw = std::min(min_bw, link_bw(t, ga, gb));
      if (numa_of(t, ga) != numa_of(t, gb)) ++numa_mix;
    }
  if (!any_pair) min_bw = 0.f;
  // Policy intent over the GPUs touched: binpack prefers GPUs already partly used (keeps
  // untouched GPUs whole); spread prefers GPUs with the most free capacity.
  float intent = 0.f;
  for (int a = 0; a < k; ++a) {
    const int g = w.dev[set[a]].gpu;
    int64_t gfree = 0, gtot = 0;
    for (int i = 0; i < w.n; ++i)
      if (w.dev[i].gpu == g) {
        gfree += w.dev[i].pct_free;
        gtot += w.dev[i].pct_total;
      }
    const float frac = gtot > 0 ? static_cast<float>(gfree) / gtot : 0.f;
    intent += o.policy == Policy::kSpread ? frac : (1.f - frac);
  }
  const float sib_w = o.policy == Policy::kSpread ? 20.f : 200.f;
  return o.topo_weight * (sib_w * siblings + min_bw - 50.f * numa_mix) + 100.f * intent;
}

bool pick_group(Work& w, const Topology* t, int k, const Options& o, uint64_t rnd, int* out) {
  int cand[kMaxDevs];
  int m = 0;
  for (int i = 0; i < w.n; ++i)
    if (whole_free(w.dev[i])) cand[m++] = i;
  if (m < k) return false;
  if (o.policy == Policy::kFirstFit) {
    for (int a = 0; a < k; ++a) out[a] = cand[a];
    return true;
  }
  if (o.policy == Policy::kRandom) {
    // partial Fisher-Yates with the pod's deterministic stream
    for (int a = 0; a < k; ++a) {
      rnd = mix64(rnd);
      const int j = a + static_cast<int>(rnd % static_cast<uint64_t>(m - a));
      std::swap(cand[a], cand[j]);
      out[a] = cand[a];
    }
    return true;
  }
  float best = -1e30f;
  int set[kMaxDevs];
  for (int s = 0; s < m; ++s) {
    int sz = 0;
    set[sz++] = cand[s];
    bool used[kMaxDevs] = {false};
    used[s] = true;
    while (sz < k) {
      int bj = -1;
      float bs = -1e30f;
      for (int j = 0; j < m; ++j) {
        if (used[j]) continue;
        set[sz] = cand[j];
        const float sc = group_score(w, t, set, sz + 1, o);
        if (sc > bs) {
          bs = sc;
          bj = j;
        }
      }
      used[bj] = true;
      set[sz++] = cand[bj];
    }
    const float sc = group_score(w, t, set, k, o);
    if (sc > best + 1e-4f) {
      best = sc;
      std::copy(set, set + k, out);
    }
  }
  return true;
}

}  // namespace

// Greedy placement of every container (hardest first) on a working copy of the devices.
// `forced` pins the first container to one device (-1 = free choice). `cost` accumulates
// the policy's per-container keys (binpack: leftover percent; spread: minus free percent)
// so whole-pod alternatives can be compared.
struct Placement {
  int16_t start[kMaxContainers], count[kMaxContainers];
  int16_t idx[kMaxPlanIdx];
  int total = 0;
  int64_t cost = 0, cost_mib = 0;   // cost includes 100 per unit of dead capacity created
};

static int32_t place_all(Work& w, const Topology* topo, const Demand& d, const Options& o, const int* order,
                         int forced, Placement* pl) {
  uint64_t rnd = mix64(o.seed ^ d.hash());
  const bool spread = o.policy == Policy::kSpread;
  for (int q = 0; q < d.n; ++q) {
    const int c = order[q];
    const ContainerDemand& cd = d.c[c];
    const int need = devices_needed(cd);
    rnd = mix64(rnd + static_cast<uint64_t>(q));
    if (need == 0) {
      if (pl->total >= kMaxPlanIdx) return kErrBadDemand;
      pl->start[c] = static_cast<int16_t>(pl->total);
      pl->count[c] = 1;
      pl->idx[pl->total++] = kNotNeedGPU;
      continue;
    }
    if (cd.pct > kPercentPerDevice && cd.pct % kPercentPerDevice != 0) return kErrBadDemand;
    if (pl->total + need > kMaxPlanIdx) return kErrBadDemand;
    pl->start[c] = static_cast<int16_t>(pl->total);
    pl->count[c] = static_cast<int16_t>(need);
    if (need == 1) {
      int i;
      if (q == 0 && forced >= 0) {
        if (!share_fits(w.dev[forced], cd)) return kErrNoFit;
        i = forced;
      } else {
        i = pick_share(w, topo, cd, o, rnd);
      }
      if (i < 0) return kErrNoFit;
      const int64_t left = w.dev[i].pct_free - cd.pct;
      pl->cost += spread ? -w.dev[i].pct_free : left + 100 * std::max(0, waste_delta(o, w.dev[i].pct_free, cd.pct));
      if (w.dev[i].mib_total > 0 && cd.mib > 0)
        pl->cost_mib += (spread ? -1 : 1) * (w.dev[i].mib_free - cd.mib) * 1000 / w.dev[i].mib_total;
      w.dev[i].pct_free -= cd.pct;
      mib_adjust(w.dev, w.n, i, -cd.mib);
      pl->idx[pl->total++] = static_cast<int16_t>(i);
      w.chosen[w.n_chosen++] = static_cast<int16_t>(i);
    } else {
      int set[kMaxDevs];
      if (!pick_group(w, topo, need, o, rnd, set)) return kErrNoFit;
      for (int a = 0; a < need; ++a) {
        Device& dv = w.dev[set[a]];
        dv.pct_free = 0;
        mib_adjust(w.dev, w.n, set[a], -whole_mib(dv));
        pl->idx[pl->total++] = static_cast<int16_t>(set[a]);
        w.chosen[w.n_chosen++] = static_cast<int16_t>(set[a]);
      }
    }
  }
  return kOk;
}

namespace {
// pick_share's ordering key of a device for the first container of a pod (nothing chosen yet,
// so the affinity term is 0), packed so that unsigned order is pick_share's order: mem-bound
// neighbours, waste, leftover percent, leftover HBM share (smaller is better; equal keys go to
// the lower index). kNoKey: a component out of the packed range (not covered).
constexpr uint64_t kNoKey = ~0ull;

uint64_t binpack_key(const Device& d, const ContainerDemand& c, const Options& o) {
  const bool membound = (c.flags & kFlagMemBound) != 0;
  const int64_t k0 = membound ? d.mem_bound + (d.mem_hot ? 1 : 0) : 0;
  const int64_t kw = (o.waste_aware() ? waste_delta(o, d.pct_free, c.pct) : 0) + 32768;
  const int64_t k1 = d.pct_free - c.pct;
  const int64_t k2 = d.mib_total > 0 && c.mib > 0 ? (d.mib_free - c.mib) * 1000 / d.mib_total : 0;
  if (k0 < 0 || k0 > 0xfffe || kw < 0 || kw > 0xffff || k1 < 0 || k1 > 0xffff || k2 < 0 || k2 > 0xffff) return kNoKey;
  return (static_cast<uint64_t>(k0) << 48) | (static_cast<uint64_t>(kw) << 32) | (static_cast<uint64_t>(k1) << 16) |
         static_cast<uint64_t>(k2);
}

bool covered(const Demand& d, const Options& o, int n) {
  return !o.compat && o.policy == Policy::kBinpack && !o.load_aware && d.n == 1 && n > 0 && n <= kMaxDevs &&
         d.c[0].pct > 0 && d.c[0].pct <= kPercentPerDevice;
}
}  // namespace

uint64_t plan_touch_mask(const Device* devs, int n, const Plan& p) {
  uint64_t m = 0;
  const int total = p.n > 0 ? p.off[p.n] : 0;
  for (int a = 0; a < total && a < kMaxPlanIdx; ++a) {
    const int i = p.idx[a];
    if (i < 0 || i >= n) continue;
    m |= 1ull << i;
    if (devs[i].pool >= 0)
      for (int k = 0; k < n; ++k)
        if (devs[k].pool == devs[i].pool) m |= 1ull << k;
  }
  return m;
}

namespace {
// (key, index) pairs: pick_share's choice is the least pair among the devices that fit
inline bool pair_less(uint64_t ka, int ia, uint64_t kb, int ib) { return ka < kb || (ka == kb && ia < ib); }
}  // namespace

bool share_fast_path(const Demand& d, const Options& o, int n) { return covered(d, o, n); }

int32_t scan_share(const Device* devs, int n, const Demand& d, const Options& o, Plan* plan, ShareMemo* next) {
  // pick_share for the first container, every device compared: the least (key, index) pair of
  // the devices that fit (what choose() places on), and the runner-up for re-validation
  if (!covered(d, o, n)) return kRevalidateNo;
  const ContainerDemand& c = d.c[0];
  uint64_t k1 = kNoKey, k2 = kNoKey;
  int i1 = kMaxDevs, i2 = kMaxDevs;
  for (int j = 0; j < n; ++j) {
    if (!share_fits(devs[j], c)) continue;
    const uint64_t k = binpack_key(devs[j], c, o);
    if (k == kNoKey) return kRevalidateNo;
    if (pair_less(k, j, k1, i1)) {
      k2 = k1;
      i2 = i1;
      k1 = k;
      i1 = j;
    } else if (pair_less(k, j, k2, i2)) {
      k2 = k;
      i2 = j;
    }
  }
  next->runner_key = k2;
  next->runner_idx = i2;
  next->runner_exact = i2 != kMaxDevs;
  if (i1 == kMaxDevs) {
    next->rc = kErrNoFit;
    next->dev = -1;
    next->score = 0;
    return kErrNoFit;
  }
  plan_init(plan, 1);
  plan->off[0] = 0;
  plan->idx[0] = static_cast<int16_t>(i1);
  plan->off[1] = 1;
  plan->score = rate(devs, n, d, o, plan);
  next->rc = kOk;
  next->dev = i1;
  next->score = plan->score;
  return kOk;
}

int32_t revalidate(const Device* devs, int n, const Demand& d, const Options& o, const ShareMemo& prev,
                   uint64_t changed, Plan* plan, ShareMemo* next) {
  // covered: native binpack, no load term, one container asking a share of one device. Its
  // device is pick_share's least (key, index) pair over the devices that fit, each device's key
  // read from that device alone, and its score (binpack_penalty, crowding) reads the chosen
  // device alone. A device that did not change kept its pair (or still does not fit), so:
  //   * prev.dev and the changed devices are compared exactly;
  //   * so is the runner-up device when its pair is exact (it was that device's pair when the
  //     memo was made, and the device has not changed since);
  //   * every other device is bounded below by the runner-up pair (a device that did not fit
  //     then still does not).
  // The least exact pair wins when it is below that bound (or is the runner-up itself); else an
  // unchanged device might: kRevalidateNo.
  if (!covered(d, o, n)) return kRevalidateNo;
  if (prev.rc != kOk && prev.rc != kErrNoFit) return kRevalidateNo;
  const ContainerDemand& c = d.c[0];
  const bool have_runner = prev.rc == kOk && prev.runner_idx != kMaxDevs;
  const bool runner_exact = have_runner && prev.runner_exact && !((changed >> prev.runner_idx) & 1u);
  uint64_t k1 = kNoKey, k2 = kNoKey;   // least and second least exact pairs
  int i1 = kMaxDevs, i2 = kMaxDevs;
  for (int j = 0; j < n; ++j) {
    const bool exact = ((changed >> j) & 1u) || (prev.rc == kOk && j == prev.dev) || (runner_exact && j == prev.runner_idx);
    if (!exact || !share_fits(devs[j], c)) continue;
    const uint64_t k = binpack_key(devs[j], c, o);
    if (k == kNoKey) return kRevalidateNo;
    if (pair_less(k, j, k1, i1)) {
      k2 = k1;
      i2 = i1;
      k1 = k;
      i1 = j;
    } else if (pair_less(k, j, k2, i2)) {
      k2 = k;
      i2 = j;
    }
  }
  // The devices not compared exactly: none fits (no runner-up), or every one is above the
  // runner-up pair when that is an exact device's (compared above, so the least exact pair is at
  // or below it), else at or above the bound, so the least exact pair must be below it.
  if (have_runner && !runner_exact && (i1 == kMaxDevs || !pair_less(k1, i1, prev.runner_key, prev.runner_idx)))
    return kRevalidateNo;
  if (i1 == kMaxDevs) {
    next->rc = kErrNoFit;
    next->dev = -1;
    next->score = 0;
    next->runner_key = kNoKey;
    next->runner_idx = kMaxDevs;
    next->runner_exact = false;
    return kErrNoFit;
  }
  // the new runner-up: the second exact pair when it is below the old bound (exact), else the
  // old bound, which still bounds the devices it covered (exact only while its device is not the
  // new choice)
  if (!have_runner || (i2 != kMaxDevs && pair_less(k2, i2, prev.runner_key, prev.runner_idx))) {
    next->runner_key = k2;
    next->runner_idx = i2;
    next->runner_exact = i2 != kMaxDevs;
  } else {
    next->runner_key = prev.runner_key;
    next->runner_idx = prev.runner_idx;
    next->runner_exact = runner_exact && i1 != prev.runner_idx;
  }
  plan_init(plan, 1);
  plan->off[0] = 0;
  plan->idx[0] = static_cast<int16_t>(i1);
  plan->off[1] = 1;
  // the score reads the chosen device: unchanged, or computed as choose() does
  plan->score = prev.rc == kOk && i1 == prev.dev && !((changed >> i1) & 1u) ? prev.score : rate(devs, n, d, o, plan);
  next->rc = kOk;
  next->dev = i1;
  next->score = plan->score;
  return kOk;
}

static int32_t native_choose(const Device* devs, int n, const Topology* topo, const Demand& d,
                             const Options& o, Plan* plan) {
  Work w0;
  w0.n = n;
  w0.n_chosen = 0;
  std::memcpy(w0.dev, devs, sizeof(Device) * n);

  // Hardest first: whole-device groups, then larger shares, then HBM; stable on index.
  int order[kMaxContainers];
  for (int i = 0; i < d.n; ++i) order[i] = i;
  std::stable_sort(order, order + d.n, [&](int a, int b) {
    const int na = devices_needed(d.c[a]), nb = devices_needed(d.c[b]);
    if ((na > 1) != (nb > 1)) return na > nb;
    if (d.c[a].pct != d.c[b].pct) return d.c[a].pct > d.c[b].pct;
    return d.c[a].mib > d.c[b].mib;
  });

  // A pod whose containers land on several devices (TP/EP ranks, RCCL peers) is placed as
  // a whole: every feasible device for its hardest single-device container is tried, the
  // rest placed greedily, and the complete placements are ranked by the policy's summed
  // keys, then by the set's topology score (partition siblings, min xGMI bandwidth, NUMA
  // span). A greedy first pick alone would settle ties by device index and could split a
  // group across sockets or over a degraded link.
  int gpu_containers = 0;
  for (int i = 0; i < d.n; ++i) gpu_containers += devices_needed(d.c[i]) > 0;
  const bool joint = gpu_containers >= 2 && d.n > 0 && devices_needed(d.c[order[0]]) == 1 &&
                     (o.policy == Policy::kBinpack || o.policy == Policy::kSpread) && o.topo_weight > 0.f;
  Placement best;
  int32_t best_rc = kErrNoFit;
  if (!joint) {
    Work w = w0;
    best_rc = place_all(w, topo, d, o, order, -1, &best);
  } else {
    float best_topo = -1e30f;
    for (int f = 0; f < n; ++f) {
      if (!share_fits(w0.dev[f], d.c[order[0]])) continue;
      Work w = w0;
      Placement pl;
      if (place_all(w, topo, d, o, order, f, &pl) != kOk) continue;
      int set[kMaxPlanIdx];
      int k = 0;
      for (int a = 0; a < pl.total; ++a)
        if (pl.idx[a] >= 0) set[k++] = pl.idx[a];
      const float ts = group_score(w0, topo, set, k, o);
      const bool better = best_rc != kOk || pl.cost < best.cost ||
                          (pl.cost == best.cost && (pl.cost_mib < best.cost_mib ||
                                                    (pl.cost_mib == best.cost_mib && ts > best_topo + 1e-4f)));
      if (better) {
        best = pl;
        best_topo = ts;
        best_rc = kOk;
      }
    }
  }
  if (best_rc != kOk) return best_rc;
  plan_init(plan, d.n);
  int pos = 0;
  for (int c = 0; c < d.n; ++c) {
    plan->off[c] = static_cast<int16_t>(pos);
    for (int a = 0; a < best.count[c]; ++a) plan->idx[pos++] = best.idx[best.start[c] + a];
  }
  plan->off[d.n] = static_cast<int16_t>(pos);
  return kOk;
}

// Binpack node penalty (0 = perfect, 100 = worst) of `plan` on `devs`, averaged over the
// pod's containers: a share scores the percent it leaves free on its device, plus 40 if it
// turns fillable capacity into dead capacity (see Options::waste); a whole-device container
// scores the fraction of the node's devices still whole after the placement (a node it
// fills up is the tight fit, an idle node the loose one). `after` is the node post-plan.
static double binpack_penalty(const Device* devs, int n, const Demand& d, const Options& o, const Plan& plan,
                              const Device* after) {
  Device cur[kMaxDevs];
  std::memcpy(cur, devs, sizeof(Device) * n);
  double pen = 0.0;
  int parts = 0, whole = 0;
  for (int c = 0; c < plan.n && c < d.n; ++c) {
    const ContainerDemand& cd = d.c[c];
    for (int k = plan.off[c]; k < plan.off[c + 1]; ++k) {
      const int i = plan.idx[k];
      if (i < 0 || i >= n) continue;
      if (cd.pct > kPercentPerDevice) {
        ++whole;
        continue;
      }
      if (cd.pct <= 0) continue;
      const int32_t left = cur[i].pct_free - cd.pct;
      pen += std::max(0, left) + (waste_delta(o, cur[i].pct_free, cd.pct) > 0 ? 40.0 : 0.0);
      cur[i].pct_free = left;
      ++parts;
    }
  }
  if (whole) {
    int still_whole = 0, healthy = 0;
    for (int i = 0; i < n; ++i) {
      if (!after[i].healthy) continue;
      ++healthy;
      still_whole += after[i].pct_free == after[i].pct_total;
    }
    pen += whole * (healthy ? 100.0 * still_whole / healthy : 0.0);
  }
  const int m = parts + whole;
  return m ? std::min(100.0, pen / m) : 0.0;
}

static int32_t native_rate(const Device* devs, int n, const Demand& d, const Options& o,
                           const Plan* plan) {
  if (n == 0) return 0;
  Device after[kMaxDevs];
  std::memcpy(after, devs, sizeof(Device) * n);
  if (plan) apply(after, n, d, *plan);
  int64_t pct_tot = 0, pct_used = 0, mib_tot = 0, mib_used = 0;
  int full_free = 0;
  float load = 0.f;
  for (int i = 0; i < n; ++i) {
    pct_tot += after[i].pct_total;
    pct_used += after[i].pct_total - after[i].pct_free;
    if (after[i].pct_free == after[i].pct_total) ++full_free;
    load += devs[i].load_usage;
  }
  {
    int64_t mfree = 0;
    hbm_totals(after, n, &mib_tot, &mfree);
    mib_used = mib_tot - mfree;
  }
  double util = pct_tot > 0 ? static_cast<double>(pct_used) / pct_tot : 0.0;
  if (mib_tot > 0) util = 0.5 * util + 0.5 * static_cast<double>(mib_used) / mib_tot;
  const double avg_load = o.load_aware ? load / (kLoadTotal * n) : 0.0;  // 0..1
  double s;
  switch (o.policy) {
    case Policy::kBinpack:
      // Fit quality of the plan, not node utilisation: kube-scheduler takes the arg-max over
      // nodes, so this makes binpack a cluster-wide best fit. Frag% counts free capacity on
      // partly used devices, which a tight fit anywhere in the cluster keeps low and filling
      // the busiest node does not (a busy node's last holes rarely fit the next request).
      // Ties stay ties (kube-scheduler picks one at random): breaking them toward the busier
      // node measured worse on frag% (tools/fragsim.py: 0.45 vs 0.34 on the bench burst).
      s = plan ? 100.0 - binpack_penalty(devs, n, d, o, *plan, after) : 100.0 * util;
      if (o.load_aware) s = 0.8 * s + 20.0 * avg_load;  // reference binpack rewards load (rater.go:69)
      break;
    case Policy::kSpread:
      s = 50.0 * (1.0 - util) + 50.0 * static_cast<double>(full_free) / n;
      if (o.load_aware) s = 0.8 * s + 20.0 * (1.0 - avg_load);
      break;
    case Policy::kRandom:
      s = static_cast<double>(mix64(o.seed ^ d.hash() ^ static_cast<uint64_t>(pct_used) ^
                                    (static_cast<uint64_t>(n) << 32)) %
                              101);
      break;
    default:
      s = 100.0;
  }
  if (plan && o.policy != Policy::kRandom) {
    // a memory-bound share that would sit next to another memory-bound tenant costs this node
    // points, so priorities prefer a node where it can pair with compute-bound neighbours
    int crowded = 0;
    for (int c = 0; c < plan->n && c < d.n; ++c) {
      if (!(d.c[c].flags & kFlagMemBound) || d.c[c].pct > kPercentPerDevice) continue;
      for (int k = plan->off[c]; k < plan->off[c + 1]; ++k)
        if (plan->idx[k] >= 0 && (devs[plan->idx[k]].mem_bound > 0 || devs[plan->idx[k]].mem_hot))
          ++crowded;
    }
    s -= 15.0 * crowded;
  }
  return static_cast<int32_t>(std::clamp(s, 0.0, 100.0));
}

int32_t choose(const Device* devs, int n, const Topology* topo, const Demand& d,
               const Options& o, Plan* plan) {
  if (d.n < 0 || d.n > kMaxContainers) return kErrBadDemand;
  if (n <= 0) return kErrNoDevices;
  if (n > kMaxDevs) return kErrBadPlan;
  int32_t rc;
  if (o.compat && o.policy != Policy::kRandom) {
    rc = compat_choose(devs, n, d, o, plan);
  } else {
    rc = native_choose(devs, n, topo, d, o, plan);
  }
  if (rc != kOk) return rc;
  plan->score = rate(devs, n, d, o, plan);
  return kOk;
}

int32_t rate(const Device* devs, int n, const Demand& d, const Options& o, const Plan* plan) {
  if (o.compat && o.policy != Policy::kRandom) return compat_rate(devs, n, o);
  return native_rate(devs, n, d, o, plan);
}

static bool plan_shape_ok(int n, const Demand& d, const Plan& p) {
  if (p.n != d.n || p.n < 0 || p.n > kMaxContainers) return false;
  if (p.off[0] != 0 || p.off[p.n] > kMaxPlanIdx) return false;
  for (int c = 0; c < p.n; ++c) {
    if (p.off[c + 1] < p.off[c]) return false;
    for (int k = p.off[c]; k < p.off[c + 1]; ++k)
      if (p.idx[k] >= n || p.idx[k] < kNotNeedGPU) return false;
  }
  return true;
}

// Whole-device entries (pct > 100) debit the full device (and its HBM, or its share of
// the HBM pool); share entries debit (pct, mib).
static inline void debit(Device* devs, int n, int i, const ContainerDemand& cd, int sign) {
  Device& dv = devs[i];
  if (cd.pct > kPercentPerDevice) {
    dv.pct_free = sign < 0 ? 0 : dv.pct_total;
    mib_adjust(devs, n, i, sign * whole_mib(dv));
    return;
  }
  dv.pct_free += sign * cd.pct;
  mib_adjust(devs, n, i, sign * cd.mib);
  if (cd.flags & kFlagMemBound) dv.mem_bound = static_cast<int16_t>(std::max(0, dv.mem_bound - sign));
}

static inline bool can_debit(const Device& dv, const ContainerDemand& cd) {
  if (cd.pct > kPercentPerDevice)
    return dv.pct_free == dv.pct_total && (dv.mib_total <= 0 || dv.mib_free >= whole_mib(dv));
  return dv.pct_free >= cd.pct && hbm_fits(dv, cd.mib);
}

int32_t apply(Device* devs, int n, const Demand& d, const Plan& p) {
  if (!plan_shape_ok(n, d, p)) return kErrBadPlan;
  for (int c = 0; c < p.n; ++c) {
    for (int k = p.off[c]; k < p.off[c + 1]; ++k) {
      const int i = p.idx[k];
      if (i < 0) continue;
      if (!can_debit(devs[i], d.c[c])) {
        // roll back exactly what this call debited
        for (int c2 = 0; c2 <= c; ++c2) {
          const int end = c2 == c ? k : p.off[c2 + 1];
          for (int k2 = p.off[c2]; k2 < end; ++k2)
            if (p.idx[k2] >= 0) debit(devs, n, p.idx[k2], d.c[c2], +1);
        }
        return kErrPlanNoLongerFits;
      }
      debit(devs, n, i, d.c[c], -1);
    }
  }
  return kOk;
}

int32_t unapply(Device* devs, int n, const Demand& d, const Plan& p) {
  if (!plan_shape_ok(n, d, p)) return kErrBadPlan;
  for (int c = 0; c < p.n; ++c)
    for (int k = p.off[c]; k < p.off[c + 1]; ++k) {
      const int i = p.idx[k];
      if (i < 0) continue;
      debit(devs, n, i, d.c[c], +1);
      devs[i].pct_free = std::min(devs[i].pct_free, devs[i].pct_total);
    }
  for (int i = 0; i < n; ++i)
    if (devs[i].mib_total > 0) devs[i].mib_free = std::min(devs[i].mib_free, devs[i].mib_total);
  return kOk;
}

void frag_accumulate(const Device* devs, int n, int32_t min_request, FragStats* s) {
  uint64_t pool_seen = 0, pool_partial = 0;
  for (int i = 0; i < n; ++i) {
    const Device& d = devs[i];
    if (!d.healthy) continue;
    ++s->devices;
    s->pct_free_total += d.pct_free;
    const bool partial = d.pct_free > 0 && d.pct_free < d.pct_total;
    if (d.mib_total > 0) {
      if (d.pool < 0) {
        s->mib_free_total += d.mib_free;
        if (partial) s->mib_free_partial += d.mib_free;
      } else {  // a pool counts once; its free HBM is "partial" if any member is partly used
        const uint64_t bit = 1ULL << (d.pool & 63);
        if (!(pool_seen & bit)) {
          pool_seen |= bit;
          s->mib_free_total += d.mib_free;
        }
        if (partial && !(pool_partial & bit)) {
          pool_partial |= bit;
          s->mib_free_partial += d.mib_free;
        }
      }
    }
    const bool full = d.pct_free == d.pct_total;
    if (full) ++s->devices_full_free;
    if (d.pct_free < d.pct_total) ++s->devices_used;
    if (partial) s->pct_free_partial += d.pct_free;
    if (d.pct_free > 0 && d.pct_free < min_request) s->pct_stranded += d.pct_free;
  }
}

std::string plan_to_string(const Plan& p) {
  std::ostringstream os;
  os << "[";
  for (int c = 0; c < p.n; ++c) {
    if (c) os << " ";
    for (int k = p.off[c]; k < p.off[c + 1]; ++k) {
      if (k > p.off[c]) os << ",";
      os << p.idx[k];
    }
  }
  os << "]";
  return os.str();
}

}  // namespace nanogpu
