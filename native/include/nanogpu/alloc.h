// Allocation algebra for fine-grained AMD Instinct scheduling.
//
// Reference parity map (reference = alex337/nano-gpu-scheduler):
//   Device            ~ GPUResource{Percent, PercentTotal, RemainLoad}  pkg/dealer/allocate.go:141-161
//   Demand            ~ Demand ([]GPUResource, one per container)      pkg/dealer/allocate.go:52-62
//   Plan              ~ Plan{Demand, GPUIndexes, Score}                 pkg/dealer/allocate.go:23-27
//   choose()/rate()   ~ Rater.Choose / Rater.Rate                       pkg/dealer/rater.go:16-163
//   apply()/unapply() ~ GPUs.Allocate / GPUs.Release                    pkg/dealer/allocate.go:102-131
//
// MI355X-first extensions (not in the reference):
//   * a second resource dimension, HBM MiB (288 GB per MI355X; read, never assumed);
//   * schedulable devices may be compute partitions (SPX/DPX/QPX/CPX) that record
//     their parent physical GPU, NUMA node, XCD and CU counts;
//   * containers may request whole devices (gpu-percent 200, 300, ... => k devices),
//     chosen as a set by an xGMI-link / partition-sibling / NUMA topology score;
//   * native policies (best-fit binpack, worst-fit spread, random, first-fit) that
//     are deterministic and HBM-aware, next to a bit-exact `compat` (Go 1.16) mode.
#pragma once

#include <cstdint>
#include <string>

namespace nanogpu {

constexpr int kMaxDevs = 64;         // 8 GPUs x CPX (8 XCD partitions each)
constexpr int kMaxGpus = 16;         // physical GPUs per node
// containers per pod: every GPU-requesting container takes at least one plan index, so a pod
// never needs more than kMaxPlanIdx (a ledger pod slot holds 16 inline, larger pods spill into
// the ledger's overflow records)
constexpr int kMaxContainers = 64;
constexpr int kMaxPlanIdx = 64;      // device indices per pod plan
constexpr int kNotNeedGPU = -1;      // reference NotNeedGPU, allocate.go:15
constexpr int kLoadTotal = 2;        // reference LoadTotal, allocate.go:16
constexpr int kPercentPerDevice = 100;
constexpr int kWasteSlots = kPercentPerDevice + 1;
constexpr int32_t kRevalidateNoMemo = -2;   // ShareMemo::rc of a memo entry that cannot be re-validated

enum class Policy : int32_t { kBinpack = 0, kSpread = 1, kRandom = 2, kFirstFit = 3 };

enum Err : int32_t {
  kOk = 0,
  kErrNoFit = 1,         // demand cannot be placed on this node
  kErrNoDevices = 2,     // node advertises no devices (reference divides by zero: rater.go:68)
  kErrBadPlan = 3,       // plan indices out of range / shape mismatch
  kErrPlanNoLongerFits = 4,
  kErrUnknownNode = 5,
  kErrUnknownPod = 6,
  kErrPodExists = 7,     // pod already allocated on a different node
  kErrTableFull = 8,
  kErrBadDemand = 9,
  kOkExisting = 10,      // not an error: the pod was already reserved/committed on that node
};

const char* err_str(int32_t e);

struct Device {
  int32_t pct_free;
  int32_t pct_total;
  int64_t mib_free;
  int64_t mib_total;    // 0 => HBM not tracked on this device
  float load_usage;     // sum over fresh metrics of ceil(10u)/10 (reference allocate.go:173-195)
  int16_t remain_load;  // reference RemainLoad = LoadTotal - int(load_usage)
  int16_t gpu;          // physical GPU index within the node
  int16_t part;         // partition index within the physical GPU (0 in SPX)
  int16_t numa;         // NUMA node of the GPU, -1 unknown
  int16_t healthy;      // 0 => never chosen
  int16_t xcds;         // XCDs backing this device (8 for an SPX MI355X, 1 in CPX)
  int32_t cus;          // compute units backing this device (256 for SPX MI355X)
  // HBM pool: compute partitions that share one memory partition (CPX/QPX/DPX under
  // NPS1, CPX under NPS2) draw from one pool. Every member mirrors the pool's
  // mib_free/mib_total and every debit updates all members. -1: the device's own HBM.
  int16_t pool;
  int16_t mem_bound;    // memory-bound share containers placed here (see kFlagMemBound)
  int16_t mem_hot;      // measured: the device's HBM activity is above the policy threshold
                        // (telemetry, Ledger::set_mem_hot), whatever its tenants declared
  int16_t mem_busy;     // the averaged HBM activity itself, percent (Ledger::set_mem_busy): the
                        // streaming-owner learner compares it with a threshold per tenant share
  int64_t mib_share;    // HBM a whole-device grant of a pooled member takes (pool / members)
};

struct Topology {
  int32_t n_gpus;
  int16_t numa[kMaxGpus];
  float link_bw[kMaxGpus * kMaxGpus];  // GB/s between physical GPUs, 0 = no direct link
};

// Container flags. kFlagMemBound: the container streams HBM (pod annotation
// nano-gpu/memory-bound). CU masks split the compute units but not the memory system: on
// the MI355X box two streaming tenants with 25 % / 75 % masks split the HBM bandwidth
// 25 / 75, while a 25 % tenant alone reaches 51 % of it (profiles/gpu_calibration.md). So
// native policies place a memory-bound share on the device with the fewest memory-bound
// tenants first, next to compute-bound neighbours, before the policy's own order. A device
// whose measured HBM activity is high (Device::mem_hot) counts as holding one more streaming
// tenant, so undeclared streaming workloads are seen too.
constexpr int32_t kFlagMemBound = 1;

struct ContainerDemand {
  int32_t pct;    // 0 => no GPU; <=100 => share of one device; k*100 => k whole devices
  int32_t flags;  // kFlag* bits
  int64_t mib;    // HBM MiB requested (per device for whole-device requests it is ignored)
};

struct Demand {
  int32_t n;
  int32_t pad;
  ContainerDemand c[kMaxContainers];
  uint64_t hash() const;
};

struct Plan {
  int32_t n;                          // containers
  int32_t score;
  int16_t off[kMaxContainers + 1];    // container c uses idx[off[c] .. off[c+1])
  int16_t idx[kMaxPlanIdx];           // device indices; a single -1 for "no GPU"
};

// Request-size model of native binpack. A hole of h percent left on a device is only as
// useful as the share requests that can still fill it: with {10, 25, 50} % requests a 5 %
// hole is dead and a 15 % hole ends as 5 % whatever arrives. waste[h] = h minus the largest
// sum of common request sizes that fits in h (unbounded knapsack over `sizes`), so binpack
// avoids placements that turn a fillable hole into a dead one (a 10 % share into a 25 % hole,
// where the 25 % hole would have paired with the next 25 % request). `sizes` is a 101-bit set
// (bit s: s % requests are common); the ledger learns it from the requests it sees
// (Ledger::note_request) unless fixed by the operator (--request-sizes).
struct SizeSet {
  uint64_t bits[2] = {0, 0};
  bool empty() const { return (bits[0] | bits[1]) == 0; }
  bool has(int s) const { return s >= 0 && s < 128 && ((bits[s >> 6] >> (s & 63)) & 1u); }
  void add(int s) {
    if (s > 0 && s <= kPercentPerDevice) bits[s >> 6] |= 1ULL << (s & 63);
  }
  bool operator==(const SizeSet& o) const { return bits[0] == o.bits[0] && bits[1] == o.bits[1]; }
};

struct Options {
  Policy policy = Policy::kBinpack;
  int32_t compat = 0;        // 1 => reproduce the reference (Go 1.16) bit for bit
  int32_t load_aware = 0;    // reference --isLoadSchedule
  float topo_weight = 1.0f;  // weight of the xGMI/partition term in native mode
  uint64_t seed = 0;         // random policy seed (mixed with the demand hash)
  int32_t learn_sizes = 1;   // native binpack: add the ledger's learned request sizes
  int32_t pad = 0;
  SizeSet sizes;             // request sizes in force (fixed ones, plus learned ones)
  uint8_t waste[kWasteSlots] = {};   // derived from `sizes` by set_sizes()
  void set_sizes(const SizeSet& s);
  bool waste_aware() const { return !sizes.empty(); }
  uint64_t hash() const;
};

// Devices needed by one container (0 for "no GPU").
int devices_needed(const ContainerDemand& c);

// Computes a placement for `d` on `devs` (not modified). Returns kOk and fills `plan`
// (including plan->score from rate()), or an error code.
int32_t choose(const Device* devs, int n, const Topology* topo, const Demand& d,
               const Options& o, Plan* plan);

// Node score for `d` on the pre-placement state (reference semantics: rater.go:59-70,
// 113-123 in compat mode; 0..100 utilisation/fragmentation score in native mode).
int32_t rate(const Device* devs, int n, const Demand& d, const Options& o, const Plan* plan);

// Devices a plan's debit changes: its device indices and, for pooled HBM, every member of
// their pools (a debit mirrors the pool's free MiB onto each member).
uint64_t plan_touch_mask(const Device* devs, int n, const Plan& p);

// Single-share fast path and re-validation of a memoised placement (Ledger::assume_many). A
// placement decided device by device (native binpack, one container asking a share of one
// device, no load awareness: share_fast_path) is pick_share's least (key, index) pair over the
// devices that fit, each key read from that device alone. scan_share computes it over every
// device, as choose() would (same device, same score), and keeps the runner-up pair;
// revalidate answers a node that changed from its memo (ShareMemo), the devices that changed
// (`changed`: bit i = device i) and the runner-up bound alone, or says kRevalidateNo when an
// unchanged device could now be the best.
struct ShareMemo {
  int32_t rc = kRevalidateNoMemo;   // kOk / kErrNoFit for a memo that can be re-validated
  int32_t dev = -1;                 // the chosen device (kOk)
  int32_t score = 0;
  int32_t runner_idx = kMaxDevs;    // kMaxDevs: no other device fitted
  uint64_t runner_key = ~0ull;      // every other fitting device's pair is at or above this one
  bool runner_exact = false;        // ... which is device runner_idx's own pair
};
constexpr int32_t kRevalidateNo = -1;
bool share_fast_path(const Demand& d, const Options& o, int n);
// kOk (*plan with its score) or kErrNoFit, *next set; kRevalidateNo when not covered
int32_t scan_share(const Device* devs, int n, const Demand& d, const Options& o, Plan* plan, ShareMemo* next);
int32_t revalidate(const Device* devs, int n, const Demand& d, const Options& o, const ShareMemo& prev,
                   uint64_t changed, Plan* plan, ShareMemo* next);

// Debits the plan; on any misfit restores what was taken and returns an error.
// (Fixes reference allocate.go:108-113, which restores Demand[i] instead of Demand[j].)
int32_t apply(Device* devs, int n, const Demand& d, const Plan& p);
int32_t unapply(Device* devs, int n, const Demand& d, const Plan& p);

struct FragStats {
  int64_t pct_free_total;
  int64_t pct_free_partial;   // free percent on partially used devices
  int64_t mib_free_total;
  int64_t mib_free_partial;
  int64_t pct_stranded;       // free percent on devices whose free < min_request
  int32_t devices;
  int32_t devices_full_free;
  int32_t devices_used;
};
void frag_accumulate(const Device* devs, int n, int32_t min_request, FragStats* s);

std::string plan_to_string(const Plan& p);

}  // namespace nanogpu
