// Cluster GPU ledger: the state cache of the scheduler, native and shareable.
//
// Reference: DealerImpl (pkg/dealer/dealer.go:76-87) keeps NodeMaps / PodMaps /
// ReleasedPodMap behind ONE sync.Mutex that is held across filter fan-out, scoring and
// the API-server writes of bind (dealer.go:90-91, 139-140, 156-203).  Here:
//   * the state lives in one flat region (heap, or a /dev/shm file shared by several
//     extender worker processes: SO_REUSEPORT replicas on one host see one ledger);
//   * every node has its own robust, process-shared mutex and a generation counter;
//     filter/score copy a node snapshot (3 KB) under the lock and compute outside it;
//   * bind = reserve (allocate + record pod, microseconds under the node lock), the
//     API-server I/O happens with no lock held, then commit or rollback;
//   * pods live in a sharded open-addressing table (64 shards, one mutex each).
// Lock order is always node -> pod shard.
#pragma once

#include <pthread.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <memory>
#include <unordered_map>
#include <vector>

#include "nanogpu/alloc.h"

namespace nanogpu {

constexpr int kNameLen = 256;
constexpr int kKeyLen = 64;
constexpr int kPodShards = 64;
// learned streaming owners (Ledger::set_stream_owner): direct-mapped, a collision forgets the
// older owner (it falls back to its pods' own annotation)
constexpr int kStreamOwners = 4096;

// Hash of an owner's UID (ownerReferences[controller].uid), never 0.
uint64_t owner_hash(std::string_view uid);

// Nominated: taken tentatively at priorities for the top-scored node (see nominate()).
enum PodState : int32_t { kPodEmpty = 0, kPodReserved = 1, kPodCommitted = 2, kPodTombstone = 3, kPodNominated = 4 };

// Cache-line layout: a filter reads, per node, the name and in_use (verifying its id cache)
// and the generation (its plan-cache key) without locking. Those live apart from the mutex,
// whose line every lock/unlock by any worker process dirties, so lock traffic on a node does
// not turn the filters of the other workers into cross-CCD misses; the generation has a
// line of its own as it changes on every mutation.
// The devices each of a node's last kChangeRing generation bumps touched (Ledger::bump): a
// placement memoised at an older generation is re-validated against the devices that changed
// since (Ledger::assume_many) instead of being recomputed from scratch.
constexpr int kChangeRing = 64;

struct NodeSlot {
  char name[kNameLen];                              // written at registration only
  int32_t in_use;
  int32_t n_devs;
  alignas(64) pthread_mutex_t mu;
  int32_t n_pods;                                   // under mu
  // entry g % kChangeRing: the bump from generation g to g + 1 (tag chg_gen = g) changed the
  // devices in chg_mask (bit i: device i; every bit: the node as a whole). Written under mu.
  alignas(64) std::atomic<uint64_t> chg_gen[kChangeRing];
  std::atomic<uint64_t> chg_mask[kChangeRing];
  alignas(64) Topology topo;
  Device devs[kMaxDevs];
};

// What a filter reads of every node it is sent: its generation (the plan cache's key) and
// whether the slot is live. One dense array (16 bytes a node) instead of a line inside each
// 20 KB node slot: a request over 420 nodes reads 105 consecutive cache lines, which the
// hardware prefetches, instead of 420 scattered ones. A bind's write shares its line with three
// other nodes' entries, a small cost against the reads (hundreds per bind).
struct NodeHot {
  std::atomic<uint64_t> gen;      // bumps on every change to the node (under its mutex)
  std::atomic<int32_t> in_use;
  int32_t pad;
};

struct alignas(64) PaddedMutex {   // one line per pod-shard lock (no false sharing)
  pthread_mutex_t m;
};

// A pod slot keeps up to kSlotContainers containers inline (the common case, and what keeps
// the table small: it is scanned by the sweepers); a pod with more spills its demand and plan
// into an overflow record (Ledger::put_record). Every pod is read through get_record.
constexpr int kSlotContainers = 16;

struct SlotDemand {
  int32_t n;
  int32_t pad;
  ContainerDemand c[kSlotContainers];
};

struct SlotPlan {
  int32_t n;
  int32_t score;
  int16_t off[kSlotContainers + 1];
  int16_t idx[kMaxPlanIdx];
};

struct PodSlot {
  uint64_t hash;
  char key[kKeyLen];
  int32_t node;
  int32_t state;
  double t_reserved;   // CLOCK_MONOTONIC seconds at reservation
  SlotDemand demand;   // inline record (ext == 0)
  SlotPlan plan;
  uint64_t owner;      // owner_hash of the pod's controlling owner (set_pod_owner), 0: unknown
  int32_t ext;         // 0: inline; k > 0: overflow record k - 1
  int32_t wide;        // 0: none; k > 0: wide record k - 1 (a wide pod's per-container plan)
};

// Overflow record of a pod with more than kSlotContainers containers (shared region, claimed
// with a CAS on `used`, owned by exactly one pod slot).
struct ExtRecord {
  std::atomic<int32_t> used;
  int32_t pad;
  Demand demand;
  Plan plan;
};

// A wide pod (more GPU containers than a Demand holds, pu.is_wide) is accounted as one record
// folded per device; its per-container plan, what its bind answers and its annotations carry,
// lives beside it in a wide record (shared region, claimed with a CAS on `used`, owned by one
// pod slot), so every worker answers a retried bind with the plan the ledger holds and a
// restart rebuilds it from the ledger or the annotations alike.
constexpr int kWideContainers = 1024;   // GPU containers a wide record holds
constexpr int kWideIdx = 2048;          // device indices (whole-device containers take several)
struct WideRecord {
  std::atomic<int32_t> used;
  int32_t n;                            // containers
  int16_t off[kWideContainers + 1];     // container c: idx[off[c] .. off[c+1])
  int16_t idx[kWideIdx];
};
using WidePlan = std::vector<std::vector<int32_t>>;   // per container, its device indices (-1: none)

// Bind handoff between the worker processes of a replica (Frontend): what a filter parsed
// from a pod (namespace, name, containers, demand, owner), for its bind when another worker
// process receives it. kube-scheduler sends binds from per-pod goroutines on other keep-alive
// connections than its scheduling cycle's, and SO_REUSEPORT spreads connections over the
// workers, so with several workers the bind usually lands on a worker whose own pod cache
// never saw the pod. Buckets of kPodInfoWays slots by key hash, the oldest entry of a full
// bucket replaced; an entry a newer pod replaced just sends its bind the slow way (Python,
// which reads the pod from the API server).
constexpr int kPodInfoBytes = 1000;
constexpr int kPodInfoWays = 4;
struct PodInfoSlot {
  uint64_t hash;    // key_hash(key), 0: empty
  uint64_t stamp;   // insertion order within the region (the oldest of a full bucket goes)
  char key[kKeyLen];
  uint32_t len;
  uint32_t pad;
  char data[kPodInfoBytes];
};

struct LedgerHeader {
  uint64_t magic;
  uint32_t version;
  uint32_t max_nodes;
  uint32_t pods_per_shard;
  uint32_t pad;
  std::atomic<int32_t> n_nodes;
  std::atomic<int32_t> attached;    // processes attached
  pthread_mutex_t registry_mu;
  alignas(64) std::atomic<uint64_t> epoch;      // bumps on every mutation anywhere
  // bumps when a node slot is created or removed: what caches of node ids (the front door's
  // name -> id lists, assume_many's score memo) must re-check; every other change is visible
  // through the node's own generation
  std::atomic<uint64_t> node_epoch;
  // 1 while this replica may schedule: the worker running the leader elector writes it, every
  // worker (front door, Python router, /readyz) reads it. 1 without leader election.
  std::atomic<int32_t> serving;
  // nominations (Ledger::nominate): made, adopted by their pod's bind on the same node, moved
  // (the bind went to another node: kube-scheduler's own scores overrode ours), and the score
  // lead a node needs over the runner-up before priorities nominate it (adaptive)
  alignas(64) std::atomic<uint64_t> nom_made;
  std::atomic<int32_t> nom_margin;   // read by every priorities call
  // written by the binds, which land on any worker: a line apart from what priorities read
  alignas(64) std::atomic<uint64_t> nom_adopted;
  std::atomic<uint64_t> nom_moved;
  // nominations a worker left for after its answer (Frontend::run_deferred): begun before the
  // answer went out, done once made; a filter on another worker waits while they differ
  // (wait_deferred_nominations), so it never reads the ledger without a pod answered before it
  alignas(64) std::atomic<uint64_t> nom_deferred_begun;
  std::atomic<uint64_t> nom_deferred_done;
  alignas(64) std::atomic<int64_t> n_pods;
  // learned request-size mix (Ledger::note_request): decayed counts of share sizes and the
  // set of the common ones, which native binpack's waste model uses (alloc.h SizeSet)
  alignas(64) std::atomic<uint32_t> size_total;
  std::atomic<uint64_t> size_bits[2];
  std::atomic<uint32_t> size_hist[kWasteSlots];
  // owners (ReplicaSet, Job, ...) whose pods were measured streaming HBM: a device at or above
  // the HBM-activity threshold while it held one of their pods alone. Their new pods count as
  // memory-bound unless annotated otherwise. Written by the telemetry worker, read by every
  // worker's front door without a lock.
  alignas(64) std::atomic<uint64_t> stream_owner[kStreamOwners];
  PaddedMutex shard_mu[kPodShards];
  int32_t shard_live[kPodShards];   // guarded by shard_mu[s]
  int32_t shard_tomb[kPodShards];
  uint32_t ext_cap;                 // overflow records (pods over kSlotContainers containers)
  std::atomic<uint32_t> ext_hint;   // where the next claim starts looking
  std::atomic<int32_t> ext_used;
  uint32_t wide_cap;                // wide records (WideRecord)
  std::atomic<uint32_t> wide_hint;
  std::atomic<int32_t> wide_used;
  uint32_t info_cap;                // bind-handoff slots (PodInfoSlot), a multiple of kPodInfoWays
  std::atomic<uint64_t> info_stamp;
  PaddedMutex info_mu[kPodShards];  // bucket b is guarded by info_mu[b % kPodShards]
};

struct NodeSnapshot {
  int32_t n_devs;
  uint64_t generation;
  Topology topo;
  Device devs[kMaxDevs];
};

struct PodRecord {
  std::string key;
  int32_t node;
  int32_t state;
  double t_reserved;
  Demand demand;
  Plan plan;
  uint64_t owner = 0;
};

class Ledger {
 public:
  // path empty => private heap ledger. Otherwise a /dev/shm file (created if absent,
  // attached if present with the same geometry).
  Ledger(const std::string& path, uint32_t max_nodes, uint32_t max_pods, bool create);
  ~Ledger();
  Ledger(const Ledger&) = delete;
  Ledger& operator=(const Ledger&) = delete;

  // Registers or updates a node. Existing allocations are preserved: free = new_total - used.
  // Devices that disappear while still in use are kept, marked unhealthy.
  int32_t upsert_node(const std::string& name, const Device* devs, int n, const Topology& topo);
  int32_t find_node(const std::string& name) const;
  // Name of node `id` if it is registered (no lock: slot names are written before in_use).
  bool node_named(int32_t id, std::string_view name) const;
  std::string node_name(int32_t id) const;
  int32_t n_nodes() const { return hdr_->n_nodes.load(std::memory_order_acquire); }
  bool remove_node(int32_t id);  // only when no pods are on it
  bool snapshot(int32_t id, NodeSnapshot* out) const;
  // This process's plan cache for node `id`: the entries still valid at the node's current
  // generation (the reference's NodeInfo.PlanCache dump in /status, node.go:18-23).
  struct CachedPlan {
    uint64_t demand_hash, options_hash;
    int32_t rc;
    Plan plan;
  };
  std::vector<CachedPlan> cached_plans(int32_t id) const;
  uint64_t generation(int32_t id) const;
  uint64_t epoch() const { return hdr_->epoch.load(std::memory_order_acquire); }
  uint64_t node_epoch() const { return hdr_->node_epoch.load(std::memory_order_acquire); }
  bool serving() const { return hdr_->serving.load(std::memory_order_acquire) != 0; }
  // Score lead over the runner-up a top node needs before priorities nominate it. Starts at
  // 0 (any unique top node); each nomination a bind moves elsewhere raises it by 2 (to 40),
  // every 16 adopted ones lower it by 1: nominations stay where kube-scheduler agrees.
  int32_t nomination_margin() const { return hdr_->nom_margin.load(std::memory_order_relaxed); }
  // a nomination this worker makes after its answer: begin() before the answer is written,
  // end() once Ledger::nominate ran (Frontend::run_deferred)
  void deferred_nomination_begin() { hdr_->nom_deferred_begun.fetch_add(1, std::memory_order_release); }
  void deferred_nomination_end() { hdr_->nom_deferred_done.fetch_add(1, std::memory_order_release); }
  // before a filter reads the ledger: until every nomination another worker deferred past its
  // answer is made, at most `max_ns` (a worker that died in between cannot hold filters up for
  // longer). False: it timed out.
  bool wait_deferred_nominations(uint64_t max_ns) const;
  // nominations made so far, anywhere in the region (a change marker)
  uint64_t nominations_made() const { return hdr_->nom_made.load(std::memory_order_acquire); }
  void nomination_counts(uint64_t* made, uint64_t* adopted, uint64_t* moved) const {
    *made = hdr_->nom_made.load(std::memory_order_relaxed);
    *adopted = hdr_->nom_adopted.load(std::memory_order_relaxed);
    *moved = hdr_->nom_moved.load(std::memory_order_relaxed);
  }
  void set_serving(bool on) { hdr_->serving.store(on ? 1 : 0, std::memory_order_release); }

  // Filter/score: plan for `d` on node `id`, cached per (node, generation, demand, options).
  int32_t assume(int32_t id, const Demand& d, const Options& o, Plan* plan);
  // assume() over many nodes for one demand (the filter / priorities verbs): the demand and
  // option hashes are computed once and only rc + score leave the plan cache.
  void assume_many(const int32_t* ids, int n, const Demand& d, const Options& o, int32_t* rc, int32_t* score);

  // Bind: choose (cache hit if the node is unchanged) and allocate atomically; records the
  // pod as Reserved. Idempotent for the same key on the same node. A nomination of the
  // key on this node is adopted (kOk: the caller owns it, e.g. rolls it back on failure);
  // one on another node is released first.
  int32_t reserve(int32_t id, std::string_view key, const Demand& d, const Options& o, Plan* plan);
  // Priorities: takes `d` tentatively on node `id` for pod `key` (state Nominated), the node
  // kube-scheduler is about to pick, so the filters of the pods scheduled right behind it
  // (kube-scheduler's cycle does not wait for the bind) already see it — the extender-side
  // counterpart of kube-scheduler's assume cache. Moves an older nomination of the key;
  // leaves a Reserved/Committed key alone (kOkExisting). Unbound ones expire (below).
  int32_t nominate(int32_t id, std::string_view key, const Demand& d, const Options& o);
  std::vector<std::string> expired_nominations(double older_than_s) const;
  // Releases `key` only while it is a nomination: every scheduling attempt of a pod starts
  // by dropping its own nomination, so its filter and scores never count it against itself.
  // kOk = dropped, kOkExisting = reserved/committed (left alone), kErrUnknownPod = none.
  int32_t drop_nomination(std::string_view key);
  // Releases `key` only while it is still a reservation (a sweep racing a commit).
  int32_t drop_reservation(std::string_view key);
  // Allocates an explicit plan (pods bound by someone else / rebuild from annotations).
  int32_t allocate_plan(int32_t id, std::string_view key, const Demand& d, const Plan& plan,
                        bool committed);
  // A wide pod: its folded record (demand / plan, as allocate_plan) and its per-container plan
  // `wide`. kOk: accounted now; kOkExisting: the pod is already on node `id` and *held is the
  // per-container plan the ledger holds for it (empty if it has none), nothing changed (a
  // `committed` call still marks it committed); kErrPodExists: it is on another node;
  // kErrTableFull: no slot or wide record free; kErrBadDemand: more than the record holds.
  int32_t reserve_wide(int32_t id, std::string_view key, const Demand& folded, const Plan& fplan,
                       const WidePlan& wide, bool committed, WidePlan* held);
  // the per-container plan of wide pod `key` (false: not a wide pod of this ledger)
  bool wide_plan(std::string_view key, WidePlan* out) const;
  int32_t wide_records_used() const { return hdr_->wide_used.load(std::memory_order_relaxed); }
  int32_t commit(std::string_view key);
  int32_t release(std::string_view key);
  bool lookup(std::string_view key, PodRecord* out) const;
  // whether the ledger holds a record for `key` (no copy of it; the pod watch's drop test)
  bool holds(std::string_view key) const;
  std::vector<PodRecord> pods_on(int32_t node) const;
  // Preemption check (extender preemptVerb): does demand `d` fit on node `id` once the
  // shares of `victims` (pod keys) are released? Simulated on a copy; nothing changes.
  int32_t fits_without(int32_t id, const std::vector<std::string>& victims, const Demand& d, const Options& o,
                       Plan* plan) const;
  std::vector<std::string> expired_reservations(double older_than_s) const;
  // Relist reconciliation (client-go reflector Replace: what a LIST no longer holds was
  // deleted). Releases every Committed pod recorded before `before` (CLOCK_MONOTONIC, taken
  // before the LIST was sent) whose key is absent from `live`, the UIDs the LIST returned.
  // Reservations (binds in flight) and nominations are left to their sweepers; a pod committed
  // after `before` may postdate the LIST's snapshot and is left alone too. Returns the keys
  // released.
  std::vector<std::string> reconcile(const std::vector<std::string>& live, double before);
  // The same over views (the binding hands the LIST's UIDs as one newline-joined string)
  std::vector<std::string> reconcile_views(const std::vector<std::string_view>& live, double before);
  // Releases `key` only while it is Committed (reconcile racing a re-bind of the same key).
  int32_t drop_committed(std::string_view key);
  int64_t n_pods() const { return hdr_->n_pods.load(std::memory_order_acquire); }
  // processes attached to the region (more than one: worker processes share it)
  int32_t attached() const { return hdr_->attached.load(std::memory_order_relaxed); }
  // Bind handoff (PodInfoSlot): `blob` is the front door's packed pod. put: false when it does
  // not fit a slot. take: the blob stored for `key`, removed (one bind per pod UID).
  bool put_pod_info(std::string_view key, std::string_view blob);
  bool take_pod_info(std::string_view key, std::string* blob);
  int32_t overflow_records_used() const { return hdr_->ext_used.load(std::memory_order_relaxed); }

  // Load-aware telemetry (reference nodeusage.go + allocate.go:173-195).
  int32_t set_load(int32_t id, int dev, float usage);
  int32_t set_health(int32_t id, int dev, bool healthy);
  // measured HBM activity above the policy threshold (Device::mem_hot)
  int32_t set_mem_hot(int32_t id, int dev, bool hot);
  // the averaged HBM activity in percent (what the learner reads; placement does not)
  int32_t set_mem_busy(int32_t id, int dev, int32_t percent);

  FragStats frag(int32_t min_request) const;

  // Request-size learning: every new reservation/allocation counts its share sizes; a size
  // is common once it is >= 2 % of the decayed count (dropped below 1 %).
  void note_request(const Demand& d);
  void set_stream_owner(uint64_t owner, bool streaming);
  bool is_stream_owner(uint64_t owner) const;
  // records the controlling owner of a pod the ledger holds (what learn_stream_owners reads)
  int32_t set_pod_owner(std::string_view key, uint64_t owner);
  // One pass over the committed pods. A device that holds exactly one pod is that pod's "lone"
  // device; only pods recorded at or before `reserved_before` (CLOCK_MONOTONIC: the start of
  // the HBM metric's averaging window, so the mark was measured on this pod and not on a
  // tenant it replaced) count. Per owner: learned if any of its lone pods sits on a device
  // marked mem_hot; with `forget_cool`, forgotten once every lone pod of it was cool (and none
  // hot) in `forget_after` consecutive passes. Returns {owners learned, owners forgotten}.
  //
  // `hot_curve` (share percent -> activity percent, ascending shares) makes the decision share
  // aware: a lone pod holding share s of its device counts as streaming when the device's
  // mem_busy is at least the curve at s (linear in between, flat outside). A streaming tenant
  // alone moves more of the device's bandwidth the more CUs it holds, so one fixed threshold
  // either misses small streamers or flags big non-streamers. Empty: the device's mem_hot mark.
  std::pair<int32_t, int32_t> learn_stream_owners(bool forget_cool, double reserved_before = 1e300,
                                                  int32_t forget_after = 1,
                                                  const std::vector<std::pair<float, float>>& hot_curve = {});
  SizeSet learned_sizes() const;
  // The options a placement runs with: native binpack gets the request-size set (fixed |
  // learned | this demand's sizes) and its waste table; everything else is unchanged.
  Options resolve(const Options& o, const Demand& d) const;

  void clear_cache();
  size_t cache_size() const;
  const std::string& path() const { return path_; }
  size_t bytes() const { return bytes_; }
  static size_t region_bytes(uint32_t max_nodes, uint32_t max_pods);

 private:
  NodeSlot* node(int32_t id) const;
  std::atomic<uint64_t>& gen_of(const NodeSlot* n) const { return hot_[n - nodes_].gen; }
  // under n->mu: records which devices this change touched (~0: all, or not device-local), then
  // bumps the node's generation
  void bump(NodeSlot* n, uint64_t devices_touched);
  // the devices changed between generations `from` and `to` (false: the ring no longer holds
  // every bump in between)
  bool changed_since(const NodeSlot* n, uint64_t from, uint64_t to, uint64_t* mask) const;
  PodSlot* shard(int s) const;
  int shard_of(uint64_t h) const { return static_cast<int>(h % kPodShards); }
  int32_t reserve_as(int32_t id, std::string_view key, const Demand& d, const Options& o, Plan* plan,
                     int32_t state);
  std::vector<std::string> expired(int32_t state, double older_than_s) const;
  int32_t release_if(std::string_view key, int32_t only_state);   // -1: any state
  PodSlot* find_pod_locked(int s, uint64_t h, const char* key) const;
  PodSlot* insert_pod_locked(int s, uint64_t h, const char* key);
  // frees slot `p` of shard `s` (shard lock held): a tombstone only where a probe may pass
  void erase_pod_locked(int s, PodSlot* p);
  // a slot's demand and plan, inline or in its overflow record (false: no record free)
  bool put_record(PodSlot* p, const Demand& d, const Plan& plan);
  void get_record(const PodSlot& p, Demand* d, Plan* plan) const;
  void free_record(PodSlot* p);
  bool put_wide(PodSlot* p, const WidePlan& w);
  void get_wide(const PodSlot& p, WidePlan* w) const;

  void lock_node(NodeSlot* n) const;
  void lock_mu(pthread_mutex_t* m) const;

  std::string path_;
  // this object's identity for per-thread caches (a later Ledger can reuse a freed address)
  uint64_t instance_ = 0;
  bool owner_;
  int fd_ = -1;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  LedgerHeader* hdr_ = nullptr;
  NodeHot* hot_ = nullptr;
  NodeSlot* nodes_ = nullptr;
  PodSlot* pods_ = nullptr;
  ExtRecord* ext_ = nullptr;
  WideRecord* wide_ = nullptr;
  PodInfoSlot* info_ = nullptr;

  struct CacheKey {
    int32_t node;
    uint64_t gen, dh, oh;
    bool operator==(const CacheKey& o) const {
      return node == o.node && gen == o.gen && dh == o.dh && oh == o.oh;
    }
  };
  // Plan cache: process-local, one small direct-mapped table per node slot (a 2-way probe
  // on the demand/options hash). Entries carry the node generation they were computed at,
  // so a change to the node invalidates them without any clearing. Writers and plan readers
  // take a per-node spin flag; the filter/priorities path (rc + score only) reads through a
  // sequence counter without any read-modify-write, so 64 nodes cost 64 plain load pairs.
  static constexpr int kCacheWays = 32;
  struct CacheEntry {
    std::atomic<uint64_t> gen{0}, dh{0}, oh{0};
    std::atomic<int32_t> rc{0}, score{0};
    std::atomic<bool> used{false};
    Plan plan{};   // under `busy`
  };
  struct NodeCache {
    std::atomic<uint32_t> seq{0};   // odd while a writer updates entries
    std::atomic<bool> busy{false};
    CacheEntry e[kCacheWays];
    void lock() {
      for (int spins = 0; busy.exchange(true, std::memory_order_acquire);)
        while (busy.load(std::memory_order_relaxed))
          if (++spins > 64) std::this_thread::yield();
    }
    void unlock() { busy.store(false, std::memory_order_release); }
  };
  // allocated on a node's first cached plan (6.6 KB each), published with a CAS
  mutable std::unique_ptr<std::atomic<NodeCache*>[]> cache_;
  uint32_t cache_nodes_ = 0;
  NodeCache* node_cache(int32_t node, bool create) const;
  bool cache_get(const CacheKey& k, int32_t* rc, Plan* plan) const;
  bool cache_get_score(const CacheKey& k, int32_t* rc, int32_t* score) const;
  void cache_put(const CacheKey& k, int32_t rc, const Plan& plan);
  // learner (one telemetry worker per replica): consecutive all-cool passes per learned owner
  std::mutex learn_mu_;
  std::unordered_map<uint64_t, int32_t> cool_streak_;
  mutable std::mutex names_mu_;
  mutable std::unordered_map<std::string, int32_t> names_;  // process-local name index
};

uint64_t key_hash(const char* key);
double mono_now();

}  // namespace nanogpu
