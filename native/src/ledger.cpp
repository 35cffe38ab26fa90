// Native cluster ledger (see ledger.h). Reference parity: pkg/dealer/dealer.go
// (Assume :89-136, Score :138-153, Bind :155-203, Allocate :205-228, Release :230-255,
// KnownPod :257-262, getNodeInfo :271-301) and pkg/dealer/node.go (PlanCache :18-98).
#include "nanogpu/iotally.h"
#include "nanogpu/ledger.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <unordered_set>

namespace nanogpu {

static constexpr uint64_t kMagic = 0x4e414e4f47505531ULL;  // "NANOGPU1"
static constexpr uint32_t kVersion = 18;  // 4: HBM pools; 5: cache lines; 6: sizes; 7: serving; 8: nominations; 9: stream owners; 10: overflow records; 11: node epoch; 12-13: bind handoff; 14: dense node generations; 15: device change ring; 16: wide records; 17: deferred nominations; 18: adoption counters on a line of their own

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

uint64_t key_hash(const char* key) {
  uint64_t h = 0xcbf29ce484222325ULL;
  for (const unsigned char* p = reinterpret_cast<const unsigned char*>(key); *p; ++p) {
    h ^= *p;
    h *= 0x100000001b3ULL;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  return h;
}

// A pod key as the C string the table stores (NUL-terminated, < kKeyLen bytes) on the stack:
// the key APIs take a view, so the front door's UIDs reach the table without a heap copy. A
// key no slot can hold (empty, too long) reads as the empty key, which no slot holds either.
struct KeyBuf {
  char b[kKeyLen];
  explicit KeyBuf(std::string_view k) {
    const size_t n = k.size() < static_cast<size_t>(kKeyLen) ? k.size() : 0;
    std::memcpy(b, k.data(), n);
    b[n] = '\0';
  }
  const char* c_str() const { return b; }
};

double mono_now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + 1e-9 * static_cast<double>(ts.tv_nsec);
}

static void init_mutex(pthread_mutex_t* m) {
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(m, &a);
  pthread_mutexattr_destroy(&a);
}

void Ledger::lock_mu(pthread_mutex_t* m) const {
  const int rc = pthread_mutex_lock(m);
  if (rc == EOWNERDEAD) {
    // A worker died inside a critical section. Every mutation below validates before it
    // writes and writes counters last, so the protected state is consistent enough to go on.
    pthread_mutex_consistent(m);
  } else if (rc != 0) {
    throw std::runtime_error("ledger: pthread_mutex_lock failed");
  }
}

void Ledger::lock_node(NodeSlot* n) const { lock_mu(&n->mu); }

namespace {
struct Unlock {
  pthread_mutex_t* m;
  ~Unlock() {
    if (m) pthread_mutex_unlock(m);
  }
};
uint32_t pods_per_shard_for(uint32_t max_pods) {
  uint64_t per = (static_cast<uint64_t>(max_pods) * 3 / 2 + kPodShards - 1) / kPodShards;
  return static_cast<uint32_t>(std::max<uint64_t>(per, 16));
}
// pods with more than kSlotContainers containers are rare (one in 32 pods at most)
uint32_t ext_records_for(uint32_t max_pods) { return std::max<uint32_t>(64, max_pods / 32); }
// pods with more GPU containers than a Demand holds are rarer still
uint32_t wide_records_for(uint32_t max_pods) { return std::max<uint32_t>(16, max_pods / 512); }
// bind handoffs in flight at once: pods between their filter and their bind
uint32_t info_slots_for(uint32_t max_pods) {
  return std::clamp<uint32_t>(max_pods / 16, 1024, 16384) / kPodInfoWays * kPodInfoWays;
}
}  // namespace

size_t Ledger::region_bytes(uint32_t max_nodes, uint32_t max_pods) {
  const size_t h = align_up(sizeof(LedgerHeader), 4096) + align_up(sizeof(NodeHot) * max_nodes, 4096);
  const size_t n = align_up(sizeof(NodeSlot) * max_nodes, 4096);
  const size_t p = align_up(sizeof(PodSlot) * kPodShards * pods_per_shard_for(max_pods), 4096);
  const size_t e = align_up(sizeof(ExtRecord) * ext_records_for(max_pods), 4096);
  const size_t w = align_up(sizeof(WideRecord) * wide_records_for(max_pods), 4096);
  const size_t i = align_up(sizeof(PodInfoSlot) * info_slots_for(max_pods), 4096);
  return h + n + p + e + w + i;
}

Ledger::Ledger(const std::string& path, uint32_t max_nodes, uint32_t max_pods, bool create)
    : path_(path), owner_(false) {
  static std::atomic<uint64_t> instances{0};
  instance_ = instances.fetch_add(1, std::memory_order_relaxed) + 1;
  if (max_nodes == 0 || max_pods == 0) throw std::invalid_argument("ledger: zero capacity");
  bytes_ = region_bytes(max_nodes, max_pods);
  bool init = false;
  if (path.empty()) {
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::runtime_error("ledger: mmap anonymous failed");
    base_ = static_cast<char*>(p);
    init = true;
    owner_ = true;
  } else {
    if (create) {
      fd_ = open(path.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
      if (fd_ >= 0) {
        init = true;
        owner_ = true;
        if (ftruncate(fd_, static_cast<off_t>(bytes_)) != 0) {
          close(fd_);
          unlink(path.c_str());
          throw std::runtime_error("ledger: ftruncate failed");
        }
      }
    }
    if (fd_ < 0) {
      fd_ = open(path.c_str(), O_RDWR);
      if (fd_ < 0) throw std::runtime_error("ledger: cannot open " + path);
      // wait for the creator to size the file; a file that stays short (another geometry, or a
      // creator that died before ftruncate) is refused here: touching a page past its end
      // would raise SIGBUS
      bool sized = false;
      for (int i = 0; i < 2000 && !sized; ++i) {
        struct stat st;
        sized = fstat(fd_, &st) == 0 && static_cast<size_t>(st.st_size) >= bytes_;
        if (!sized) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (!sized) {
        close(fd_);
        throw std::runtime_error("ledger: shared region is smaller than this geometry needs: " + path);
      }
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) {
      close(fd_);
      throw std::runtime_error("ledger: mmap shared failed (geometry mismatch?)");
    }
    base_ = static_cast<char*>(p);
  }
  hdr_ = reinterpret_cast<LedgerHeader*>(base_);
  hot_ = reinterpret_cast<NodeHot*>(base_ + align_up(sizeof(LedgerHeader), 4096));
  nodes_ = reinterpret_cast<NodeSlot*>(reinterpret_cast<char*>(hot_) + align_up(sizeof(NodeHot) * max_nodes, 4096));
  pods_ = reinterpret_cast<PodSlot*>(reinterpret_cast<char*>(nodes_) +
                                     align_up(sizeof(NodeSlot) * max_nodes, 4096));
  ext_ = reinterpret_cast<ExtRecord*>(
      reinterpret_cast<char*>(pods_) +
      align_up(sizeof(PodSlot) * kPodShards * pods_per_shard_for(max_pods), 4096));
  wide_ = reinterpret_cast<WideRecord*>(reinterpret_cast<char*>(ext_) +
                                        align_up(sizeof(ExtRecord) * ext_records_for(max_pods), 4096));
  info_ = reinterpret_cast<PodInfoSlot*>(reinterpret_cast<char*>(wide_) +
                                         align_up(sizeof(WideRecord) * wide_records_for(max_pods), 4096));
  if (init) {
    hdr_->version = kVersion;
    hdr_->max_nodes = max_nodes;
    hdr_->pods_per_shard = pods_per_shard_for(max_pods);
    hdr_->n_nodes.store(0);
    hdr_->epoch.store(1);
    hdr_->node_epoch.store(1);
    hdr_->serving.store(1);
    hdr_->nom_made.store(0);
    hdr_->nom_adopted.store(0);
    hdr_->nom_moved.store(0);
    hdr_->nom_margin.store(0);
    hdr_->n_pods.store(0);
    hdr_->attached.store(0);
    hdr_->size_total.store(0);
    hdr_->size_bits[0].store(0);
    hdr_->size_bits[1].store(0);
    for (auto& c : hdr_->size_hist) c.store(0);
    for (auto& o : hdr_->stream_owner) o.store(0);
    hdr_->ext_cap = ext_records_for(max_pods);
    hdr_->ext_hint.store(0);
    hdr_->ext_used.store(0);
    hdr_->wide_cap = wide_records_for(max_pods);
    hdr_->wide_hint.store(0);
    hdr_->wide_used.store(0);
    hdr_->info_cap = info_slots_for(max_pods);
    hdr_->info_stamp.store(0);
    for (auto& m : hdr_->info_mu) init_mutex(&m.m);
    init_mutex(&hdr_->registry_mu);
    for (int s = 0; s < kPodShards; ++s) {
      init_mutex(&hdr_->shard_mu[s].m);
      hdr_->shard_live[s] = 0;
      hdr_->shard_tomb[s] = 0;
    }
    std::atomic_thread_fence(std::memory_order_release);
    __atomic_store_n(&hdr_->magic, kMagic, __ATOMIC_RELEASE);
  } else {
    bool ok = false;
    for (int i = 0; i < 5000; ++i) {
      if (__atomic_load_n(&hdr_->magic, __ATOMIC_ACQUIRE) == kMagic) {
        ok = true;
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (!ok || hdr_->version != kVersion || hdr_->max_nodes != max_nodes ||
        hdr_->pods_per_shard != pods_per_shard_for(max_pods)) {
      munmap(base_, bytes_);
      close(fd_);
      throw std::runtime_error("ledger: shared region has a different layout: " + path);
    }
  }
  hdr_->attached.fetch_add(1);
  cache_nodes_ = hdr_->max_nodes;
  cache_.reset(new std::atomic<NodeCache*>[cache_nodes_]);
  for (uint32_t i = 0; i < cache_nodes_; ++i) cache_[i].store(nullptr, std::memory_order_relaxed);
}

Ledger::NodeCache* Ledger::node_cache(int32_t node, bool create) const {
  if (static_cast<uint32_t>(node) >= cache_nodes_) return nullptr;
  NodeCache* c = cache_[node].load(std::memory_order_acquire);
  if (c || !create) return c;
  auto* fresh = new NodeCache();
  if (cache_[node].compare_exchange_strong(c, fresh, std::memory_order_acq_rel)) return fresh;
  delete fresh;   // another thread published first
  return c;
}

Ledger::~Ledger() {
  if (cache_)
    for (uint32_t i = 0; i < cache_nodes_; ++i) delete cache_[i].load(std::memory_order_relaxed);
  if (hdr_) hdr_->attached.fetch_sub(1);
  if (base_) munmap(base_, bytes_);
  if (fd_ >= 0) close(fd_);
}

NodeSlot* Ledger::node(int32_t id) const {
  if (id < 0 || id >= hdr_->n_nodes.load(std::memory_order_acquire)) return nullptr;
  return &nodes_[id];
}

PodSlot* Ledger::shard(int s) const {
  return pods_ + static_cast<size_t>(s) * hdr_->pods_per_shard;
}

PodSlot* Ledger::find_pod_locked(int s, uint64_t h, const char* key) const {
  PodSlot* t = shard(s);
  const uint32_t cap = hdr_->pods_per_shard;
  uint32_t i = static_cast<uint32_t>((h / kPodShards) % cap);
  for (uint32_t probe = 0; probe < cap; ++probe, i = (i + 1) % cap) {
    PodSlot& p = t[i];
    if (p.state == kPodEmpty) return nullptr;
    if (p.state != kPodTombstone && p.hash == h && std::strncmp(p.key, key, kKeyLen) == 0)
      return &p;
  }
  return nullptr;
}

void Ledger::erase_pod_locked(int s, PodSlot* p) {
  // Linear probing needs a tombstone only where a later entry's probe may run through the
  // slot. With the next slot empty none can; nor then through the tombstones right before
  // this one (a cluster's dead tail): they all become empty (no live entry moves, so slot
  // pointers stay valid). Churn then leaves no tombstones to lengthen every miss's probe.
  PodSlot* t = shard(s);
  const uint32_t cap = hdr_->pods_per_shard;
  const uint32_t i = static_cast<uint32_t>(p - t);
  --hdr_->shard_live[s];
  if (t[(i + 1) % cap].state != kPodEmpty) {
    p->state = kPodTombstone;
    ++hdr_->shard_tomb[s];
    return;
  }
  p->state = kPodEmpty;
  for (uint32_t k = (i + cap - 1) % cap; k != i && t[k].state == kPodTombstone; k = (k + cap - 1) % cap) {
    t[k].state = kPodEmpty;
    --hdr_->shard_tomb[s];
  }
}

PodSlot* Ledger::insert_pod_locked(int s, uint64_t h, const char* key) {
  const uint32_t cap = hdr_->pods_per_shard;
  // rehash when the table is nearly full, or when tombstones alone are a quarter of it (the
  // probe of every miss runs through them)
  if (hdr_->shard_live[s] + hdr_->shard_tomb[s] + 1 > static_cast<int32_t>(cap * 9 / 10) ||
      hdr_->shard_tomb[s] > static_cast<int32_t>(cap / 4)) {
    if (hdr_->shard_tomb[s] == 0) return nullptr;  // genuinely full
    // compact: rehash live entries, dropping tombstones
    PodSlot* t = shard(s);
    std::vector<PodSlot> live;
    live.reserve(hdr_->shard_live[s]);
    for (uint32_t i = 0; i < cap; ++i)
      if (t[i].state == kPodReserved || t[i].state == kPodCommitted || t[i].state == kPodNominated)
        live.push_back(t[i]);
    for (uint32_t i = 0; i < cap; ++i) t[i].state = kPodEmpty;
    for (const PodSlot& p : live) {
      uint32_t i = static_cast<uint32_t>((p.hash / kPodShards) % cap);
      while (t[i].state != kPodEmpty) i = (i + 1) % cap;
      t[i] = p;
    }
    hdr_->shard_tomb[s] = 0;
  }
  PodSlot* t = shard(s);
  uint32_t i = static_cast<uint32_t>((h / kPodShards) % cap);
  PodSlot* reuse = nullptr;
  for (uint32_t probe = 0; probe < cap; ++probe, i = (i + 1) % cap) {
    PodSlot& p = t[i];
    if (p.state == kPodTombstone) {
      if (!reuse) reuse = &p;
      continue;
    }
    if (p.state == kPodEmpty) {
      if (!reuse) reuse = &p;
      break;
    }
  }
  if (!reuse) return nullptr;
  if (reuse->state == kPodTombstone) --hdr_->shard_tomb[s];
  std::memset(reuse, 0, sizeof(PodSlot));
  reuse->hash = h;
  std::strncpy(reuse->key, key, kKeyLen - 1);
  ++hdr_->shard_live[s];
  return reuse;
}

bool Ledger::put_record(PodSlot* p, const Demand& d, const Plan& plan) {
  free_record(p);
  if (d.n <= kSlotContainers && plan.n <= kSlotContainers) {
    p->demand.n = d.n;
    std::memcpy(p->demand.c, d.c, sizeof(ContainerDemand) * static_cast<size_t>(std::max(0, d.n)));
    p->plan.n = plan.n;
    p->plan.score = plan.score;
    std::memcpy(p->plan.off, plan.off, sizeof(int16_t) * static_cast<size_t>(std::max(0, plan.n) + 1));
    std::memcpy(p->plan.idx, plan.idx, sizeof(plan.idx));
    return true;
  }
  const uint32_t cap = hdr_->ext_cap;
  const uint32_t start = hdr_->ext_hint.load(std::memory_order_relaxed);
  for (uint32_t k = 0; k < cap; ++k) {
    const uint32_t i = (start + k) % cap;
    int32_t free_ = 0;
    if (ext_[i].used.load(std::memory_order_relaxed) == 0 &&
        ext_[i].used.compare_exchange_strong(free_, 1, std::memory_order_acquire)) {
      ext_[i].demand = d;
      ext_[i].plan = plan;
      p->ext = static_cast<int32_t>(i) + 1;
      p->demand.n = d.n;
      p->plan.n = plan.n;
      p->plan.score = plan.score;
      hdr_->ext_hint.store((i + 1) % cap, std::memory_order_relaxed);
      hdr_->ext_used.fetch_add(1, std::memory_order_relaxed);
      return true;
    }
  }
  return false;
}

void Ledger::get_record(const PodSlot& p, Demand* d, Plan* plan) const {
  if (p.ext > 0 && static_cast<uint32_t>(p.ext) <= hdr_->ext_cap) {
    const ExtRecord& e = ext_[p.ext - 1];
    if (d) *d = e.demand;
    if (plan) *plan = e.plan;
    return;
  }
  if (d) {
    std::memset(d, 0, sizeof(Demand));
    d->n = std::clamp(p.demand.n, 0, kSlotContainers);
    std::memcpy(d->c, p.demand.c, sizeof(ContainerDemand) * static_cast<size_t>(d->n));
  }
  if (plan) {
    std::memset(plan, 0, sizeof(Plan));
    plan->n = std::clamp(p.plan.n, 0, kSlotContainers);
    plan->score = p.plan.score;
    std::memcpy(plan->off, p.plan.off, sizeof(int16_t) * static_cast<size_t>(plan->n + 1));
    std::memcpy(plan->idx, p.plan.idx, sizeof(p.plan.idx));
  }
}

void Ledger::free_record(PodSlot* p) {
  if (p->ext > 0 && static_cast<uint32_t>(p->ext) <= hdr_->ext_cap) {
    ext_[p->ext - 1].used.store(0, std::memory_order_release);
    hdr_->ext_used.fetch_sub(1, std::memory_order_relaxed);
  }
  p->ext = 0;
  if (p->wide > 0 && static_cast<uint32_t>(p->wide) <= hdr_->wide_cap) {
    wide_[p->wide - 1].used.store(0, std::memory_order_release);
    hdr_->wide_used.fetch_sub(1, std::memory_order_relaxed);
  }
  p->wide = 0;
}

bool Ledger::put_wide(PodSlot* p, const WidePlan& w) {
  size_t total = 0;
  for (const auto& c : w) total += c.size();
  if (w.size() > static_cast<size_t>(kWideContainers) || total > static_cast<size_t>(kWideIdx)) return false;
  const uint32_t cap = hdr_->wide_cap;
  const uint32_t start = hdr_->wide_hint.load(std::memory_order_relaxed);
  for (uint32_t k = 0; k < cap; ++k) {
    const uint32_t i = (start + k) % cap;
    int32_t free_ = 0;
    if (wide_[i].used.load(std::memory_order_relaxed) == 0 &&
        wide_[i].used.compare_exchange_strong(free_, 1, std::memory_order_acquire)) {
      WideRecord& r = wide_[i];
      r.n = static_cast<int32_t>(w.size());
      int pos = 0;
      for (size_t c = 0; c < w.size(); ++c) {
        r.off[c] = static_cast<int16_t>(pos);
        for (int32_t x : w[c]) r.idx[pos++] = static_cast<int16_t>(x);
      }
      r.off[w.size()] = static_cast<int16_t>(pos);
      p->wide = static_cast<int32_t>(i) + 1;
      hdr_->wide_hint.store((i + 1) % cap, std::memory_order_relaxed);
      hdr_->wide_used.fetch_add(1, std::memory_order_relaxed);
      return true;
    }
  }
  return false;
}

void Ledger::get_wide(const PodSlot& p, WidePlan* w) const {
  w->clear();
  if (p.wide <= 0 || static_cast<uint32_t>(p.wide) > hdr_->wide_cap) return;
  const WideRecord& r = wide_[p.wide - 1];
  const int n = std::clamp(r.n, 0, kWideContainers);
  w->resize(static_cast<size_t>(n));
  for (int c = 0; c < n; ++c) {
    const int a = std::clamp<int>(r.off[c], 0, kWideIdx), b = std::clamp<int>(r.off[c + 1], a, kWideIdx);
    (*w)[static_cast<size_t>(c)].assign(r.idx + a, r.idx + b);
  }
}

int32_t Ledger::upsert_node(const std::string& name, const Device* devs, int n,
                            const Topology& topo) {
  if (n < 0 || n > kMaxDevs || name.empty() || name.size() >= kNameLen) return -kErrBadPlan;
  lock_mu(&hdr_->registry_mu);
  Unlock ur{&hdr_->registry_mu};
  const int32_t count = hdr_->n_nodes.load(std::memory_order_acquire);
  int32_t id = -1;
  for (int32_t i = 0; i < count; ++i)
    if (nodes_[i].in_use && std::strncmp(nodes_[i].name, name.c_str(), kNameLen) == 0) {
      id = i;
      break;
    }
  if (id < 0) {
    if (static_cast<uint32_t>(count) >= hdr_->max_nodes) return -kErrTableFull;
    id = count;
    NodeSlot& s = nodes_[id];
    std::memset(s.name, 0, kNameLen);
    std::strncpy(s.name, name.c_str(), kNameLen - 1);
    init_mutex(&s.mu);
    hot_[id].gen.store(1);
    s.n_devs = n;
    s.n_pods = 0;
    s.topo = topo;
    std::memcpy(s.devs, devs, sizeof(Device) * n);
    for (int i = 0; i < n; ++i) {
      s.devs[i].pct_free = s.devs[i].pct_total;
      s.devs[i].mib_free = s.devs[i].mib_total;
      s.devs[i].mem_bound = 0;
      s.devs[i].mem_hot = 0;
      s.devs[i].mem_busy = 0;
    }
    s.in_use = 1;
    hot_[id].in_use.store(1, std::memory_order_release);
    hdr_->n_nodes.store(count + 1, std::memory_order_release);
    hdr_->node_epoch.fetch_add(1, std::memory_order_release);
  } else {
    NodeSlot& s = nodes_[id];
    lock_node(&s);
    Unlock un{&s.mu};
    Device merged[kMaxDevs];
    int m = n;
    for (int i = 0; i < n; ++i) {
      merged[i] = devs[i];
      if (i < s.n_devs) {
        const Device& old = s.devs[i];
        const int32_t used = old.pct_total - old.pct_free;
        const int64_t mused = old.mib_total > 0 ? old.mib_total - old.mib_free : 0;
        merged[i].pct_free = std::max(0, merged[i].pct_total - used);
        merged[i].mib_free = merged[i].mib_total > 0 ? std::max<int64_t>(0, merged[i].mib_total - mused) : 0;
        merged[i].load_usage = old.load_usage;
        merged[i].remain_load = old.remain_load;
        merged[i].mem_bound = old.mem_bound;
        merged[i].mem_hot = old.mem_hot;
        merged[i].mem_busy = old.mem_busy;
      } else {
        merged[i].pct_free = merged[i].pct_total;
        merged[i].mib_free = merged[i].mib_total;
        merged[i].mem_bound = 0;
        merged[i].mem_hot = 0;
        merged[i].mem_busy = 0;
      }
    }
    // Devices that vanished while still in use stay (unhealthy) until their pods release.
    for (int i = n; i < s.n_devs; ++i)
      if (s.devs[i].pct_free != s.devs[i].pct_total) m = i + 1;
    for (int i = n; i < m; ++i) {
      merged[i] = s.devs[i];
      merged[i].healthy = 0;
    }
    std::memcpy(s.devs, merged, sizeof(Device) * m);
    s.n_devs = m;
    s.topo = topo;
    bump(&s, ~0ull);
  }
  hdr_->epoch.fetch_add(1);
  {
    std::lock_guard<std::mutex> g(names_mu_);
    names_[name] = id;
  }
  return id;
}

int32_t Ledger::find_node(const std::string& name) const {
  {
    std::lock_guard<std::mutex> g(names_mu_);
    auto it = names_.find(name);
    if (it != names_.end() && nodes_[it->second].in_use) return it->second;
  }
  const int32_t count = hdr_->n_nodes.load(std::memory_order_acquire);
  for (int32_t i = 0; i < count; ++i)
    if (nodes_[i].in_use && std::strncmp(nodes_[i].name, name.c_str(), kNameLen) == 0) {
      std::lock_guard<std::mutex> g(names_mu_);
      names_[name] = i;
      return i;
    }
  return -1;
}

std::string Ledger::node_name(int32_t id) const {
  NodeSlot* n = node(id);
  return n ? std::string(n->name) : std::string();
}

bool Ledger::remove_node(int32_t id) {
  NodeSlot* n = node(id);
  if (!n) return false;
  lock_node(n);
  Unlock un{&n->mu};
  if (n->n_pods > 0) return false;
  n->in_use = 0;
  hot_[id].in_use.store(0, std::memory_order_release);
  bump(n, ~0ull);
  hdr_->epoch.fetch_add(1);
  hdr_->node_epoch.fetch_add(1, std::memory_order_release);
  std::lock_guard<std::mutex> g(names_mu_);
  names_.erase(n->name);
  return true;
}

bool Ledger::snapshot(int32_t id, NodeSnapshot* out) const {
  NodeSlot* n = node(id);
  if (!n || !n->in_use) return false;
  lock_node(n);
  Unlock un{&n->mu};
  out->n_devs = n->n_devs;
  out->generation = gen_of(n).load(std::memory_order_relaxed);
  out->topo = n->topo;
  std::memcpy(out->devs, n->devs, sizeof(Device) * n->n_devs);
  return true;
}

uint64_t Ledger::generation(int32_t id) const {
  NodeSlot* n = node(id);
  return n ? gen_of(n).load(std::memory_order_acquire) : 0;
}

void Ledger::bump(NodeSlot* n, uint64_t devices_touched) {
  const uint64_t g = gen_of(n).load(std::memory_order_relaxed);
  const int k = static_cast<int>(g % kChangeRing);
  // the tag is cleared while the mask is rewritten: a reader that sees the tag before and after
  // its mask read equal to g read the mask of this bump
  n->chg_gen[k].store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  n->chg_mask[k].store(devices_touched, std::memory_order_relaxed);
  n->chg_gen[k].store(g, std::memory_order_release);
  gen_of(n).fetch_add(1, std::memory_order_release);
}

bool Ledger::changed_since(const NodeSlot* n, uint64_t from, uint64_t to, uint64_t* mask) const {
  if (to < from || to - from > static_cast<uint64_t>(kChangeRing)) return false;
  uint64_t m = 0;
  for (uint64_t g = from; g < to; ++g) {
    const int k = static_cast<int>(g % kChangeRing);
    if (n->chg_gen[k].load(std::memory_order_acquire) != g) return false;
    const uint64_t x = n->chg_mask[k].load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (n->chg_gen[k].load(std::memory_order_relaxed) != g) return false;
    m |= x;
  }
  *mask = m;
  return true;
}

namespace {
inline int cache_way(uint64_t dh, uint64_t oh) {
  return static_cast<int>((dh ^ (oh * 0x9e3779b97f4a7c15ULL)) >> 59);   // top 5 bits: 0..31
}
}  // namespace

namespace {
constexpr auto kRlx = std::memory_order_relaxed;

template <class E>
inline bool entry_is(const E& e, uint64_t gen, uint64_t dh, uint64_t oh) {
  return e.used.load(kRlx) && e.gen.load(kRlx) == gen && e.dh.load(kRlx) == dh && e.oh.load(kRlx) == oh;
}
}  // namespace

bool Ledger::cache_get(const CacheKey& k, int32_t* rc, Plan* plan) const {
  NodeCache* cp = node_cache(k.node, false);
  if (!cp) return false;
  NodeCache& c = *cp;
  const int w = cache_way(k.dh, k.oh);
  c.lock();
  for (int j = 0; j < 2; ++j) {
    const CacheEntry& e = c.e[(w + j) % kCacheWays];
    if (entry_is(e, k.gen, k.dh, k.oh)) {
      *rc = e.rc.load(kRlx);
      *plan = e.plan;
      c.unlock();
      return true;
    }
  }
  c.unlock();
  return false;
}

// Sequence-counter read (no read-modify-write): sample seq, read the entry's atomic fields,
// and accept them if seq is even and unchanged; a writer in between makes the reader retry,
// and a reader that keeps losing falls back to the lock.
bool Ledger::cache_get_score(const CacheKey& k, int32_t* rc, int32_t* score) const {
  NodeCache* cp = node_cache(k.node, false);
  if (!cp) return false;
  NodeCache& c = *cp;
  const int w = cache_way(k.dh, k.oh);
  for (int tries = 0; tries < 4; ++tries) {
    const uint32_t s0 = c.seq.load(std::memory_order_acquire);
    if (s0 & 1u) continue;
    int found = -1;
    int32_t r = 0, sc = 0;
    for (int j = 0; j < 2 && found < 0; ++j) {
      const CacheEntry& e = c.e[(w + j) % kCacheWays];
      if (entry_is(e, k.gen, k.dh, k.oh)) {
        found = j;
        r = e.rc.load(kRlx);
        sc = e.score.load(kRlx);
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (c.seq.load(kRlx) != s0) continue;
    if (found < 0) return false;
    *rc = r;
    *score = sc;
    return true;
  }
  c.lock();
  for (int j = 0; j < 2; ++j) {
    const CacheEntry& e = c.e[(w + j) % kCacheWays];
    if (entry_is(e, k.gen, k.dh, k.oh)) {
      *rc = e.rc.load(kRlx);
      *score = e.score.load(kRlx);
      c.unlock();
      return true;
    }
  }
  c.unlock();
  return false;
}

std::vector<Ledger::CachedPlan> Ledger::cached_plans(int32_t id) const {
  std::vector<CachedPlan> out;
  NodeSlot* n = node(id);
  NodeCache* cp = n ? node_cache(id, false) : nullptr;
  if (!cp) return out;
  const uint64_t gen = gen_of(n).load(std::memory_order_acquire);
  cp->lock();
  for (const CacheEntry& e : cp->e)
    if (e.used.load(kRlx) && e.gen.load(kRlx) == gen)
      out.push_back(CachedPlan{e.dh.load(kRlx), e.oh.load(kRlx), e.rc.load(kRlx), e.plan});
  cp->unlock();
  return out;
}

void Ledger::cache_put(const CacheKey& k, int32_t rc, const Plan& plan) {
  NodeCache* cp = node_cache(k.node, true);
  if (!cp) return;
  NodeCache& c = *cp;
  const int w = cache_way(k.dh, k.oh);
  c.lock();
  // same key or an unused/stale way first; else replace the older-generation one
  CacheEntry* a = &c.e[w];
  CacheEntry* b = &c.e[(w + 1) % kCacheWays];
  CacheEntry* dst = a;
  auto same_key = [&](const CacheEntry* e) { return e->dh.load(kRlx) == k.dh && e->oh.load(kRlx) == k.oh; };
  if (a->used.load(kRlx) && a->gen.load(kRlx) == k.gen && !same_key(a))
    dst = (!b->used.load(kRlx) || b->gen.load(kRlx) != k.gen || same_key(b)) ? b : a;
  const uint32_t s = c.seq.load(kRlx);
  c.seq.store(s + 1, kRlx);                              // odd: lock-free readers retry
  std::atomic_thread_fence(std::memory_order_release);
  dst->gen.store(k.gen, kRlx);
  dst->dh.store(k.dh, kRlx);
  dst->oh.store(k.oh, kRlx);
  dst->rc.store(rc, kRlx);
  dst->score.store(plan.score, kRlx);
  dst->used.store(true, kRlx);
  dst->plan = plan;
  c.seq.store(s + 2, std::memory_order_release);
  c.unlock();
}

bool Ledger::node_named(int32_t id, std::string_view name) const {
  const NodeSlot* n = node(id);
  return n && n->in_use && name.size() < kNameLen && std::strncmp(n->name, name.data(), name.size()) == 0 &&
         n->name[name.size()] == '\0';
}

namespace {
// Per-thread memo of (rc, score) per node for the few demands a burst repeats: a flat array
// indexed by node id, valid while the node's generation is the one it was computed at. A
// filter or priorities request over 64 nodes then reads 64 generations and 64 contiguous
// entries instead of probing 64 separately allocated plan-cache tables (~100 ns a node).
// Any node added or removed (the ledger's node epoch) clears it; every other change shows in the
// node's generation, which each entry carries.
struct ScoreMemo {
  uint64_t owner = 0;   // Ledger::instance_ (0: unused)
  uint64_t dh = 0, oh = 0, epoch = 0, used = 0;
  struct E {
    uint64_t gen;   // generation + 1; 0 = empty
    int32_t rc, score;
    ShareMemo sm;   // what re-validates it after the node changed (sm.rc kRevalidateNoMemo: nothing)
  };
  std::vector<E> e;
};
constexpr int kMemoSlots = 16;
thread_local ScoreMemo t_memo[kMemoSlots];
thread_local uint64_t t_memo_clock = 0;

ScoreMemo& memo_for(uint64_t owner, uint64_t dh, uint64_t oh, uint64_t epoch, uint32_t n_nodes) {
  ScoreMemo* lru = &t_memo[0];
  for (ScoreMemo& m : t_memo) {
    if (m.owner == owner && m.dh == dh && m.oh == oh) {
      if (m.epoch != epoch) {
        m.e.assign(n_nodes, ScoreMemo::E{0, 0, 0, ShareMemo{}});
        m.epoch = epoch;
      }
      if (m.e.size() < n_nodes) m.e.resize(n_nodes, ScoreMemo::E{0, 0, 0, ShareMemo{}});
      m.used = ++t_memo_clock;
      return m;
    }
    if (m.used < lru->used) lru = &m;
  }
  lru->owner = owner;
  lru->dh = dh;
  lru->oh = oh;
  lru->epoch = epoch;
  lru->e.assign(n_nodes, ScoreMemo::E{0, 0, 0, ShareMemo{}});
  lru->used = ++t_memo_clock;
  return *lru;
}
}  // namespace

void Ledger::assume_many(const int32_t* ids, int count, const Demand& d, const Options& o_in, int32_t* rc,
                         int32_t* score) {
  const Options o = resolve(o_in, d);
  const uint64_t dh = d.hash(), oh = o.hash();
  const int32_t n_nodes = hdr_->n_nodes.load(std::memory_order_acquire);
  ScoreMemo& memo = memo_for(instance_, dh, oh, hdr_->node_epoch.load(std::memory_order_acquire),
                             static_cast<uint32_t>(std::max(0, n_nodes)));
  Plan plan;
  const bool fast = share_fast_path(d, o, kMaxDevs);
  for (int i = 0; i < count; ++i) {
    const int32_t id = ids[i];
    score[i] = 0;
    // only the dense NodeHot array on a memo hit: the node slot is touched on a miss alone
    if (id < 0 || id >= n_nodes || !hot_[id].in_use.load(std::memory_order_acquire)) {
      rc[i] = kErrUnknownNode;
      continue;
    }
    const uint64_t gen = hot_[id].gen.load(std::memory_order_acquire);
    ScoreMemo::E* me = static_cast<size_t>(id) < memo.e.size() ? &memo.e[id] : nullptr;
    if (me && me->gen == gen + 1) {
      rc[i] = me->rc;
      score[i] = me->score;
      continue;
    }
    const uint64_t io0 = io_t0();
    if (cache_get_score(CacheKey{id, gen, dh, oh}, &rc[i], &score[i])) {
      if (me) *me = ScoreMemo::E{gen + 1, rc[i], score[i], ShareMemo{}};
      io_end(kLedgerCacheHit, io0);
      continue;
    }
    // One share container under native binpack (the common pod): answered in place under the
    // node's lock, no snapshot copy. From an older memo entry and the devices changed since when
    // that decides it (alloc.h revalidate), else by the fast full scan (scan_share: what
    // choose() computes for such a pod).
    if (fast) {
      const uint64_t io1 = io_t0();
      NodeSlot* ns = node(id);
      int32_t r = kRevalidateNo;
      int kind = kLedgerRevalidate;
      uint64_t g = 0, changed;
      ShareMemo next;
      if (ns) {
        lock_node(ns);
        Unlock un{&ns->mu};
        g = gen_of(ns).load(std::memory_order_relaxed);
        if (!ns->in_use) {
          r = kErrUnknownNode;
        } else {
          if (!me || !me->gen || me->sm.rc == kRevalidateNoMemo || me->gen - 1 >= g) io_count(kLedgerMemoCold);
          else if (!changed_since(ns, me->gen - 1, g, &changed)) io_count(kLedgerRingGap);
          else if ((r = revalidate(ns->devs, ns->n_devs, d, o, me->sm, changed, &plan, &next)) == kRevalidateNo)
            io_count(kLedgerRevalUndecided);
          if (r == kRevalidateNo) {
            r = scan_share(ns->devs, ns->n_devs, d, o, &plan, &next);
            kind = kLedgerScan;
          }
        }
      }
      if (r == kErrUnknownNode || !ns) {
        rc[i] = kErrUnknownNode;
        continue;
      }
      if (r != kRevalidateNo) {
        rc[i] = r;
        score[i] = r == kOk ? plan.score : 0;
        cache_put(CacheKey{id, g, dh, oh}, r, plan);
        if (me) *me = ScoreMemo::E{g + 1, r, score[i], next};
        io_end(kind, io1);
        continue;
      }
    }
    IoTimer it{kLedgerChoose};
    NodeSnapshot snap;
    if (!snapshot(id, &snap)) {
      rc[i] = kErrUnknownNode;
      continue;
    }
    rc[i] = choose(snap.devs, snap.n_devs, &snap.topo, d, o, &plan);
    score[i] = rc[i] == kOk ? plan.score : 0;
    cache_put(CacheKey{id, snap.generation, dh, oh}, rc[i], plan);
    if (me) *me = ScoreMemo::E{snap.generation + 1, rc[i], score[i], ShareMemo{}};
  }
}

int32_t Ledger::assume(int32_t id, const Demand& d, const Options& o_in, Plan* plan) {
  // Fast path: the node's generation is read without copying its snapshot; a cached plan
  // for (node, generation, demand, options) is exact for that generation.
  NodeSlot* n = node(id);
  if (!n || !n->in_use) return kErrUnknownNode;
  const Options o = resolve(o_in, d);
  const uint64_t dh = d.hash(), oh = o.hash();
  int32_t rc;
  if (cache_get(CacheKey{id, gen_of(n).load(std::memory_order_acquire), dh, oh}, &rc, plan)) return rc;
  NodeSnapshot snap;
  if (!snapshot(id, &snap)) return kErrUnknownNode;
  rc = choose(snap.devs, snap.n_devs, &snap.topo, d, o, plan);
  cache_put(CacheKey{id, snap.generation, dh, oh}, rc, *plan);
  return rc;
}

namespace {
constexpr int32_t kNominatedElsewhere = -1000;   // internal: release the nomination, retry

// a bind adopted its pod's nomination: every 16th lowers the nomination margin by one
void note_adopted(LedgerHeader* h) {
  if ((h->nom_adopted.fetch_add(1, std::memory_order_relaxed) + 1) % 16 != 0) return;
  int32_t m = h->nom_margin.load(std::memory_order_relaxed);
  while (m > 0 && !h->nom_margin.compare_exchange_weak(m, m - 1, std::memory_order_relaxed)) {
  }
}
}  // namespace

int32_t Ledger::reserve(int32_t id, std::string_view key, const Demand& d, const Options& o,
                        Plan* plan) {
  int32_t rc = reserve_as(id, key, d, o, plan, kPodReserved);
  if (rc == kNominatedElsewhere) {
    // kube-scheduler bound the pod elsewhere than its nomination: nominate less eagerly
    hdr_->nom_moved.fetch_add(1, std::memory_order_relaxed);
    int32_t m = hdr_->nom_margin.load(std::memory_order_relaxed);
    while (m < 40 && !hdr_->nom_margin.compare_exchange_weak(m, std::min(40, m + 2), std::memory_order_relaxed)) {
    }
    release(key);
    rc = reserve_as(id, key, d, o, plan, kPodReserved);
    if (rc == kNominatedElsewhere) rc = kErrPodExists;   // re-nominated concurrently
  }
  return rc;
}

int32_t Ledger::nominate(int32_t id, std::string_view key, const Demand& d, const Options& o) {
  Plan plan;
  int32_t rc = reserve_as(id, key, d, o, &plan, kPodNominated);
  if (rc == kNominatedElsewhere) {
    release(key);
    rc = reserve_as(id, key, d, o, &plan, kPodNominated);
    if (rc == kNominatedElsewhere) rc = kOkExisting;
  }
  return rc;
}

int32_t Ledger::reserve_as(int32_t id, std::string_view key, const Demand& d, const Options& o_in, Plan* plan,
                           int32_t state) {
  NodeSlot* n = node(id);
  const Options o = resolve(o_in, d);
  if (!n || !n->in_use) return kErrUnknownNode;
  if (key.empty() || key.size() >= kKeyLen) return kErrBadDemand;
  const KeyBuf kb(key);
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  if (state == kPodReserved) {
    // A bind adopting its nomination changes the pod's state only, never the node's devices:
    // under the pod shard's lock alone (a pod's state is written under it; release_if re-checks
    // under node + shard lock). The node's lock line then stays with the worker that runs the
    // scheduling cycle instead of moving to whichever worker took the bind.
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = find_pod_locked(s, h, kb.c_str());
    if (p && p->state == kPodNominated && p->node == id) {
      note_adopted(hdr_);
      p->state = state;
      p->t_reserved = mono_now();
      get_record(*p, nullptr, plan);
      return kOk;
    }
  }
  lock_node(n);
  Unlock un{&n->mu};
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = find_pod_locked(s, h, kb.c_str());
    if (p) {
      if (p->state == kPodNominated) {
        if (p->node != id) return kNominatedElsewhere;
        // adopt (bind) or refresh (a repeated priorities call) the nomination
        if (state == kPodReserved) note_adopted(hdr_);
        p->state = state;
        p->t_reserved = mono_now();
        get_record(*p, nullptr, plan);
        return state == kPodReserved ? kOk : kOkExisting;
      }
      if (state == kPodNominated) return kOkExisting;   // already bound or binding
      if (p->node != id) return kErrPodExists;
      get_record(*p, nullptr, plan);
      return kOkExisting;
    }
  }
  const uint64_t gen = gen_of(n).load(std::memory_order_relaxed);
  const CacheKey k{id, gen, d.hash(), o.hash()};
  int32_t rc = kOk;
  const bool hit = cache_get(k, &rc, plan);
  if (!hit) rc = choose(n->devs, n->n_devs, &n->topo, d, o, plan);
  if (rc != kOk) return rc;
  rc = apply(n->devs, n->n_devs, d, *plan);
  if (rc != kOk) return rc;
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = insert_pod_locked(s, h, kb.c_str());
    if (p && !put_record(p, d, *plan)) {
      erase_pod_locked(s, p);       // no overflow record free: give the slot back
      p = nullptr;
    }
    if (!p) {
      unapply(n->devs, n->n_devs, d, *plan);
      return kErrTableFull;
    }
    p->node = id;
    p->t_reserved = mono_now();
    p->owner = 0;
    p->state = state;
  }
  ++n->n_pods;
  bump(n, plan_touch_mask(n->devs, n->n_devs, *plan));
  hdr_->n_pods.fetch_add(1);
  hdr_->epoch.fetch_add(1);
  if (state == kPodNominated) hdr_->nom_made.fetch_add(1, std::memory_order_relaxed);
  note_request(d);
  return kOk;
}

int32_t Ledger::allocate_plan(int32_t id, std::string_view key, const Demand& d,
                              const Plan& plan, bool committed) {
  NodeSlot* n = node(id);
  if (!n || !n->in_use) return kErrUnknownNode;
  if (key.empty() || key.size() >= kKeyLen) return kErrBadDemand;
  {
    // the annotations are the truth: a nomination of ours (maybe another node/plan) yields
    PodRecord r;
    if (lookup(key, &r) && r.state == kPodNominated) release(key);
  }
  const KeyBuf kb(key);
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  lock_node(n);
  Unlock un{&n->mu};
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = find_pod_locked(s, h, kb.c_str());
    if (p) {
      if (p->node != id) return kErrPodExists;
      if (committed) p->state = kPodCommitted;
      return kOk;  // already accounted (reference dealer.go:214-216)
    }
  }
  int32_t rc = apply(n->devs, n->n_devs, d, plan);
  if (rc != kOk) return rc;
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = insert_pod_locked(s, h, kb.c_str());
    if (p && !put_record(p, d, plan)) {
      erase_pod_locked(s, p);
      p = nullptr;
    }
    if (!p) {
      unapply(n->devs, n->n_devs, d, plan);
      return kErrTableFull;
    }
    p->node = id;
    p->t_reserved = mono_now();
    p->owner = 0;
    p->state = committed ? kPodCommitted : kPodReserved;
  }
  ++n->n_pods;
  bump(n, plan_touch_mask(n->devs, n->n_devs, plan));
  hdr_->n_pods.fetch_add(1);
  hdr_->epoch.fetch_add(1);
  note_request(d);
  return kOk;
}

int32_t Ledger::reserve_wide(int32_t id, std::string_view key, const Demand& folded, const Plan& fplan,
                             const WidePlan& wide, bool committed, WidePlan* held) {
  NodeSlot* n = node(id);
  if (!n || !n->in_use) return kErrUnknownNode;
  if (key.empty() || key.size() >= kKeyLen) return kErrBadDemand;
  {
    // the annotations are the truth: a nomination of ours yields (as in allocate_plan)
    PodRecord r;
    if (lookup(key, &r) && r.state == kPodNominated) release(key);
  }
  const KeyBuf kb(key);
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  lock_node(n);
  Unlock un{&n->mu};
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = find_pod_locked(s, h, kb.c_str());
    if (p) {
      if (p->node != id) return kErrPodExists;
      if (committed) p->state = kPodCommitted;
      if (held) get_wide(*p, held);
      return kOkExisting;   // a retried bind, another worker's reservation, an informer replay
    }
  }
  size_t total = 0;
  for (const auto& c : wide) total += c.size();
  if (wide.size() > static_cast<size_t>(kWideContainers) || total > static_cast<size_t>(kWideIdx)) return kErrBadDemand;
  int32_t rc = apply(n->devs, n->n_devs, folded, fplan);
  if (rc != kOk) return rc;
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = insert_pod_locked(s, h, kb.c_str());
    if (p && (!put_record(p, folded, fplan) || !put_wide(p, wide))) {
      free_record(p);
      erase_pod_locked(s, p);
      p = nullptr;
    }
    if (!p) {
      unapply(n->devs, n->n_devs, folded, fplan);
      return kErrTableFull;
    }
    p->node = id;
    p->t_reserved = mono_now();
    p->owner = 0;
    p->state = committed ? kPodCommitted : kPodReserved;
  }
  ++n->n_pods;
  bump(n, plan_touch_mask(n->devs, n->n_devs, fplan));
  hdr_->n_pods.fetch_add(1);
  hdr_->epoch.fetch_add(1);
  note_request(folded);
  return kOk;
}

bool Ledger::wide_plan(std::string_view key, WidePlan* out) const {
  if (key.empty() || key.size() >= kKeyLen) return false;
  const KeyBuf kb(key);
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  lock_mu(&hdr_->shard_mu[s].m);
  Unlock us{&hdr_->shard_mu[s].m};
  const PodSlot* p = find_pod_locked(s, h, kb.c_str());
  if (!p || p->wide <= 0) return false;
  get_wide(*p, out);
  return true;
}

int32_t Ledger::commit(std::string_view key) {
  const KeyBuf kb(key);
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  lock_mu(&hdr_->shard_mu[s].m);
  Unlock us{&hdr_->shard_mu[s].m};
  PodSlot* p = find_pod_locked(s, h, kb.c_str());
  if (!p) return kErrUnknownPod;
  p->state = kPodCommitted;
  return kOk;
}

int32_t Ledger::release(std::string_view key) { return release_if(key, -1); }

int32_t Ledger::drop_nomination(std::string_view key) { return release_if(key, kPodNominated); }

bool Ledger::wait_deferred_nominations(uint64_t max_ns) const {
  if (hdr_->nom_deferred_done.load(std::memory_order_acquire) ==
      hdr_->nom_deferred_begun.load(std::memory_order_acquire))
    return true;
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::nanoseconds(max_ns);
  for (;;) {
    for (int k = 0; k < 32; ++k) __builtin_ia32_pause();
    if (hdr_->nom_deferred_done.load(std::memory_order_acquire) >=
        hdr_->nom_deferred_begun.load(std::memory_order_acquire))
      return true;
    if (std::chrono::steady_clock::now() > t_end) return false;
  }
}

int32_t Ledger::drop_reservation(std::string_view key) { return release_if(key, kPodReserved); }

int32_t Ledger::release_if(std::string_view key, int32_t only_state) {
  const KeyBuf kb(key);
  const bool only = only_state >= 0;
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  int32_t id;
  {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* p = find_pod_locked(s, h, kb.c_str());
    if (!p) return kErrUnknownPod;
    if (only && p->state != only_state) return kOkExisting;
    id = p->node;
  }
  NodeSlot* n = node(id);
  if (!n) return kErrUnknownNode;
  lock_node(n);
  Unlock un{&n->mu};
  lock_mu(&hdr_->shard_mu[s].m);
  Unlock us{&hdr_->shard_mu[s].m};
  PodSlot* p = find_pod_locked(s, h, kb.c_str());
  if (!p || p->node != id) return kErrUnknownPod;  // raced with another release
  if (only && p->state != only_state) return kOkExisting;   // adopted / committed meanwhile
  uint64_t touched;
  {
    Demand pd;
    Plan pp;
    get_record(*p, &pd, &pp);
    unapply(n->devs, n->n_devs, pd, pp);
    touched = plan_touch_mask(n->devs, n->n_devs, pp);
  }
  free_record(p);
  erase_pod_locked(s, p);
  --n->n_pods;
  bump(n, touched);
  hdr_->n_pods.fetch_sub(1);
  hdr_->epoch.fetch_add(1);
  return kOk;
}

bool Ledger::holds(std::string_view key) const {
  if (key.empty() || key.size() >= kKeyLen) return false;
  uint64_t h = 0xcbf29ce484222325ULL;   // key_hash over the view's bytes
  for (const char c : key) {
    if (c == '\0') return false;
    h ^= static_cast<unsigned char>(c);
    h *= 0x100000001b3ULL;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  const int s = shard_of(h);
  lock_mu(&hdr_->shard_mu[s].m);
  Unlock us{&hdr_->shard_mu[s].m};
  const PodSlot* t = shard(s);
  const uint32_t cap = hdr_->pods_per_shard;
  uint32_t i = static_cast<uint32_t>((h / kPodShards) % cap);
  for (uint32_t probe = 0; probe < cap; ++probe, i = (i + 1) % cap) {
    const PodSlot& p = t[i];
    if (p.state == kPodEmpty) return false;
    if (p.state != kPodTombstone && p.hash == h && std::memcmp(p.key, key.data(), key.size()) == 0 &&
        p.key[key.size()] == '\0')
      return true;
  }
  return false;
}

bool Ledger::lookup(std::string_view key, PodRecord* out) const {
  const KeyBuf kb(key);
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  lock_mu(&hdr_->shard_mu[s].m);
  Unlock us{&hdr_->shard_mu[s].m};
  PodSlot* p = find_pod_locked(s, h, kb.c_str());
  if (!p) return false;
  out->key = p->key;
  out->node = p->node;
  out->state = p->state;
  out->t_reserved = p->t_reserved;
  get_record(*p, &out->demand, &out->plan);
  out->owner = p->owner;
  return true;
}

int32_t Ledger::set_pod_owner(std::string_view key, uint64_t owner) {
  const KeyBuf kb(key);
  if (key.empty() || key.size() >= kKeyLen) return kErrUnknownPod;
  const uint64_t h = key_hash(kb.c_str());
  const int s = shard_of(h);
  lock_mu(&hdr_->shard_mu[s].m);
  Unlock us{&hdr_->shard_mu[s].m};
  PodSlot* p = find_pod_locked(s, h, kb.c_str());
  if (!p) return kErrUnknownPod;
  p->owner = owner;
  return kOk;
}

static float curve_at(const std::vector<std::pair<float, float>>& c, float x) {
  if (x <= c.front().first) return c.front().second;
  if (x >= c.back().first) return c.back().second;
  for (size_t i = 1; i < c.size(); ++i)
    if (x <= c[i].first) {
      const auto& [x0, y0] = c[i - 1];
      const auto& [x1, y1] = c[i];
      return x1 > x0 ? y0 + (y1 - y0) * (x - x0) / (x1 - x0) : y1;
    }
  return c.back().second;
}

std::pair<int32_t, int32_t> Ledger::learn_stream_owners(bool forget_cool, double reserved_before,
                                                        int32_t forget_after,
                                                        const std::vector<std::pair<float, float>>& hot_curve) {
  // (node, device) -> tenant pods, and the owner / record time / share of the last one seen
  struct Tenancy {
    int32_t pods = 0;
    uint64_t owner = 0;
    double t = 0;
    int32_t share = 0;   // percent of the device the last pod holds there
  };
  std::unordered_map<uint64_t, Tenancy> dev;
  for (int s = 0; s < kPodShards; ++s) {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    const PodSlot* t = shard(s);
    for (uint32_t i = 0; i < hdr_->pods_per_shard; ++i) {
      const PodSlot& p = t[i];
      if (p.state != kPodCommitted || p.node < 0) continue;
      int16_t seen[kMaxPlanIdx];
      int32_t share[kMaxPlanIdx];
      int n_seen = 0;
      Demand dm;
      Plan pl;
      get_record(p, &dm, &pl);
      for (int c = 0; c < pl.n && c < dm.n; ++c) {
        // a share container takes its percent of one device; a whole-device one all of each
        const int32_t s = std::min(dm.c[c].pct, kPercentPerDevice);
        for (int k = pl.off[c]; k < pl.off[c + 1] && k < kMaxPlanIdx; ++k) {
          const int16_t x = pl.idx[k];
          if (x < 0) continue;
          int16_t* at = std::find(seen, seen + n_seen, x);
          if (at != seen + n_seen) {
            share[at - seen] = std::min(kPercentPerDevice, share[at - seen] + s);
            continue;
          }
          share[n_seen] = s;
          seen[n_seen++] = x;
        }
      }
      for (int k = 0; k < n_seen; ++k) {
        Tenancy& te = dev[(static_cast<uint64_t>(p.node) << 16) | static_cast<uint16_t>(seen[k])];
        ++te.pods;
        te.owner = p.owner;
        te.t = p.t_reserved;
        te.share = share[k];
      }
    }
  }
  // per owner: any lone replica on a hot device / any on a cool one (a decision per owner, not
  // per device, so one replica on a hot and one on a cool device cannot flip it back and forth)
  struct Verdict {
    bool hot = false, cool = false;
  };
  std::unordered_map<uint64_t, Verdict> owners;
  for (const auto& [key, te] : dev) {
    if (te.pods != 1 || te.owner == 0 || te.t > reserved_before) continue;
    const int32_t id = static_cast<int32_t>(key >> 16);
    const int x = static_cast<int>(key & 0xffff);
    NodeSlot* n = node(id);
    if (!n) continue;
    bool hot;
    {
      lock_node(n);
      Unlock un{&n->mu};
      if (x >= n->n_devs) continue;
      hot = hot_curve.empty() ? n->devs[x].mem_hot != 0
                              : n->devs[x].mem_busy >= curve_at(hot_curve, static_cast<float>(te.share));
    }
    Verdict& v = owners[te.owner];
    (hot ? v.hot : v.cool) = true;
  }
  int32_t learned = 0, forgotten = 0;
  std::lock_guard<std::mutex> g(learn_mu_);
  for (const auto& [owner, v] : owners) {
    if (v.hot) {
      cool_streak_.erase(owner);
      if (!is_stream_owner(owner)) {
        set_stream_owner(owner, true);
        ++learned;
      }
    } else if (forget_cool && is_stream_owner(owner)) {
      if (++cool_streak_[owner] >= std::max(1, forget_after)) {
        cool_streak_.erase(owner);
        set_stream_owner(owner, false);
        ++forgotten;
      }
    }
  }
  // an owner with no lone replica this pass keeps its streak where it was; owners no longer
  // learned drop out of the map
  for (auto it = cool_streak_.begin(); it != cool_streak_.end();)
    it = is_stream_owner(it->first) ? std::next(it) : cool_streak_.erase(it);
  return {learned, forgotten};
}

int32_t Ledger::fits_without(int32_t id, const std::vector<std::string>& victims, const Demand& d,
                             const Options& o, Plan* plan) const {
  NodeSnapshot snap;
  if (!snapshot(id, &snap)) return kErrUnknownNode;
  // take the victims' shares back on a copy of the node (a victim the ledger does not hold,
  // or holds on another node, frees nothing here)
  for (const std::string& key : victims) {
    if (key.empty() || key.size() >= kKeyLen) continue;
    const KeyBuf kb(key);
    const uint64_t h = key_hash(kb.c_str());
    const int s = shard_of(h);
    Demand vd;
    Plan vp;
    {
      lock_mu(&hdr_->shard_mu[s].m);
      Unlock us{&hdr_->shard_mu[s].m};
      const PodSlot* p = find_pod_locked(s, h, kb.c_str());
      if (!p || p->node != id) continue;
      get_record(*p, &vd, &vp);
    }
    unapply(snap.devs, snap.n_devs, vd, vp);
  }
  const Options ro = resolve(o, d);
  return choose(snap.devs, snap.n_devs, &snap.topo, d, ro, plan);
}

std::vector<PodRecord> Ledger::pods_on(int32_t node_id) const {
  std::vector<PodRecord> out;
  for (int s = 0; s < kPodShards; ++s) {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* t = shard(s);
    for (uint32_t i = 0; i < hdr_->pods_per_shard; ++i) {
      const PodSlot& p = t[i];
      if ((p.state == kPodReserved || p.state == kPodCommitted || p.state == kPodNominated) &&
          (node_id < 0 || p.node == node_id))
      {
        PodRecord r{p.key, p.node, p.state, p.t_reserved, {}, {}, p.owner};
        get_record(p, &r.demand, &r.plan);
        out.push_back(std::move(r));
      }
    }
  }
  return out;
}

std::vector<std::string> Ledger::expired(int32_t state, double older_than_s) const {
  std::vector<std::string> out;
  const double now = mono_now();
  for (int s = 0; s < kPodShards; ++s) {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    PodSlot* t = shard(s);
    for (uint32_t i = 0; i < hdr_->pods_per_shard; ++i)
      if (t[i].state == state && now - t[i].t_reserved > older_than_s) out.emplace_back(t[i].key);
  }
  return out;
}

std::vector<std::string> Ledger::expired_reservations(double older_than_s) const {
  return expired(kPodReserved, older_than_s);
}

int32_t Ledger::drop_committed(std::string_view key) { return release_if(key, kPodCommitted); }

std::vector<std::string> Ledger::reconcile(const std::vector<std::string>& live, double before) {
  std::vector<std::string_view> v(live.begin(), live.end());
  return reconcile_views(v, before);
}

// Cost at 100k listed pods: one hash set of the views, one pass over every pod slot with each
// shard's lock held for that shard's slots only (a reserve waits for at most one shard's pass),
// then the releases one by one (native/tests/stress_main.cpp relist_scale pins both).
std::vector<std::string> Ledger::reconcile_views(const std::vector<std::string_view>& live, double before) {
  // the listed keys in a flat open-addressing table keyed by the hash every pod slot already
  // stores (key_hash): one probe per committed slot, the key bytes compared only on a match
  size_t cap = 64;
  while (cap < live.size() * 2) cap <<= 1;
  std::vector<uint64_t> th(cap, 0);
  std::vector<uint32_t> ti(cap, 0);
  for (size_t i = 0; i < live.size(); ++i) {
    const std::string_view k = live[i];
    uint64_t h = 0xcbf29ce484222325ULL;   // key_hash over the view's bytes
    for (const unsigned char c : k) {
      h ^= c;
      h *= 0x100000001b3ULL;
    }
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33;
    h |= 1;   // 0 marks an empty cell
    size_t j = h & (cap - 1);
    while (th[j]) j = (j + 1) & (cap - 1);
    th[j] = h;
    ti[j] = static_cast<uint32_t>(i);
  }
  auto listed = [&](const PodSlot& p) {
    const uint64_t h = p.hash | 1;
    for (size_t j = h & (cap - 1); th[j]; j = (j + 1) & (cap - 1))
      if (th[j] == h && live[ti[j]] == std::string_view(p.key)) return true;
    return false;
  };
  std::vector<std::string> gone;
  for (int s = 0; s < kPodShards; ++s) {
    lock_mu(&hdr_->shard_mu[s].m);
    Unlock us{&hdr_->shard_mu[s].m};
    const PodSlot* t = shard(s);
    for (uint32_t i = 0; i < hdr_->pods_per_shard; ++i) {
      const PodSlot& p = t[i];
      if (p.state == kPodCommitted && p.t_reserved < before && !listed(p)) gone.emplace_back(p.key);
    }
  }
  std::vector<std::string> released;
  for (const std::string& k : gone)
    if (drop_committed(k) == kOk) released.push_back(k);
  return released;
}

bool Ledger::put_pod_info(std::string_view key, std::string_view blob) {
  const KeyBuf kb(key);
  if (key.empty() || key.size() >= static_cast<size_t>(kKeyLen) || blob.size() > static_cast<size_t>(kPodInfoBytes))
    return false;
  const uint64_t h = key_hash(kb.c_str());
  const uint32_t bucket = static_cast<uint32_t>(h % (hdr_->info_cap / kPodInfoWays));
  lock_mu(&hdr_->info_mu[bucket % kPodShards].m);
  Unlock u{&hdr_->info_mu[bucket % kPodShards].m};
  PodInfoSlot* b = &info_[bucket * kPodInfoWays];
  PodInfoSlot* s = nullptr;
  for (int w = 0; w < kPodInfoWays && !s; ++w)   // the key's own slot, else an empty one
    if (b[w].hash == h && std::strncmp(b[w].key, kb.c_str(), kKeyLen) == 0) s = &b[w];
  for (int w = 0; w < kPodInfoWays && !s; ++w)
    if (b[w].hash == 0) s = &b[w];
  if (!s) {   // a full bucket: the oldest entry goes
    s = &b[0];
    for (int w = 1; w < kPodInfoWays; ++w)
      if (b[w].stamp < s->stamp) s = &b[w];
  }
  s->hash = h;
  s->stamp = hdr_->info_stamp.fetch_add(1, std::memory_order_relaxed) + 1;
  std::memcpy(s->key, kb.c_str(), key.size() + 1);
  s->len = static_cast<uint32_t>(blob.size());
  std::memcpy(s->data, blob.data(), blob.size());
  return true;
}

bool Ledger::take_pod_info(std::string_view key, std::string* blob) {
  const KeyBuf kb(key);
  if (key.empty() || key.size() >= static_cast<size_t>(kKeyLen)) return false;
  const uint64_t h = key_hash(kb.c_str());
  const uint32_t bucket = static_cast<uint32_t>(h % (hdr_->info_cap / kPodInfoWays));
  lock_mu(&hdr_->info_mu[bucket % kPodShards].m);
  Unlock u{&hdr_->info_mu[bucket % kPodShards].m};
  PodInfoSlot* b = &info_[bucket * kPodInfoWays];
  for (int w = 0; w < kPodInfoWays; ++w) {
    PodInfoSlot& s = b[w];
    if (s.hash != h || std::strncmp(s.key, kb.c_str(), kKeyLen) != 0) continue;
    blob->assign(s.data, std::min<uint32_t>(s.len, kPodInfoBytes));
    s.hash = 0;
    return true;
  }
  return false;
}

std::vector<std::string> Ledger::expired_nominations(double older_than_s) const {
  return expired(kPodNominated, older_than_s);
}

int32_t Ledger::set_load(int32_t id, int dev, float usage) {
  NodeSlot* n = node(id);
  if (!n) return kErrUnknownNode;
  lock_node(n);
  Unlock un{&n->mu};
  if (dev < 0 || dev >= n->n_devs) return kErrBadPlan;
  Device& d = n->devs[dev];
  d.load_usage = usage;
  d.remain_load = static_cast<int16_t>(kLoadTotal - static_cast<int>(usage));
  bump(n, 1ull << dev);
  hdr_->epoch.fetch_add(1);
  return kOk;
}

int32_t Ledger::set_mem_busy(int32_t id, int dev, int32_t percent) {
  NodeSlot* n = node(id);
  if (!n) return kErrUnknownNode;
  lock_node(n);
  Unlock un{&n->mu};
  if (dev < 0 || dev >= n->n_devs) return kErrBadPlan;
  n->devs[dev].mem_busy = static_cast<int16_t>(std::clamp(percent, 0, 100));
  return kOk;   // read by the learner only: no generation bump, cached plans stay valid
}

int32_t Ledger::set_mem_hot(int32_t id, int dev, bool hot) {
  NodeSlot* n = node(id);
  if (!n) return kErrUnknownNode;
  lock_node(n);
  Unlock un{&n->mu};
  if (dev < 0 || dev >= n->n_devs) return kErrBadPlan;
  Device& d = n->devs[dev];
  if ((d.mem_hot != 0) == hot) return kOk;   // unchanged: cached plans stay valid
  d.mem_hot = hot ? 1 : 0;
  bump(n, 1ull << dev);
  hdr_->epoch.fetch_add(1);
  return kOk;
}

int32_t Ledger::set_health(int32_t id, int dev, bool healthy) {
  NodeSlot* n = node(id);
  if (!n) return kErrUnknownNode;
  lock_node(n);
  Unlock un{&n->mu};
  if (dev < 0 || dev >= n->n_devs) return kErrBadPlan;
  n->devs[dev].healthy = healthy ? 1 : 0;
  bump(n, 1ull << dev);
  hdr_->epoch.fetch_add(1);
  return kOk;
}

FragStats Ledger::frag(int32_t min_request) const {
  FragStats s{};
  const int32_t count = n_nodes();
  for (int32_t i = 0; i < count; ++i) {
    NodeSlot* n = &nodes_[i];
    if (!n->in_use) continue;
    lock_node(n);
    Unlock un{&n->mu};
    frag_accumulate(n->devs, n->n_devs, min_request, &s);
  }
  return s;
}

namespace {
constexpr uint32_t kSizeDecayAt = 4096;   // halve the counts when they reach this many
inline bool size_common(uint32_t cnt, uint32_t total) { return cnt * 50u >= total && cnt > 0; }
inline bool size_rare(uint32_t cnt, uint32_t total) { return cnt * 100u < total; }
}  // namespace

uint64_t owner_hash(std::string_view uid) {
  uint64_t h = 0xcbf29ce484222325ULL;   // FNV-1a
  for (unsigned char c : uid) h = (h ^ c) * 0x100000001b3ULL;
  return h ? h : 1;
}

void Ledger::set_stream_owner(uint64_t owner, bool streaming) {
  std::atomic<uint64_t>& slot = hdr_->stream_owner[owner % kStreamOwners];
  if (streaming) {
    slot.store(owner, std::memory_order_relaxed);
  } else {
    uint64_t cur = owner;
    slot.compare_exchange_strong(cur, 0, std::memory_order_relaxed);
  }
}

bool Ledger::is_stream_owner(uint64_t owner) const {
  return hdr_->stream_owner[owner % kStreamOwners].load(std::memory_order_relaxed) == owner;
}

void Ledger::note_request(const Demand& d) {
  for (int c = 0; c < d.n; ++c) {
    const int s = d.c[c].pct;
    if (s <= 0 || s > kPercentPerDevice) continue;
    const uint32_t cnt = hdr_->size_hist[s].fetch_add(1, kRlx) + 1;
    uint32_t total = hdr_->size_total.fetch_add(1, kRlx) + 1;
    if (total >= kSizeDecayAt) {
      // one process wins the halving; counts racing with it are off by a request or two
      if (hdr_->size_total.compare_exchange_strong(total, total / 2, kRlx)) {
        uint64_t bits[2] = {0, 0};
        for (int q = 1; q <= kPercentPerDevice; ++q) {
          const uint32_t h = hdr_->size_hist[q].load(kRlx) / 2;
          hdr_->size_hist[q].store(h, kRlx);
          const bool was = (hdr_->size_bits[q >> 6].load(kRlx) >> (q & 63)) & 1u;
          if (size_common(h, total / 2) || (was && !size_rare(h, total / 2))) bits[q >> 6] |= 1ULL << (q & 63);
        }
        hdr_->size_bits[0].store(bits[0], std::memory_order_release);
        hdr_->size_bits[1].store(bits[1], std::memory_order_release);
      }
      continue;
    }
    if (size_common(cnt, total)) hdr_->size_bits[s >> 6].fetch_or(1ULL << (s & 63), std::memory_order_release);
  }
}

SizeSet Ledger::learned_sizes() const {
  SizeSet s;
  s.bits[0] = hdr_->size_bits[0].load(std::memory_order_acquire);
  s.bits[1] = hdr_->size_bits[1].load(std::memory_order_acquire);
  // sizes that went rare since they were set (no decay pass yet) are dropped on read
  const uint32_t total = hdr_->size_total.load(kRlx);
  for (int w = 0; w < 2; ++w)
    for (uint64_t b = s.bits[w]; b; b &= b - 1) {
      const int q = w * 64 + __builtin_ctzll(b);
      if (q > kPercentPerDevice || size_rare(hdr_->size_hist[q].load(kRlx), total)) s.bits[w] &= ~(1ULL << (q & 63));
    }
  return s;
}

Options Ledger::resolve(const Options& o, const Demand& d) const {
  if (o.compat || o.policy != Policy::kBinpack) return o;
  SizeSet s = o.sizes;
  if (o.learn_sizes) {
    const SizeSet l = learned_sizes();
    s.bits[0] |= l.bits[0];
    s.bits[1] |= l.bits[1];
  }
  for (int c = 0; c < d.n; ++c) s.add(d.c[c].pct);
  if (s.empty()) return o;
  // the knapsack table costs ~5k operations: keep the last one per thread
  thread_local SizeSet last_set;
  thread_local uint8_t last_waste[kWasteSlots];
  thread_local bool have = false;
  Options r = o;
  if (have && last_set == s) {
    r.sizes = s;
    std::memcpy(r.waste, last_waste, sizeof(last_waste));
    return r;
  }
  r.set_sizes(s);
  last_set = s;
  std::memcpy(last_waste, r.waste, sizeof(last_waste));
  have = true;
  return r;
}

void Ledger::clear_cache() {
  for (uint32_t i = 0; i < cache_nodes_; ++i) {
    NodeCache* cp = node_cache(static_cast<int32_t>(i), false);
    if (!cp) continue;
    NodeCache& c = *cp;
    c.lock();
    const uint32_t sq = c.seq.load(kRlx);
    c.seq.store(sq + 1, kRlx);
    std::atomic_thread_fence(std::memory_order_release);
    for (auto& e : c.e) e.used.store(false, kRlx);
    c.seq.store(sq + 2, std::memory_order_release);
    c.unlock();
  }
}

size_t Ledger::cache_size() const {
  size_t n = 0;
  for (uint32_t i = 0; i < cache_nodes_; ++i) {
    NodeCache* cp = node_cache(static_cast<int32_t>(i), false);
    if (!cp) continue;
    NodeCache& c = *cp;
    c.lock();
    for (const auto& e : c.e) n += e.used.load(kRlx);
    c.unlock();
  }
  return n;
}

}  // namespace nanogpu
