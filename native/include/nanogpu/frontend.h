// Native HTTP front door of the extender: kube-scheduler's filter / priorities verbs are
// answered entirely in C++ (epoll workers, no GIL, no Python objects), everything else
// (bind, /status, /metrics, /debug/*, and any request the fast path declines) is handed
// to the Python asyncio runtime through a queue + eventfd and answered when it responds.
//
// Reference: pkg/routes/routes.go:40-122 (filter / prioritize routes) with the verbs of
// pkg/scheduler/predicate.go:19-41 and priority.go:19-42 over dealer.go:89-153. The
// reference serves every verb through net/http goroutines that all contend on the
// dealer's one mutex; here N SO_REUSEPORT workers each own their connections and read
// the ledger through per-node snapshots and its (node, generation)-keyed plan cache.
// Responses are byte-identical to the Python verbs (nanogpu/extender/verbs.py), which
// remain the fallback and the reference implementation for the tests.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "nanogpu/bindhops.h"
#include "nanogpu/iotally.h"
#include "nanogpu/alloc.h"
#include "nanogpu/kubewriter.h"
#include "nanogpu/ledger.h"

namespace nanogpu {

// Kubernetes resource.Quantity -> int64 rounded up (Quantity.Value()); false if invalid
// or out of range. `mib` = memory semantics: a bare integer is MiB, anything else is
// bytes rounded up to MiB (nanogpu/k8s/quantity.py::quantity_to_mib).
bool quantity_value(std::string_view s, bool mib, int64_t* out);

// Bind whose ledger half ran natively: the pod was seen by filter/prioritize, its demand
// reserved on the ledger here; Python only performs the API writes and commits or rolls back.
struct PreparedBind {
  bool ok = false;                 // false: Python runs the whole bind (pod_json if cached)
  int32_t rc = 0;                  // ledger reserve result (kOk, kOkExisting or an error)
  std::string ns, name, uid, node;
  std::vector<std::string> containers;
  std::vector<std::vector<int32_t>> plan;
  std::vector<std::pair<int32_t, int64_t>> demand;
};

struct PyRequest {
  uint64_t id;
  std::string method, path, query, body;
  std::string pod_json;   // bind: the Pod seen by filter/prioritize for this UID ("" if none)
  PreparedBind bind;
  double t_arrival;
};

struct CachedPod {
  std::string raw, ns, name;
  std::vector<std::string> containers;
  Demand demand;
  bool completed = false;
  uint64_t owner = 0;   // owner_hash of the controlling owner's UID, 0: none
};

struct VerbStats {
  std::atomic<uint64_t> count{0}, errors{0}, deferred{0};
  std::atomic<uint64_t> ns_total{0};
  std::atomic<uint64_t> max_ns{0};     // slowest observation since the last reset_max()
  std::atomic<uint64_t> buckets[16];   // latency histogram, bucket k: < 2^k * 8 us
  VerbStats() {
    for (auto& b : buckets) b.store(0);
  }
  void observe(uint64_t ns);
};

// Grows this process's file-descriptor table to `want` slots (capped by RLIMIT_NOFILE) up
// front. The kernel grows the table by doubling when an fd past its end is allocated, and in
// a multi-threaded process each growth waits for an RCU grace period: on the 256-CPU MI355X
// host that froze a front-door worker inside accept4() for 110-130 ms whenever a burst of new
// connections crossed a power of two. Tables never shrink, so paying it once at start-up
// removes the stall. Returns the number of slots now available (0 if nothing was done).
int presize_fd_table(int want = 16384);

class Frontend {
 public:
  Frontend(std::shared_ptr<Ledger> ledger, const std::string& host, int port, int threads);
  ~Frontend();
  Frontend(const Frontend&) = delete;
  Frontend& operator=(const Frontend&) = delete;

  int port() const { return port_; }
  int notify_fd() const { return py_efd_; }
  // nominate: priorities tentatively reserve the pod on its unique top-scored node
  // (Ledger::nominate) so the next pods' filters see it before the bind arrives.
  // decisive: filter answers the one node priorities would rank first (ties broken by the pod's
  // UID hash, as priorities breaks them) and nominates it; kube-scheduler skips scoring for a
  // single feasible node, so a pod's cycle is one round trip (off: the reference's filter)
  void set_options(const Options& o, bool score_normalize, bool nominate = false, bool decisive = false,
                   int32_t lead = 0);
  // false: every request goes to Python (a standby replica answers 503 from there).
  void set_serving(bool on) { serving_.store(on, std::memory_order_release); }
  // this process's switch AND the replica's shared flag in the ledger (leader election runs
  // in one worker; every worker's front door follows it)
  bool serving() const { return serving_.load(std::memory_order_acquire) && ledger_->serving(); }
  // After any event a worker keeps polling (epoll timeout 0) for this long before it
  // blocks again: trades a little CPU during bursts for no wake-up latency per request.
  void set_busy_poll_us(int us) { busy_poll_ns_.store(static_cast<int64_t>(us) * 1000, std::memory_order_relaxed); }
  // the window after a priorities answer (kube-scheduler then picks the host, sends the bind and
  // builds the next pod's filter: a longer gap than after a filter answer); < 0: the same window
  void set_busy_poll_prio_us(int us) { busy_poll_prio_ns_.store(us < 0 ? -1 : static_cast<int64_t>(us) * 1000, std::memory_order_relaxed); }
  // Binds read in the same batch as a filter / priorities request are reserved first (placement
  // quality: the next pod's filter sees the pod just bound) instead of after (cycle latency).
  void set_bind_first(bool on) { bind_first_.store(on, std::memory_order_relaxed); }
  // The busy-poll window is slept (epoll_pwait2 with a microsecond timeout) instead of polled.
  void set_spin_nap(bool on) { spin_nap_.store(on, std::memory_order_relaxed); }
  // busy poll: probe the connection the last cycle answer went out on with a non-blocking
  // recv before each epoll_wait(0) (the request that follows usually comes back on it;
  // profiles/ab_results_r04.md r04sr: +6 % pods/s, -1.3 us a pod). Off while binds go first.
  void set_spin_recv(bool on) { spin_recv_.store(on, std::memory_order_relaxed); }
  // ... and, when that finds nothing, the connection the last bind answer went out on
  void set_spin_recv_binds(bool on) { spin_recv_binds_.store(on, std::memory_order_relaxed); }
  // Drains requests waiting for Python (non-blocking).
  std::vector<PyRequest> take();
  // Completes request `id` (any thread). Unknown ids (connection gone) are dropped.
  // notify=false queues the response without waking its worker: the caller batches
  // several and wakes each worker once with wake_workers().
  void respond(uint64_t id, int status, const std::string& content_type, const std::string& body,
               bool notify = true);
  void wake_workers();
  void stop();
  // Native bind writes: from now on a bind whose reservation succeeded here is finished by
  // KubeWriter threads (PATCH + binding + commit / rollback) without Python. Set once.
  // `inline_io`: each worker drives the API requests of the binds it parsed from its own epoll
  // loop and answers them itself (BindIo, bindio.h); else the writer's own io thread does.
  void set_kube_writer(const KubeTarget& t, int threads, int retries, bool record_events,
                       bool evented = true, bool label = true, double timeout_s = 30.0, bool inline_io = false,
                       bool batch_labels = false, int max_binds = 0);
  const KubeWriter* kube_writer() const { return writer_.load(std::memory_order_acquire); }
  // evented writer: workers send each bind's requests themselves (KubeWriter::send_from_caller)
  void set_fe_send(bool on) {
    if (KubeWriter* w = writer_.load(std::memory_order_acquire)) w->set_fe_send(on);
  }
  void set_lazy_labels(bool on) {
    if (KubeWriter* w = writer_.load(std::memory_order_acquire)) w->set_lazy_labels(on);
  }
  // The native filter / priorities verb on a request body (what a worker runs per request);
  // false = the request needs the Python path.
  bool filter_verb(std::string_view body, bool prioritize, std::string* out);
  struct VerbScratch;   // a worker's per-request scratch (frontend.cpp)
  bool filter_verb(std::string_view body, bool prioritize, std::string* out, VerbScratch& s);

  VerbStats filter_stats, prio_stats, py_stats, bind_stats;   // bind_stats: native reserve half
  // a native verb's residence: first request byte read -> whole answer handed to the kernel
  VerbStats filter_wall_stats, prio_wall_stats;
  std::atomic<uint64_t> connections{0}, requests{0};
  std::atomic<uint64_t> spin_hits{0};     // event batches a busy-polling worker caught
  std::atomic<uint64_t> mb_wakeups{0};    // posted responses that had to wake a parked worker
  // binds this process answered natively with a pod another worker process's filter parsed
  // (Ledger::take_pod_info), and pods it handed to the other workers that way
  std::atomic<uint64_t> bind_handoffs{0}, pods_published{0};
  // binds whose pod another worker had not published yet when they came (they waited for it)
  std::atomic<uint64_t> handoff_waits{0};
  static constexpr uint64_t kHandoffWaitNs = 200'000;
  static constexpr uint64_t kDeferredNominationWaitNs = 100'000;
  std::atomic<uint64_t> loop_max_ns{0};   // longest event-batch a worker spent between epoll_waits
  // longest single step of a batch: 0 accept, 1 mailbox, 2 read+cycle verbs, 3 deferred binds,
  // 4 pod-cache lock wait (bind), 5 node lookup (bind), 6 Python hand-off (defer)
  std::atomic<uint64_t> phase_max_ns[7] = {};
  void reset_max();
  size_t pod_cache_size() const;
  // Extender-side wall time of each POST /scheduler/bind answered since the last call: from
  // the first request bytes read to the response handed to the kernel (BASELINE's "p50 bind
  // latency"). Bounded at kMaxWallSamples between calls.
  std::vector<uint64_t> take_bind_wall();
  static constexpr size_t kMaxWallSamples = 1u << 20;
  // Per-hop split of the native binds answered since the last call (bindhops.h), each the seven
  // durations in ns between its eight stamps: parse+reserve, hand-off to the writer, wait for the
  // admission window, build+send, API answer, commit+post, reply. Recorded only while switched on (off by default; false
  // when this host has no invariant TSC to stamp with).
  bool set_bind_hops(bool on);
  std::vector<std::array<uint32_t, kHopSplits>> take_bind_hops();
  // how many of each are waiting to be taken (a marker between steps, no copy)
  std::pair<size_t, size_t> bind_samples_waiting();

 private:
  struct Conn;
  struct Worker;
  void run(Worker* w);
  bool read_in(Worker* w, Conn* c, bool* eof);      // false: connection closed
  void after_read(Worker* w, Conn* c, bool eof);    // parse + answer what is buffered
  bool spin_recv_hot(Worker* w);                     // true: a request was read and handled
  bool spin_recv_conn(Worker* w, uint64_t cid);
  void process(Worker* w, Conn* c);
  // the verb's whole HTTP answer appended to *out (false: not a native verb, nothing written)
  bool handle_native(Worker* w, Conn* c, std::string_view method, std::string_view path, std::string_view body,
                     std::string* out);
  void defer(Worker* w, Conn* c, std::string method, std::string path, std::string query, std::string body);
  void flush(Worker* w, Conn* c, int io_kind = kFeSendOther);
  void close_conn(Worker* w, Conn* c);
  void put_pod(std::string_view uid, const CachedPod& meta, std::string_view raw, const Demand& dem);
  bool has_pod(std::string_view uid) const;
  void prepare_bind(std::string_view body, PyRequest* r, VerbScratch& s);
  void cache_pod(VerbScratch& s, std::string_view uid, const CachedPod& cached, std::string_view raw, const Demand& dem);
  void run_deferred(VerbScratch& s);   // a worker verb's work left for after its answer went out
  // a nomination may wait until after the answer with one worker thread (this worker reads
  // nothing in between). kube-scheduler's next filter may reach another worker process: the
  // ledger counts the deferred nominations, and that filter waits until they are made
  // (Ledger::wait_deferred_nominations), so it never sees the ledger without this pod's devices
  bool defer_nominate_ok(const VerbScratch& s) const;
  // priorities right behind its pod's filter, nothing changed since: the filter's placements
  bool reuse_assume(VerbScratch& s, std::string_view uid, const Demand& dem, const std::vector<int32_t>& ids,
                    std::vector<int32_t>* rcs, std::vector<int32_t>* scores);
  void note_bind_wall(uint64_t ns);
  // a response for connection `conn` of worker w, on w's thread: sent, then its next request
  struct Reply;
  void deliver_reply(Worker* w, const Reply& r);
  void drain_local(Worker* w);   // the replies w's BindIo queued during its last call
  static void append_http(std::string* out, int status, std::string_view content_type, std::string_view body);

  std::shared_ptr<Ledger> ledger_;
  std::unique_ptr<KubeWriter> writer_owner_;
  std::atomic<KubeWriter*> writer_{nullptr};
  int port_ = 0;
  int py_efd_ = -1;
  std::atomic<bool> stopping_{false};   // stop() entered (idempotence)
  std::atomic<bool> stop_{false};       // the workers leave their loops
  std::atomic<bool> serving_{true};
  std::atomic<int64_t> busy_poll_ns_{0};
  std::atomic<int64_t> busy_poll_prio_ns_{-1};
  std::atomic<bool> bind_first_{false};
  std::atomic<bool> spin_nap_{false};
  std::atomic<bool> spin_recv_{false};
  std::atomic<bool> spin_recv_binds_{false};
  std::vector<std::unique_ptr<Worker>> workers_;

  // this instance among every Frontend the process made: thread_local caches (the verbs'
  // scratch for callers off the workers) are keyed by it, not by an address a later instance
  // (or its ledger) may reuse
  const uint64_t serial_ = next_serial();
  static uint64_t next_serial() {
    static std::atomic<uint64_t> n{0};
    return n.fetch_add(1, std::memory_order_relaxed) + 1;
  }
  mutable std::mutex opt_mu_;
  Options opt_;
  std::atomic<uint64_t> opt_version_{1};   // bumped by every set_options (workers re-copy then)
  bool normalize_ = false;
  bool nominate_ = false;
  bool decisive_ = false;
  int32_t lead_ = 0;   // priorities: the nominated node's lead over every other node (0: off)

  std::mutex py_mu_;
  std::deque<PyRequest> py_q_;

  std::mutex wall_mu_;
  std::vector<uint64_t> bind_wall_ns_;
  std::vector<std::array<uint32_t, kHopSplits>> bind_hops_;

  mutable std::mutex pod_mu_;
  // filter -> bind pod cache: kPodWays-way buckets by UID hash whose entries keep their
  // strings' capacity from pod to pod (no allocation per pod once warm); a full bucket gives
  // up its oldest entry (a pod filtered long ago and never bound)
  struct PodEntry {
    uint64_t h = 0;   // 0: empty
    uint64_t stamp = 0;
    std::string uid;
    CachedPod pod;
  };
  static constexpr size_t kPodWays = 4;
  std::vector<PodEntry> pod_slots_ = std::vector<PodEntry>(16384);
  uint64_t pod_stamp_ = 0;
  size_t pod_live_ = 0;
  PodEntry* find_pod_locked(std::string_view uid, uint64_t h);
  const PodEntry* find_pod_locked(std::string_view uid, uint64_t h) const;
};

}  // namespace nanogpu
