// Per-call-site tally of the extender's system calls and hot phases: how many times each ran
// and how long it took (TSC ticks), process-wide. The sampler (sampler.h) says which functions
// the CPU time lands in; this says how much each kind of call costs on the box and how many of
// them a pod takes, which is what separates the protocol's floor (the HTTP exchanges and API
// writes every pod needs) from work that can go. Off unless switched on (bench.py
// --io-tally); when off a site costs one relaxed load.
#pragma once

#include <x86intrin.h>

#include <atomic>
#include <cstdint>

namespace nanogpu {

enum IoKind : int {
  // front-door worker threads
  kFeSpinEmpty,     // polling epoll_wait that found nothing (the busy poll)
  kFeSpinHit,       // polling epoll_wait that returned events
  kFeSpinAfterPrio, // the part of fe_spin_empty spent after a priorities answer (the rest: after a filter's)
  kFeWait,          // blocking epoll_wait (time includes sleep: count only is CPU-meaningful)
  kFeRecv,          // recv() of a kube-scheduler request
  kFeSendCycle,     // send() of a filter / priorities answer
  kFeSendOther,     // send() of any other answer (binds, Python's)
  kFeEfdRead,       // mailbox eventfd read
  kFeSubmit,        // bind handed to the writer (queue + eventfd write when it sleeps)
  kFeParseBind,     // bind arguments parsed, pod looked up, reserve
  kFeVerb,          // filter / priorities verb (JSON in, answer out); its parts:
  kFeVerbPod,       //   the args framed, the pod parsed (or matched with the last one)
  kFeVerbNames,     //   the node list matched / scanned, ids resolved
  kFeVerbCache,     //   nomination dropped, the pod cached for its bind
  kFeVerbAssume,    //   Ledger::assume_many
  kFeVerbNominate,  //   Ledger::nominate (priorities)
  kLedgerChoose,    // a node's plan computed (snapshot + choose) on a score-memo and plan-cache miss
  kLedgerCacheHit,  // a node's score taken from the plan cache on a memo miss
  // bind writer thread (evented) / BindIo
  kWrWait,          // epoll_wait (count only)
  kWrEfdRead,
  kWrSend,          // one send() of a bind's pipelined binding + label PATCH
  kWrRecv,          // recv() of API answers
  kWrBuild,         // binding / label request bodies built
  kWrCommit,        // ledger commit + answer posted to the front door
  // pod watch thread
  kPwRecv,          // blocking read of watch bytes (count only)
  kPwFilter,        // one event line through the filter
  kFeSpinRecv,      // busy poll: non-blocking recv on the last cycle answer's connection (set_spin_recv)
  kLedgerRevalidate,  // a node's memoised answer re-validated against the devices changed since (no choose)
  kLedgerScan,        // a one-share binpack pod's placement computed by the fast full scan (scan_share)
  // why a memo miss ran choose() (counts): no memo entry to re-validate, more bumps since it than
  // the change ring holds, re-validation undecided (an unchanged device may now be the best)
  kLedgerMemoCold,
  kLedgerRingGap,
  kLedgerRevalUndecided,
  kIoKinds
};

inline const char* io_kind_name(int k) {
  static const char* const names[kIoKinds] = {
      "fe_spin_empty", "fe_spin_hit", "fe_spin_after_prio", "fe_wait", "fe_recv", "fe_send_cycle", "fe_send_other", "fe_efd_read",
      "fe_submit", "fe_parse_bind", "fe_verb", "fe_verb_pod", "fe_verb_names", "fe_verb_cache",
      "fe_verb_assume", "fe_verb_nominate", "ledger_choose", "ledger_cache_hit", "wr_wait", "wr_efd_read", "wr_send", "wr_recv",
      "wr_build", "wr_commit", "pw_recv", "pw_filter", "fe_spin_recv", "ledger_revalidate", "ledger_scan",
      "ledger_memo_cold", "ledger_ring_gap", "ledger_reval_undecided"};
  return k >= 0 && k < kIoKinds ? names[k] : "?";
}

struct IoTally {
  std::atomic<bool> on{false};
  // one cache line per kind: the kinds belong to different threads
  struct alignas(64) Slot {
    std::atomic<uint64_t> n{0}, ticks{0};
  };
  Slot s[kIoKinds];
  void add(int k, uint64_t ticks) {
    s[k].n.fetch_add(1, std::memory_order_relaxed);
    s[k].ticks.fetch_add(ticks, std::memory_order_relaxed);
  }
  void reset() {
    for (auto& x : s) x.n.store(0, std::memory_order_relaxed), x.ticks.store(0, std::memory_order_relaxed);
  }
};

inline IoTally g_io;

// RAII: times the enclosing scope into kind k when the tally is on
struct IoTimer {
  int k;
  uint64_t t0;
  explicit IoTimer(int kind) : k(kind), t0(g_io.on.load(std::memory_order_relaxed) ? __rdtsc() : 0) {}
  ~IoTimer() {
    if (t0) g_io.add(k, __rdtsc() - t0);
  }
  IoTimer(const IoTimer&) = delete;
  IoTimer& operator=(const IoTimer&) = delete;
};

// the same by hand, where the kind is known only afterwards
inline uint64_t io_t0() { return g_io.on.load(std::memory_order_relaxed) ? __rdtsc() : 0; }
inline void io_end(int k, uint64_t t0) {
  if (t0) g_io.add(k, __rdtsc() - t0);
}
// an event counted, not timed
inline void io_count(int k) {
  if (g_io.on.load(std::memory_order_relaxed)) g_io.add(k, 0);
}

// ns per TSC tick (calibrated by the front door; 0 when the TSC is not invariant)
double io_ns_per_tick();

}  // namespace nanogpu
