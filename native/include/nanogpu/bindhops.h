// Per-hop timestamps of the native binds: where a POST /scheduler/bind spends its time between
// the front door reading it and the front door handing kube-scheduler its answer. The front
// door opens a record when it hands a reserved bind to the writer, the writer stamps the hops
// it owns, and the front door closes the record when the reply went to the kernel. bench.py
// reports the hops' p50 / p99 and the hop mix of the slowest 1 % of binds, so a tail in one
// driver run can be traced to its hop.
//
// Hops (TSC ticks; the invariant TSC is one clock for every thread):
//   kRead      first bytes of the bind request read by the front-door worker
//   kReserved  arguments parsed, pod found, ledger reserve done; handed to the writer
//   kPickup    the writer's loop took the bind (io thread woken, or the caller's send)
//   kLaunched  the admission window had room for it (kube-apiserver's max-in-flight share:
//              with every slot held by unanswered requests, a bind waits here)
//   kSent      binding (+ label PATCH) written to the API server connection
//   kAnswer    the binding's answer parsed
//   kPosted    ledger committed, reply posted to the front-door worker
//   kReplied   reply handed to the kernel by the front-door worker
//
// Off unless switched on (Frontend::set_bind_hops); when off each site costs one relaxed load.
// A record is a slot of a fixed table keyed by the front-door request id (one bind at a time
// per kube-scheduler connection, so ids of binds in flight differ); two binds in flight that
// hash to one slot lose the first one's record, which only thins the sample.
#pragma once

#include <x86intrin.h>

#include <atomic>
#include <cstdint>

namespace nanogpu {

enum BindHop : int { kHopRead, kHopReserved, kHopPickup, kHopLaunched, kHopSent, kHopAnswer, kHopPosted, kHopReplied,
                     kBindHops };
constexpr int kHopSplits = kBindHops - 1;   // the time between consecutive hops

struct BindHopTable {
  static constexpr size_t kSlots = 8192;   // power of two
  std::atomic<bool> on{false};
  struct alignas(64) Slot {
    std::atomic<uint64_t> id{0};
    std::atomic<uint64_t> t[kBindHops];
  };
  Slot s[kSlots];

  static size_t slot_of(uint64_t id) { return static_cast<size_t>((id * 0x9E3779B97F4A7C15ull) >> 51) & (kSlots - 1); }
  bool enabled() const { return on.load(std::memory_order_relaxed); }
  // a new record for bind `id`, read at TSC `t_read`
  void open(uint64_t id, uint64_t t_read) {
    if (!enabled()) return;
    Slot& x = s[slot_of(id)];
    x.id.store(0, std::memory_order_relaxed);
    for (auto& t : x.t) t.store(0, std::memory_order_relaxed);
    x.t[kHopRead].store(t_read, std::memory_order_relaxed);
    x.t[kHopReserved].store(__rdtsc(), std::memory_order_relaxed);
    x.id.store(id, std::memory_order_release);
  }
  void stamp(uint64_t id, int hop) {
    if (!enabled()) return;
    Slot& x = s[slot_of(id)];
    if (x.id.load(std::memory_order_acquire) == id) x.t[hop].store(__rdtsc(), std::memory_order_relaxed);
  }
  // stamps kReplied and takes the record: true with every hop's TSC in out[] when the record
  // is whole and in order
  bool close(uint64_t id, uint64_t out[kBindHops]) {
    if (!enabled()) return false;
    Slot& x = s[slot_of(id)];
    if (x.id.load(std::memory_order_acquire) != id) return false;
    x.t[kHopReplied].store(__rdtsc(), std::memory_order_relaxed);
    bool ok = true;
    for (int h = 0; h < kBindHops; ++h) {
      out[h] = x.t[h].load(std::memory_order_relaxed);
      if (!out[h] || (h > 0 && out[h] < out[h - 1])) ok = false;
    }
    x.id.store(0, std::memory_order_relaxed);
    return ok;
  }
};

inline BindHopTable g_hops;

}  // namespace nanogpu
