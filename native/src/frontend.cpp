// Native extender front door (see frontend.h).
#include "nanogpu/frontend.h"

#include "nanogpu/bindhops.h"
#include "nanogpu/bindio.h"
#include "nanogpu/iotally.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cpuid.h>
#include <x86intrin.h>

#include <algorithm>
#include <charconv>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "nanogpu/json.h"

namespace nanogpu {

namespace {

constexpr size_t kMaxHeader = 64 * 1024;
constexpr size_t kMaxBody = 64u * 1024 * 1024;
constexpr const char* kPercent = "nano-gpu/gpu-percent";
constexpr const char* kMemory = "nano-gpu/gpu-memory";

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
uint64_t now_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count());
}

// The front door's own timers (busy-poll windows, phase and verb timings, the extender-side
// bind wall): durations measured on one worker thread, read several times a request. The
// invariant TSC (CPUID 8000_0007h EDX bit 8) scaled to nanoseconds costs a few cycles where
// the vDSO clock read costs tens (6.5 % of the front door's samples, profiles/extender_cpu_profile.md).
// Values handed to other threads (BindJob::t0_ns) stay on now_ns().
struct TscClock {
  double ns_per_tick = 0.0;   // 0: no invariant TSC, fast_ns() is now_ns()
  uint64_t tick0 = 0, ns0 = 0;
};

TscClock calibrate_tsc() {
  TscClock c;
  unsigned a = 0, b = 0, cx = 0, d = 0;
  if (!__get_cpuid(0x80000007u, &a, &b, &cx, &d) || !((d >> 8) & 1u)) return c;
  const uint64_t n0 = now_ns(), t0 = __rdtsc();
  uint64_t n1;
  do {
    n1 = now_ns();
  } while (n1 - n0 < 2'000'000);   // 2 ms
  const uint64_t t1 = __rdtsc();
  if (t1 <= t0) return c;
  const double r = static_cast<double>(n1 - n0) / static_cast<double>(t1 - t0);
  if (r < 0.05 || r > 2.0) return c;   // 0.5-20 GHz, else not a clock to trust
  c.ns_per_tick = r;
  c.tick0 = t1;
  c.ns0 = n1;
  return c;
}

const TscClock& tsc_clock() {
  static const TscClock c = calibrate_tsc();
  return c;
}

uint64_t fast_ns() {
  const TscClock& c = tsc_clock();
  if (c.ns_per_tick == 0.0) return now_ns();
  return c.ns0 + static_cast<uint64_t>(static_cast<double>(__rdtsc() - c.tick0) * c.ns_per_tick);
}

// the TSC reading a fast_ns() value was taken at (the bind hop stamps are raw TSC)
uint64_t tsc_of(uint64_t fast) {
  const TscClock& c = tsc_clock();
  if (c.ns_per_tick == 0.0 || fast < c.ns0) return __rdtsc();
  return c.tick0 + static_cast<uint64_t>(static_cast<double>(fast - c.ns0) / c.ns_per_tick);
}

}  // namespace

double io_ns_per_tick() {
  const double r = tsc_clock().ns_per_tick;
  return r > 0.0 ? r : 1.0;
}

namespace {

bool ieq(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i]))) return false;
  return true;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

const char* reason(int status) {
  switch (status) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Payload Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

using i128 = __int128;

bool mul_ok(i128 a, i128 b, i128* out) { return !__builtin_mul_overflow(a, b, out); }

bool pow10(int e, i128* out) {
  i128 v = 1;
  for (int i = 0; i < e; ++i)
    if (!mul_ok(v, 10, &v)) return false;
  *out = v;
  return true;
}

}  // namespace

// ------------------------------------------------------------------------------ quantity
bool quantity_value(std::string_view s, bool mib, int64_t* out) {
  s = trim(s);
  while (!s.empty() && (s.back() == '\n')) s.remove_suffix(1);
  if (s.empty()) return false;
  bool bare = true;
  for (char c : s)
    if (c < '0' || c > '9') bare = false;
  if (mib && bare) {
    if (s.size() > 18) return false;
    *out = std::strtoll(std::string(s).c_str(), nullptr, 10);
    return true;
  }
  // [+-]?[0-9.]+ ([eE][+-]?[0-9]+)? suffix?
  size_t p = 0;
  bool neg = false;
  if (s[p] == '+' || s[p] == '-') neg = s[p++] == '-';
  i128 m = 0;
  int frac = 0, ndig = 0;
  bool dot = false, any = false;
  for (; p < s.size() && ((s[p] >= '0' && s[p] <= '9') || s[p] == '.'); ++p) {
    if (s[p] == '.') {
      if (dot) return false;  // "1.2.3": Decimal rejects it too
      dot = true;
      continue;
    }
    any = true;
    if (m == 0 && s[p] == '0') {
      if (dot) ++frac;
      continue;
    }
    if (++ndig > 30) return false;
    m = m * 10 + (s[p] - '0');
    if (dot) ++frac;
  }
  if (!any) return false;
  int e10 = 0;
  if (p < s.size() && (s[p] == 'e' || s[p] == 'E')) {
    // "E" alone is the exa suffix; an exponent needs digits after it
    size_t q = p + 1;
    bool eneg = false;
    if (q < s.size() && (s[q] == '+' || s[q] == '-')) eneg = s[q++] == '-';
    if (q < s.size() && s[q] >= '0' && s[q] <= '9') {
      int v = 0;
      for (; q < s.size() && s[q] >= '0' && s[q] <= '9'; ++q) {
        v = v * 10 + (s[q] - '0');
        if (v > 60) return false;
      }
      e10 = eneg ? -v : v;
      p = q;
    }
  }
  const std::string_view suf = s.substr(p);
  int bin = 0, dec = 0;
  if (suf.empty()) {
  } else if (suf == "Ki") bin = 10;
  else if (suf == "Mi") bin = 20;
  else if (suf == "Gi") bin = 30;
  else if (suf == "Ti") bin = 40;
  else if (suf == "Pi") bin = 50;
  else if (suf == "Ei") bin = 60;
  else if (suf == "n") dec = -9;
  else if (suf == "u") dec = -6;
  else if (suf == "m") dec = -3;
  else if (suf == "k") dec = 3;
  else if (suf == "M") dec = 6;
  else if (suf == "G") dec = 9;
  else if (suf == "T") dec = 12;
  else if (suf == "P") dec = 15;
  else if (suf == "E") dec = 18;
  else return false;
  if (neg && m != 0) {  // every caller clamps negatives to 0
    *out = 0;
    return true;
  }
  // value = m * 10^(e10 + dec - frac) * 2^bin ; result = ceil(value / (mib ? 2^20 : 1))
  int e = e10 + dec - frac;
  int b = bin - (mib ? 20 : 0);
  i128 num = m, den = 1, t;
  if (e > 0) {
    if (!pow10(e, &t) || !mul_ok(num, t, &num)) return false;
  } else if (e < 0) {
    if (!pow10(-e, &den)) return false;
  }
  if (b > 0) {
    if (!mul_ok(num, static_cast<i128>(1) << b, &num)) return false;
  } else if (b < 0) {
    if (!mul_ok(den, static_cast<i128>(1) << (-b), &den)) return false;
  }
  const i128 q = num / den + (num % den != 0 ? 1 : 0);
  if (q > static_cast<i128>(INT64_MAX)) return false;
  *out = static_cast<int64_t>(q);
  return true;
}

constexpr const char* kMemBoundAnnotation = "nano-gpu/memory-bound";   // nanogpu/types.py

// `name` is one of the comma-separated items of `list` (items trimmed of spaces).
static bool list_has(std::string_view list, std::string_view name) {
  while (!list.empty()) {
    const size_t c = list.find(',');
    std::string_view item = list.substr(0, c);
    while (!item.empty() && item.front() == ' ') item.remove_prefix(1);
    while (!item.empty() && item.back() == ' ') item.remove_suffix(1);
    if (!item.empty() && item == name) return true;
    if (c == std::string_view::npos) break;
    list.remove_prefix(c + 1);
  }
  return false;
}

// UID of the controlling owner in a pod's ownerReferences (the first entry with
// controller: true, else the first entry); empty when there is none.
static std::string_view controller_uid(const json::Doc& d, int32_t refs) {
  if (!d.is(refs, json::Type::kArr)) return {};
  std::string_view first;
  for (int32_t r = d.at(refs).first; r >= 0; r = d.at(r).next) {
    if (!d.is(r, json::Type::kObj)) continue;
    const int32_t u = d.get(r, "uid");
    if (!d.is(u, json::Type::kStr)) continue;
    const int32_t ctl = d.get(r, "controller");
    if (d.is(ctl, json::Type::kBool) && d.at(ctl).b) return d.str(u);
    if (first.empty()) first = d.str(u);
  }
  return first;
}

// 64-bit hash of a byte string, eight bytes per step (keys the per-worker node-id cache;
// hits are verified name by name, so a collision costs a lookup, never a wrong answer).
static uint64_t text_hash(std::string_view s) {
  uint64_t h = 0x9e3779b97f4a7c15ULL ^ s.size();
  size_t i = 0;
  for (; i + 8 <= s.size(); i += 8) {
    uint64_t w;
    std::memcpy(&w, s.data() + i, 8);
    h = (h ^ w) * 0xff51afd7ed558ccdULL;
    h ^= h >> 32;
  }
  uint64_t tail = 0;
  std::memcpy(&tail, s.data() + i, s.size() - i);
  h = (h ^ tail) * 0xc4ceb9fe1a85ec53ULL;
  return h ^ (h >> 29);
}

// A JSON array of plain strings written compactly, `["a","b"]` (what kube-scheduler's Go encoder
// sends), into its tokens' (offset, length), quotes included. false: any other shape (spaces,
// escapes, non-strings), which the caller hands to the JSON parser. One pass, 16 bytes a step:
// the quotes' positions from a byte compare, and any backslash or control byte anywhere sends
// the list the parser's way (sampled windows of 420 names are 5 KB: a window not seen before
// is scanned whole on the scheduling cycle's path).
static bool scan_string_array(std::string_view t, std::vector<std::pair<uint32_t, uint32_t>>* toks) {
  const size_t n = t.size();
  if (n < 2 || t.front() != '[' || t.back() != ']') return false;
  if (n == 2) return true;
  const char* b = t.data();
  const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\'), space = _mm_set1_epi8(0x20);
  size_t expect = 1;   // where the next name's opening quote must be
  size_t open = 0;
  bool in_str = false, closed = false;
  for (size_t base = 0; base < n; base += 16) {
    __m128i v;
    if (base + 16 <= n) {
      v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(b + base));
    } else {
      alignas(16) char tail[16];
      std::memset(tail, ' ', sizeof tail);
      std::memcpy(tail, b + base, n - base);
      v = _mm_load_si128(reinterpret_cast<const __m128i*>(tail));
    }
    // a byte below 0x20 (unsigned) or a backslash: not the plain shape
    const __m128i ctl = _mm_andnot_si128(_mm_cmpeq_epi8(_mm_max_epu8(v, space), v), _mm_set1_epi8(-1));
    if (_mm_movemask_epi8(_mm_or_si128(ctl, _mm_cmpeq_epi8(v, bslash)))) return false;
    for (uint32_t m = static_cast<uint32_t>(_mm_movemask_epi8(_mm_cmpeq_epi8(v, quote))); m; m &= m - 1) {
      const size_t q = base + static_cast<size_t>(__builtin_ctz(m));
      if (closed) return false;
      if (!in_str) {
        if (q != expect) return false;
        open = q;
        in_str = true;
        continue;
      }
      in_str = false;
      toks->emplace_back(static_cast<uint32_t>(open), static_cast<uint32_t>(q - open + 1));
      if (q + 2 == n) {
        closed = true;
      } else {
        if (b[q + 1] != ',') return false;
        expect = q + 2;
      }
    }
  }
  return closed;
}

namespace {
// name -> node id for this thread, valid for one node epoch: open addressing on the name's hash,
// names kept in an arena so a lookup compares bytes in a few cache lines of its own
struct NameTable {
  uint64_t owner = 0;   // Frontend::serial_ (a thread_local table outlives the Frontend it served)
  uint64_t epoch = 0;
  struct Slot {
    uint64_t h = 0;   // 0: empty
    uint32_t off = 0, len = 0;
    int32_t id = -1;
  };
  std::vector<Slot> slots;
  std::string arena;
  size_t used = 0;
  // by node id: its name in the arena, and the id that followed it in the last list resolved.
  // kube-scheduler's lists are windows of its own node order, so the next name is nearly always
  // the successor seen before (one compare of bytes laid out in id order, no hash); a node that
  // filled up, left out of the window, costs one lookup and moves the successor
  std::vector<std::pair<uint32_t, uint32_t>> at;
  std::vector<int32_t> succ;
  void reset(uint64_t o, uint64_t e) {
    owner = o;
    epoch = e;
    slots.assign(1024, Slot{});
    arena.clear();
    used = 0;
    at.clear();
    succ.clear();
  }
  bool is(int32_t id, std::string_view name) const {
    if (id < 0 || static_cast<size_t>(id) >= at.size()) return false;
    const auto& [off, len] = at[static_cast<size_t>(id)];
    if (len != name.size() || len == 0) return false;
    const char* a = arena.data() + off;
    if (len >= 8 && len <= 16) {   // node names: two overlapping 8-byte words, no call
      uint64_t x0, y0, x1, y1;
      std::memcpy(&x0, a, 8);
      std::memcpy(&y0, name.data(), 8);
      std::memcpy(&x1, a + len - 8, 8);
      std::memcpy(&y1, name.data() + len - 8, 8);
      return ((x0 ^ y0) | (x1 ^ y1)) == 0;
    }
    return std::memcmp(a, name.data(), len) == 0;
  }
  int32_t next_of(int32_t id) const {
    return id >= 0 && static_cast<size_t>(id) < succ.size() ? succ[static_cast<size_t>(id)] : -1;
  }
  void set_next(int32_t id, int32_t next) {
    if (id < 0) return;
    if (static_cast<size_t>(id) >= succ.size()) succ.resize(static_cast<size_t>(id) + 1, -1);
    succ[static_cast<size_t>(id)] = next;
  }
  int32_t find(std::string_view name) const {
    if (slots.empty()) return -1;
    const uint64_t h = text_hash(name) | 1;
    const size_t mask = slots.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& s = slots[i];
      if (s.h == 0) return -1;
      if (s.h == h && s.len == name.size() && std::memcmp(arena.data() + s.off, name.data(), name.size()) == 0)
        return s.id;
    }
  }
  void insert(std::string_view name, int32_t id) {
    if ((used + 1) * 2 > slots.size()) {   // keep it at most half full
      std::vector<Slot> old;
      old.swap(slots);
      slots.assign(old.size() * 2, Slot{});
      used = 0;
      for (const Slot& s : old)
        if (s.h) place(s);
    }
    Slot s;
    s.h = text_hash(name) | 1;
    s.off = static_cast<uint32_t>(arena.size());
    s.len = static_cast<uint32_t>(name.size());
    s.id = id;
    arena.append(name);
    place(s);
    if (id >= 0) {
      if (static_cast<size_t>(id) >= at.size()) at.resize(static_cast<size_t>(id) + 1, {0u, 0u});
      at[static_cast<size_t>(id)] = {s.off, s.len};
    }
  }
  void place(const Slot& s) {
    const size_t mask = slots.size() - 1;
    for (size_t i = s.h & mask;; i = (i + 1) & mask)
      if (slots[i].h == 0) {
        slots[i] = s;
        ++used;
        return;
      }
  }
};
}  // namespace

// The fitting node with the top score; a tie at the top goes to the tied node (in the
// request's order) the pod's UID hash picks: as even over the tied nodes as kube-scheduler's
// random pick among equal scores, but the same on every worker. -1: nothing fits.
static int64_t top_pick(const std::vector<int32_t>& scores, const std::vector<int32_t>& rcs, std::string_view uid) {
  int64_t best = -1;
  uint64_t n_best = 0;
  for (size_t i = 0; i < scores.size(); ++i) {
    if (rcs[i] != kOk) continue;
    if (best < 0 || scores[i] > scores[best]) {
      best = static_cast<int64_t>(i);
      n_best = 1;
    } else if (scores[i] == scores[best]) {
      ++n_best;
    }
  }
  if (n_best < 2 || uid.empty()) return best;
  uint64_t k = owner_hash(uid) % n_best;
  const int32_t top = scores[best];
  for (size_t i = static_cast<size_t>(best); i < scores.size(); ++i)
    if (rcs[i] == kOk && scores[i] == top && k-- == 0) return static_cast<int64_t>(i);
  return best;
}

static bool wants_devices(const Demand& d) {
  for (int i = 0; i < d.n; ++i)
    if (d.c[i].pct > 0 || d.c[i].mib > 0) return true;
  return false;
}

static void atomic_max(std::atomic<uint64_t>* m, uint64_t v) {
  uint64_t cur = m->load(std::memory_order_relaxed);
  while (v > cur && !m->compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
  }
}

void VerbStats::observe(uint64_t ns) {
  count.fetch_add(1, std::memory_order_relaxed);
  ns_total.fetch_add(ns, std::memory_order_relaxed);
  uint64_t us8 = ns / 8000;
  int k = 0;
  while (us8 > 0 && k < 15) {
    us8 >>= 1;
    ++k;
  }
  buckets[k].fetch_add(1, std::memory_order_relaxed);
  atomic_max(&max_ns, ns);
}

void Frontend::note_bind_wall(uint64_t ns) {
  std::lock_guard<std::mutex> g(wall_mu_);
  if (bind_wall_ns_.size() < kMaxWallSamples) bind_wall_ns_.push_back(ns);
}

std::vector<uint64_t> Frontend::take_bind_wall() {
  std::lock_guard<std::mutex> g(wall_mu_);
  std::vector<uint64_t> out;
  out.swap(bind_wall_ns_);
  return out;
}

bool Frontend::set_bind_hops(bool on) {
  on = on && tsc_clock().ns_per_tick > 0.0;
  g_hops.on.store(on, std::memory_order_relaxed);
  return on;
}

std::pair<size_t, size_t> Frontend::bind_samples_waiting() {
  std::lock_guard<std::mutex> g(wall_mu_);
  return {bind_wall_ns_.size(), bind_hops_.size()};
}

std::vector<std::array<uint32_t, kHopSplits>> Frontend::take_bind_hops() {
  std::lock_guard<std::mutex> g(wall_mu_);
  std::vector<std::array<uint32_t, kHopSplits>> out;
  out.swap(bind_hops_);
  return out;
}

void Frontend::reset_max() {
  for (VerbStats* v : {&filter_stats, &prio_stats, &py_stats, &bind_stats, &filter_wall_stats, &prio_wall_stats})
    v->max_ns.store(0);
  loop_max_ns.store(0);
  for (auto& p : phase_max_ns) p.store(0);
}

namespace {
struct PhaseTimer {
  std::atomic<uint64_t>* m;
  uint64_t t0 = fast_ns();
  ~PhaseTimer() { atomic_max(m, fast_ns() - t0); }
};
}  // namespace

namespace {
// priorities follows its cycle's filter with the same Pod text on the same connection, so on
// the same worker: the pod a worker parsed last is reused when the text is identical (demand,
// identity, containers); only the learned-owner flag is read again
struct LastPod {
  std::string raw, uid;
  Demand dem{};
  CachedPod cached;
  bool mb_annotated = false;
  bool valid = false;
};

// The node lists of the last kListSlots distinct texts a worker resolved (LRU). With
// kube-scheduler's node sampling (numFeasibleNodesToFind from a rotating start) the list is a
// window of the cluster that moves every cycle, but the windows repeat: 1000 nodes sampled 420
// at a time cycle through 50 of them, so a few dozen slots catch them all. A slot is found by
// its text alone (length, then bytes; the last slot used is tried first): no hash pass over the
// list.
constexpr int kListSlots = 64;
struct IdCache {
  uint64_t owner = 0;   // Frontend::serial_
  bool valid[kListSlots] = {};         // an escape-free list whose ids can be reused
  uint64_t epoch[kListSlots] = {};     // the ledger's node epoch the ids were checked at
  uint64_t used[kListSlots] = {};
  size_t len[kListSlots] = {};
  bool compact[kListSlots] = {};       // the text is `["a","b",...]` exactly: a reply may copy it whole
  std::vector<int32_t> ids[kListSlots];
  std::vector<std::pair<uint32_t, uint32_t>> tok[kListSlots];   // token (offset, length) in the list text
  std::string text[kListSlots];        // the list text itself
  int mru = 0;
  uint64_t clock = 0;
  // equal-length lists are told apart by their last bytes first (sampled windows of one
  // cluster's names are mostly the same length), then compared whole
  bool same(int k, std::string_view t) const {
    if (!valid[k] || len[k] != t.size()) return false;
    const size_t tail = std::min<size_t>(16, t.size());
    return std::memcmp(text[k].data() + t.size() - tail, t.data() + t.size() - tail, tail) == 0 &&
           std::memcmp(text[k].data(), t.data(), t.size()) == 0;
  }
  int find(std::string_view t) const {
    if (same(mru, t)) return mru;
    for (int k = 0; k < kListSlots; ++k)
      if (k != mru && same(k, t)) return k;
    return -1;
  }
  // The nodes of list `src` that a filter answered as fitting (`rcs[i] == kOk`), kept as a list
  // of its own: kube-scheduler sends priorities exactly that list, in that order, re-encoded the
  // way a compact escape-free list is written. Once nodes fill up, the answer is a subset of the
  // request's window, so without this every priorities call would scan and resolve its whole
  // list again (6 us at 420 nodes).
  void remember_subset(int src, const std::vector<int32_t>& rcs) {
    if (src < 0 || !valid[src] || tok[src].size() != rcs.size()) return;
    int k = src == 0 ? 1 : 0;
    for (int j = 0; j < kListSlots; ++j)
      if (j != src && used[j] < used[k]) k = j;
    std::string& t = text[k];
    t.clear();
    t += '[';
    tok[k].clear();
    ids[k].clear();
    for (size_t i = 0; i < rcs.size(); ++i) {
      if (rcs[i] != kOk) continue;
      if (t.size() > 1) t += ',';
      const auto& [off, n] = tok[src][i];
      tok[k].emplace_back(static_cast<uint32_t>(t.size()), n);
      t.append(text[src], off, n);
      ids[k].push_back(ids[src][i]);
    }
    t += ']';
    valid[k] = true;
    compact[k] = true;
    len[k] = t.size();
    epoch[k] = epoch[src];
    used[k] = ++clock;
    mru = k;   // the next request is this pod's priorities
  }
};
}  // namespace

// A front-door worker's scratch for the verbs: DOMs, name views, result arrays, the last pod
// and the node-list cache keep their capacity from one request to the next (every cycle of a
// burst sends the same-sized bodies). Owned by the worker and handed down, not thread_local:
// in a shared library every thread_local access is a __tls_get_addr call (10 % of the verbs'
// samples when they were thread_local).
struct Frontend::VerbScratch {
  json::Doc top, d, other, dn;
  std::vector<std::string_view> nv, nraw;                // a list in another shape (the JSON parser's)
  std::vector<std::pair<uint32_t, uint32_t>> ntok;       // a compact list scanned now: its tokens
  std::vector<int32_t> rcs, scores;
  LastPod last;
  IdCache idc;
  NameTable nid;
  std::deque<std::string> requoted;
  std::string blob, dstr, resp;
  bool nom_dropped = false;   // the last pod's own nomination was dropped ...
  uint64_t nom_mark = 0;      // ... when Ledger::nominations_made() read this
  uint64_t opt_seen = 0;   // Frontend::opt_version_ of the copy below ...
  uint64_t opt_owner = 0;   // ... of this Frontend (serial_)
  Options opt;
  bool normalize = false, nominate = false, decisive = false;
  int32_t lead = 0;
  // A worker's verbs leave two pieces of work for after their answer is on the wire
  // (Frontend::run_deferred, before the worker reads anything else): the pod cached for its bind
  // (filter) and the priorities-time nomination. Neither changes the answer, and kube-scheduler's
  // next request of the cycle no longer waits on them. Off for callers off the workers (tests,
  // time_verb), which get the work done in the verb.
  bool defer = false;
  bool defer_cache = false;   // the pod-cache put too: only with one worker thread (see filter_verb)
  bool defer_put = false;
  bool defer_nominate = false;
  int defer_list = -1;   // the filter's node-list slot whose fitting subset priorities will send
  // The last filter's placements (Ledger::assume_many) and the ledger's mutation epoch before
  // them: kube-scheduler's priorities call for the same pod follows, over the same nodes or
  // the fitting ones, and with no mutation anywhere in between (a bind adopting its nomination
  // and a commit change no device) the answers are the same, so priorities reads them here
  // instead of walking the nodes again on the scheduling cycle's path. One use.
  struct LastAssume {
    bool valid = false;
    uint64_t epoch = 0, dem_hash = 0, opt_seen = 0;
    std::string uid;
    std::vector<int32_t> ids, rcs, scores;
  } last_assume;
  int32_t defer_node = -1;
  Demand defer_dem{};
};

// ------------------------------------------------------------------------------ plumbing
struct Frontend::Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in, out;
  size_t out_off = 0;
  bool waiting = false;      // a request is with Python; later requests wait their turn
  bool close_after = false;
  bool want_out = false;
  bool bind_waiting = false; // the request with Python is a bind (its wall time is recorded)
  uint64_t t_in_ns = 0;      // first bytes of the request being parsed arrived
  uint64_t t_req_ns = 0;     // ... of the request now with Python
};

// An answer posted to a worker (bind writer, Python, inline BindIo): formatted into the
// connection's output by the worker itself, so posting one allocates nothing for a short
// JSON body (a bind's {"Error":""} fits the string's inline buffer).
struct Frontend::Reply {
  uint64_t conn = 0;
  int status = 200;
  std::string ctype;   // empty: application/json
  std::string body;
};

struct Frontend::Worker {
  int idx = 0;
  int lfd = -1, ep = -1, efd = -1;
  // inline bind writes (set_kube_writer inline_io): this worker's request driver, published
  // once from the setting thread, then used by this worker's thread only
  std::unique_ptr<BindIo> bio_owner;
  std::atomic<BindIo*> bio{nullptr};
  std::vector<Reply> local_replies;   // inline BindIo answers, sent after the call
  std::vector<Reply> local_spare;
  std::thread th;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;   // by conn id
  std::mutex mb_mu;
  std::vector<Reply> mailbox;        // posted by other threads (under mb_mu)
  std::vector<Reply> mb_spare;       // the worker's side of the swap (keeps its capacity)
  std::atomic<bool> unsignalled{false};                         // queued with notify=false
  bool mb_signalled = false;   // under mb_mu: the eventfd was written for what the mailbox holds
  // An awake worker (busy polling, or handling a batch) looks at the mailbox itself after
  // every epoll round, so a response posted then needs no eventfd write and no wake-up. Only
  // a worker about to block is signalled: it sets `parked` and then re-reads `mb_pending`, the
  // poster sets `mb_pending` and then reads `parked` (both seq_cst), so one of the two always
  // sees the other.
  std::atomic<bool> parked{false};
  std::atomic<bool> mb_pending{false};
  uint64_t next_conn = 1;
  uint64_t cycle_reply_ns = 0;   // last filter / priorities reply handed to the kernel
  bool cycle_was_prio = false;   // ... and whether it was a priorities answer (io tally)
  uint64_t cycle_cid = 0;        // ... and the connection it went out on (set_spin_recv)
  uint64_t bind_cid = 0;         // the connection the last bind answer went out on (set_spin_recv_binds)
  VerbScratch scratch;           // the verbs' per-request scratch (this worker's thread only)
};

static uint64_t make_id(int worker, uint64_t conn) { return (conn << 8) | static_cast<uint64_t>(worker); }
// epoll tags: 0 listen socket, 1 mailbox, bit 63 a client connection, bit 62 a BindIo connection
static constexpr uint64_t kBioTag = 1ull << 62;

int presize_fd_table(int want) {
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) != 0) return 0;
  const rlim_t cap = rl.rlim_cur == RLIM_INFINITY ? static_cast<rlim_t>(want) : rl.rlim_cur;
  const int top = static_cast<int>(std::min<rlim_t>(cap, static_cast<rlim_t>(want))) - 1;
  if (top < 64) return 0;
  // the lowest free fd >= top: allocating it sizes the table past `top`; closing keeps the size
  const int fd = fcntl(0, F_DUPFD_CLOEXEC, top);
  if (fd < 0) {
    const int alt = open("/dev/null", O_RDONLY | O_CLOEXEC);
    if (alt < 0) return 0;
    const int fd2 = fcntl(alt, F_DUPFD_CLOEXEC, top);
    close(alt);
    if (fd2 < 0) return 0;
    close(fd2);
    return top + 1;
  }
  close(fd);
  return top + 1;
}

Frontend::Frontend(std::shared_ptr<Ledger> ledger, const std::string& host, int port, int threads)
    : ledger_(std::move(ledger)) {
  if (!ledger_) throw std::invalid_argument("Frontend: ledger required");
  (void)tsc_clock();   // calibrated here (2 ms), not on the first request
  presize_fd_table();
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  py_efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (py_efd_ < 0) throw std::runtime_error("eventfd failed");
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  if (host.empty() || host == "0.0.0.0") {
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
  } else if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    throw std::invalid_argument("Frontend: host must be an IPv4 address");
  }
  for (int i = 0; i < threads; ++i) {
    auto w = std::make_unique<Worker>();
    // the verbs' pod caching / nomination run after their answer (run_deferred);
    // NANOGPU_FE_NO_DEFER=1 keeps them inside the verb (A/B measurements)
    const char* nd = std::getenv("NANOGPU_FE_NO_DEFER");
    w->scratch.defer = !(nd && nd[0] == '1');
    w->scratch.defer_cache = w->scratch.defer && threads == 1;
    w->idx = i;
    w->lfd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(w->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    setsockopt(w->lfd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    if (bind(w->lfd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || listen(w->lfd, 1024) != 0) {
      const std::string err = std::strerror(errno);
      close(w->lfd);
      for (auto& o : workers_) close(o->lfd);
      close(py_efd_);
      throw std::runtime_error("Frontend: bind/listen failed: " + err);
    }
    if (i == 0) {
      socklen_t len = sizeof(addr);
      getsockname(w->lfd, reinterpret_cast<sockaddr*>(&addr), &len);
      port_ = ntohs(addr.sin_port);
    }
    w->ep = epoll_create1(EPOLL_CLOEXEC);
    w->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 0;  // listen socket
    epoll_ctl(w->ep, EPOLL_CTL_ADD, w->lfd, &ev);
    ev.data.u64 = 1;  // mailbox
    epoll_ctl(w->ep, EPOLL_CTL_ADD, w->efd, &ev);
    workers_.push_back(std::move(w));
  }
  for (size_t i = 0; i < workers_.size(); ++i)
    workers_[i]->th = std::thread([this, p = workers_[i].get(), i] {
      // named for per-thread CPU accounting (bench.py thread_cpu, /proc/<pid>/task/<tid>/comm)
      pthread_setname_np(pthread_self(), ("ngpu-fe" + std::to_string(i)).c_str());
      run(p);
    });
}

Frontend::~Frontend() { stop(); }

void Frontend::set_kube_writer(const KubeTarget& t, int threads, int retries, bool record_events, bool evented,
                               bool label, double timeout_s, bool inline_io, bool batch_labels, int max_binds) {
  if (writer_.load()) throw std::logic_error("Frontend: the kube writer is already set");
  writer_owner_ = std::make_unique<KubeWriter>(
      t, ledger_, [this](uint64_t id, int status, const std::string& body) { respond(id, status, "application/json", body); },
      threads, retries, record_events, evented, label, timeout_s, inline_io, max_binds);
  writer_owner_->set_batch_labels(batch_labels);
  if (inline_io) {
    for (auto& wp : workers_) {
      Worker* w = wp.get();
      // happy-path answers from w's own BindIo, on w's thread: queued, sent after the call
      w->bio_owner = writer_owner_->make_io(w->ep, kBioTag, [w](uint64_t id, int status, const std::string& body) {
        Reply r;
        r.conn = id >> 8;
        r.status = status;
        r.body = body;
        w->local_replies.push_back(std::move(r));
      });
      w->bio.store(w->bio_owner.get(), std::memory_order_release);
    }
  }
  writer_.store(writer_owner_.get(), std::memory_order_release);
}

void Frontend::stop() {
  if (stopping_.exchange(true)) return;
  // the workers still run while the writer stops: what it answers reaches kube-scheduler
  if (writer_owner_) writer_owner_->stop();
  stop_.store(true, std::memory_order_release);
  for (auto& w : workers_) {
    uint64_t one = 1;
    (void)!write(w->efd, &one, sizeof(one));
  }
  for (auto& w : workers_) {
    if (w->th.joinable()) w->th.join();
    w->bio.store(nullptr, std::memory_order_relaxed);
    w->bio_owner.reset();   // its sockets leave w->ep before the epoll fd closes
    for (auto& kv : w->conns) close(kv.second->fd);
    w->conns.clear();
    close(w->lfd);
    close(w->ep);
    close(w->efd);
  }
  if (py_efd_ >= 0) close(py_efd_);
  py_efd_ = -1;
}

void Frontend::set_options(const Options& o, bool score_normalize, bool nominate, bool decisive, int32_t lead) {
  std::lock_guard<std::mutex> g(opt_mu_);
  opt_version_.fetch_add(1, std::memory_order_release);
  opt_ = o;
  normalize_ = score_normalize;
  nominate_ = nominate;
  decisive_ = decisive;
  lead_ = std::max<int32_t>(0, lead);
}

std::vector<PyRequest> Frontend::take() {
  uint64_t v;
  (void)!read(py_efd_, &v, sizeof(v));
  std::lock_guard<std::mutex> g(py_mu_);
  std::vector<PyRequest> out(std::make_move_iterator(py_q_.begin()), std::make_move_iterator(py_q_.end()));
  py_q_.clear();
  return out;
}

void Frontend::append_http(std::string* out, int status, std::string_view content_type, std::string_view body) {
  char num[24];
  out->reserve(out->size() + body.size() + 96 + content_type.size());
  *out += "HTTP/1.1 ";
  out->append(num, static_cast<size_t>(std::to_chars(num, num + sizeof num, status).ptr - num));
  *out += ' ';
  *out += reason(status);
  *out += "\r\nContent-Type: ";
  *out += content_type;
  *out += "\r\nContent-Length: ";
  out->append(num, static_cast<size_t>(std::to_chars(num, num + sizeof num, body.size()).ptr - num));
  *out += "\r\n\r\n";
  *out += body;
}

void Frontend::respond(uint64_t id, int status, const std::string& content_type, const std::string& body,
                       bool notify) {
  const int widx = static_cast<int>(id & 0xff);
  if (widx < 0 || widx >= static_cast<int>(workers_.size())) return;
  Worker* w = workers_[widx].get();
  Reply r;
  r.conn = id >> 8;
  r.status = status;
  if (content_type != "application/json") r.ctype = content_type;
  r.body = body;
  bool signal = false;
  {
    std::lock_guard<std::mutex> g(w->mb_mu);
    w->mailbox.push_back(std::move(r));
    w->mb_pending.store(true, std::memory_order_seq_cst);
    // one eventfd write per mailbox fill, and only to a worker that may be blocked in
    // epoll_wait: the worker takes everything queued until it swaps
    if (notify && !w->mb_signalled && w->parked.load(std::memory_order_seq_cst))
      signal = w->mb_signalled = true;
  }
  if (!notify) {
    w->unsignalled.store(true, std::memory_order_release);
    return;
  }
  if (signal) {
    mb_wakeups.fetch_add(1, std::memory_order_relaxed);
    uint64_t one = 1;
    (void)!write(w->efd, &one, sizeof(one));
  }
}

void Frontend::wake_workers() {
  for (auto& w : workers_) {
    if (!w->unsignalled.exchange(false, std::memory_order_acq_rel)) continue;
    uint64_t one = 1;
    (void)!write(w->efd, &one, sizeof(one));
  }
}

namespace {
uint64_t uid_hash(std::string_view uid) {   // FNV-1a, never 0 (0 marks an empty slot)
  uint64_t h = 0xcbf29ce484222325ULL;
  for (const char c : uid) h = (h ^ static_cast<unsigned char>(c)) * 0x100000001b3ULL;
  return h | 1;
}
}  // namespace

const Frontend::PodEntry* Frontend::find_pod_locked(std::string_view uid, uint64_t h) const {
  const size_t nb = pod_slots_.size() / kPodWays;
  const PodEntry* b = &pod_slots_[((h >> 7) % nb) * kPodWays];
  for (size_t w = 0; w < kPodWays; ++w)
    if (b[w].h == h && b[w].uid == uid) return &b[w];
  return nullptr;
}

Frontend::PodEntry* Frontend::find_pod_locked(std::string_view uid, uint64_t h) {
  return const_cast<PodEntry*>(static_cast<const Frontend*>(this)->find_pod_locked(uid, h));
}

bool Frontend::has_pod(std::string_view uid) const {
  std::lock_guard<std::mutex> g(pod_mu_);
  return find_pod_locked(uid, uid_hash(uid)) != nullptr;
}

size_t Frontend::pod_cache_size() const {
  std::lock_guard<std::mutex> g(pod_mu_);
  return pod_live_;
}

namespace {
// CachedPod <-> the bytes of a bind handoff (Ledger::put_pod_info): namespace, name, container
// names, owner, completed flag and demand; not the pod's JSON text.
template <typename T>
void put_raw(std::string* o, const T& v) {
  o->append(reinterpret_cast<const char*>(&v), sizeof(T));
}
void put_str(std::string* o, std::string_view v) {
  put_raw(o, static_cast<uint16_t>(std::min<size_t>(v.size(), 0xffff)));
  o->append(v.data(), std::min<size_t>(v.size(), 0xffff));
}
void pack_pod(const CachedPod& p, const Demand& dem, std::string* o) {
  o->clear();
  put_str(o, p.ns);
  put_str(o, p.name);
  put_raw(o, static_cast<uint16_t>(p.containers.size()));
  for (const auto& c : p.containers) put_str(o, c);
  put_raw(o, p.owner);
  put_raw(o, static_cast<uint8_t>(p.completed));
  put_raw(o, dem.n);
  o->append(reinterpret_cast<const char*>(dem.c), sizeof(ContainerDemand) * static_cast<size_t>(dem.n));
}
struct Reader {
  std::string_view b;
  bool ok = true;
  template <typename T>
  T raw() {
    T v{};
    if (b.size() < sizeof(T)) return ok = false, v;
    std::memcpy(&v, b.data(), sizeof(T));
    b.remove_prefix(sizeof(T));
    return v;
  }
  std::string str() {
    const uint16_t n = raw<uint16_t>();
    if (!ok || b.size() < n) return ok = false, std::string();
    std::string v(b.substr(0, n));
    b.remove_prefix(n);
    return v;
  }
};
bool unpack_pod(std::string_view b, CachedPod* p) {
  Reader r{b};
  p->ns = r.str();
  p->name = r.str();
  const uint16_t nc = r.raw<uint16_t>();
  for (uint16_t i = 0; r.ok && i < nc; ++i) p->containers.push_back(r.str());
  p->owner = r.raw<uint64_t>();
  p->completed = r.raw<uint8_t>() != 0;
  std::memset(&p->demand, 0, sizeof(p->demand));
  p->demand.n = r.raw<int32_t>();
  if (!r.ok || p->demand.n < 0 || p->demand.n > kMaxContainers ||
      r.b.size() != sizeof(ContainerDemand) * static_cast<size_t>(p->demand.n))
    return false;
  std::memcpy(p->demand.c, r.b.data(), r.b.size());
  return true;
}
}  // namespace

void Frontend::put_pod(std::string_view uid, const CachedPod& meta, std::string_view raw, const Demand& dem) {
  if (uid.empty()) return;
  const uint64_t h = uid_hash(uid);
  std::lock_guard<std::mutex> g(pod_mu_);
  PodEntry* e = find_pod_locked(uid, h);
  if (!e) {   // an empty way of the bucket, else its oldest entry (a pod filtered but never bound)
    const size_t nb = pod_slots_.size() / kPodWays;
    PodEntry* b = &pod_slots_[((h >> 7) % nb) * kPodWays];
    e = &b[0];
    for (size_t w = 0; w < kPodWays; ++w) {
      if (b[w].h == 0) {
        e = &b[w];
        break;
      }
      if (b[w].stamp < e->stamp) e = &b[w];
    }
    if (e->h == 0) ++pod_live_;
    e->h = h;
    e->uid.assign(uid);
  }
  // assigned member by member: the entry's strings keep their capacity from pod to pod
  e->stamp = ++pod_stamp_;
  CachedPod& p = e->pod;
  p.raw.assign(raw);
  p.ns.assign(meta.ns);
  p.name.assign(meta.name);
  p.containers.resize(meta.containers.size());
  for (size_t i = 0; i < meta.containers.size(); ++i) p.containers[i].assign(meta.containers[i]);
  p.demand = dem;
  p.completed = meta.completed;
  p.owner = meta.owner;
}

void Frontend::prepare_bind(std::string_view body, PyRequest* r, VerbScratch& s) {
  thread_local json::Doc d;   // keeps its capacity across binds
  if (!d.parse(body) || !d.is(d.root(), json::Type::kObj)) return;
  auto str = [&](const char* k) -> std::string {
    const int32_t v = d.get(d.root(), k, true);
    return d.is(v, json::Type::kStr) ? std::string(d.str(v)) : std::string();
  };
  std::string uid = str("PodUID"), name = str("PodName"), node = str("Node");
  std::string ns = str("PodNamespace");
  if (ns.empty()) ns = "default";
  if (uid.empty() || name.empty() || node.empty()) return;
  int32_t id;
  {
    PhaseTimer pt{&phase_max_ns[5]};
    id = ledger_->find_node(node);
  }
  CachedPod pod;
  bool cached = false;
  {
    const uint64_t h = uid_hash(uid);
    const uint64_t tw = fast_ns();
    std::lock_guard<std::mutex> g(pod_mu_);
    atomic_max(&phase_max_ns[4], fast_ns() - tw);
    if (PodEntry* e = find_pod_locked(uid, h)) {   // one bind per pod UID: the entry is freed
      const CachedPod& c = e->pod;
      cached = true;
      if (c.name != name || c.ns != ns || c.completed || id < 0) {
        r->pod_json = c.raw;   // unusual: Python decides (and reports) with the object
      } else {
        pod.containers = c.containers;
        pod.demand = c.demand;
        pod.owner = c.owner;
      }
      e->h = 0;
      --pod_live_;
    }
  }
  if (cached && !r->pod_json.empty()) return;
  if (!cached) {
    // another worker process's filter parsed it (its bind came over another connection). That
    // worker publishes it just after its filter answer (Frontend::run_deferred): a bind that
    // overtook the publish waits for it a little, then goes to Python (which reads the pod)
    std::string blob;
    bool got = ledger_->take_pod_info(uid, &blob);
    if (!got && ledger_->attached() > 1) {
      const uint64_t t_end = fast_ns() + kHandoffWaitNs;
      while (!got && fast_ns() < t_end) {
        for (int k = 0; k < 64; ++k) __builtin_ia32_pause();
        got = ledger_->take_pod_info(uid, &blob);
      }
      if (got) handoff_waits.fetch_add(1, std::memory_order_relaxed);
    }
    if (!got || !unpack_pod(blob, &pod)) return;
    bind_handoffs.fetch_add(1, std::memory_order_relaxed);
    if (pod.name != name || pod.ns != ns || pod.completed || id < 0) return;   // Python reads the pod itself
  }
  // the options as of the last policy change this worker saw (as the verbs read them)
  if (s.opt_seen != opt_version_.load(std::memory_order_acquire) || s.opt_owner != serial_) {
    std::lock_guard<std::mutex> g(opt_mu_);
    s.opt = opt_;
    s.normalize = normalize_;
    s.nominate = nominate_;
    s.decisive = decisive_;
    s.lead = lead_;
    s.opt_owner = serial_;   // a thread_local scratch serves every Frontend of its thread
    s.opt_seen = opt_version_.load(std::memory_order_relaxed);
  }
  const Options& o = s.opt;
  const uint64_t t0 = fast_ns();
  Plan plan;
  std::memset(&plan, 0, sizeof(plan));
  PreparedBind& b = r->bind;
  b.rc = ledger_->reserve(id, uid, pod.demand, o, &plan);
  if ((b.rc == kOk || b.rc == kOkExisting) && pod.owner) ledger_->set_pod_owner(uid, pod.owner);
  bind_stats.observe(fast_ns() - t0);
  b.ok = true;
  b.ns = std::move(ns);
  b.name = std::move(name);
  b.uid = std::move(uid);
  b.node = std::move(node);
  b.containers = std::move(pod.containers);
  for (int c = 0; c < pod.demand.n; ++c) b.demand.emplace_back(pod.demand.c[c].pct, pod.demand.c[c].mib);
  if (b.rc == kOk || b.rc == kOkExisting)
    for (int c = 0; c < plan.n; ++c) b.plan.emplace_back(plan.idx + plan.off[c], plan.idx + plan.off[c + 1]);
}

// ------------------------------------------------------------------------------ event loop
void Frontend::run(Worker* w) {
  epoll_event evs[128];
  std::vector<uint64_t> later;   // connections whose next request is a bind
  std::vector<std::pair<uint64_t, uint32_t>> bio_later;   // BindIo events of this batch
  // Busy polling only where a wake-up would sit on kube-scheduler's critical path: after this
  // worker replied to a filter or priorities request. kube-scheduler's scheduling cycle is
  // serial (filter, then priorities, then the next pod's filter a few microseconds later), so
  // the next cycle request is due soon; a bind is asynchronous and its reply, or a writer's
  // completion, never starts a spin. Adaptive on top: the first event after a cycle reply is a
  // hit if it came within the spin window; a worker spins while at least half of its last 16
  // were hits (a slow scheduler, tens of microseconds between verbs, is not spun for).
  uint32_t gaps = 0xffffu;   // 1 bits: hits among the last 16 cycle replies (start hot)
  uint64_t scored = 0;       // the cycle reply the last hit/miss was scored for
  // responses posted by the bind writer or Python: sent, then the connection's next request
  auto drain_mailbox = [&] {
    PhaseTimer pt{&phase_max_ns[1]};
    std::vector<Reply>& mb = w->mb_spare;
    mb.clear();
    {
      std::lock_guard<std::mutex> g(w->mb_mu);
      mb.swap(w->mailbox);
      w->mb_signalled = false;
      w->mb_pending.store(false, std::memory_order_relaxed);
    }
    for (Reply& m : mb) deliver_reply(w, m);
    mb.clear();
  };
  while (!stop_.load(std::memory_order_acquire)) {
    const int64_t prio_spin = busy_poll_prio_ns_.load(std::memory_order_relaxed);
    const int64_t spin = w->cycle_was_prio && prio_spin >= 0 ? prio_spin : busy_poll_ns_.load(std::memory_order_relaxed);
    const bool hot = __builtin_popcount(gaps & 0xffffu) >= 8;
    const uint64_t since = w->cycle_reply_ns;
    const uint64_t t_now = fast_ns();
    const bool polling = spin > 0 && hot && since && t_now - since < static_cast<uint64_t>(spin);
    // nap: the spin window is slept in the kernel (epoll_pwait2 with the window's remaining
    // microseconds) instead of polled: a request that arrives wakes the worker, and idle
    // periods that short keep the core in its shallowest idle state (fast exit), while the
    // window costs no CPU time
    const bool nap = polling && spin_nap_.load(std::memory_order_relaxed);
    if (!polling || nap) {
      w->parked.store(true, std::memory_order_seq_cst);
      if (w->mb_pending.load(std::memory_order_seq_cst)) {   // posted before we parked
        w->parked.store(false, std::memory_order_relaxed);
        drain_mailbox();
        continue;
      }
    }
    BindIo* bio = w->bio.load(std::memory_order_acquire);
    if (polling && !nap && spin_recv_.load(std::memory_order_relaxed) && !bind_first_.load(std::memory_order_relaxed) &&
        spin_recv_hot(w)) {   // (binds first: a bind on another connection must not wait behind it)
      if (since != scored) {   // caught inside the window
        gaps = (gaps << 1) | 1u;
        scored = since;
      }
      spin_hits.fetch_add(1, std::memory_order_relaxed);
      if (bio) {
        bio->pump();
        drain_local(w);
      }
      if (w->mb_pending.load(std::memory_order_acquire)) drain_mailbox();
      continue;
    }
    int n;
    const uint64_t io0 = io_t0();
    if (nap) {
      const timespec ts{0, static_cast<long>(static_cast<uint64_t>(spin) - (t_now - since))};
      n = epoll_pwait2(w->ep, evs, 128, &ts, nullptr);
    } else {
      // with bind answers due, wake at least for the BindIo's deadline scan
      n = epoll_wait(w->ep, evs, 128, polling ? 0 : bio && bio->labels_waiting() ? 1 : bio && bio->inflight() ? 100 : 200);
    }
    if (io0 && polling && !nap && n <= 0 && w->cycle_was_prio) g_io.add(kFeSpinAfterPrio, __rdtsc() - io0);
    io_end(polling && !nap ? (n > 0 ? kFeSpinHit : kFeSpinEmpty) : kFeWait, io0);
    w->parked.store(false, std::memory_order_relaxed);
    const uint64_t t_batch = n > 0 ? fast_ns() : 0;
    if (n > 0) {
      if (spin > 0 && since && since != scored) {
        gaps = (gaps << 1) | (t_batch - since < static_cast<uint64_t>(spin) ? 1u : 0u);
        scored = since;
      }
      if (polling) spin_hits.fetch_add(1, std::memory_order_relaxed);   // caught without a wake-up
    }
    struct BatchTimer {
      Frontend* f;
      uint64_t t0;
      ~BatchTimer() {
        if (t0) atomic_max(&f->loop_max_ns, fast_ns() - t0);
      }
    } batch_timer{this, t_batch};
    for (int i = 0; i < n; ++i) {
      const uint64_t tag = evs[i].data.u64;
      if (tag == 0) {
        PhaseTimer pt{&phase_max_ns[0]};
        for (;;) {
          const int fd = accept4(w->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (fd < 0) break;
          int one = 1;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          auto c = std::make_unique<Conn>();
          c->fd = fd;
          c->id = w->next_conn++;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.u64 = (c->id << 1) | (1ull << 63);
          epoll_ctl(w->ep, EPOLL_CTL_ADD, fd, &ev);
          connections.fetch_add(1, std::memory_order_relaxed);
          w->conns.emplace(c->id, std::move(c));
        }
      } else if (tag == 1) {
        uint64_t v;
        {
          IoTimer it{kFeEfdRead};
          (void)!read(w->efd, &v, sizeof(v));
        }
        drain_mailbox();
      } else if (!(tag >> 63) && (tag & kBioTag)) {
        // API answers after this batch's scheduling-cycle requests: a bind's answer only ends
        // an asynchronous binding, the cycle's next pod waits on filter / priorities
        const uint32_t ev = evs[i].events;   // epoll_event is packed: no reference into it
        bio_later.emplace_back(tag & ~kBioTag, ev);
      } else {
        PhaseTimer pt{&phase_max_ns[2]};
        const uint64_t cid = (tag & ~(1ull << 63)) >> 1;
        auto it = w->conns.find(cid);
        if (it == w->conns.end()) continue;
        Conn* c = it->second.get();
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
          close_conn(w, c);
          continue;
        }
        if (evs[i].events & EPOLLOUT) {
          flush(w, c);
          if (!w->conns.count(cid)) continue;
        }
        if (evs[i].events & (EPOLLIN | EPOLLRDHUP)) {
          bool eof = false;
          if (!read_in(w, c, &eof)) continue;
          // Which verb of a batch goes first. Cycle first: kube-scheduler's next pod waits on
          // filter / priorities, while a bind's reply only ends an asynchronous binding
          // goroutine. Binds first (set_bind_first): the bind of pod i is reserved before
          // pod i+1's filter reads the ledger, so a pod kube-scheduler placed off its
          // nomination (or never nominated) is not invisible to the next pod's placement.
          const bool is_bind = c->in.compare(0, 20, "POST /scheduler/bind") == 0;
          if (!eof && is_bind != bind_first_.load(std::memory_order_relaxed)) {
            later.push_back(cid);
            continue;
          }
          after_read(w, c, eof);
        }
      }
    }
    for (uint64_t cid : later) {
      PhaseTimer pt{&phase_max_ns[3]};
      auto it = w->conns.find(cid);
      if (it != w->conns.end()) after_read(w, it->second.get(), false);
    }
    later.clear();
    if (bio)
      for (const auto& e : bio_later) bio->on_event(e.first, e.second);
    bio_later.clear();
    if (bio) {   // the binds this batch parsed go out now; answers that came in are replied
      bio->pump();
      drain_local(w);
    }
    if (w->mb_pending.load(std::memory_order_acquire)) drain_mailbox();   // posted while awake
  }
  // stopping: the binds this worker has in flight finish (bounded), else the slow path takes
  // them; their answers still reach kube-scheduler on the open connections
  if (BindIo* bio = w->bio.load(std::memory_order_acquire)) {
    const uint64_t until = fast_ns() + 5'000'000'000ull;
    while (bio->inflight() + bio->waiting() > 0 && fast_ns() < until) {
      const int n = epoll_wait(w->ep, evs, 128, 10);
      for (int i = 0; i < n; ++i) {
        const uint64_t tag = evs[i].data.u64;
        if (!(tag >> 63) && (tag & kBioTag)) bio->on_event(tag & ~kBioTag, evs[i].events);
      }
      bio->pump();
      drain_local(w);
    }
    bio->abandon("extender shutting down");
    drain_local(w);
  }
  drain_mailbox();
}

void Frontend::deliver_reply(Worker* w, const Reply& r) {
  const uint64_t conn = r.conn;
  auto it = w->conns.find(conn);
  if (it == w->conns.end()) return;
  Conn* c = it->second.get();
  append_http(&c->out, r.status, r.ctype.empty() ? std::string_view("application/json") : std::string_view(r.ctype), r.body);
  c->waiting = false;
  const bool was_bind = c->bind_waiting;
  const uint64_t t_req = c->t_req_ns;
  c->bind_waiting = false;
  flush(w, c);   // may close the connection (Connection: close, a peer reset): c is gone then
  if (was_bind) {
    note_bind_wall(fast_ns() - t_req);   // handed to the kernel: extender-side wall time
    w->bind_cid = conn;   // back in kube-scheduler's idle pool, the next bind's likeliest (LIFO)
    uint64_t hv[kBindHops];
    if (g_hops.close(make_id(w->idx, conn), hv)) {
      const double k = io_ns_per_tick();
      std::array<uint32_t, kHopSplits> d{};
      for (int h = 0; h < kHopSplits; ++h)
        d[h] = static_cast<uint32_t>(std::min(4.0e9, static_cast<double>(hv[h + 1] - hv[h]) * k));
      std::lock_guard<std::mutex> g(wall_mu_);
      if (bind_hops_.size() < kMaxWallSamples) bind_hops_.push_back(d);
    }
  }
  if (w->conns.count(conn)) process(w, c);
}

void Frontend::drain_local(Worker* w) {
  // process() below may parse the next bind and queue more: swap first, loop until empty
  std::vector<Reply>& batch = w->local_spare;
  while (!w->local_replies.empty()) {
    batch.clear();
    batch.swap(w->local_replies);
    for (const Reply& r : batch) deliver_reply(w, r);
    if (BindIo* bio = w->bio.load(std::memory_order_relaxed)) bio->pump();
  }
}

bool Frontend::read_in(Worker* w, Conn* c, bool* eof) {
  char buf[65536];
  *eof = false;
  for (;;) {
    ssize_t r;
    {
      IoTimer it{kFeRecv};
      r = recv(c->fd, buf, sizeof(buf), 0);
    }
    if (r > 0) {
      if (c->in.empty()) c->t_in_ns = fast_ns();
      c->in.append(buf, static_cast<size_t>(r));
      if (c->in.size() > kMaxBody + kMaxHeader) {
        close_conn(w, c);
        return false;
      }
      // a short read drained the socket: no second recv() just to see EAGAIN (the epoll is
      // level-triggered, so bytes that arrive after this are reported again)
      if (static_cast<size_t>(r) < sizeof(buf)) break;
      continue;
    }
    if (r == 0) *eof = true;
    else if (errno == EINTR) continue;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) *eof = true;
    break;
  }
  return true;
}

bool Frontend::spin_recv_hot(Worker* w) {
  if (spin_recv_conn(w, w->cycle_cid)) return true;
  return spin_recv_binds_.load(std::memory_order_relaxed) && w->bind_cid != w->cycle_cid &&
         spin_recv_conn(w, w->bind_cid);
}

bool Frontend::spin_recv_conn(Worker* w, uint64_t cid) {
  // one non-blocking recv on the connection the last cycle answer went out on: a request
  // found there is handled without the epoll_wait that would report it and the recv after it
  auto it = w->conns.find(cid);
  if (it == w->conns.end()) return false;
  Conn* c = it->second.get();
  if (c->waiting || c->close_after) return false;
  char buf[16384];
  ssize_t r;
  {
    IoTimer t{kFeSpinRecv};
    r = recv(c->fd, buf, sizeof(buf), MSG_DONTWAIT);
  }
  if (r < 0) return false;   // EAGAIN (nothing yet) or an error epoll reports next
  if (r == 0) {
    after_read(w, c, true);
    return true;
  }
  if (c->in.empty()) c->t_in_ns = fast_ns();
  c->in.append(buf, static_cast<size_t>(r));
  if (static_cast<size_t>(r) == sizeof(buf)) {   // more behind it: the usual reader takes it
    bool eof = false;
    if (!read_in(w, c, &eof)) return true;
    after_read(w, c, eof);
    return true;
  }
  after_read(w, c, false);
  return true;
}

void Frontend::after_read(Worker* w, Conn* c, bool eof) {
  const uint64_t id = c->id;
  process(w, c);
  if (!w->conns.count(id)) return;
  if (eof && !c->waiting && c->out.size() == c->out_off) close_conn(w, c);
  else if (eof) c->close_after = true;
}

void Frontend::process(Worker* w, Conn* c) {
  const uint64_t id = c->id;
  while (!c->waiting) {
    const size_t he = c->in.find("\r\n\r\n");
    if (he == std::string::npos) {
      if (c->in.size() > kMaxHeader) close_conn(w, c);
      return;
    }
    const std::string_view head(c->in.data(), he);
    const size_t le = head.find("\r\n");
    const std::string_view line = head.substr(0, le);
    const size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string_view::npos || s2 == s1) {
      close_conn(w, c);
      return;
    }
    const std::string_view method = line.substr(0, s1);
    const std::string_view target = line.substr(s1 + 1, s2 - s1 - 1);
    const bool http10 = line.substr(s2 + 1) == "HTTP/1.0";
    size_t clen = 0;
    bool chunked = false, close = http10, keep = false, have_clen = false;
    size_t pos = le == std::string_view::npos ? head.size() : le + 2;
    while (pos < head.size()) {
      size_t e = head.find("\r\n", pos);
      if (e == std::string_view::npos) e = head.size();
      const std::string_view h = head.substr(pos, e - pos);
      const size_t colon = h.find(':');
      if (colon != std::string_view::npos) {
        const std::string_view k = trim(h.substr(0, colon)), v = trim(h.substr(colon + 1));
        if (ieq(k, "content-length")) {
          // no allocation per request; a malformed length (trailing bytes included: "12abc",
          // "12, 34") or a repeated header that disagrees reads as too large (refused below)
          size_t v_len = 0;
          const auto r = std::from_chars(v.data(), v.data() + v.size(), v_len);
          if (r.ec != std::errc() || r.ptr != v.data() + v.size() || v.empty() || (have_clen && v_len != clen))
            v_len = SIZE_MAX;
          clen = have_clen && clen == SIZE_MAX ? SIZE_MAX : v_len;
          have_clen = true;
        } else if (ieq(k, "transfer-encoding")) {
          chunked = v.find("chunked") != std::string_view::npos;
        } else if (ieq(k, "connection")) {
          if (ieq(v, "close")) close = true;
          if (ieq(v, "keep-alive")) keep = true;
        }
      }
      pos = e + 2;
    }
    if (http10 && keep) close = false;
    if (chunked && have_clen) {   // both framings: request smuggling territory, refused
      close_conn(w, c);
      return;
    }
    // the body stays a view into the connection's input unless it came chunked; the input is
    // consumed only after the request is handled (the views point into it)
    thread_local std::string chunked_body;
    std::string_view body;
    size_t consumed;
    if (chunked) {
      chunked_body.clear();
      size_t p = he + 4;
      for (;;) {
        const size_t le2 = c->in.find("\r\n", p);
        if (le2 == std::string::npos) return;  // need more
        const size_t n = std::strtoull(c->in.substr(p, le2 - p).c_str(), nullptr, 16);
        if (c->in.size() < le2 + 2 + n + 2) return;
        if (n == 0) {
          // last chunk: optional trailer lines, then the blank line
          const size_t end = c->in.find("\r\n\r\n", le2);
          if (end == std::string::npos) return;  // need more
          consumed = end + 4;
          break;
        }
        chunked_body.append(c->in, le2 + 2, n);
        if (chunked_body.size() > kMaxBody) {
          close_conn(w, c);
          return;
        }
        p = le2 + 2 + n + 2;
      }
      body = chunked_body;
    } else {
      if (clen > kMaxBody) {
        close_conn(w, c);
        return;
      }
      if (c->in.size() < he + 4 + clen) return;  // need more
      body = std::string_view(c->in).substr(he + 4, clen);
      consumed = he + 4 + clen;
    }
    if (close) c->close_after = true;
    requests.fetch_add(1, std::memory_order_relaxed);
    std::string_view path = target, query;
    const size_t qm = target.find('?');
    if (qm != std::string_view::npos) {
      path = target.substr(0, qm);
      query = target.substr(qm + 1);
    }
    const bool prio = path == "/scheduler/priorities";   // `path` views c->in, erased below
    if (handle_native(w, c, method, path, body, &c->out)) {   // the answer lands in c->out
      const uint64_t t_in = c->t_in_ns;
      c->in.erase(0, consumed);
      if (!c->in.empty()) c->t_in_ns = fast_ns();   // a pipelined request behind it: its own clock
      flush(w, c, kFeSendCycle);
      w->cycle_reply_ns = fast_ns();   // the scheduling cycle's next request is due: spin for it
      if (t_in) (prio ? prio_wall_stats : filter_wall_stats).observe(w->cycle_reply_ns - t_in);
      w->cycle_was_prio = prio;
      w->cycle_cid = id;
      run_deferred(w->scratch);        // the answer is out: the pod cache / nomination now
      if (!w->conns.count(id)) return;
    } else {
      std::string m(method), pth(path), q(query), b(body);   // owned: the Python side keeps them
      c->in.erase(0, consumed);
      defer(w, c, std::move(m), std::move(pth), std::move(q), std::move(b));
    }
  }
}

void Frontend::defer(Worker* w, Conn* c, std::string method, std::string path, std::string query, std::string body) {
  PyRequest r;
  r.id = make_id(w->idx, c->id);
  if (method == "POST" && path == "/scheduler/bind" && serving()) {
    {
      IoTimer it{kFeParseBind};
      prepare_bind(body, &r, w->scratch);
    }
    KubeWriter* kw = writer_.load(std::memory_order_acquire);
    BindIo* bio = w->bio.load(std::memory_order_acquire);
    if (kw && r.bind.ok && (r.bind.rc == kOk || r.bind.rc == kOkExisting) && (bio || !kw->inline_io())) {
      // the whole bind stays native: API writes and commit on the writer's threads
      BindJob j;
      j.id = r.id;
      j.ns = std::move(r.bind.ns);
      j.name = std::move(r.bind.name);
      j.uid = std::move(r.bind.uid);
      j.node = std::move(r.bind.node);
      j.containers = std::move(r.bind.containers);
      j.plan = std::move(r.bind.plan);
      j.fresh = r.bind.rc == kOk;
      j.t0_ns = now_ns();   // read by the writer's threads: the shared clock
      c->waiting = true;
      c->bind_waiting = true;
      c->t_req_ns = c->t_in_ns ? c->t_in_ns : fast_ns();
      c->t_in_ns = c->in.empty() ? 0 : fast_ns();
      g_hops.open(j.id, tsc_of(c->t_req_ns));
      IoTimer it{kFeSubmit};
      if (bio) bio->submit(std::move(j));   // sent by pump() after this batch of events
      else if (!kw->send_from_caller(j)) kw->submit(std::move(j));   // sent here, or by the writer
      return;
    }
  }
  r.method = std::move(method);
  r.path = std::move(path);
  r.query = std::move(query);
  r.body = std::move(body);
  r.t_arrival = now_s();
  c->waiting = true;
  c->bind_waiting = r.path == "/scheduler/bind";
  c->t_req_ns = c->t_in_ns ? c->t_in_ns : fast_ns();
  c->t_in_ns = c->in.empty() ? 0 : fast_ns();   // pipelined bytes behind it: their clock starts now
  py_stats.deferred.fetch_add(1, std::memory_order_relaxed);
  PhaseTimer pt{&phase_max_ns[6]};
  {
    std::lock_guard<std::mutex> g(py_mu_);
    py_q_.push_back(std::move(r));
  }
  uint64_t one = 1;
  (void)!write(py_efd_, &one, sizeof(one));
}

void Frontend::flush(Worker* w, Conn* c, int io_kind) {
  while (c->out_off < c->out.size()) {
    ssize_t n;
    {
      IoTimer it{io_kind};
      n = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    }
    if (n > 0) {
      c->out_off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      if (!c->want_out) {
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
        ev.data.u64 = (c->id << 1) | (1ull << 63);
        epoll_ctl(w->ep, EPOLL_CTL_MOD, c->fd, &ev);
        c->want_out = true;
      }
      return;
    }
    close_conn(w, c);
    return;
  }
  c->out.clear();
  c->out_off = 0;
  if (c->want_out) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = (c->id << 1) | (1ull << 63);
    epoll_ctl(w->ep, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = false;
  }
  if (c->close_after && !c->waiting) close_conn(w, c);
}

void Frontend::close_conn(Worker* w, Conn* c) {
  epoll_ctl(w->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
  w->conns.erase(c->id);   // destroys c
}

// ------------------------------------------------------------------------------ verbs
void Frontend::cache_pod(VerbScratch& s, std::string_view uid, const CachedPod& cached, std::string_view raw,
                         const Demand& dem) {
  if (ledger_->attached() > 1) {
    // other worker processes share the ledger: the bind may reach one of them
    std::string& blob = s.blob;
    pack_pod(cached, dem, &blob);
    if (ledger_->put_pod_info(uid, blob)) pods_published.fetch_add(1, std::memory_order_relaxed);
  }
  put_pod(uid, cached, raw, dem);
}

bool Frontend::defer_nominate_ok(const VerbScratch& s) const { return s.defer_cache; }

bool Frontend::reuse_assume(VerbScratch& s, std::string_view uid, const Demand& dem, const std::vector<int32_t>& ids,
                            std::vector<int32_t>* rcs, std::vector<int32_t>* scores) {
  VerbScratch::LastAssume& la = s.last_assume;
  if (!la.valid) return false;
  la.valid = false;   // one use: the priorities call right behind its filter
  if (uid.empty() || uid != la.uid || la.opt_seen != s.opt_seen || la.dem_hash != dem.hash() ||
      la.epoch != ledger_->epoch())
    return false;
  if (ids == la.ids) {
    std::copy(la.rcs.begin(), la.rcs.end(), rcs->begin());
    std::copy(la.scores.begin(), la.scores.end(), scores->begin());
    return true;
  }
  // the filter's fitting nodes, in the filter's order (what kube-scheduler sends when some
  // nodes did not fit)
  size_t j = 0;
  for (size_t i = 0; i < ids.size(); ++i) {
    while (j < la.ids.size() && la.rcs[j] != kOk) ++j;
    if (j == la.ids.size() || la.ids[j] != ids[i]) return false;
    (*rcs)[i] = kOk;
    (*scores)[i] = la.scores[j++];
  }
  return true;
}

void Frontend::run_deferred(VerbScratch& s) {
  if (s.defer_list >= 0) {
    IoTimer it{kFeVerbNames};
    s.idc.remember_subset(s.defer_list, s.rcs);
    s.defer_list = -1;
  }
  if (!s.defer_put && !s.defer_nominate) return;
  const LastPod& last = s.last;
  if (s.defer_put) {
    IoTimer it{kFeVerbCache};
    cache_pod(s, last.uid, last.cached, last.raw, s.defer_dem);
  }
  if (s.defer_nominate) {
    IoTimer it{kFeVerbNominate};
    ledger_->nominate(s.defer_node, last.uid, s.defer_dem, s.opt);
    ledger_->deferred_nomination_end();
  }
  s.defer_put = s.defer_nominate = false;
}

bool Frontend::handle_native(Worker* w, Conn* c, std::string_view method, std::string_view path,
                             std::string_view body, std::string* out) {
  (void)c;
  if (method != "POST" || !serving()) return false;
  const bool prio = path == "/scheduler/priorities";
  if (!prio && path != "/scheduler/filter") return false;
  const uint64_t t0 = fast_ns();
  std::string& resp = w->scratch.resp;   // keeps its capacity: no allocation per request
  IoTimer it{kFeVerb};
  if (!filter_verb(body, prio, &resp, w->scratch)) return false;
  (prio ? prio_stats : filter_stats).observe(fast_ns() - t0);
  constexpr std::string_view kHead = "HTTP/1.1 200 OK\r\nContent-Type: application/json; charset=utf-8\r\nContent-Length: ";
  char len[24];
  const char* e = std::to_chars(len, len + sizeof len, resp.size()).ptr;
  out->reserve(out->size() + kHead.size() + 24 + resp.size());
  *out += kHead;
  out->append(len, static_cast<size_t>(e - len));
  *out += "\r\n\r\n";
  *out += resp;
  return true;
}

bool Frontend::filter_verb(std::string_view body, bool prioritize, std::string* out) {
  thread_local VerbScratch s;   // callers off the workers (tests, time_verb)
  return filter_verb(body, prioritize, out, s);
}

bool Frontend::filter_verb(std::string_view body, bool prioritize, std::string* out, VerbScratch& s) {
  json::Doc& top = s.top;
  json::Doc& d = s.d;
  std::vector<std::string_view>& nv = s.nv;
  std::vector<std::string_view>& nraw = s.nraw;
  std::vector<int32_t>& rcs = s.rcs;
  std::vector<int32_t>& scores = s.scores;
  LastPod& last = s.last;
  IdCache& idc = s.idc;
  uint64_t io0 = io_t0();
  if (idc.owner != serial_) idc = IdCache{}, idc.owner = serial_;
  if (body.empty()) return false;
  // kube-scheduler's ExtenderArgs as Go's encoding/json writes them (struct field order, no
  // spaces): {"Pod":{...},"Nodes":null,"NodeNames":[...]}. In that exact layout the pod's text
  // is found by comparing it with the last pod's (priorities, and every retry, sends the same
  // text) or by parsing it where it starts, and the node list runs to the closing brace: no
  // pass over the body just to find where its members end. Any other layout takes the general
  // path below (a shallow parse of the top level, then the members).
  constexpr std::string_view kHead = "{\"Pod\":", kMid = ",\"Nodes\":null,\"NodeNames\":";
  std::string_view pod_text, raw_names;
  bool framed = false, reused = false, has_pod_text = false;
  bool scanned = false;   // s.ntok holds raw_names' tokens (a list not in the cache)
  int found = -2;         // the list's cache slot when the framing looked it up (-1: none)
  int32_t pod = -1;
  nv.clear();
  nraw.clear();
  if (body.size() > kHead.size() + kMid.size() + 4 && body.compare(0, kHead.size(), kHead) == 0 &&
      body[kHead.size()] == '{' && body.back() == '}') {
    const std::string_view rest = body.substr(kHead.size());
    size_t pe = 0;
    bool same = false;
    if (last.valid && rest.size() > last.raw.size() && std::memcmp(rest.data(), last.raw.data(), last.raw.size()) == 0) {
      pe = last.raw.size();
      same = true;
    } else if (!d.parse_prefix(rest, &pe) || !d.is(d.root(), json::Type::kObj)) {
      pe = 0;
    }
    if (pe) {
      const std::string_view tail = rest.substr(pe);
      if (tail.size() > kMid.size() + 2 && tail.compare(0, kMid.size(), kMid) == 0 && tail[kMid.size()] == '[' &&
          tail[tail.size() - 2] == ']') {
        raw_names = tail.substr(kMid.size(), tail.size() - kMid.size() - 1);
        // the list must be one: a cached text, or a compact string array scanned whole
        // (anything else, members after it included, goes the general way)
        found = idc.find(raw_names);
        if (found < 0) s.ntok.clear();
        framed = found >= 0 || (scanned = scan_string_array(raw_names, &s.ntok));
        if (framed) {
          has_pod_text = true;
          pod_text = rest.substr(0, pe);
          reused = same;
          if (!same) pod = d.root();
        } else {
          nv.clear();
          nraw.clear();
        }
      }
    }
  }
  if (!framed) {
    // The body's top level only (Pod and NodeNames stay unparsed text), then the Pod on its own
    // (`d`); the node-name list is parsed only when this worker has not seen that exact text.
    if (!top.parse_shallow(body, 1)) return false;
    const int32_t root = top.root();
    if (!top.is(root, json::Type::kObj)) return false;
    const int32_t names = top.get(root, "NodeNames", true);
    if (!top.is(names, json::Type::kArr)) return false;     // null / Nodes-only: Python path
    const int32_t pod_top = top.get(root, "Pod", true);
    // any other member that is an object or array was only bracket-checked: the whole body
    // must be valid JSON, as for the Python verb (which answers 400 otherwise)
    for (int32_t c = top.at(root).first; c >= 0; c = top.at(c).next) {
      if (c == names || c == pod_top) continue;
      if (top.is(c, json::Type::kObj) || top.is(c, json::Type::kArr)) {
        if (!s.other.parse(top.raw(c))) return false;
      }
    }
    raw_names = top.raw(names);
    has_pod_text = pod_top >= 0 && !top.is(pod_top, json::Type::kNull);
    if (has_pod_text) pod_text = top.raw(pod_top);
    reused = has_pod_text && last.valid && top.is(pod_top, json::Type::kObj) && pod_text == last.raw;
    if (has_pod_text && !reused) {
      if (!top.is(pod_top, json::Type::kObj) || !d.parse(pod_text)) return false;
      pod = d.root();
    }
  }
  Demand dem;
  std::memset(&dem, 0, sizeof(dem));
  std::string_view uid;
  // the pod's identity and containers are parsed into the last-pod record itself (its strings
  // keep their capacity); it is valid again only once the parse succeeded with a UID
  CachedPod& cached = last.cached;
  bool mb_annotated = false;
  if (reused) {
    dem = last.dem;
    uid = last.uid;
    mb_annotated = last.mb_annotated;
  } else {
    last.valid = false;
    cached.ns.clear();
    cached.name.clear();
    cached.containers.clear();
    cached.completed = false;
    cached.owner = 0;
    if (pod >= 0 && !d.is(pod, json::Type::kNull)) {
      if (!d.is(pod, json::Type::kObj)) return false;
      const int32_t md = d.get(pod, "metadata");
      if (md >= 0 && !d.is(md, json::Type::kNull)) {
        if (!d.is(md, json::Type::kObj)) return false;
        const int32_t u = d.get(md, "uid");
        if (u >= 0) {
          if (!d.is(u, json::Type::kStr)) return false;
          uid = d.str(u);
        }
        const int32_t nm = d.get(md, "name"), ns = d.get(md, "namespace"), del = d.get(md, "deletionTimestamp");
        if (d.is(nm, json::Type::kStr)) cached.name.assign(d.str(nm));
        cached.ns.assign(d.is(ns, json::Type::kStr) ? d.str(ns) : std::string_view("default"));
        if (del >= 0 && !d.is(del, json::Type::kNull) && !(d.is(del, json::Type::kStr) && d.str(del).empty()))
          cached.completed = true;
      }
      const int32_t stt = d.get(pod, "status");
      if (d.is(stt, json::Type::kObj)) {
        const int32_t ph = d.get(stt, "phase");
        if (d.is(ph, json::Type::kStr) && (d.str(ph) == "Succeeded" || d.str(ph) == "Failed")) cached.completed = true;
      }
      const int32_t spec = d.get(pod, "spec");
      int32_t cons = -1;
      if (spec >= 0 && !d.is(spec, json::Type::kNull)) {
        if (!d.is(spec, json::Type::kObj)) return false;
        cons = d.get(spec, "containers");
      }
      if (cons >= 0 && !d.is(cons, json::Type::kNull)) {
        if (!d.is(cons, json::Type::kArr)) return false;
        if (d.at(cons).count > kMaxContainers) return false;
        for (int32_t c = d.at(cons).first; c >= 0; c = d.at(c).next) {
          if (!d.is(c, json::Type::kObj)) return false;
          ContainerDemand& cd = dem.c[dem.n++];
          const int32_t cn = d.get(c, "name");
          cached.containers.emplace_back(d.is(cn, json::Type::kStr) ? d.str(cn) : std::string_view());
          const int32_t res = d.get(c, "resources");
          int32_t lim = -1;
          if (res >= 0 && !d.is(res, json::Type::kNull)) {
            if (!d.is(res, json::Type::kObj)) return false;
            lim = d.get(res, "limits");
          }
          if (lim >= 0 && !d.is(lim, json::Type::kNull)) {
            if (!d.is(lim, json::Type::kObj)) return false;
            for (int k = 0; k < 2; ++k) {
              const int32_t q = d.get(lim, k == 0 ? kPercent : kMemory);
              if (q < 0 || d.is(q, json::Type::kNull)) continue;
              if (!d.is(q, json::Type::kStr) && !d.is(q, json::Type::kNum)) return false;
              int64_t v;
              if (!quantity_value(d.str(q), k == 1, &v)) return false;  // Python logs + treats as 0
              if (k == 0) {
                if (v > INT32_MAX) return false;
                cd.pct = static_cast<int32_t>(v);
              } else {
                cd.mib = v;
              }
            }
          }
        }
      }
    }
    // nano-gpu/memory-bound: "true" (every container) or a comma list of container names. With
    // no annotation, a pod whose controlling owner was measured streaming (Ledger stream owners,
    // nanogpu.telemetry.poller.OwnerLearner) counts as memory-bound; "false" opts out.
    if (pod >= 0 && d.is(pod, json::Type::kObj)) {
      const int32_t md = d.get(pod, "metadata");
      const int32_t ann = d.is(md, json::Type::kObj) ? d.get(md, "annotations") : -1;
      const int32_t mb = d.is(ann, json::Type::kObj) ? d.get(ann, kMemBoundAnnotation) : -1;
      if (d.is(mb, json::Type::kStr)) {
        const std::string_view v = d.str(mb);
        for (int c = 0; c < dem.n; ++c)
          if (v == "true" || list_has(v, cached.containers[c])) dem.c[c].flags |= kFlagMemBound;
      }
      if (d.is(md, json::Type::kObj)) {
        const std::string_view owner = controller_uid(d, d.get(md, "ownerReferences"));
        if (!owner.empty()) cached.owner = owner_hash(owner);
      }
      mb_annotated = d.is(mb, json::Type::kStr);
    }
    if (pod >= 0 && !uid.empty()) {
      last.raw.assign(pod_text);
      last.uid.assign(uid);
      last.dem = dem;
      last.mb_annotated = mb_annotated;
      last.valid = true;
      uid = last.uid;   // `d` is reparsed by the next request; the uid outlives it here
    }
  }
  // A learned streaming owner marks an unannotated pod memory-bound. Read per request, not
  // memoised per pod: a learning pass between a pod's priorities and its bind can change the
  // flag. The bind then adopts the priorities-time nomination, whose plan and demand the ledger
  // keeps (Ledger::reserve), so the pod lands where it was scored
  // (tests/test_frontend.py::test_owner_learned_between_priorities_and_bind_is_tolerated).
  {
    const uint64_t owner = reused ? last.cached.owner : cached.owner;
    if (!mb_annotated && owner && ledger_->is_stream_owner(owner))
      for (int c = 0; c < dem.n; ++c) dem.c[c].flags |= kFlagMemBound;
  }
  // node ids: any unknown node goes to Python, which can register it from its informer.
  // kube-scheduler sends the same node list over and over, so each worker remembers the ids
  // of the last lists it resolved (keyed by the array's raw text) and only checks that slot
  // `id` still carries that name; a miss falls back to the ledger's name index.
  io_end(kFeVerbPod, io0);
  io0 = io_t0();
  const uint64_t epoch = ledger_->node_epoch();
  int slot = scanned ? -1 : framed && found != -2 ? found : idc.find(raw_names);
  // a list's names are read through its token offsets into this request's text (no per-request
  // copy of 2 x N views); only a list in another shape fills nv / nraw
  const std::vector<std::pair<uint32_t, uint32_t>>* toks = nullptr;
  if (slot >= 0) {
    // the same list text as before: its tokens sit at the same offsets (escape-free lists
    // only are cached); names and ids come from the cache
    toks = &idc.tok[slot];
  } else {
    // the common shape first, scanned directly: ["a","b",...] with no escapes; anything else
    // (whitespace, escapes, other types) goes through the JSON parser
    if (!scanned) s.ntok.clear();
    const bool compact = scanned || scan_string_array(raw_names, &s.ntok);
    bool plain = compact;
    if (!plain) {
      nv.clear();
      nraw.clear();
      json::Doc& dn = s.dn;
      if (!dn.parse(raw_names) || !dn.is(dn.root(), json::Type::kArr)) return false;
      plain = true;
      for (int32_t c = dn.at(dn.root()).first; c >= 0; c = dn.at(c).next) {
        if (!dn.is(c, json::Type::kStr)) return false;
        nv.push_back(dn.str(c));
        // the token is reused as written unless it holds an escape (then it is re-quoted, so
        // the reply stays byte-identical to the Python verb's json.dumps)
        const std::string_view tok = dn.raw(c);
        if (tok.size() == nv.back().size() + 2) {
          nraw.push_back(tok);
        } else {
          plain = false;
          std::deque<std::string>& requoted = s.requoted;   // stable storage for this request
          if (nraw.empty()) requoted.clear();
          requoted.emplace_back();
          json::append_quoted(&requoted.back(), nv.back());
          nraw.push_back(requoted.back());
        }
      }
    }
    slot = 0;
    for (int k = 1; k < kListSlots; ++k)
      if (idc.used[k] < idc.used[slot]) slot = k;
    idc.valid[slot] = plain;   // a list with escapes is parsed every time
    idc.len[slot] = raw_names.size();
    if (plain) idc.text[slot].assign(raw_names.data(), raw_names.size());
    else idc.text[slot].clear();
    idc.epoch[slot] = 0;                // ids checked below
    if (compact) {
      idc.tok[slot].swap(s.ntok);       // the scan's tokens become the slot's (no copy)
      idc.compact[slot] = true;
    } else {
      idc.tok[slot].clear();
      size_t joined = nraw.empty() ? 2 : 1 + nraw.size();   // brackets and commas
      if (plain)
        for (const std::string_view t : nraw) {
          idc.tok[slot].emplace_back(static_cast<uint32_t>(t.data() - raw_names.data()), static_cast<uint32_t>(t.size()));
          joined += t.size();
        }
      idc.compact[slot] = plain && joined == raw_names.size();
    }
    idc.ids[slot].assign(plain ? idc.tok[slot].size() : nv.size(), -1);
    if (plain) toks = &idc.tok[slot];   // names through the slot's offsets from here on
  }
  idc.used[slot] = ++idc.clock;
  idc.mru = slot;
  auto raw_at = [&](size_t i) -> std::string_view {
    return toks ? raw_names.substr((*toks)[i].first, (*toks)[i].second) : nraw[i];
  };
  auto name_at = [&](size_t i) -> std::string_view {
    if (!toks) return nv[i];
    const auto& t = (*toks)[i];
    return raw_names.substr(t.first + 1, t.second - 2);
  };
  const int32_t nn = static_cast<int32_t>(toks ? toks->size() : nv.size());
  // node ids: any unknown node goes to Python, which can register it from its informer. The
  // ids of a cached list are re-checked (slot `id` still carries that name, else the ledger's
  // name index) only when a node was added or removed since (the ledger's epoch moved).
  std::vector<int32_t>& ids = idc.ids[slot];
  if (idc.epoch[slot] != epoch) {
    // names this worker resolved before, by a hash of the name (no string, no lock): with
    // kube-scheduler's node sampling the list is a different window of the cluster every
    // cycle, so the per-list cache above misses while every name in it is known
    NameTable& nid = s.nid;
    if (nid.owner != serial_ || nid.epoch != epoch) nid.reset(serial_, epoch);
    int32_t prev = -1;
    for (size_t i = 0; i < static_cast<size_t>(nn); ++i) {
      const std::string_view name = name_at(i);
      // the successor of the previous name last time, else the table (its own copy of every
      // name in a compact arena): a hit touches neither the ledger's node slots nor its lock,
      // and is exact (names compared, not only hashed)
      int32_t id = nid.next_of(prev);
      if (!nid.is(id, name)) {
        id = nid.find(name);
        if (id < 0) {
          id = ledger_->find_node(std::string(name));
          if (id < 0) {
            idc.valid[slot] = false;
            return false;
          }
          nid.insert(name, id);
        }
        nid.set_next(prev, id);
      }
      ids[i] = id;
      prev = id;
    }
    idc.epoch[slot] = epoch;
  }
  // the options as of the last policy change this worker saw (one atomic load a request; the
  // lock and the copy only after a change)
  if (s.opt_seen != opt_version_.load(std::memory_order_acquire) || s.opt_owner != serial_) {
    std::lock_guard<std::mutex> g(opt_mu_);
    s.opt = opt_;
    s.normalize = normalize_;
    s.nominate = nominate_;
    s.decisive = decisive_;
    s.lead = lead_;
    s.opt_owner = serial_;   // a thread_local scratch serves every Frontend of its thread
    s.opt_seen = opt_version_.load(std::memory_order_relaxed);
  }
  const Options& o = s.opt;
  const bool normalize = s.normalize, nominate = s.nominate, decisive = s.decisive && !o.compat;
  io_end(kFeVerbNames, io0);
  // a nomination another worker left for after its answer is made before this verb reads the
  // ledger (this worker's own ran before it read this request); bounded
  if (nominate && ledger_->attached() > 1) ledger_->wait_deferred_nominations(kDeferredNominationWaitNs);
  io0 = io_t0();
  // not against itself; priorities right behind this worker's filter of the same pod text
  // (`reused`) with no nomination made anywhere since find it dropped already: no second trip
  // to the pod table
  if (nominate && !uid.empty() &&
      !(prioritize && reused && s.nom_dropped && ledger_->nominations_made() == s.nom_mark)) {
    s.nom_mark = ledger_->nominations_made();
    ledger_->drop_nomination(uid);
    s.nom_dropped = reused || (pod >= 0 && last.valid);   // about the pod `last` holds
  }
  if ((pod >= 0 || reused) && !uid.empty() && !(prioritize && has_pod(uid))) {
    // filter caches the pod for its bind (and, with other worker processes on the ledger,
    // publishes it for their binds); priorities of the same cycle find it there. After the
    // answer with one worker thread: the pod's own bind is the only reader, and it follows the
    // answer. A bind on another worker process that comes before the deferred publish waits
    // for it (prepare_bind, kHandoffWaitNs); one on this thread comes after it
    if (s.defer_cache && last.valid && uid.data() == last.uid.data()) {
      s.defer_put = true;   // the pod is last.raw / last.uid / last.cached: stable until the next request
      s.defer_dem = dem;
    } else {
      cache_pod(s, uid, cached, reused ? std::string_view(last.raw) : d.raw(pod), dem);
    }
  }
  std::string& r = *out;
  r.reserve(64 + 128 * static_cast<size_t>(nn));   // room for a FailedNodes entry per node
  if (!prioritize) {
    rcs.resize(ids.size());
    scores.resize(ids.size());
    io_end(kFeVerbCache, io0);
    {
      IoTimer it{kFeVerbAssume};
      const uint64_t epoch0 = ledger_->epoch();
      ledger_->assume_many(ids.data(), static_cast<int>(ids.size()), dem, o, rcs.data(), scores.data());
      VerbScratch::LastAssume& la = s.last_assume;
      la.valid = !uid.empty();
      if (la.valid) {
        la.epoch = epoch0;
        la.dem_hash = dem.hash();
        la.opt_seen = s.opt_seen;
        la.uid.assign(uid);
        la.ids.assign(ids.begin(), ids.end());
        la.rcs.assign(rcs.begin(), rcs.end());
        la.scores.assign(scores.begin(), scores.end());
      }
    }
    // decisive: the node priorities would rank first is the only one answered (and nominated)
    const int64_t pick = decisive ? top_pick(scores, rcs, uid) : -1;
    // one fitting node: kube-scheduler binds it without a priorities call, so the filter
    // nominates it (otherwise the pod is invisible to the next filters until its bind reserves)
    int64_t only = -1;
    if (!decisive && nominate && !o.compat) {
      for (size_t i = 0; i < ids.size(); ++i) {
        if (rcs[i] != kOk) continue;
        if (only >= 0) {
          only = -1;
          break;
        }
        only = static_cast<int64_t>(i);
      }
    }
    const int64_t nom = pick >= 0 ? pick : only;
    if (nom >= 0 && nominate && !uid.empty() && wants_devices(dem)) {
      if (s.defer && defer_nominate_ok(s) && last.valid && uid.data() == last.uid.data()) {
        s.defer_nominate = true;
        s.defer_node = ids[nom];
        s.defer_dem = dem;
        ledger_->deferred_nomination_begin();   // other workers' filters wait for it
      } else {
        IoTimer it{kFeVerbNominate};
        ledger_->nominate(ids[nom], uid, dem, o);
      }
      s.nom_dropped = false;
    }
    // written straight into the reply; a fitting node's name is its request token, as is
    r.clear();
    r += "{\"Nodes\":null,\"NodeNames\":";
    bool any_failed = false;
    for (size_t i = 0; i < ids.size() && !any_failed; ++i) any_failed = rcs[i] != kOk;
    bool first = true;
    if (pick >= 0) {
      r += '[';
      r += raw_at(static_cast<size_t>(pick));
      r += ']';
    } else if (!any_failed && toks && idc.compact[slot]) {
      r += raw_names;   // every node fits: the request's own list is the answer
    } else {
      r += '[';
      for (size_t i = 0; i < ids.size(); ++i) {
        if (rcs[i] != kOk) continue;
        if (!first) r += ',';
        r += raw_at(i);
        first = false;
      }
      r += ']';
    }
    r += ",\"FailedNodes\":{";
    if (any_failed) {
      // "can't allocate <demand> on node <name>: <reason>" per failing node, written in place:
      // the demand text, the reasons (alloc.cpp err_str) and an escape-free name (its request
      // token is the name in quotes) need no escaping
      std::string& dstr = s.dstr;
      dstr.clear();
      char num[24];
      for (int i = 0; i < dem.n; ++i) {
        dstr += '(';
        dstr.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof num, dem.c[i].pct).ptr - num));
        if (dem.c[i].mib) {
          dstr += ',';
          dstr.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof num, dem.c[i].mib).ptr - num));
          dstr += "Mi";
        }
        dstr += ')';
      }
      first = true;
      for (size_t i = 0; i < ids.size(); ++i) {
        if (rcs[i] == kOk) continue;
        if (!first) r += ',';
        const std::string_view tok = raw_at(i), name = name_at(i);
        r += tok;
        if (tok.size() == name.size() + 2) {
          r += ":\"can't allocate ";
          r += dstr;
          r += " on node ";
          r += name;
          r += ": ";
          r += err_str(rcs[i]);
          r += '"';
        } else {
          r += ':';
          json::append_quoted(&r, "can't allocate " + dstr + " on node " + std::string(name) + ": " + err_str(rcs[i]));
        }
        first = false;
      }
    }
    r += "},\"Error\":\"\"}";
    if (any_failed && pick < 0 && slot >= 0 && idc.valid[slot] && idc.epoch[slot] == epoch) {
      size_t n_ok = 0;
      for (const int32_t rc : rcs) n_ok += rc == kOk;
      if (n_ok > 1) {   // one node: kube-scheduler skips priorities
        if (s.defer) s.defer_list = slot;
        else idc.remember_subset(slot, rcs);
      }
    }
    return true;
  }
  scores.resize(ids.size());
  rcs.resize(ids.size());
  io_end(kFeVerbCache, io0);
  {
    IoTimer it{kFeVerbAssume};
    if (!reuse_assume(s, uid, dem, ids, &rcs, &scores))
      ledger_->assume_many(ids.data(), static_cast<int>(ids.size()), dem, o, rcs.data(), scores.data());
  }
  int64_t best = -1;
  int n_best = 0;
  int32_t second = -1;   // best score among the other fitting nodes
  for (size_t i = 0; i < ids.size(); ++i) {
    const int32_t rc = rcs[i];
    if (rc != kOk) scores[i] = 0;
    if (rc != kOk) continue;
    if (best < 0 || scores[i] > scores[best]) {
      if (best >= 0) second = scores[best];
      best = static_cast<int64_t>(i);
      n_best = 1;
    } else if (scores[i] == scores[best]) {
      ++n_best;
    } else {
      second = std::max(second, scores[i]);
    }
  }
  // a unique winner is the node kube-scheduler picks (ties are broken at random there) when
  // its lead survives kube-scheduler's own score plugins (Ledger::nomination_margin). A tie at
  // the top is broken here by one point, for the tied node the pod's UID hash picks, and that
  // node nominated: a pod without a nomination is invisible to the filters of the pods
  // behind it until its bind reserves, and on identical nodes the top nearly always ties. Only
  // while kube-scheduler has been following the nominations (margin 0): a moved one raises the
  // margin and turns this off (cluster.py::score applies the same rule on the Python path).
  const int32_t margin = ledger_->nomination_margin();
  if (nominate && !o.compat && n_best > 1 && margin == 0 && !uid.empty()) {
    best = top_pick(scores, rcs, uid);
    ++scores[best];
    second = scores[best] - 1;
    n_best = 1;
  }
  const bool lead = n_best == 1 && (second < 0 || scores[best] - second >= margin);
  bool nominated = false;
  if (nominate && lead && !uid.empty() && dem.n > 0) {
    if (wants_devices(dem)) {
      if (s.defer && defer_nominate_ok(s) && last.valid && uid.data() == last.uid.data()) {
        s.defer_nominate = true;
        s.defer_node = ids[best];
        s.defer_dem = dem;
        ledger_->deferred_nomination_begin();   // other workers' filters wait for it
      } else {
        IoTimer it{kFeVerbNominate};
        ledger_->nominate(ids[best], uid, dem, o);
      }
      s.nom_dropped = false;
      nominated = true;
    }
  }
  // The nomination is the pod's placement from this answer on: every later filter sees its
  // devices held. kube-scheduler adds its own score plugins (LeastAllocated, BalancedAllocation,
  // PodTopologySpread: about 800 points between nodes at most) to 10 x the extender's score, so a
  // close second can still win. A pod bound elsewhere than its nomination was invisible on the
  // node it went to until its bind reserved there, and the filters kube-scheduler ran meanwhile
  // (its next cycles start before its binds land) stacked onto the same free devices: steady-
  // churn frag grew from 0.6 % with no such lag to 3.6 % with one cycle of it and 12 % with four
  // (tests/test_lag.py). With a lead, the nominated node is answered `lead` points above every
  // other fitting node (normalised scores: 10 and 0), so kube-scheduler binds where the ledger
  // already holds the pod, whichever worker the bind reaches and however late.
  if (nominated && s.lead > 0 && !o.compat) {
    int32_t other = INT32_MIN;
    for (size_t i = 0; i < ids.size(); ++i)
      if (static_cast<int64_t>(i) != best && rcs[i] == kOk) other = std::max(other, scores[i]);
    if (other != INT32_MIN) {
      if (normalize) {
        for (size_t i = 0; i < ids.size(); ++i) scores[i] = static_cast<int64_t>(i) == best ? 100 : 0;
      } else if (scores[best] - other < s.lead) {
        scores[best] = other + s.lead;
      }
    }
  }
  if (normalize && !scores.empty()) {
    // nanogpu/state/cluster.py::_normalize (Python round(): half to even)
    if (o.compat) {
      int32_t lo = scores[0], hi = scores[0];
      for (int32_t s : scores) lo = std::min(lo, s), hi = std::max(hi, s);
      for (int32_t& s : scores)
        s = hi == lo ? (hi > 0 ? 10 : 0) : static_cast<int32_t>(std::nearbyint(10.0 * (s - lo) / (hi - lo)));
    } else {
      for (int32_t& s : scores) s = std::max(0, std::min(10, static_cast<int32_t>(std::nearbyint(s / 10.0))));
    }
  }
  // [{"Host":<token>,"Score":<n>},...] written through a pointer into a buffer sized for the
  // worst case (no per-append capacity checks: 420 nodes are 2,000 small writes)
  constexpr std::string_view kHost = "{\"Host\":", kScore = ",\"Score\":";
  size_t cap = 2;
  for (size_t i = 0; i < ids.size(); ++i) cap += raw_at(i).size() + kHost.size() + kScore.size() + 14;
  r.resize(cap);
  char* w = r.data();
  *w++ = '[';
  for (size_t i = 0; i < ids.size(); ++i) {
    if (i) *w++ = ',';
    const std::string_view tok = raw_at(i);
    std::memcpy(w, kHost.data(), kHost.size());
    w += kHost.size();
    std::memcpy(w, tok.data(), tok.size());
    w += tok.size();
    std::memcpy(w, kScore.data(), kScore.size());
    w += kScore.size();
    w = std::to_chars(w, w + 12, scores[i]).ptr;
    *w++ = '}';
  }
  *w++ = ']';
  r.resize(static_cast<size_t>(w - r.data()));
  return true;
}

}  // namespace nanogpu
