// Native in-memory Kubernetes API server (see apiserver.h).
//
// Behaviour mirrors nanogpu/k8s/fake_apiserver.py (the Python store the in-process tests use):
// same routes, status codes and Status bodies, merge-patch semantics, binding conflicts, and
// the watch cache (bounded history per kind, resume from a resourceVersion, 410 Gone when the
// version is older than what the cache holds).
#include "nanogpu/apiserver.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <charconv>
#include <chrono>
#include <cmath>
#include <cstring>
#include <ctime>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <stdexcept>
#include <tuple>
#include <unordered_map>

#include "nanogpu/frontend.h"
#include "nanogpu/json.h"

namespace nanogpu::apisrv {

// ------------------------------------------------------------------------------ JSON value
const JV* JV::get(std::string_view k) const {
  if (t != T::kObj) return nullptr;
  for (const auto& kv : o)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
JV* JV::get(std::string_view k) { return const_cast<JV*>(static_cast<const JV*>(this)->get(k)); }

JV& JV::set(std::string_view k, JV v) {
  if (t != T::kObj) {
    *this = obj();
  }
  for (auto& kv : o)
    if (kv.first == k) return kv.second = std::move(v);
  o.emplace_back(std::string(k), std::move(v));
  return o.back().second;
}

JV& JV::child(std::string_view k) {
  JV* c = get(k);
  if (c && c->t == T::kObj) return *c;
  return set(k, obj());
}

void JV::erase(std::string_view k) {
  for (size_t i = 0; i < o.size(); ++i)
    if (o[i].first == k) {
      o.erase(o.begin() + static_cast<long>(i));
      return;
    }
}

namespace {
JV from_doc(const json::Doc& d, int32_t i) {
  JV v;
  const json::Node& n = d.at(i);
  switch (n.type) {
    case json::Type::kNull: break;
    case json::Type::kBool: v.t = JV::T::kBool, v.b = n.b; break;
    case json::Type::kNum: v.t = JV::T::kNum, v.s = std::string(d.str(i)); break;
    case json::Type::kStr: v.t = JV::T::kStr, v.s = std::string(d.str(i)); break;
    case json::Type::kArr:
      v.t = JV::T::kArr;
      v.a.reserve(static_cast<size_t>(n.count));
      for (int32_t c = n.first; c >= 0; c = d.at(c).next) v.a.push_back(from_doc(d, c));
      break;
    case json::Type::kObj:
      v.t = JV::T::kObj;
      v.o.reserve(static_cast<size_t>(n.count));
      for (int32_t c = n.first; c >= 0; c = d.at(c).next) v.o.emplace_back(std::string(d.key(c)), from_doc(d, c));
      break;
  }
  return v;
}
}  // namespace

bool parse(std::string_view text, JV* out) {
  json::Doc d;
  if (!d.parse(text) || d.root() < 0) return false;
  *out = from_doc(d, d.root());
  return true;
}

void dump(const JV& v, std::string* out) {
  switch (v.t) {
    case JV::T::kNull: out->append("null"); break;
    case JV::T::kBool: out->append(v.b ? "true" : "false"); break;
    case JV::T::kNum: out->append(v.s); break;
    case JV::T::kStr: json::append_quoted(out, v.s); break;
    case JV::T::kArr:
      out->push_back('[');
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) out->push_back(',');
        dump(v.a[i], out);
      }
      out->push_back(']');
      break;
    case JV::T::kObj:
      out->push_back('{');
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) out->push_back(',');
        json::append_quoted(out, v.o[i].first);
        out->push_back(':');
        dump(v.o[i].second, out);
      }
      out->push_back('}');
      break;
  }
}

void merge_patch(JV* target, const JV& patch) {
  if (patch.t != JV::T::kObj) {
    *target = patch;
    return;
  }
  if (target->t != JV::T::kObj) *target = JV::obj();
  for (const auto& kv : patch.o) {
    if (kv.second.t == JV::T::kNull) {
      target->erase(kv.first);
    } else if (kv.second.t == JV::T::kObj) {
      JV* cur = target->get(kv.first);
      if (!cur) cur = &target->set(kv.first, JV::obj());
      merge_patch(cur, kv.second);
    } else {
      target->set(kv.first, kv.second);
    }
  }
}

namespace {

// ------------------------------------------------------------------------------ helpers
std::string str_of(const JV* v) { return v && v->t == JV::T::kStr ? v->s : std::string(); }

std::string now_rfc3339() {
  // one-second resolution: formatted once per second per thread (a bulk create stamps
  // thousands of pods within the same second)
  thread_local std::time_t last = -1;
  thread_local char buf[32];
  const std::time_t t = std::time(nullptr);
  if (t != last) {
    std::tm g{};
    gmtime_r(&t, &g);
    std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &g);
    last = t;
  }
  return buf;
}

std::string new_uid() {
  static thread_local std::mt19937_64 rng{std::random_device{}() ^
                                           static_cast<uint64_t>(std::hash<std::thread::id>{}(std::this_thread::get_id()))};
  const uint64_t a = rng(), b = rng();
  char buf[40];
  std::snprintf(buf, sizeof buf, "%08x-%04x-4%03x-%04x-%012llx", static_cast<unsigned>(a >> 32),
                static_cast<unsigned>((a >> 16) & 0xffff), static_cast<unsigned>(a & 0xfff),
                static_cast<unsigned>(0x8000 | ((b >> 48) & 0x3fff)),
                static_cast<unsigned long long>(b & 0xffffffffffffULL));
  return buf;
}

std::string url_decode(std::string_view s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '+') {
      out.push_back(' ');
    } else if (s[i] == '%' && i + 2 < s.size() && std::isxdigit(static_cast<unsigned char>(s[i + 1])) &&
               std::isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out.push_back(static_cast<char>(std::stoi(std::string(s.substr(i + 1, 2)), nullptr, 16)));
      i += 2;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

std::vector<std::string_view> split(std::string_view s, char c) {
  std::vector<std::string_view> out;
  size_t p = 0;
  while (p <= s.size()) {
    const size_t q = s.find(c, p);
    const size_t e = q == std::string_view::npos ? s.size() : q;
    out.push_back(s.substr(p, e - p));
    if (q == std::string_view::npos) break;
    p = q + 1;
  }
  return out;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

std::string status_body(int code, std::string_view reason, std::string_view message) {
  std::string b = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"status\":\"Failure\",\"message\":";
  json::append_quoted(&b, message);
  b += ",\"reason\":";
  json::append_quoted(&b, reason);
  b += ",\"code\":" + std::to_string(code) + "}";
  return b;
}

const char* reason_phrase(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 413: return "Payload Too Large";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    default: return "Status";
  }
}

// ------------------------------------------------------------------------------ store
enum Kind { kPods = 0, kNodes = 1, kKinds = 2 };

// One stored version of an object: its JSON text (what every read and watch event sends)
// and, built on first need only, its tree (what a patch edits and label selectors read).
// A create or delete whose text only gains a resourceVersion never builds the tree.
struct Obj {
  std::string json;
  std::string ns, name, uid, node, phase;
  uint64_t rv = 0;
  // where metadata.resourceVersion's digits sit in `json` (rv_len 0: not known), so a new
  // version is spliced without searching the text
  uint32_t rv_at = 0, rv_len = 0;
  // set before the object is published (seal, restamp), or once by v(); read through
  // atomic_load because restamp may copy it while another thread is building it
  mutable std::once_flag once;
  mutable std::shared_ptr<const JV> tree;
  const JV& v() const {
    std::call_once(once, [this] {
      if (std::atomic_load(&tree)) return;
      auto t = std::make_shared<JV>();
      parse(json, t.get());
      std::atomic_store(&tree, std::shared_ptr<const JV>(std::move(t)));
    });
    return *std::atomic_load(&tree);
  }
  const JV* labels() const {
    const JV* m = v().get("metadata");
    return m ? m->get("labels") : nullptr;
  }
};
using ObjP = std::shared_ptr<const Obj>;

// Stamps the resourceVersion, extracts the indexed fields and serializes once.
ObjP seal(JV v, uint64_t rv) {
  auto o = std::make_shared<Obj>();
  JV& m = v.child("metadata");
  m.set("resourceVersion", JV::str(std::to_string(rv)));
  o->ns = str_of(m.get("namespace"));
  o->name = str_of(m.get("name"));
  o->uid = str_of(m.get("uid"));
  if (const JV* sp = v.get("spec")) o->node = str_of(sp->get("nodeName"));
  if (const JV* st = v.get("status")) o->phase = str_of(st->get("phase"));
  o->rv = rv;
  auto t = std::make_shared<JV>(std::move(v));
  dump(*t, &o->json);
  o->tree = std::move(t);
  const std::string digits = std::to_string(rv);
  const size_t at = o->json.find("\"resourceVersion\":\"" + digits + "\"");
  if (at != std::string::npos) {
    o->rv_at = static_cast<uint32_t>(at + 19);   // past "resourceVersion":"
    o->rv_len = static_cast<uint32_t>(digits.size());
  }
  return o;
}

// The same object at a new resourceVersion, text spliced (a delete's final version).
ObjP restamp(const ObjP& cur, uint64_t rv) {
  size_t at = cur->rv_at, len = cur->rv_len;
  if (len == 0) {
    const std::string digits = std::to_string(cur->rv);
    const size_t hit = cur->json.find("\"resourceVersion\":\"" + digits + "\"");
    if (hit == std::string::npos) return seal(cur->v(), rv);   // (not ours: no stamp to splice)
    at = hit + 19;
    len = digits.size();
  }
  char buf[24];
  const auto res = std::to_chars(buf, buf + sizeof buf, rv);
  const size_t n = static_cast<size_t>(res.ptr - buf);
  auto o = std::make_shared<Obj>();
  o->json.reserve(cur->json.size() + 4);
  o->json.append(cur->json, 0, at);
  o->json.append(buf, n);
  o->json.append(cur->json, at + len, std::string::npos);
  o->rv_at = static_cast<uint32_t>(at);
  o->rv_len = static_cast<uint32_t>(n);
  o->ns = cur->ns, o->name = cur->name, o->uid = cur->uid, o->node = cur->node, o->phase = cur->phase;
  o->rv = rv;
  // the tree (if built) stays usable as the base of later patches, which re-stamp anyway
  if (auto t = std::atomic_load(&cur->tree)) o->tree = std::move(t);
  return o;
}

// A create whose body already has everything the store fills in except the resourceVersion
// (and maybe the creationTimestamp): the stored text is the body with those spliced into
// metadata, no tree. Anything else goes through the tree path (create_pod_locked).
struct FastCreate {
  bool ok = false;
  std::string ns, name, uid, node, phase;
  std::string_view text;
  size_t meta_open = 0;   // offset just past metadata's '{'
  bool need_ts = false;
};

FastCreate fast_create(std::string_view text, std::string_view ns_path) {
  FastCreate f;
  json::Doc d;
  if (!d.parse(text) || !d.is(d.root(), json::Type::kObj)) return f;
  const int32_t m = d.get(d.root(), "metadata");
  if (!d.is(m, json::Type::kObj) || d.at(m).count == 0) return f;
  auto sget = [&](int32_t obj, const char* k) -> std::string {
    const int32_t v = d.get(obj, k);
    return d.is(v, json::Type::kStr) ? std::string(d.str(v)) : std::string();
  };
  f.ns = sget(m, "namespace");
  f.name = sget(m, "name");
  f.uid = sget(m, "uid");
  if (f.name.empty() || f.uid.empty() || f.ns.empty() || (!ns_path.empty() && f.ns != ns_path)) return f;
  if (d.get(m, "resourceVersion") >= 0) return f;
  f.need_ts = d.get(m, "creationTimestamp") < 0;
  const int32_t st = d.get(d.root(), "status");
  if (!d.is(st, json::Type::kObj)) return f;
  f.phase = sget(st, "phase");
  if (f.phase.empty()) return f;
  const int32_t sp = d.get(d.root(), "spec");
  if (d.is(sp, json::Type::kObj)) f.node = sget(sp, "nodeName");
  const uint32_t b = d.at(m).src_begin;
  if (b >= text.size() || text[b] != '{') return f;
  f.meta_open = b + 1;
  f.text = text;
  f.ok = true;
  return f;
}

struct Selector {
  struct Term {
    std::string k, v;
    int op;  // 0 =, 1 !=, 2 exists
  };
  std::vector<Term> terms;
  static Selector parse(std::string_view s) {
    Selector out;
    for (std::string_view t : split(s, ',')) {
      t = trim(t);
      if (t.empty()) continue;
      Term x;
      size_t p;
      if ((p = t.find("!=")) != std::string_view::npos) {
        x = {std::string(trim(t.substr(0, p))), std::string(trim(t.substr(p + 2))), 1};
      } else if ((p = t.find('=')) != std::string_view::npos) {
        std::string_view v = t.substr(p + 1);
        if (!v.empty() && v.front() == '=') v.remove_prefix(1);
        x = {std::string(trim(t.substr(0, p))), std::string(trim(v)), 0};
      } else {
        x = {std::string(t), std::string(), 2};
      }
      out.terms.push_back(std::move(x));
    }
    return out;
  }
  bool labels_match(const Obj& o) const {
    if (terms.empty()) return true;   // no selector: never build the object's tree for it
    const JV* l = o.labels();
    for (const Term& t : terms) {
      const JV* v = l ? l->get(t.k) : nullptr;
      if (t.op == 0 && (!v || v->sv() != t.v)) return false;
      if (t.op == 1 && v && v->sv() == t.v) return false;
      if (t.op == 2 && !v) return false;
    }
    return true;
  }
  bool fields_match(const Obj& o) const {
    for (const Term& t : terms) {
      std::string_view have;
      if (t.k == "spec.nodeName") have = o.node;
      else if (t.k == "metadata.name") have = o.name;
      else if (t.k == "metadata.namespace") have = o.ns;
      else if (t.k == "status.phase") have = o.phase;
      else continue;
      if ((t.op == 0) != (have == t.v)) return false;
    }
    return true;
  }
};

struct Ev {
  uint64_t rv;
  ObjP obj;
  std::shared_ptr<const std::string> line;   // {"type":..,"object":..}\n
};

// Versions a thread's writes evicted from the watch history (a full history evicts one per
// event: its text, its parsed tree, a few hundred frees). They are freed by the same thread
// once it has left the store's lock (release_evicted), not while every other request waits on
// that lock: a soak of 300 bursts had its bulk creates 60 % slower once the history was full.
thread_local std::vector<Ev> tl_evicted;

void release_evicted() { tl_evicted.clear(); }

std::shared_ptr<const std::string> ev_line(const char* type, const std::string& obj_json) {
  auto s = std::make_shared<std::string>();
  s->reserve(obj_json.size() + 32);
  *s += "{\"type\":\"";
  *s += type;
  *s += "\",\"object\":";
  *s += obj_json;
  *s += "}\n";
  return s;
}

struct Conn;

struct Watch {
  int kind;
  Selector ls, fs;
  std::shared_ptr<Conn> conn;
};

struct ApiErr {
  int code;
  std::string reason, message;
};

}  // namespace

// ------------------------------------------------------------------------------ connection
namespace {
struct IoThread;

struct Conn {
  int fd = -1;
  IoThread* owner = nullptr;
  std::string in;
  std::string out;                 // owner thread only
  // watch stream state
  std::mutex mu;                   // guards pending / ended (written by store writers)
  std::string pending;             // event lines not yet framed
  bool ended = false;              // the stream is to be terminated after pending
  std::atomic<bool> queued{false}; // on the owner's flush list
  bool watching = false;
  double deadline = 0;             // steady seconds; 0 = none
  bool close_after = false;
};

double steady_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct IoThread {
  int ep = -1, efd = -1;
  std::thread th;
  // modelled round trip: responses held until due, in arrival order (one latency for all)
  // (due, connection, bytes, a mutating request's answer: its in-flight slot is freed when written)
  std::deque<std::tuple<double, std::weak_ptr<Conn>, std::string, bool>> delayed;
  double last_flush = 0, flush_due = 0;   // watch output coalescing (Impl::flush_watches)
  double last_event = 0;                  // the spin window (set_spin) runs from here
  std::atomic<bool> urgent{false};        // flush now, without the linger (a bulk write ended)
  std::mutex mu;
  std::vector<std::shared_ptr<Conn>> flush;   // watch conns with pending output
  std::unordered_map<int, std::shared_ptr<Conn>> conns;
  void wake(const std::shared_ptr<Conn>& c) {
    if (c->queued.exchange(true)) return;
    {
      std::lock_guard<std::mutex> g(mu);
      flush.push_back(c);
    }
    const uint64_t one = 1;
    (void)!write(efd, &one, sizeof one);
  }
};
}  // namespace

struct Server::Impl {
  Config cfg;
  int lfd = -1;
  std::atomic<double> latency_s{0.0};
  std::atomic<double> spin_s{0.0};   // poll this long after the last event before sleeping (0: never)
  // max-in-flight admission (set_max_mutating_inflight): mutating requests handled whose answer
  // is not written yet, the limit (0: none) and the 429s answered
  std::atomic<int> mutating_inflight{0};
  std::atomic<int> max_mutating{0};
  std::atomic<uint64_t> n_429{0};
  std::atomic<int> peak_mutating{0};
  double linger_s = 200e-6;   // watch output coalescing window under load
  std::atomic<bool> stopping{false};
  std::vector<std::unique_ptr<IoThread>> io;

  // ---- store (under mu)
  mutable std::mutex mu;
  uint64_t rv = 0;
  std::unordered_map<std::string, ObjP> pods;          // "ns/name"
  std::map<std::string, ObjP> nodes;
  std::map<std::string, ObjP> leases;                  // "ns/name"
  std::deque<Ev> hist[kKinds];
  uint64_t compacted[kKinds] = {0, 0};
  std::vector<Watch> watches;
  std::atomic<uint64_t> n_create{0}, n_get{0}, n_patch{0}, n_bind{0}, n_delete{0}, n_list{0}, n_watch{0},
      n_events{0}, n_requests{0}, n_lease{0};
  // bulk create/delete phases (steady ns): parse outside the lock, store + emit under it
  std::atomic<uint64_t> bulk_parse_ns{0}, bulk_insert_ns{0}, bulk_delete_ns{0};
  uint64_t bindings = 0;

  static std::string key(std::string_view ns, std::string_view name) {
    std::string k(ns);
    k.push_back('/');
    k.append(name);
    return k;
  }

  // A bulk write is complete: its last events leave now rather than after the linger.
  void flush_now() {
    for (auto& t : io) {
      t->urgent.store(true, std::memory_order_relaxed);
      const uint64_t one = 1;
      (void)!write(t->efd, &one, sizeof one);
    }
  }

  // -- emit under mu
  void emit(int kind, const char* type, const ObjP& o) { emit_line(kind, o, ev_line(type, o->json)); }
  // `line` built beforehand (bulk paths build them on several threads)
  void emit_line(int kind, const ObjP& o, std::shared_ptr<const std::string> line) {
    Ev e{o->rv, o, std::move(line)};
    for (const Watch& w : watches) {
      if (w.kind != kind) continue;
      if (!w.ls.labels_match(*o) || !w.fs.fields_match(*o)) continue;
      {
        std::lock_guard<std::mutex> g(w.conn->mu);
        if (w.conn->ended) continue;
        w.conn->pending += *e.line;
      }
      w.conn->owner->wake(w.conn);
    }
    auto& h = hist[kind];
    h.push_back(std::move(e));
    while (h.size() > cfg.history) {
      tl_evicted.push_back(std::move(h.front()));   // freed after the lock (release_evicted)
      h.pop_front();
    }
  }

  // -- pods
  ObjP create_pod_locked(JV v, std::string_view ns_path) {
    JV& m = v.child("metadata");
    if (!ns_path.empty()) m.set("namespace", JV::str(std::string(ns_path)));
    if (str_of(m.get("namespace")).empty()) m.set("namespace", JV::str("default"));
    if (str_of(m.get("name")).empty()) throw ApiErr{422, "Invalid", "metadata.name: Required value"};
    if (str_of(m.get("uid")).empty()) m.set("uid", JV::str(new_uid()));
    if (!m.get("creationTimestamp")) m.set("creationTimestamp", JV::str(now_rfc3339()));
    JV& st = v.child("status");
    if (!st.get("phase")) st.set("phase", JV::str("Pending"));
    const std::string k = key(str_of(m.get("namespace")), str_of(m.get("name")));
    if (pods.count(k)) throw ApiErr{409, "AlreadyExists", "pods \"" + str_of(m.get("name")) + "\" already exists"};
    ObjP o = seal(std::move(v), ++rv);
    pods.emplace(k, o);
    emit(kPods, "ADDED", o);
    return o;
  }
  // `f` from fast_create (parsed outside the lock)
  ObjP create_fast_locked(const FastCreate& f) {
    const std::string k = key(f.ns, f.name);
    if (pods.count(k)) throw ApiErr{409, "AlreadyExists", "pods \"" + f.name + "\" already exists"};
    auto o = std::make_shared<Obj>();
    o->rv = ++rv;
    std::string ins = "\"resourceVersion\":\"" + std::to_string(o->rv) + "\"";
    if (f.need_ts) ins += ",\"creationTimestamp\":\"" + now_rfc3339() + "\"";
    ins += ',';
    o->json.reserve(f.text.size() + ins.size());
    o->json.append(f.text.substr(0, f.meta_open));
    o->json += ins;
    o->json.append(f.text.substr(f.meta_open));
    o->rv_at = static_cast<uint32_t>(f.meta_open + 19);
    o->rv_len = static_cast<uint32_t>(std::to_string(o->rv).size());
    o->ns = f.ns, o->name = f.name, o->uid = f.uid, o->node = f.node, o->phase = f.phase;
    pods.emplace(k, o);
    emit(kPods, "ADDED", o);
    return o;
  }
  ObjP pod_or_404(std::string_view ns, std::string_view name) const {
    auto it = pods.find(key(ns, name));
    if (it == pods.end()) throw ApiErr{404, "NotFound", "pods \"" + std::string(name) + "\" not found"};
    return it->second;
  }
  // Writes that derive the new version from the current one: the tree copy, the edit and
  // the serialization run outside the store lock against a snapshot; the lock is held only
  // to check the snapshot is still current, splice the resourceVersion in and publish.
  // A concurrent write to the same pod makes the loser redo its edit (optimistic).
  template <class Edit>
  ObjP write_pod(std::string_view ns, std::string_view name, Edit edit) {
    const std::string k = key(ns, name);
    for (;;) {
      ObjP cur;
      {
        std::lock_guard<std::mutex> g(mu);
        cur = pod_or_404(ns, name);
      }
      JV v = cur->v();
      edit(*cur, &v);                       // may throw ApiErr (checked against this version)
      ObjP draft = seal(std::move(v), 0);
      std::lock_guard<std::mutex> g(mu);
      auto it = pods.find(k);
      if (it == pods.end()) throw ApiErr{404, "NotFound", "pods \"" + std::string(name) + "\" not found"};
      if (it->second != cur) continue;       // someone wrote in between: redo on theirs
      ObjP o = restamp(draft, ++rv);
      it->second = o;
      emit(kPods, "MODIFIED", o);
      return o;
    }
  }
  ObjP patch_pod(std::string_view ns, std::string_view name, const JV& patch) {
    return write_pod(ns, name, [&](const Obj& cur, JV* v) {
      merge_patch(v, patch);
      // kube-apiserver's pod update validation: spec.nodeName is set by a Binding only, so a
      // patch that would change it is refused (and one that restates it is a precondition)
      const JV* sp = v->get("spec");
      if ((sp ? str_of(sp->get("nodeName")) : std::string()) != cur.node)
        throw ApiErr{422, "Invalid",
                     "Pod \"" + std::string(name) + "\" is invalid: spec: Forbidden: pod updates may not change "
                     "fields other than `spec.containers[*].image`, `spec.initContainers[*].image`, "
                     "`spec.activeDeadlineSeconds`, `spec.tolerations` (only additions to existing tolerations) "
                     "or `spec.terminationGracePeriodSeconds`"};
    });
  }
  // pods/binding; the Binding's metadata.annotations land on the pod with spec.nodeName, as
  // kube-apiserver's setPodHostAndAnnotations does
  void bind_pod(std::string_view ns, std::string_view name, std::string_view uid, std::string_view node,
                const JV* annotations = nullptr) {
    {
      std::lock_guard<std::mutex> g(mu);
      if (!nodes.count(std::string(node))) {
        (void)pod_or_404(ns, name);
        throw ApiErr{404, "NotFound", "nodes \"" + std::string(node) + "\" not found"};
      }
    }
    write_pod(ns, name, [&](const Obj& cur, JV* v) {
      if (!uid.empty() && cur.uid != uid) throw ApiErr{409, "Conflict", "pod " + std::string(name) + " uid mismatch"};
      if (!cur.node.empty())
        throw ApiErr{409, "Conflict",
                     "pod " + std::string(name) + " is already assigned to node \"" + cur.node + "\""};
      v->child("spec").set("nodeName", JV::str(std::string(node)));
      v->child("status").set("phase", JV::str("Running"));
      if (annotations && annotations->is_obj()) {
        JV& ann = v->child("metadata").child("annotations");
        for (const auto& kv : annotations->o) ann.set(kv.first, kv.second);
      }
    });
    std::lock_guard<std::mutex> g(mu);
    ++bindings;
  }
  ObjP update_pod_locked(std::string_view ns, std::string_view name, JV v) {
    ObjP cur = pod_or_404(ns, name);
    const JV* m = v.get("metadata");
    const std::string want = m ? str_of(m->get("resourceVersion")) : std::string();
    if (!want.empty() && want != std::to_string(cur->rv))
      throw ApiErr{409, "Conflict", "Operation cannot be fulfilled on pods \"" + std::string(name) +
                                        "\": the object has been modified; please apply your changes to the latest "
                                        "version and try again"};
    ObjP o = seal(std::move(v), ++rv);
    pods[key(ns, name)] = o;
    emit(kPods, "MODIFIED", o);
    return o;
  }
  bool delete_pod_locked(std::string_view ns, std::string_view name) {
    auto it = pods.find(key(ns, name));
    if (it == pods.end()) return false;
    ObjP cur = it->second;
    pods.erase(it);
    emit(kPods, "DELETED", restamp(cur, ++rv));
    return true;
  }

  // -- nodes
  ObjP put_node_locked(JV v) {
    const std::string name = str_of(v.child("metadata").get("name"));
    if (name.empty()) throw ApiErr{422, "Invalid", "metadata.name: Required value"};
    const bool existed = nodes.count(name) > 0;
    ObjP o = seal(std::move(v), ++rv);
    nodes[name] = o;
    emit(kNodes, existed ? "MODIFIED" : "ADDED", o);
    return o;
  }
  ObjP node_or_404(std::string_view name) const {
    auto it = nodes.find(std::string(name));
    if (it == nodes.end()) throw ApiErr{404, "NotFound", "nodes \"" + std::string(name) + "\" not found"};
    return it->second;
  }

  // -- listing
  std::string listing(const char* kind, const std::vector<ObjP>& items) const {
    size_t n = 96;
    for (const auto& o : items) n += o->json.size() + 1;
    std::string b;
    b.reserve(n);
    b += "{\"kind\":\"";
    b += kind;
    b += "\",\"apiVersion\":\"v1\",\"metadata\":{\"resourceVersion\":\"" + std::to_string(rv) + "\"},\"items\":[";
    for (size_t i = 0; i < items.size(); ++i) {
      if (i) b.push_back(',');
      b += items[i]->json;
    }
    b += "]}";
    return b;
  }

  // ------------------------------------------------------------------ request dispatch
  struct Req {
    std::string_view method, path;
    std::unordered_map<std::string, std::string> q;
    std::string_view body;
  };

  static bool is_watch(const Req& r) {
    auto it = r.q.find("watch");
    return it != r.q.end() && (it->second == "1" || it->second == "true");
  }

  static std::string qv(const Req& r, const char* k) {
    auto it = r.q.find(k);
    return it == r.q.end() ? std::string() : it->second;
  }

  JV body_json(const Req& r) const {
    JV v;
    if (!parse(r.body, &v)) throw ApiErr{400, "BadRequest", "request body is not valid JSON"};
    return v;
  }

  std::pair<int, std::string> handle(const Req& r) {
    n_requests.fetch_add(1, std::memory_order_relaxed);
    std::pair<int, std::string> out;
    try {
      out = route(r);
    } catch (const ApiErr& e) {
      out = {e.code, status_body(e.code, e.reason, e.message)};
    }
    release_evicted();   // no lock held here
    return out;
  }

  std::pair<int, std::string> route(const Req& r) {
    const auto parts = split(r.path.substr(r.path.empty() || r.path[0] != '/' ? 0 : 1), '/');
    const size_t n = parts.size();
    auto at = [&](size_t i) -> std::string_view { return i < n ? parts[i] : std::string_view(); };
    const std::string_view m = r.method;
    static const std::string kOk = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"status\":\"Success\"}";
    if (n == 1 && (at(0) == "healthz" || at(0) == "readyz")) return {200, "ok"};
    if (at(0) == "api" && at(1) == "v1") {
      // /api/v1/pods
      if (n == 3 && at(2) == "pods" && m == "GET") return list_pods(r, "");
      // /api/v1/nodes...
      if (at(2) == "nodes") {
        if (n == 3 && m == "GET") return list_nodes(r);
        if (n == 3 && m == "POST") {
          JV v = body_json(r);
          std::lock_guard<std::mutex> g(mu);
          return {201, put_node_locked(std::move(v))->json};
        }
        if (n == 4 || (n == 5 && at(4) == "status")) {
          const std::string name(at(3));
          if (m == "GET" && n == 4) {
            std::lock_guard<std::mutex> g(mu);
            return {200, node_or_404(name)->json};
          }
          if (m == "PATCH") {
            JV p = body_json(r);
            std::lock_guard<std::mutex> g(mu);
            JV v = node_or_404(name)->v();
            merge_patch(&v, p);
            return {200, put_node_locked(std::move(v))->json};
          }
          if (m == "DELETE" && n == 4) {
            std::lock_guard<std::mutex> g(mu);
            auto it = nodes.find(name);
            if (it == nodes.end()) throw ApiErr{404, "NotFound", "nodes \"" + name + "\" not found"};
            ObjP cur = it->second;
            nodes.erase(it);
            emit(kNodes, "DELETED", restamp(cur, ++rv));
            return {200, kOk};
          }
        }
        return {405, status_body(405, "MethodNotAllowed", "method not allowed")};
      }
      // /api/v1/namespaces/{ns}/...
      if (at(2) == "namespaces" && n >= 5) {
        const std::string_view ns = at(3);
        if (at(4) == "events" && n == 5 && m == "POST") {
          n_events.fetch_add(1, std::memory_order_relaxed);
          return {201, "{}"};
        }
        if (at(4) == "pods") {
          if (n == 5 && m == "GET") return list_pods(r, ns);
          if (n == 5 && m == "POST") {
            n_create.fetch_add(1, std::memory_order_relaxed);
            const FastCreate f = fast_create(r.body, ns);
            if (f.ok) {
              std::lock_guard<std::mutex> g(mu);
              return {201, create_fast_locked(f)->json};
            }
            JV v = body_json(r);
            std::lock_guard<std::mutex> g(mu);
            return {201, create_pod_locked(std::move(v), ns)->json};
          }
          const std::string_view name = at(5);
          if (n == 6) {
            if (m == "GET") {
              n_get.fetch_add(1, std::memory_order_relaxed);
              std::lock_guard<std::mutex> g(mu);
              return {200, pod_or_404(ns, name)->json};
            }
            if (m == "PATCH") {
              JV p = body_json(r);
              n_patch.fetch_add(1, std::memory_order_relaxed);
              return {200, patch_pod(ns, name, p)->json};
            }
            if (m == "PUT") {
              JV v = body_json(r);
              std::lock_guard<std::mutex> g(mu);
              return {200, update_pod_locked(ns, name, std::move(v))->json};
            }
            if (m == "DELETE") {
              n_delete.fetch_add(1, std::memory_order_relaxed);
              std::lock_guard<std::mutex> g(mu);
              if (!delete_pod_locked(ns, name))
                throw ApiErr{404, "NotFound", "pods \"" + std::string(name) + "\" not found"};
              return {200, kOk};
            }
          }
          if (n == 7 && at(6) == "binding" && m == "POST") {
            JV b = body_json(r);
            const JV* md = b.get("metadata");
            const JV* tg = b.get("target");
            n_bind.fetch_add(1, std::memory_order_relaxed);
            bind_pod(ns, name, md ? str_of(md->get("uid")) : std::string(), tg ? str_of(tg->get("name")) : "",
                     md ? md->get("annotations") : nullptr);
            return {201, kOk};
          }
        }
      }
    }
    // leases (coordination.k8s.io/v1)
    if (at(0) == "apis" && at(1) == "coordination.k8s.io" && at(2) == "v1" && at(3) == "namespaces" &&
        at(5) == "leases") {
      n_lease.fetch_add(1, std::memory_order_relaxed);
      const std::string_view ns = at(4);
      if (n == 6 && m == "POST") {
        JV v = body_json(r);
        v.child("metadata").set("namespace", JV::str(std::string(ns)));
        const std::string name = str_of(v.child("metadata").get("name"));
        std::lock_guard<std::mutex> g(mu);
        const std::string k = key(ns, name);
        if (leases.count(k))
          throw ApiErr{409, "AlreadyExists", "leases.coordination.k8s.io \"" + name + "\" already exists"};
        ObjP o = seal(std::move(v), ++rv);
        leases[k] = o;
        return {201, o->json};
      }
      if (n == 7) {
        const std::string k = key(ns, at(6));
        std::lock_guard<std::mutex> g(mu);
        auto it = leases.find(k);
        if (it == leases.end())
          throw ApiErr{404, "NotFound", "leases.coordination.k8s.io \"" + std::string(at(6)) + "\" not found"};
        if (m == "GET") return {200, it->second->json};
        if (m == "PUT") {
          JV v = body_json(r);
          const JV* md = v.get("metadata");
          if ((md ? str_of(md->get("resourceVersion")) : std::string()) != std::to_string(it->second->rv))
            throw ApiErr{409, "Conflict", "Operation cannot be fulfilled on leases.coordination.k8s.io \"" +
                                              std::string(at(6)) + "\": the object has been modified"};
          v.child("metadata").set("namespace", JV::str(std::string(ns)));
          ObjP o = seal(std::move(v), ++rv);
          it->second = o;
          return {200, o->json};
        }
      }
    }
    return {404, status_body(404, "NotFound", "the server could not find the requested resource")};
  }

  std::pair<int, std::string> list_pods(const Req& r, std::string_view ns) {
    n_list.fetch_add(1, std::memory_order_relaxed);
    const Selector ls = Selector::parse(qv(r, "labelSelector")), fs = Selector::parse(qv(r, "fieldSelector"));
    std::vector<ObjP> items;
    std::lock_guard<std::mutex> g(mu);
    items.reserve(pods.size());
    for (const auto& kv : pods) {
      const Obj& o = *kv.second;
      if ((ns.empty() || o.ns == ns) && ls.labels_match(o) && fs.fields_match(o)) items.push_back(kv.second);
    }
    return {200, listing("PodList", items)};
  }

  std::pair<int, std::string> list_nodes(const Req& r) {
    n_list.fetch_add(1, std::memory_order_relaxed);
    const Selector ls = Selector::parse(qv(r, "labelSelector"));
    std::vector<ObjP> items;
    std::lock_guard<std::mutex> g(mu);
    for (const auto& kv : nodes)
      if (ls.labels_match(*kv.second)) items.push_back(kv.second);
    return {200, listing("NodeList", items)};
  }

  // Registers a watch and queues its replay; returns false (and an in-stream 410) when the
  // requested version is older than the cache.
  void start_watch(const std::shared_ptr<Conn>& c, int kind, const Req& r) {
    n_watch.fetch_add(1, std::memory_order_relaxed);
    Watch w{kind, Selector::parse(qv(r, "labelSelector")), Selector::parse(qv(r, "fieldSelector")), c};
    uint64_t from = 0;
    const std::string rvs = qv(r, "resourceVersion");
    if (!rvs.empty()) from = std::strtoull(rvs.c_str(), nullptr, 10);
    const std::string to = qv(r, "timeoutSeconds");
    if (!to.empty()) c->deadline = steady_s() + std::strtod(to.c_str(), nullptr);
    std::lock_guard<std::mutex> g(mu);
    std::string replay;
    const auto& h = hist[kind];
    const bool truncated = !h.empty() && h.size() >= cfg.history && h.front().rv > from + 1;
    if (from > 0 && (from < compacted[kind] || truncated)) {
      std::string msg = "too old resource version: " + std::to_string(from) + " (" +
                        std::to_string(compacted[kind] ? compacted[kind] : (h.empty() ? 0 : h.front().rv)) + ")";
      std::lock_guard<std::mutex> cg(c->mu);
      c->pending = "{\"type\":\"ERROR\",\"object\":" + status_body(410, "Expired", msg) + "}\n";
      c->ended = true;
      c->owner->wake(c);
      return;
    }
    if (from == 0) {
      // no version: the current state as ADDED events, then live
      auto add = [&](const ObjP& o) {
        if (w.ls.labels_match(*o) && w.fs.fields_match(*o)) replay += *ev_line("ADDED", o->json);
      };
      if (kind == kPods)
        for (const auto& kv : pods) add(kv.second);
      else
        for (const auto& kv : nodes) add(kv.second);
    } else {
      for (const Ev& e : h)
        if (e.rv > from && w.ls.labels_match(*e.obj) && w.fs.fields_match(*e.obj)) replay += *e.line;
    }
    {
      std::lock_guard<std::mutex> cg(c->mu);
      c->pending += replay;
    }
    watches.push_back(std::move(w));
    if (!replay.empty()) c->owner->wake(c);
  }

  void unwatch(const Conn* c) {
    std::lock_guard<std::mutex> g(mu);
    for (size_t i = 0; i < watches.size();)
      if (watches[i].conn.get() == c) {
        watches[i] = std::move(watches.back());
        watches.pop_back();
      } else {
        ++i;
      }
  }

  void end_watches(int kind) {   // under mu
    for (size_t i = 0; i < watches.size();) {
      if (kind < 0 || watches[i].kind == kind) {
        {
          std::lock_guard<std::mutex> cg(watches[i].conn->mu);
          watches[i].conn->ended = true;
        }
        watches[i].conn->owner->wake(watches[i].conn);
        watches[i] = std::move(watches.back());
        watches.pop_back();
      } else {
        ++i;
      }
    }
  }

  // ------------------------------------------------------------------ IO
  void io_loop(IoThread* t);
  void on_readable(IoThread* t, const std::shared_ptr<Conn>& c);
  void flush_watch(const std::shared_ptr<Conn>& c);
  void flush_watches(IoThread* t);
  bool write_out(Conn* c);
  void close_conn(IoThread* t, const std::shared_ptr<Conn>& c);
};

namespace {
std::string head(int code, size_t len, bool chunked = false) {
  std::string h = "HTTP/1.1 " + std::to_string(code) + " " + reason_phrase(code) +
                  "\r\nContent-Type: application/json\r\n";
  if (code == 429) h += "Retry-After: 1\r\n";   // kube-apiserver's max-in-flight rejection
  if (chunked)
    h += "Transfer-Encoding: chunked\r\n\r\n";
  else
    h += "Content-Length: " + std::to_string(len) + "\r\n\r\n";
  return h;
}

void frame_chunk(std::string* out, std::string_view data) {
  char hex[24];
  std::snprintf(hex, sizeof hex, "%zx\r\n", data.size());
  out->append(hex);
  out->append(data);
  out->append("\r\n");
}
}  // namespace

bool Server::Impl::write_out(Conn* c) {
  while (!c->out.empty()) {
    const ssize_t w = ::send(c->fd, c->out.data(), c->out.size(), MSG_NOSIGNAL);
    if (w > 0) {
      c->out.erase(0, static_cast<size_t>(w));
      continue;
    }
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return true;
    if (w < 0 && errno == EINTR) continue;
    return false;
  }
  return true;
}

void Server::Impl::flush_watch(const std::shared_ptr<Conn>& c) {
  std::string data;
  bool end;
  {
    std::lock_guard<std::mutex> g(c->mu);
    data.swap(c->pending);
    end = c->ended;
  }
  if (!c->watching) return;
  if (!data.empty()) frame_chunk(&c->out, data);
  if (end) {
    c->out += "0\r\n\r\n";
    c->watching = false;
    c->deadline = 0;
    std::lock_guard<std::mutex> g(c->mu);
    c->ended = false;
    c->pending.clear();
  }
}

void Server::Impl::close_conn(IoThread* t, const std::shared_ptr<Conn>& c) {
  if (c->watching) unwatch(c.get());
  epoll_ctl(t->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  ::close(c->fd);
  t->conns.erase(c->fd);
}

void Server::Impl::on_readable(IoThread* t, const std::shared_ptr<Conn>& c) {
  char buf[65536];
  for (;;) {
    const ssize_t r = ::recv(c->fd, buf, sizeof buf, 0);
    if (r > 0) {
      c->in.append(buf, static_cast<size_t>(r));
      if (c->in.size() > (64u << 20)) {
        close_conn(t, c);
        return;
      }
      continue;
    }
    if (r == 0) {
      close_conn(t, c);
      return;
    }
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    if (errno == EINTR) continue;
    close_conn(t, c);
    return;
  }
  // requests (pipelined ones in order); none while a watch stream is open on the connection
  while (!c->watching) {
    const size_t he = c->in.find("\r\n\r\n");
    if (he == std::string::npos) break;
    std::string_view hdr(c->in.data(), he);
    const size_t l1 = hdr.find("\r\n");
    std::string_view line = hdr.substr(0, l1);
    const size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string_view::npos || s2 == s1) {
      close_conn(t, c);
      return;
    }
    size_t clen = 0;
    bool chunked = false, close_req = false;
    for (std::string_view h : split(l1 == std::string_view::npos ? std::string_view() : hdr.substr(l1 + 2), '\n')) {
      h = trim(h);
      const size_t colon = h.find(':');
      if (colon == std::string_view::npos) continue;
      std::string name(h.substr(0, colon));
      for (char& ch : name) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
      const std::string_view val = trim(h.substr(colon + 1));
      if (name == "content-length") clen = static_cast<size_t>(std::strtoull(std::string(val).c_str(), nullptr, 10));
      else if (name == "transfer-encoding" && val.find("chunked") != std::string_view::npos) chunked = true;
      else if (name == "connection" && (val == "close" || val == "Close")) close_req = true;
    }
    std::string body;
    size_t consumed;
    if (chunked) {
      size_t p = he + 4;
      bool done = false;
      for (;;) {
        const size_t le = c->in.find("\r\n", p);
        if (le == std::string::npos) break;
        const size_t sz = static_cast<size_t>(std::strtoull(c->in.substr(p, le - p).c_str(), nullptr, 16));
        if (sz == 0) {
          const size_t fe = c->in.find("\r\n", le + 2);
          if (fe == std::string::npos) break;
          p = fe + 2;
          done = true;
          break;
        }
        if (c->in.size() < le + 2 + sz + 2) break;
        body.append(c->in, le + 2, sz);
        p = le + 2 + sz + 2;
      }
      if (!done) break;
      consumed = p;
    } else {
      if (c->in.size() < he + 4 + clen) break;
      body.assign(c->in, he + 4, clen);
      consumed = he + 4 + clen;
    }
    Req req;
    req.method = line.substr(0, s1);
    std::string_view target = line.substr(s1 + 1, s2 - s1 - 1);
    const size_t qm = target.find('?');
    req.path = target.substr(0, qm);
    if (qm != std::string_view::npos)
      for (std::string_view kv : split(target.substr(qm + 1), '&')) {
        const size_t eq = kv.find('=');
        if (eq == std::string_view::npos) req.q[url_decode(kv)] = "";
        else req.q[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
      }
    req.body = body;
    const bool watch_pods = req.method == "GET" && req.path == "/api/v1/pods" && is_watch(req);
    const bool watch_nodes = req.method == "GET" && req.path == "/api/v1/nodes" && is_watch(req);
    if (watch_pods || watch_nodes) {
      c->out += head(200, 0, true);
      c->watching = true;
      // the rest of the buffer (nothing, from a well-behaved client) waits for the stream end
      std::string rest = c->in.substr(consumed);
      start_watch(c, watch_pods ? kPods : kNodes, req);
      c->in.swap(rest);
      break;
    }
    // kube-apiserver's max-in-flight filter: a mutating request over the limit is refused before
    // any handling (429, Retry-After: 1); one admitted holds its slot until its answer is written
    const bool mutating = req.method == "POST" || req.method == "PUT" || req.method == "PATCH" ||
                          req.method == "DELETE";
    const int limit = max_mutating.load(std::memory_order_relaxed);
    bool admitted = false;
    std::pair<int, std::string> answer;
    if (mutating && limit > 0) {
      const int now_in = mutating_inflight.fetch_add(1, std::memory_order_relaxed) + 1;
      if (now_in > limit) {
        mutating_inflight.fetch_sub(1, std::memory_order_relaxed);
        n_429.fetch_add(1, std::memory_order_relaxed);
        answer = {429, status_body(429, "TooManyRequests", "Too many requests, please try again later.")};
      } else {
        admitted = true;
        int pk = peak_mutating.load(std::memory_order_relaxed);
        while (now_in > pk && !peak_mutating.compare_exchange_weak(pk, now_in, std::memory_order_relaxed)) {
        }
      }
    }
    auto [code, resp] = admitted || !(mutating && limit > 0) ? handle(req) : std::move(answer);
    c->in.erase(0, consumed);
    const double lat = code == 429 ? 0.0 : latency_s.load(std::memory_order_relaxed);
    if (lat > 0 || !t->delayed.empty()) {
      // earlier responses of this thread may still be held: keep every connection's order
      t->delayed.emplace_back(steady_s() + lat, c, head(code, resp.size()) + resp, admitted);
    } else {
      c->out += head(code, resp.size());
      c->out += resp;
      if (admitted) mutating_inflight.fetch_sub(1, std::memory_order_relaxed);
    }
    if (close_req) c->close_after = true;
    // a pipelined request behind this one: its answer goes out first, as Go's net/http (kube-
    // apiserver) flushes every response when its handler returns; an answer never waits for
    // the next request's handling
    if (!c->in.empty() && !c->close_after && lat <= 0 && t->delayed.empty() && !write_out(c.get())) {
      close_conn(t, c);
      return;
    }
  }
  if (!write_out(c.get())) {
    close_conn(t, c);
    return;
  }
  if (c->out.empty() && c->close_after) {
    close_conn(t, c);
    return;
  }
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | (c->out.empty() ? 0u : EPOLLOUT);
  ev.data.fd = c->fd;
  epoll_ctl(t->ep, EPOLL_CTL_MOD, c->fd, &ev);
}

void Server::Impl::flush_watches(IoThread* t) {
  t->flush_due = 0;
  t->last_flush = steady_s();
  std::vector<std::shared_ptr<Conn>> fl;
  {
    std::lock_guard<std::mutex> g(t->mu);
    fl.swap(t->flush);
  }
  for (auto& c : fl) {
    c->queued.store(false);
    if (!t->conns.count(c->fd) || t->conns[c->fd] != c) continue;   // closed meanwhile
    flush_watch(c);
    if (!write_out(c.get())) {
      close_conn(t, c);
      continue;
    }
    epoll_event ce{};
    ce.events = EPOLLIN | EPOLLRDHUP | (c->out.empty() ? 0u : EPOLLOUT);
    ce.data.fd = c->fd;
    epoll_ctl(t->ep, EPOLL_CTL_MOD, c->fd, &ce);
    if (!c->watching && !c->in.empty()) on_readable(t, c);   // requests queued behind a stream
  }
}

namespace {
// epoll_pwait2's nanosecond timeout where the kernel has it (5.11+), else milliseconds
// rounded up
int wait_events(int ep, epoll_event* evs, int max, double wait_s) {
  static std::atomic<bool> no_pwait2{false};
  if (!no_pwait2.load(std::memory_order_relaxed)) {
    timespec ts;
    ts.tv_sec = static_cast<time_t>(wait_s);
    ts.tv_nsec = static_cast<long>((wait_s - static_cast<double>(ts.tv_sec)) * 1e9);
    const int n = epoll_pwait2(ep, evs, max, &ts, nullptr);
    if (n >= 0 || errno != ENOSYS) return n;
    no_pwait2.store(true, std::memory_order_relaxed);
  }
  return epoll_wait(ep, evs, max, static_cast<int>(std::ceil(wait_s * 1e3)));
}
}  // namespace

void Server::Impl::io_loop(IoThread* t) {
  epoll_event evs[256];
  while (!stopping.load(std::memory_order_acquire)) {
    // sub-millisecond deadlines (the 200 us watch linger, modelled round trips): a
    // millisecond epoll timeout would hold the last chunk of a burst up to 1 ms
    double wait_s = 0.2;
    if (!t->delayed.empty()) wait_s = std::min(wait_s, std::get<0>(t->delayed.front()) - steady_s());
    if (t->flush_due > 0) wait_s = std::min(wait_s, t->flush_due - steady_s());
    wait_s = std::max(0.0, wait_s);
    const double deadline = steady_s() + wait_s;   // the next held answer / watch flush is due
    int n = 0;
    const double spin = spin_s.load(std::memory_order_relaxed);
    if (spin > 0 && wait_s > 0) {
      // the thread polls instead of sleeping for `spin` after its last event, so its core never
      // idles between a burst's requests (or across a short gap); never past `deadline`
      const double until = std::min(t->last_event + spin, deadline);
      while ((n = wait_events(t->ep, evs, 256, 0.0)) == 0 && steady_s() < until &&
             !stopping.load(std::memory_order_relaxed)) {
      }
    }
    if (n == 0) n = wait_events(t->ep, evs, 256, std::max(0.0, deadline - steady_s()));
    if (n > 0 && spin > 0) t->last_event = steady_s();
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == lfd) {
        for (;;) {
          const int cfd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (cfd < 0) break;
          int one = 1;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          auto c = std::make_shared<Conn>();
          c->fd = cfd;
          c->owner = t;
          t->conns[cfd] = c;
          epoll_event ce{};
          ce.events = EPOLLIN | EPOLLRDHUP;
          ce.data.fd = cfd;
          epoll_ctl(t->ep, EPOLL_CTL_ADD, cfd, &ce);
        }
        continue;
      }
      if (fd == t->efd) {
        uint64_t v;
        (void)!read(t->efd, &v, sizeof v);
        // a busy stream is flushed at most once per linger window, so a burst of events
        // leaves as a few large chunks instead of one chunk per event; an idle one at once
        const double now = steady_s();
        if (t->urgent.exchange(false) || now - t->last_flush >= linger_s) flush_watches(t);
        else if (t->flush_due == 0) t->flush_due = t->last_flush + linger_s;
        continue;
      }
      auto it = t->conns.find(fd);
      if (it == t->conns.end()) continue;
      std::shared_ptr<Conn> c = it->second;
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
        close_conn(t, c);
        continue;
      }
      if (evs[i].events & EPOLLOUT) {
        if (!write_out(c.get())) {
          close_conn(t, c);
          continue;
        }
        if (c->out.empty() && c->close_after) {
          close_conn(t, c);
          continue;
        }
      }
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP)) on_readable(t, c);
      else if (c->out.empty()) {
        epoll_event ce{};
        ce.events = EPOLLIN | EPOLLRDHUP;
        ce.data.fd = c->fd;
        epoll_ctl(t->ep, EPOLL_CTL_MOD, c->fd, &ce);
      }
    }
    // held responses that are due
    const double now = steady_s();
    if (t->flush_due > 0 && now >= t->flush_due) flush_watches(t);
    while (!t->delayed.empty() && std::get<0>(t->delayed.front()) <= now) {
      auto c = std::get<1>(t->delayed.front()).lock();
      std::string bytes = std::move(std::get<2>(t->delayed.front()));
      if (std::get<3>(t->delayed.front())) mutating_inflight.fetch_sub(1, std::memory_order_relaxed);
      t->delayed.pop_front();
      if (!c || !t->conns.count(c->fd) || t->conns[c->fd] != c) continue;
      c->out += bytes;
      if (!write_out(c.get()) || (c->out.empty() && c->close_after)) {
        close_conn(t, c);
        continue;
      }
      epoll_event ce{};
      ce.events = EPOLLIN | EPOLLRDHUP | (c->out.empty() ? 0u : EPOLLOUT);
      ce.data.fd = c->fd;
      epoll_ctl(t->ep, EPOLL_CTL_MOD, c->fd, &ce);
    }
    // watch deadlines (timeoutSeconds): the stream ends cleanly
    std::vector<std::shared_ptr<Conn>> due;
    for (auto& kv : t->conns)
      if (kv.second->watching && kv.second->deadline > 0 && now >= kv.second->deadline) due.push_back(kv.second);
    for (auto& c : due) {
      unwatch(c.get());
      {
        std::lock_guard<std::mutex> g(c->mu);
        c->ended = true;
      }
      flush_watch(c);
      if (!write_out(c.get())) close_conn(t, c);
    }
  }
}

// ------------------------------------------------------------------------------ Server
Server::Server(const Config& cfg) : impl_(new Impl) {
  presize_fd_table();
  impl_->cfg = cfg;
  if (impl_->cfg.threads < 1) impl_->cfg.threads = 1;
  if (impl_->cfg.history < 16) impl_->cfg.history = 16;
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(cfg.port));
  if (cfg.host.empty() || cfg.host == "0.0.0.0") addr.sin_addr.s_addr = htonl(INADDR_ANY);
  else if (inet_pton(AF_INET, cfg.host.c_str(), &addr.sin_addr) != 1)
    throw std::invalid_argument("ApiServer: host must be an IPv4 address");
  const int lfd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (lfd < 0) throw std::runtime_error("ApiServer: socket failed");
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (bind(lfd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0 || listen(lfd, 4096) != 0) {
    ::close(lfd);
    throw std::runtime_error(std::string("ApiServer: bind/listen failed: ") + std::strerror(errno));
  }
  socklen_t len = sizeof addr;
  getsockname(lfd, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  impl_->lfd = lfd;
  for (int i = 0; i < impl_->cfg.threads; ++i) {
    auto t = std::make_unique<IoThread>();
    t->ep = epoll_create1(EPOLL_CLOEXEC);
    t->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (t->ep < 0 || t->efd < 0) throw std::runtime_error("ApiServer: epoll/eventfd failed");
    epoll_event le{};
    le.events = EPOLLIN | EPOLLEXCLUSIVE;
    le.data.fd = lfd;
    epoll_ctl(t->ep, EPOLL_CTL_ADD, lfd, &le);
    epoll_event ee{};
    ee.events = EPOLLIN;
    ee.data.fd = t->efd;
    epoll_ctl(t->ep, EPOLL_CTL_ADD, t->efd, &ee);
    impl_->io.push_back(std::move(t));
  }
  for (auto& t : impl_->io) {
    IoThread* tp = t.get();
    Impl* im = impl_.get();
    t->th = std::thread([im, tp] { im->io_loop(tp); });
  }
}

Server::~Server() { stop(); }

void Server::stop() {
  if (!impl_ || impl_->stopping.exchange(true)) return;
  for (auto& t : impl_->io) {
    const uint64_t one = 1;
    (void)!write(t->efd, &one, sizeof one);
  }
  for (auto& t : impl_->io)
    if (t->th.joinable()) t->th.join();
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    impl_->watches.clear();
  }
  for (auto& t : impl_->io) {
    for (auto& kv : t->conns) ::close(kv.first);
    t->conns.clear();
    ::close(t->ep);
    ::close(t->efd);
  }
  ::close(impl_->lfd);
}

std::pair<int, std::string> Server::call(std::string_view method, std::string_view target, std::string_view body) {
  Impl::Req r;
  r.method = method;
  const size_t qm = target.find('?');
  r.path = target.substr(0, qm);
  if (qm != std::string_view::npos)
    for (std::string_view kv : split(target.substr(qm + 1), '&')) {
      const size_t eq = kv.find('=');
      if (eq == std::string_view::npos) r.q[url_decode(kv)] = "";
      else r.q[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
    }
  r.body = body;
  if (Impl::is_watch(r)) return {400, status_body(400, "BadRequest", "watch needs a connection")};
  return impl_->handle(r);
}

namespace {
// fn(begin, end) over [0, n) on up to `workers` threads (this one included); serial below
// `min_parallel` items, where thread start-up would cost more than it saves
// threads for bulk creates and deletes (NANOGPU_APISERVER_BULK_THREADS, default 4)
size_t bulk_threads() {
  static const size_t n = [] {
    const char* e = std::getenv("NANOGPU_APISERVER_BULK_THREADS");
    const long v = e ? std::strtol(e, nullptr, 10) : 4;
    return static_cast<size_t>(std::max(1L, std::min(64L, v)));
  }();
  return n;
}

template <class Fn>
void parallel_for(size_t n, size_t workers, size_t min_parallel, Fn&& fn) {
  if (n < min_parallel || workers <= 1) {
    fn(size_t{0}, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t per = (n + workers - 1) / workers;
  for (size_t w = 1; w < workers; ++w)
    pool.emplace_back([&fn, n, per, w] { fn(std::min(n, w * per), std::min(n, (w + 1) * per)); });
  fn(0, std::min(n, per));
  for (auto& t : pool) t.join();
}
}  // namespace

constexpr size_t kBulkChunk = 128;   // pods a bulk create / delete writes per hold of the store's lock

std::vector<int> Server::create_pods(const std::vector<std::string>& texts, int threads) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<FastCreate> fast(texts.size());
  std::vector<JV> vs(texts.size());
  std::vector<int> codes(texts.size(), 201);
  // parsing needs no lock: a large batch is parsed by a few threads, only the inserts are serial
  parallel_for(texts.size(), threads > 0 ? static_cast<size_t>(threads) : bulk_threads(), 256, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      fast[i] = fast_create(texts[i], "");
      if (!fast[i].ok && !parse(texts[i], &vs[i])) codes[i] = 400;
    }
  });
  const auto t1 = std::chrono::steady_clock::now();
  // in chunks: the store's lock is let go (and what the chunk evicted freed) every kBulkChunk
  // pods, so a bind or a label patch waits for one chunk, not for the whole burst
  for (size_t b = 0; b < texts.size(); b += kBulkChunk) {
    {
      std::lock_guard<std::mutex> g(impl_->mu);
      for (size_t i = b; i < std::min(texts.size(), b + kBulkChunk); ++i) {
        if (codes[i] != 201) continue;
        try {
          if (fast[i].ok) impl_->create_fast_locked(fast[i]);
          else impl_->create_pod_locked(std::move(vs[i]), "");
          impl_->n_create.fetch_add(1, std::memory_order_relaxed);
        } catch (const ApiErr& e) {
          codes[i] = e.code;
        }
      }
      impl_->flush_now();
    }
    release_evicted();
  }
  const auto t2 = std::chrono::steady_clock::now();
  auto ns = [](auto d) { return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(d).count()); };
  impl_->bulk_parse_ns.fetch_add(ns(t1 - t0), std::memory_order_relaxed);
  impl_->bulk_insert_ns.fetch_add(ns(t2 - t1), std::memory_order_relaxed);
  return codes;
}

int Server::delete_pods(const std::vector<std::pair<std::string, std::string>>& keys) {
  const auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  // serial: measured on the box, building the final versions on several threads was slower
  // than one thread (allocator contention outweighs ~1 us of work per pod); in chunks, as the
  // bulk create
  for (size_t b = 0; b < keys.size(); b += kBulkChunk) {
    {
      std::lock_guard<std::mutex> g(impl_->mu);
      for (size_t i = b; i < std::min(keys.size(), b + kBulkChunk); ++i)
        n += impl_->delete_pod_locked(keys[i].first, keys[i].second) ? 1 : 0;
      impl_->flush_now();
    }
    release_evicted();
  }
  impl_->n_delete.fetch_add(static_cast<uint64_t>(keys.size()), std::memory_order_relaxed);
  impl_->bulk_delete_ns.fetch_add(
      static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count()),
      std::memory_order_relaxed);
  return n;
}

std::string Server::stats_json() const {
  const Impl& m = *impl_;
  std::lock_guard<std::mutex> g(m.mu);
  auto ld = [](const std::atomic<uint64_t>& a) { return std::to_string(a.load(std::memory_order_relaxed)); };
  return "{\"rv\":" + std::to_string(m.rv) + ",\"pods\":" + std::to_string(m.pods.size()) +
         ",\"nodes\":" + std::to_string(m.nodes.size()) + ",\"bindings\":" + std::to_string(m.bindings) +
         ",\"watches\":" + std::to_string(m.watches.size()) + ",\"requests\":" + ld(m.n_requests) +
         ",\"calls\":{\"create_pod\":" + ld(m.n_create) + ",\"get_pod\":" + ld(m.n_get) + ",\"patch_pod\":" +
         ld(m.n_patch) + ",\"bind_pod\":" + ld(m.n_bind) + ",\"delete_pod\":" + ld(m.n_delete) + ",\"list\":" +
         ld(m.n_list) + ",\"watch\":" + ld(m.n_watch) + ",\"events\":" + ld(m.n_events) + ",\"lease\":" +
         ld(m.n_lease) + "},\"bulk_ns\":{\"parse\":" + ld(m.bulk_parse_ns) + ",\"insert\":" +
         ld(m.bulk_insert_ns) + ",\"delete\":" + ld(m.bulk_delete_ns) + "},\"admission\":{\"max_mutating_inflight\":" +
         std::to_string(m.max_mutating.load()) + ",\"peak_mutating_inflight\":" + std::to_string(m.peak_mutating.load()) +
         ",\"too_many_requests\":" + ld(m.n_429) + "}}";
}

void Server::set_latency(double seconds) { impl_->latency_s.store(seconds > 0 ? seconds : 0.0); }
void Server::set_spin(double seconds) { impl_->spin_s.store(seconds > 0 ? seconds : 0.0); }
void Server::set_max_mutating_inflight(int n) { impl_->max_mutating.store(n > 0 ? n : 0); }

void Server::compact(std::string_view kind) {
  std::lock_guard<std::mutex> g(impl_->mu);
  for (int k = 0; k < kKinds; ++k) {
    if (!kind.empty() && kind != (k == kPods ? "pods" : "nodes")) continue;
    impl_->hist[k].clear();
    impl_->compacted[k] = impl_->rv;
  }
}

void Server::drop_watches(std::string_view kind) {
  std::lock_guard<std::mutex> g(impl_->mu);
  impl_->end_watches(kind.empty() ? -1 : (kind == "pods" ? kPods : kNodes));
}

}  // namespace nanogpu::apisrv
