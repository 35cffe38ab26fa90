// Native in-memory Kubernetes API server: the shared API server of multi-process benches and
// system tests (pods, nodes, bindings, leases, events; list + watch with resourceVersion
// resume and 410 Gone). Wire-compatible with nanogpu/k8s/fake_apiserver.py's HTTP facade and
// the paths KubeClient uses, but built to not be the bottleneck when several extender workers
// (one per bench rank) write through it at once: epoll IO threads, one store lock held only
// for the map update, every object serialized once per version and shared by every watch.
//
// Store model: objects are immutable snapshots (shared_ptr<const Obj>); a write builds the new
// version outside nothing but the store lock and publishes it with its resourceVersion. Watch
// events are appended to a bounded per-kind history (the watch cache) and pushed to each
// matching watcher's output queue; the watcher's IO thread flushes it as HTTP chunks.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <utility>
#include <vector>

namespace nanogpu::apisrv {

// Mutable JSON value (the stored objects and merge patches). Numbers keep their source text.
struct JV {
  enum class T : uint8_t { kNull, kBool, kNum, kStr, kArr, kObj };
  T t = T::kNull;
  bool b = false;
  std::string s;                                  // string value, or number text
  std::vector<JV> a;
  std::vector<std::pair<std::string, JV>> o;

  static JV str(std::string v) {
    JV j;
    j.t = T::kStr;
    j.s = std::move(v);
    return j;
  }
  static JV obj() {
    JV j;
    j.t = T::kObj;
    return j;
  }
  bool is_obj() const { return t == T::kObj; }
  const JV* get(std::string_view k) const;
  JV* get(std::string_view k);
  JV& set(std::string_view k, JV v);              // replaces or appends
  JV& child(std::string_view k);                  // object member, created as {} when absent
  void erase(std::string_view k);
  std::string_view sv() const { return t == T::kStr ? std::string_view(s) : std::string_view(); }
};

bool parse(std::string_view text, JV* out);
void dump(const JV& v, std::string* out);
// RFC 7386 JSON merge patch.
void merge_patch(JV* target, const JV& patch);

struct Config {
  std::string host = "127.0.0.1";
  int port = 0;
  int threads = 4;
  size_t history = 200000;     // watch-cache events kept per kind
};

class Server {
 public:
  explicit Server(const Config& cfg);
  ~Server();
  Server(const Server&) = delete;
  Server& operator=(const Server&) = delete;

  int port() const { return port_; }
  void stop();
  // One request handled in-process (the harness's client path, no socket): returns
  // (status, body). Watches are not served this way.
  std::pair<int, std::string> call(std::string_view method, std::string_view target, std::string_view body);
  // Creates many pods (JSON texts, namespace taken from each object) under one lock hold.
  // `threads`: parse workers for a large batch (0: NANOGPU_APISERVER_BULK_THREADS, default 4)
  std::vector<int> create_pods(const std::vector<std::string>& pods, int threads = 0);
  // Deletes (namespace, name) pairs; returns how many existed.
  int delete_pods(const std::vector<std::pair<std::string, std::string>>& keys);
  std::string stats_json() const;
  // Modelled API round trip: every HTTP response is held this long after its request was
  // handled (watch events are not delayed). 0 = none.
  void set_latency(double seconds);
  // IO threads poll for `seconds` after their last event before sleeping (0: sleep at once)
  void set_spin(double seconds);
  // kube-apiserver's --max-mutating-requests-inflight (its default 200; 0: no limit): a
  // POST / PUT / PATCH / DELETE arriving while this many are in flight (handled, answer not yet
  // written: with a modelled round trip, until it is due) is answered 429 TooManyRequests with
  // `Retry-After: 1`, as kube-apiserver's max-in-flight filter does, without being handled.
  void set_max_mutating_inflight(int n);
  // Watch-cache control for tests: forget history (a resumed watch gets 410 Gone), end every
  // open watch of `kind` ("pods" | "nodes" | "" = both).
  void compact(std::string_view kind);
  void drop_watches(std::string_view kind);

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
  int port_ = 0;
};

}  // namespace nanogpu::apisrv
