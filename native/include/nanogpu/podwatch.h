// The pod informer's watch, native side (nanogpu/k8s/informer.py, client.py).
//
// PodWatchFilter: the pod controller's ledger-only work on a watch event, decided from a few
// shallow fields (type, metadata identity, nodeName, phase): ADDED / MODIFIED of pending pods
// and of bound pods the ledger holds are dropped, DELETED of pods Python never saw is released
// from the ledger right here and dropped; every event of a pod once handed to Python keeps
// going to Python (controller/pods.py decides the rest).
//
// PodWatchStream: one watch request read by a native thread (plain HTTP or TLS, chunked
// transfer), each event line run through the filter, the kept lines queued for the Python
// loop, which an eventfd wakes. The event loop no longer reads or splits the stream: at the
// bench's 4 events per pod, 3 of them dropped, that was most of its work per pod.
#pragma once

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_set>
#include <vector>

#include "nanogpu/json.h"
#include "nanogpu/kubewriter.h"
#include "nanogpu/ledger.h"

namespace nanogpu {

struct PodWatchFilter {
  std::shared_ptr<Ledger> ledger;
  std::unordered_set<std::string> forwarded;   // "ns/name" in the Python store
  uint64_t released = 0, dropped = 0;
  // compat (reference pod.go:15-24): a deletionTimestamp alone ends the share; otherwise a
  // terminating pod keeps it until Succeeded/Failed or DELETED (controller/pods.py)
  std::atomic<bool> release_on_terminating{false};   // set from Python while the watch thread reads it
  std::mutex mu;   // a stream thread and the Python loop (reset, counters) share it
  std::string key_buf;   // under mu: the event's "ns/name" (no allocation per event)
};

// Runs one event line through the filter. `d` is parsed (shallow) by the call. Returns true
// when the event goes on to Python; `rv` gets the event object's resourceVersion either way
// (empty when it has none). Throws std::invalid_argument on a line that is not JSON.
bool filter_pod_event(PodWatchFilter& f, std::string_view line, json::Doc& d, std::string* rv);

class PodWatchStream {
 public:
  // `path`: the watch request's path and query (/api/v1/pods?watch=1&resourceVersion=...).
  PodWatchStream(KubeTarget target, std::string path, std::shared_ptr<PodWatchFilter> filter, int read_timeout_s);
  ~PodWatchStream();
  PodWatchStream(const PodWatchStream&) = delete;
  PodWatchStream& operator=(const PodWatchStream&) = delete;

  int notify_fd() const { return efd_; }
  enum State { kStreaming = 0, kEnded = 1, kHttpError = 2, kTransportError = 3 };
  struct Batch {
    std::vector<std::string> lines;   // kept event lines, in order
    std::string last_rv;              // resourceVersion of the last event read (kept or dropped)
    int state = kStreaming;
    int status = 0;                   // kHttpError: the HTTP status; its body in `message`
    std::string message;
  };
  Batch take();
  void stop();

 private:
  void run();
  void push(std::vector<std::string>* lines, bool dropped, const std::string& tail_rv, int state, int status,
            std::string msg);

  KubeTarget t_;
  std::string path_;
  std::shared_ptr<PodWatchFilter> f_;
  int timeout_s_;
  void* ctx_ = nullptr;   // SSL_CTX*
  int efd_ = -1;
  std::atomic<bool> stop_{false};
  std::mutex sock_mu_;   // stop() shuts the socket down only while the thread holds it open
  int sock_ = -1;
  std::mutex mu_;        // pending_
  // backpressure: with this many kept lines not taken yet the thread stops reading (the
  // socket's buffers then push back on the API server) until the event loop catches up
  static constexpr size_t kMaxPending = 65536;
  std::condition_variable drained_;

  Batch pending_;
  std::thread th_;
};

}  // namespace nanogpu
