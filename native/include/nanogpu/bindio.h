// The evented half of the native bind writer (see kubewriter.h): the API requests of every bind
// in flight on non-blocking keep-alive connections (plain or TLS), driven by an epoll set that
// belongs to whoever owns the BindIo:
//   * the writer's own io thread (KubeWriter evented mode: ngpu-wr-io), or
//   * a front-door worker (inline mode): the worker that parsed the bind sends its binding
//     from its own epoll loop, takes the API answer there and writes kube-scheduler's reply
//     on the same thread. No hand-off to a writer thread and back (eventfd, two wake-ups and
//     a mailbox per bind); a busy-polling worker catches the API answer in its spin.
// Happy path only: a bind whose binding (and label PATCH) answer 2xx is committed and answered
// here. Every other outcome goes to the writer's slow-path threads (KubeWriter::finish).
#pragma once

#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <string>
#include <sys/socket.h>
#include <vector>

#include "nanogpu/kubewriter.h"

namespace nanogpu {

class BindIo {
 public:
  using Reply = std::function<void(uint64_t id, int status, const std::string& body)>;
  // Registers its sockets in `ep` with epoll data `tag_bit | k` (k: connection index); `reply`
  // answers a bind that completed on the happy path (from the owning thread).
  BindIo(KubeWriter* kw, int ep, uint64_t tag_bit, int max_inflight, Reply reply);
  ~BindIo();
  BindIo(const BindIo&) = delete;
  BindIo& operator=(const BindIo&) = delete;

  void submit(BindJob j);                      // launches it now, or when a slot frees up
  void on_event(uint64_t k, uint32_t events);  // an epoll event of connection k
  void pump();                                 // after a batch of events: drive what is due
  // binds and batched label PATCHes not finished yet
  size_t inflight() const { return inflight_ + labels_out_ + label_wait_.size() + deferred_.size(); }
  size_t waiting() const { return waiting_.size(); }
  // label PATCHes held for a batch: the owner's loop must come back within about a millisecond
  bool labels_waiting() const { return !label_wait_.empty() || !lazy_.empty() || !deferred_.empty(); }
  // Stop: every bind still in flight or waiting goes to the slow path with what it got
  // (`why` for answers that never came). The connections are closed.
  void abandon(const char* why);
  // front-door sends (KubeWriter::send_from_caller): takes over the binds handed over since
  // the last call (their connections are in this loop's epoll set already)
  void adopt_handoffs();
  // lazy label answers (KubeWriter::set_lazy_labels)
  void go_lazy(size_t k);
  void drain_lazy(uint64_t now);
  // connection k is handed out for front-door sends instead of waiting in idle_
  bool publish(size_t k);
  uint64_t timeouts() const { return timeouts_; }
  double window() const { return window_; }

 private:
  struct Conn;
  struct Job;
  struct Label;
  bool resolve();
  void close_conn(Conn& c);
  bool open_conn(size_t k);
  void request(std::string* r, const char* method, const BindJob& j, bool binding, std::string_view ctype,
               const std::string& body);
  void complete(int64_t s);
  void deliver(Conn& c, int status, std::string body, double retry_after = -1);
  void deliver_rest(Conn& c, const char* why);
  void fail(size_t k, const char* why);
  void drive(size_t k, uint32_t events);
  void launch(int64_t s);
  void start_waiting();
  void scan_deadlines(uint64_t now);
  void queue_label(BindJob&& j, std::string&& patch);
  void label_done(int64_t ls, int status, std::string body);
  void launch_labels(size_t room);
  // kube-apiserver's max-in-flight admission (429 TooManyRequests, Retry-After): the binds in
  // flight are capped by an AIMD window, halved on a 429 (once per window: only an answer to a
  // request sent after the last cut cuts again), one bind wider after a window's worth of clean
  // binds, never above the configured maximum. A throttled bind (its binding refused before any
  // handling, so nothing of it landed) or label goes out again after the Retry-After, from this
  // loop; after kMaxThrottled refusals the slow path finishes it (retries, then rollback).
  void throttle(uint64_t seq);
  void widen();
  void defer(BindJob&& j, std::string&& patch, bool label_only, double retry_after);
  void resend_due(uint64_t now);
  static constexpr int kMaxThrottled = 8;
  static constexpr double kMaxRetryAfterS = 2.0;
  double window_ = 1, max_window_ = 1, clean_ = 0;
  uint64_t launch_seq_ = 0, cut_seq_ = 0;
  struct Deferred {
    uint64_t due_ns;
    BindJob j;
    std::string patch;
    bool label_only;
  };
  std::deque<Deferred> deferred_;

  KubeWriter* kw_;
  int ep_;
  uint64_t tag_bit_;
  Reply reply_;
  std::vector<std::unique_ptr<Conn>> conns_;   // index = epoll tag (without tag_bit)
  std::vector<size_t> idle_;
  std::vector<std::unique_ptr<Job>> slots_;
  std::vector<int64_t> free_slots_;
  std::deque<BindJob> waiting_;
  std::vector<size_t> kick_;                   // connections to drive in pump()
  sockaddr_storage addr_{};
  socklen_t addr_len_ = 0;
  int family_ = 0;
  std::string auth_;
  uint64_t auth_at_ = 0;
  std::string host_hdr_;
  size_t inflight_ = 0;
  uint64_t timeout_ns_ = 0;
  uint64_t scanned_at_ = 0;
  uint64_t timeouts_ = 0;
  // Label PATCHes (the reference's assume label, guarded by spec.nodeName): pipelined behind
  // their binding on its connection by default; with KubeWriter::set_batch_labels they go out
  // after their binding answered, batched: up to kLabelBatch pipelined on one connection, one
  // send and a read or two for all of them, held at most kLabelHoldNs for the batch to fill.
  static constexpr size_t kLabelBatch = 32;
  static constexpr uint64_t kLabelHoldNs = 500'000;
  // a label left waiting for room in the admission window this long goes before more binds
  static constexpr uint64_t kLabelStarveNs = 50'000'000;
  int64_t req_inflight_ = 0;   // requests of the binds in flight (2: binding + label, 1: alone)
  std::vector<std::unique_ptr<Label>> lslots_;
  std::vector<int64_t> lfree_;
  std::deque<int64_t> label_wait_;
  uint64_t label_oldest_ns_ = 0;
  size_t labels_out_ = 0;   // sent, answer due
  // lazy label answers: connections whose only due answers are label answers of answered binds
  // (their low-water mark raised), read kLazyNs or more after they went lazy
  static constexpr uint64_t kLazyNs = 20'000;
  std::vector<size_t> lazy_;
  void reset_lowat(Conn& c);
};

}  // namespace nanogpu
