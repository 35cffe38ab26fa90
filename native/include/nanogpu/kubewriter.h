// Native second half of the extender's bind: the two API writes (the pods/binding POST, which
// carries the placement annotations, then the assume-label PATCH guarded by spec.nodeName) and
// the ledger commit / rollback, done by C++ threads on keep-alive connections to
// kube-apiserver instead of the Python event loop.
//
// Reference: pkg/dealer/dealer.go:155-203 (Bind: the plan annotated on the pod, the binding
// posted, the node's cache debited; the reference holds its global lock across both writes)
// and pkg/scheduler/bind.go. Semantics follow nanogpu/extender/verbs.py::Extender._write,
// which stays the fallback and the spec for the tests: 5xx / 429 are retried with backoff,
// a binding 409 whose pod already sits on the requested node is success (a retried POST
// whose first attempt landed), and any failure of a fresh reservation rolls the ledger back
// (the reference's defects D1/D2 fixed). No write of a refused bind lands on the pod.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <sys/socket.h>

#include "nanogpu/ledger.h"

namespace nanogpu {

struct KubeTarget {
  std::string host;
  int port = 443;
  bool tls = true;
  std::string token;        // bearer token (may be empty)
  std::string token_file;   // re-read on 401 and when it changes (projected tokens rotate)
  std::string ca_file, cert_file, key_file;
  bool insecure = false;    // skip server certificate verification
};

// SSL_CTX* for the target's CA / client certificate (throws std::runtime_error); nullptr for
// plain HTTP. The caller frees it with free_ssl_ctx.
void* make_ssl_ctx(const KubeTarget& t);
void free_ssl_ctx(void* ctx);
// The bearer token now: the token file's contents when it has any, else the target's token.
std::string kube_token(const KubeTarget& t);
// TCP keepalive probes and TCP_USER_TIMEOUT (timeout_s) on an API server connection.
void tcp_liveness(int fd, double timeout_s);
// The Host header's value: host:port, an IPv6 address in brackets.
std::string host_header(const KubeTarget& t);

// One blocking HTTP/1.1 keep-alive connection (plain or TLS).
class HttpConn {
 public:
  HttpConn(const KubeTarget* t, void* ssl_ctx, int timeout_s = 30) : t_(t), ctx_(ssl_ctx), timeout_s_(timeout_s) {}
  ~HttpConn();
  // status 0 = transport failure (message in *body); reconnects once for a request that
  // failed on a connection the server had already closed.
  int request(const char* method, const std::string& path, const std::string& content_type,
              const std::string& body, const std::string& auth, std::string* resp);
  // The same in two halves, so that requests on two connections are in flight together:
  // start() sends, finish() reads the answer (with request()'s one retry on a fresh connection).
  bool start(const char* method, const std::string& path, const std::string& content_type,
             const std::string& body, const std::string& auth);
  int finish(std::string* resp);
  // A streamed answer (a watch): after start(), stream_head() reads the status line and
  // headers; an answer other than 200 is read whole into *body. stream_read() then appends
  // the next decoded body bytes (chunked or to the end of the connection) to *out: > 0 bytes,
  // 0 at the end of the body, -1 on a transport failure or a read timeout (timeout_s).
  int stream_head(std::string* body);
  long stream_read(std::string* out);
  int fd() const { return fd_; }
  // the last answer's Retry-After (seconds; -1: none), as kube-apiserver sends with a 429
  double retry_after() const { return retry_after_; }

 private:
  struct Head {
    int status = 0;
    long clen = -1;
    bool chunked = false, close_after = false;
    double retry_after = -1;
  };
  double retry_after_ = -1;
  bool connect_();
  void close_();
  bool send_all(const char* p, size_t n);
  long recv_some(char* p, size_t n);
  int receive(std::string* resp, bool* retryable);
  bool read_head(Head* h, bool* retryable);
  int read_body(const Head& h, std::string* resp);
  bool stream_chunked_ = false, stream_end_ = false;
  long chunk_left_ = -1;   // bytes of the current chunk still to read, its CRLF included; -1: a size line next
  std::string req_;
  bool reused_ = false, sent_ = false;

  const KubeTarget* t_;
  void* ctx_;               // SSL_CTX* (nullptr: plain HTTP)
  int timeout_s_;           // send / receive timeout of the socket
  int fd_ = -1;
  void* ssl_ = nullptr;     // SSL*
  std::string buf_;
};

struct BindJob {
  uint64_t id = 0;                       // front-door request id (Frontend::respond)
  std::string ns, name, uid, node;
  std::vector<std::string> containers;
  std::vector<std::vector<int32_t>> plan;
  bool fresh = true;                     // this bind made the reservation (rollback on failure)
  uint64_t t0_ns = 0;
  int throttled = 0;                     // times kube-apiserver answered it 429 (re-sent after Retry-After)
};

struct KubeWriterStats {
  std::atomic<uint64_t> ok{0}, failed{0}, rollbacks{0}, retries{0}, patch_ns{0}, binding_ns{0}, inflight{0},
      label_failures{0}, timeouts{0};
  // kube-apiserver's max-in-flight admission: answers 429 TooManyRequests, the binds and labels
  // re-sent after their Retry-After, the window cuts, and the bind window now (evented: the
  // smallest over the writer's BindIo drivers)
  std::atomic<uint64_t> throttled{0}, throttle_resends{0}, window_cuts{0};
  std::atomic<int64_t> window{0};
  // bindings sent ahead of their label because the window had no room for both (the labels
  // followed in batches when it had)
  std::atomic<uint64_t> bindings_first{0};
};

// Two ways to run the writes:
//   * evented (default): ONE epoll thread drives every bind's two requests on non-blocking
//     keep-alive connections (plain or TLS), `threads` x kBatch binds in flight. A bind whose
//     two answers are 2xx commits right there; anything else (a 5xx / 429 / 401 to retry, a
//     409 to check, a failure to roll back, no answer within timeout_s) goes to a slow-path
//     thread that finishes it with
//     the blocking code below. One wake-up serves every answer that arrived together, where
//     a thread per batch sleeps and wakes once per request (kubewriter_evented.cpp);
//   * threads: `threads` blocking threads, each pipelining up to kBatch binds.
class BindIo;

class KubeWriter {
 public:
  using Respond = std::function<void(uint64_t id, int status, const std::string& body)>;
  // `label`: also PATCH the assume label behind the binding, the reference's pod contract;
  // false: the binding alone, which carries the annotations. `timeout_s`: an API request
  // unanswered this long fails (a half-open connection never answers, nor resets).
  // `inline_io` (evented only): no io thread; the owners of epoll loops (front-door workers)
  // drive the requests themselves through make_io(), and submit() is not used.
  // `max_binds` (evented / inline): binds in flight per request driver, the start and the ceiling
  // of its admission window (0: threads x kBatch); size it under kube-apiserver's
  // --max-mutating-requests-inflight (each bind is 2 mutating requests with the label PATCH).
  KubeWriter(KubeTarget target, std::shared_ptr<Ledger> ledger, Respond respond, int threads, int retries,
             bool record_events, bool evented = true, bool label = true, double timeout_s = 30.0,
             bool inline_io = false, int max_binds = 0);
  ~KubeWriter();
  void submit(BindJob job);
  void stop();
  // An evented request driver on the caller's epoll set `ep` (tags `tag_bit | k`); `reply`
  // answers its happy-path binds on the caller's thread. Failures go to this writer's slow path.
  std::unique_ptr<BindIo> make_io(int ep, uint64_t tag_bit, Respond reply);
  bool inline_io() const { return inline_io_; }
  // evented / inline: false pipelines each label PATCH behind its binding instead of batching
  void set_batch_labels(bool on) { batch_labels_.store(on, std::memory_order_relaxed); }
  // Front-door sends (evented mode with its io thread, plain TCP, labels pipelined): the
  // calling thread (a front-door worker, inside the poll window it would otherwise spin
  // through) writes the bind's requests itself on an idle connection the io thread published,
  // adds the connection to the io thread's epoll set and hands it over; the io thread reads
  // the answers, commits and answers kube-scheduler as for any bind, and is not woken for the
  // submission. false: nothing was sent (mode off, no connection idle): submit() the job.
  bool send_from_caller(BindJob& job);
  void set_fe_send(bool on) { fe_send_.store(on, std::memory_order_relaxed); }
  // evented / inline: a label PATCH's answer is read by a later pass of the loop instead of
  // waking it (the connection's SO_RCVLOWAT raised once its binding answered)
  void set_lazy_labels(bool on) { lazy_labels_.store(on, std::memory_order_relaxed); }
  KubeWriterStats stats;

 private:
  // binds one writer thread pipelines together (two connections each)
  static constexpr int kBatch = 8;
  void run();
  void build(BindJob& j, std::string* patch, std::string* binding);
  void process_batch(std::vector<BindJob>& jobs, std::vector<std::unique_ptr<HttpConn>>& conns);
  void finish(HttpConn* c, HttpConn* c2, BindJob& j, const std::string& patch, const std::string& binding, int sp,
              std::string* rp, int sb, std::string* rb);
  // the binding's outcome (retried, checked): committed and answered (true), or rolled back
  // and answered with the error
  bool finish_binding(HttpConn* c2, BindJob& j, const std::string& binding, int sb, std::string* rb);
  // a bound pod's label PATCH that failed (transiently, or refused by its nodeName guard
  // before the binding had landed): sent again; a lasting failure is counted
  void finish_label(HttpConn* c, const BindJob& j, const std::string& patch, int sp, std::string* rp);
  void refuse(BindJob& j);
  int call(HttpConn* c, const char* method, const std::string& path, const std::string& ctype,
           const std::string& body, std::string* resp, bool retry);
  std::string auth();

  friend class BindIo;
  // evented mode (kubewriter_evented.cpp)
  struct SlowJob {
    BindJob j;
    std::string patch, binding, rp, rb;
    int sp = 0, sb = 0;
    bool answered = false;   // bound and answered already: only the label is left
  };
  void io_loop();
  void run_slow();
  void to_slow(SlowJob&& sj);    // the slow path takes it (or, once its threads are gone, the caller)
  bool inline_io_ = false;
  std::atomic<bool> batch_labels_{false};  // evented: label PATCHes batched after their bindings (BindIo)
  bool slow_gone_ = false;       // under mu_: the slow-path threads have exited
  bool evented_ = false;
  int max_inflight_ = 0;
  int efd_ = -1;                 // wakes the io thread (new jobs, stop)
  // the io thread is about to block in epoll_wait: only then does a submit write efd_ (it sets
  // io_parked_ and re-reads q_len_; a submit stores q_len_ and reads io_parked_, both seq_cst)
  std::atomic<bool> io_parked_{false};
  std::atomic<size_t> q_len_{0};
  std::thread io_;
  std::atomic<bool> io_done_{false};   // the io thread has handed everything to the slow path
  // front-door sends (send_from_caller): connections the io thread published (taken out of its
  // epoll set), the binds sent on them waiting to be adopted, all under fe_mu_
  struct Handoff {
    size_t k = 0;                 // BindIo connection index
    BindJob j;
    std::string patch, binding, out;
    size_t sent = 0;              // bytes of `out` the caller's send took
    bool broken = false;          // the send failed: the io thread retries on a fresh connection
  };
  std::atomic<bool> fe_send_{false};
  std::atomic<bool> lazy_labels_{false};
  std::mutex fe_mu_;
  std::vector<std::pair<size_t, int>> fe_idle_;   // (connection index, fd)
  std::vector<Handoff> adopt_;
  bool fe_closed_ = true;        // no io thread to hand over to (not started, or stopping)
  int fe_busy_ = 0;              // front-door threads between taking a connection and its handoff
  int io_ep_ = -1;               // the io thread's epoll set (under fe_mu_)
  std::string host_hdr_;
  // the API server's address, resolved at construction (evented / inline); addr_len_ 0: not
  // resolved then, each BindIo resolves it itself
  sockaddr_storage addr_{};
  socklen_t addr_len_ = 0;
  int family_ = 0;
  std::deque<SlowJob> slow_q_;   // under mu_, signalled on cv_

  KubeTarget t_;
  std::shared_ptr<Ledger> ledger_;
  Respond respond_;
  int retries_;
  double timeout_s_ = 30.0;
  bool events_;
  bool label_ = true;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<BindJob> q_;
  bool stop_ = false;
  std::vector<std::thread> threads_;
  void* ctx_ = nullptr;     // SSL_CTX*
  std::mutex tok_mu_;
  std::string token_;
  int64_t token_mtime_ = 0;
  double token_checked_ = 0;
};

}  // namespace nanogpu
