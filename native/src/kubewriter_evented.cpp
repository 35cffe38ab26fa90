// Evented bind writer (see kubewriter.h, bindio.h): BindIo drives the two API requests of every
// bind in flight on non-blocking keep-alive connections, plain HTTP or TLS, from an epoll set
// that belongs to the writer's io thread or, inline, to a front-door worker.
//
// Why: the threaded writer keeps a thread per batch of binds that blocks in recv() for each
// answer; at the bench's 40 binds per millisecond with a fast API server that is one sleep and
// one wake-up per request (~17 us of CPU per bind on the MI355X box, profiles/). Here one
// epoll_wait returns every answer that arrived together.
//
// Scope: the happy path only. A bind whose binding and label PATCH both answer 2xx is committed
// on this thread and answered. Every other outcome (transport failure after the one reconnect a
// stale keep-alive connection gets, 5xx / 429 / 401 to retry, 409 to check, a rollback) goes,
// with the answers received, to a slow-path thread running KubeWriter::finish, the same code the
// threaded writer uses, so retry and rollback semantics are identical in both modes.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/epoll.h>

#include <charconv>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <deque>
#include <memory>
#include <vector>

#include "nanogpu/bindhops.h"
#include "nanogpu/bindio.h"
#include "nanogpu/iotally.h"
#include "nanogpu/kubewriter.h"

namespace nanogpu {

namespace {

constexpr const char* kMergePatchE = "application/merge-patch+json";
constexpr const char* kJsonE = "application/json";

uint64_t ns_now() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count());
}

// One HTTP/1.1 response at the front of `b`: 1 = complete, 0 = need more, -1 = malformed.
// `eof`: the peer closed (completes a response without a length).
bool ieq_ascii(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower(static_cast<unsigned char>(a[i])) != b[i]) return false;
  return true;
}

// One answer at the front of `b`: 1 = complete (status, body, bytes consumed), 0 = more bytes
// needed, -1 = not HTTP. Headers are read in place; the body is copied only for an answer
// outside 2xx, the only one anybody reads (the slow path reports or inspects it).
int parse_response(const std::string& b, bool eof, int* status, std::string* body, size_t* consumed, bool* close,
                   double* retry_after) {
  *retry_after = -1;
  const size_t he = b.find("\r\n\r\n");
  if (he == std::string::npos) return b.size() > (256u << 10) ? -1 : 0;
  if (he < 12 || b.compare(0, 5, "HTTP/") != 0) return -1;
  *status = std::atoi(b.c_str() + 9);
  const bool keep_body = *status < 200 || *status >= 300;
  long clen = -1;
  bool chunked = false;
  *close = false;
  const std::string_view bv(b);
  size_t p = b.find("\r\n");
  while (p < he) {
    const size_t e = b.find("\r\n", p + 2);
    const size_t end = e == std::string::npos || e > he ? he : e;
    const size_t colon = b.find(':', p + 2);
    if (colon != std::string::npos && colon < end) {
      const std::string_view k = bv.substr(p + 2, colon - p - 2);
      size_t v0 = colon + 1;
      while (v0 < end && b[v0] == ' ') ++v0;
      const std::string_view v = bv.substr(v0, end - v0);
      if (ieq_ascii(k, "content-length")) clen = std::strtol(b.c_str() + v0, nullptr, 10);
      else if (ieq_ascii(k, "transfer-encoding") && v.find("chunked") != std::string_view::npos) chunked = true;
      else if (ieq_ascii(k, "connection") && (v == "close" || v == "Close")) *close = true;
      else if (*status == 429 && ieq_ascii(k, "retry-after")) *retry_after = std::strtod(b.c_str() + v0, nullptr);
    }
    if (end == he) break;
    p = end;
  }
  size_t q = he + 4;
  body->clear();
  if (chunked) {
    for (;;) {
      const size_t le = b.find("\r\n", q);
      if (le == std::string::npos) return 0;
      const size_t sz = std::strtoul(b.c_str() + q, nullptr, 16);
      if (b.size() < le + 2 + sz + 2) return 0;
      if (keep_body) body->append(b, le + 2, sz);
      q = le + 2 + sz + 2;
      if (sz == 0) break;
    }
    *consumed = q;
    return 1;
  }
  if (clen >= 0) {
    if (b.size() < q + static_cast<size_t>(clen)) return 0;
    if (keep_body) body->assign(b, q, static_cast<size_t>(clen));
    *consumed = q + static_cast<size_t>(clen);
    return 1;
  }
  if (!eof) return 0;   // the body runs to the end of the connection
  if (keep_body) body->assign(b, q, std::string::npos);
  *consumed = b.size();
  *close = true;
  return 1;
}

// kPublished: handed out for front-door sends (KubeWriter::send_from_caller), out of this
// loop's epoll set until a handoff brings it back
enum ConnState { kIdle, kConnecting, kHandshake, kSending, kReceiving, kPublished };

// One API request: method, the pod's path, headers, body (`r`'s capacity is kept).
void compose_request(std::string* r, const char* method, const BindJob& j, bool binding, std::string_view ctype,
                     const std::string& body, const std::string& host_hdr, const std::string& auth) {
  r->clear();
  *r += method;
  *r += " /api/v1/namespaces/";
  *r += j.ns;
  *r += "/pods/";
  *r += j.name;
  if (binding) *r += "/binding";
  *r += " HTTP/1.1\r\nHost: ";
  *r += host_hdr;
  *r += "\r\nUser-Agent: nano-gpu-scheduler-amd/0.1\r\nAccept: application/json\r\n";
  if (!auth.empty()) {
    *r += "Authorization: Bearer ";
    *r += auth;
    *r += "\r\n";
  }
  *r += "Content-Type: ";
  *r += ctype;
  char len[24];
  *r += "\r\nContent-Length: ";
  r->append(len, static_cast<size_t>(std::to_chars(len, len + sizeof len, body.size()).ptr - len));
  *r += "\r\n\r\n";
  *r += body;
}

// A bind's two requests go out pipelined on ONE connection, the binding first: one send and,
// usually, one read for both answers (HTTP/1.1 answers come back in request order; kube-
// apiserver's Go server and the bench's API server both serve pipelined requests in order).
struct Pending {
  int64_t job;   // in-flight job slot (label slot for a batched label)
  int which;     // 0: label PATCH pipelined behind its binding, 1: binding, 2: batched label PATCH
};

}  // namespace

struct BindIo::Conn {
  int fd = -1;
  SSL* ssl = nullptr;
  int st = kIdle;
  bool reused = false;   // the requests went out on a connection used before
  bool got_any = false;  // response bytes seen since the requests went out
  bool retried = false;  // the one fresh-connection retry is spent
  std::string out, in;
  size_t off = 0;
  std::vector<Pending> pend;   // answers still due, in request order, from `head`
  size_t head = 0;
  uint64_t deadline_ns = 0;   // the answers are due by then (KubeWriter timeout_s)
  bool missed = false;        // kPublished: an arrival's edge came before the handoff was adopted
  bool lowat = false;         // SO_RCVLOWAT raised (lazy label answers): arrivals do not wake the loop
  uint64_t lazy_since = 0;    // in lazy_ since (0: not lazy)
  int npend() const { return static_cast<int>(pend.size() - head); }
};

struct BindIo::Job {
  BindJob j;
  std::string patch, binding, rp, rb;
  int sp = 0, sb = 0;
  int left = 2;
  uint64_t seq = 0;           // launch order (the admission window's cut rule)
  double retry_after = -1;    // a 429's Retry-After (seconds)
  bool answered = false;   // kube-scheduler has its answer (the binding landed; the label may follow)
  bool batch_label = false;   // the label goes in a later batch (queue_label), not behind the binding
  int reqs = 2;               // requests it holds against the admission window (binding + label, or 1)
};

struct BindIo::Label {
  BindJob j;
  std::string patch;
  uint64_t seq = 0;
  double retry_after = -1;   // a 429's Retry-After (seconds)
};

namespace {
bool ok2xx(int st) { return st >= 200 && st < 300; }
}  // namespace

BindIo::BindIo(KubeWriter* kw, int ep, uint64_t tag_bit, int max_inflight, Reply reply)
    : kw_(kw), ep_(ep), tag_bit_(tag_bit), reply_(std::move(reply)) {
  // the window counts binds (a binding and its label); under a backlog a binding may go alone
  // (start_waiting), so twice the slots
  slots_.resize(static_cast<size_t>(std::max(1, max_inflight)) * (kw_->label_ ? 2 : 1));
  for (int64_t i = static_cast<int64_t>(slots_.size()) - 1; i >= 0; --i) free_slots_.push_back(i);
  window_ = max_window_ = static_cast<double>(std::max(1, max_inflight));
  auth_ = kw_->auth();
  auth_at_ = ns_now();
  host_hdr_ = host_header(kw_->t_);
  timeout_ns_ = static_cast<uint64_t>(kw_->timeout_s_ * 1e9);
  scanned_at_ = ns_now();
}

BindIo::~BindIo() {
  for (auto& c : conns_) close_conn(*c);
}

bool BindIo::resolve() {
  if (addr_len_) return true;
  if (kw_->addr_len_) {   // resolved when the writer was set up (not on this loop)
    std::memcpy(&addr_, &kw_->addr_, kw_->addr_len_);
    addr_len_ = kw_->addr_len_;
    family_ = kw_->family_;
    return true;
  }
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  if (getaddrinfo(kw_->t_.host.c_str(), std::to_string(kw_->t_.port).c_str(), &hints, &res) != 0 || !res) return false;
  std::memcpy(&addr_, res->ai_addr, res->ai_addrlen);
  addr_len_ = res->ai_addrlen;
  family_ = res->ai_family;
  freeaddrinfo(res);
  return true;
}

void BindIo::close_conn(Conn& c) {
  if (c.ssl) SSL_free(c.ssl);
  c.ssl = nullptr;
  c.lowat = false;
  c.lazy_since = 0;   // drain_lazy drops its entry
  if (c.fd >= 0) {
    epoll_ctl(ep_, EPOLL_CTL_DEL, c.fd, nullptr);
    ::close(c.fd);
  }
  c.fd = -1;
  c.in.clear();
  c.st = kIdle;
}

// a fresh non-blocking connection (connect in progress); false: cannot even start
bool BindIo::open_conn(size_t k) {
  Conn& c = *conns_[k];
  close_conn(c);
  if (!resolve()) return false;
  const int fd = socket(family_, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (fd < 0) return false;
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  tcp_liveness(fd, kw_->timeout_s_);
  const int cr = ::connect(fd, reinterpret_cast<sockaddr*>(&addr_), addr_len_);
  if (cr != 0 && errno != EINPROGRESS) {
    ::close(fd);
    return false;
  }
  c.fd = fd;
  c.st = cr == 0 ? (kw_->ctx_ ? kHandshake : kSending) : kConnecting;
  if (kw_->ctx_) {
    c.ssl = SSL_new(static_cast<SSL_CTX*>(kw_->ctx_));
    if (!c.ssl) {
      close_conn(c);
      return false;
    }
    SSL_set_fd(c.ssl, fd);
    const std::string& host = kw_->t_.host;
    in6_addr a6{};
    const bool ip = inet_pton(AF_INET, host.c_str(), &a6) == 1 || inet_pton(AF_INET6, host.c_str(), &a6) == 1;
    if (!ip) SSL_set_tlsext_host_name(c.ssl, host.c_str());
    if (!kw_->t_.insecure) {
      if (ip) X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(c.ssl), host.c_str());
      else SSL_set1_host(c.ssl, host.c_str());
    }
  }
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP | EPOLLET;
  ev.data.u64 = tag_bit_ | k;
  epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
  return true;
}

// a request written into the connection's own buffer (its capacity is kept across binds)
void BindIo::request(std::string* r, const char* method, const BindJob& j, bool binding, std::string_view ctype,
                     const std::string& body) {
  compose_request(r, method, j, binding, ctype, body, host_hdr_, auth_);
}

// both answers of a slot are in: commit on the happy path, else the slow path finishes it
void BindIo::complete(int64_t s) {
  std::unique_ptr<Job> jb = std::move(slots_[static_cast<size_t>(s)]);
  free_slots_.push_back(s);
  --inflight_;
  req_inflight_ -= jb->reqs;
  KubeWriterStats& st = kw_->stats;
  if (jb->answered && ok2xx(jb->sp)) {   // bound and answered earlier; the label landed too
    widen();
    st.inflight.fetch_sub(1, std::memory_order_relaxed);
    return;
  }
  // kube-apiserver refused the binding at admission (429): nothing of this bind landed (the
  // label PATCH behind it was refused by its nodeName guard, or throttled too); the whole bind
  // goes out again after the Retry-After, on its reservation
  if (!jb->answered && jb->sb == 429 && jb->j.throttled < kMaxThrottled) {
    ++jb->j.throttled;
    defer(std::move(jb->j), std::string(), false, jb->retry_after);
    return;   // still in flight for the writer's stats
  }
  // bound and answered; only its label PATCH was throttled
  if (jb->answered && jb->sp == 429 && jb->j.throttled < kMaxThrottled) {
    ++jb->j.throttled;
    defer(std::move(jb->j), std::move(jb->patch), true, jb->retry_after);
    return;
  }
  IoTimer it{kWrCommit};
  const bool ok2 = ok2xx(jb->sb) && (jb->batch_label || ok2xx(jb->sp));
  if (ok2) widen();
  if (!jb->answered) st.binding_ns.fetch_add(ns_now() - jb->j.t0_ns, std::memory_order_relaxed);
  if (ok2) {
    kw_->ledger_->commit(jb->j.uid);
    st.ok.fetch_add(1, std::memory_order_relaxed);
    g_hops.stamp(jb->j.id, kHopPosted);
    reply_(jb->j.id, 200, "{\"Error\":\"\"}");
    if (jb->batch_label) {   // bound: the label follows in a batch (stats.inflight until then)
      queue_label(std::move(jb->j), std::move(jb->patch));
      return;
    }
    st.inflight.fetch_sub(1, std::memory_order_relaxed);
    return;
  }
  KubeWriter::SlowJob sj;
  sj.answered = jb->answered;   // then only the label is left to retry
  sj.j = std::move(jb->j);
  sj.patch = std::move(jb->patch);
  sj.binding = std::move(jb->binding);
  sj.rp = std::move(jb->rp);
  sj.rb = std::move(jb->rb);
  sj.sp = jb->sp;
  sj.sb = jb->sb;
  kw_->to_slow(std::move(sj));
}

// the answer to connection c's oldest pending request
void BindIo::deliver(Conn& c, int status, std::string body, double retry_after) {
  const Pending p = c.pend[c.head++];
  if (c.head == c.pend.size()) {
    c.pend.clear();
    c.head = 0;
  }
  if (p.which == 2) {
    if (status == 429) lslots_[static_cast<size_t>(p.job)]->retry_after = retry_after;
    return label_done(p.job, status, std::move(body));
  }
  Job& jb = *slots_[static_cast<size_t>(p.job)];
  if (status == 429) {
    throttle(jb.seq);
    jb.retry_after = std::max(jb.retry_after, retry_after);
  }
  if (p.which == 1) g_hops.stamp(jb.j.id, kHopAnswer);
  (p.which ? jb.sb : jb.sp) = status;
  (p.which ? jb.rb : jb.rp) = std::move(body);
  if (--jb.left == 0) {
    complete(p.job);
  } else if (p.which == 1 && ok2xx(status)) {
    // bound, with the placement annotations: kube-scheduler's bind is answered now; the
    // label PATCH behind it is the reference's selector contract only (a failure there goes
    // to the slow path's label retry, never to a rollback)
    IoTimer it{kWrCommit};
    jb.answered = true;
    KubeWriterStats& st = kw_->stats;
    st.binding_ns.fetch_add(ns_now() - jb.j.t0_ns, std::memory_order_relaxed);
    kw_->ledger_->commit(jb.j.uid);
    st.ok.fetch_add(1, std::memory_order_relaxed);
    g_hops.stamp(jb.j.id, kHopPosted);
    reply_(jb.j.id, 200, "{\"Error\":\"\"}");
  }
}

// every answer still due on connection c fails with `why` (status 0: the slow path retries)
void BindIo::deliver_rest(Conn& c, const char* why) {
  while (c.npend() > 0) deliver(c, 0, why);
}

// a transport failure: one retry on a fresh connection when a reused keep-alive connection
// failed before any answer byte (the server closed it while idle), else status 0
void BindIo::fail(size_t k, const char* why) {
  Conn& c = *conns_[k];
  if (c.npend() > 0 && c.reused && !c.got_any && !c.retried) {
    c.retried = true;   // nothing was answered: the whole pipeline goes out again
    c.reused = false;
    c.off = 0;
    if (open_conn(k)) {
      kick_.push_back(k);
      return;
    }
  }
  close_conn(c);
  deliver_rest(c, why);
  idle_.push_back(k);
}

// drives connection k as far as it goes without blocking (`events`: the epoll events that
// woke it, 0 when kicked)
void BindIo::drive(size_t k, uint32_t events) {
  Conn& c = *conns_[k];
  char tmp[16384];
  if (c.st == kPublished) {   // a front-door thread owns it until its handoff is adopted
    if (events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) c.missed = true;   // read at adoption
    return;
  }
  for (;;) {
    if (c.fd < 0) return;
    if (c.st == kConnecting) {
      // a non-blocking connect is done when the socket turns writable (or errors)
      if (!(events & (EPOLLOUT | EPOLLERR | EPOLLHUP))) return;
      int err = 0;
      socklen_t len = sizeof err;
      if (getsockopt(c.fd, SOL_SOCKET, SO_ERROR, &err, &len) != 0 || err != 0)
        return fail(k, "cannot connect to the API server");
      c.st = c.ssl ? kHandshake : kSending;
      continue;
    }
    if (c.st == kHandshake) {
      const int r = SSL_connect(c.ssl);
      if (r == 1) {
        c.st = kSending;
        continue;
      }
      const int e = SSL_get_error(c.ssl, r);
      if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return;
      return fail(k, "TLS handshake with the API server failed");
    }
    if (c.st == kSending) {
      while (c.off < c.out.size()) {
        long w;
        if (c.ssl) {
          const int r = SSL_write(c.ssl, c.out.data() + c.off, static_cast<int>(c.out.size() - c.off));
          if (r <= 0) {
            const int e = SSL_get_error(c.ssl, r);
            if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) return;
            return fail(k, "connection to the API server failed");
          }
          w = r;
        } else {
          {
            IoTimer it{kWrSend};
            w = ::send(c.fd, c.out.data() + c.off, c.out.size() - c.off, MSG_NOSIGNAL);
          }
          if (w < 0 && errno == EINTR) continue;
          if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;
          if (w <= 0) return fail(k, "connection to the API server failed");
        }
        c.off += static_cast<size_t>(w);
      }
      if (g_hops.enabled())
        for (size_t i = c.head; i < c.pend.size(); ++i)
          if (c.pend[i].which == 1 && slots_[static_cast<size_t>(c.pend[i].job)])
            g_hops.stamp(slots_[static_cast<size_t>(c.pend[i].job)]->j.id, kHopSent);
      c.st = kReceiving;
      // the answer cannot be there yet: wait for its edge (edge-triggered epoll reports
      // the bytes that arrive from now on) instead of a recv() that would see EAGAIN
      if (!events) return;
      continue;
    }
    if (c.st == kReceiving || c.st == kIdle) {
      // a writable edge alone brings no bytes (every arrival is an EPOLLIN edge of its own)
      if (events && !(events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR))) return;
      bool eof = false;
      for (;;) {
        long r;
        if (c.ssl) {
          r = SSL_read(c.ssl, tmp, sizeof tmp);
          if (r <= 0) {
            const int e = SSL_get_error(c.ssl, static_cast<int>(r));
            if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
            eof = true;
            break;
          }
        } else {
          {
            IoTimer it{kWrRecv};
            r = ::recv(c.fd, tmp, sizeof tmp, 0);
          }
          if (r < 0 && errno == EINTR) continue;
          if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
          if (r <= 0) {
            eof = true;
            break;
          }
        }
        c.in.append(tmp, static_cast<size_t>(r));
        c.got_any = true;
        // plain TCP: a short read drained the socket, and edge-triggered epoll reports the
        // next bytes as a new edge; TLS hands out a record at a time, so it reads on
        if (!c.ssl && static_cast<size_t>(r) < sizeof tmp) break;
      }
      if (c.st == kIdle) {   // an idle keep-alive connection the server closed (or junk)
        if (eof || !c.in.empty()) close_conn(c);
        return;
      }
      // every complete answer in order; a pipeline cut short leaves its later answers to
      // the slow path (the label PATCH there is idempotent)
      bool delivered = false;
      while (c.npend() > 0) {
        int status = 0;
        std::string body;
        size_t used = 0;
        bool close = false;
        double retry_after = -1;
        const int rc = parse_response(c.in, eof && c.npend() == 1, &status, &body, &used, &close, &retry_after);
        if (rc < 0) return fail(k, "bad answer from the API server");
        if (rc == 0) {
          if (!eof) return go_lazy(k);   // more bytes to come
          if (c.got_any && c.in.empty() && (delivered || c.head > 0)) break;   // answered some, then closed
          return fail(k, "connection to the API server failed");
        }
        c.in.erase(0, used);
        delivered = true;
        deliver(c, status, std::move(body), retry_after);
        if (close) {
          eof = true;
          break;
        }
      }
      if (c.npend() > 0 || eof) {
        close_conn(c);
        deliver_rest(c, "connection to the API server closed before every answer");
      }
      c.st = kIdle;
      c.lazy_since = 0;   // every answer is in: its lazy_ entry (if any) is stale
      if (!publish(k)) idle_.push_back(k);
      return;
    }
    return;
  }
}

// More bytes are due on connection k. When they are only label answers of binds already
// answered (--lazy-label-answers), the connection's receive low-water mark goes up, so their
// arrival wakes nobody, and a later pass of the loop reads them (drain_lazy).
void BindIo::go_lazy(size_t k) {
  Conn& c = *conns_[k];
  if (!kw_->lazy_labels_.load(std::memory_order_relaxed) || c.ssl || c.fd < 0 || c.npend() <= 0) return;
  for (size_t i = c.head; i < c.pend.size(); ++i) {
    const Pending& p = c.pend[i];
    if (p.which != 0 || !slots_[static_cast<size_t>(p.job)] || !slots_[static_cast<size_t>(p.job)]->answered) return;
  }
  if (!c.lowat) {
    const int big = 1 << 30;
    if (setsockopt(c.fd, SOL_SOCKET, SO_RCVLOWAT, &big, sizeof big) != 0) return;
    c.lowat = true;
  }
  if (!c.lazy_since) {
    c.lazy_since = ns_now();
    lazy_.push_back(k);
  }
}

// lazy connections whose label answers are due by now are read (one recv each; an answer still
// on its way leaves the connection lazy for the next pass)
void BindIo::drain_lazy(uint64_t now) {
  size_t keep = 0;
  for (size_t i = 0; i < lazy_.size(); ++i) {
    const size_t k = lazy_[i];
    Conn& c = *conns_[k];
    if (!c.lazy_since || c.fd < 0 || c.st != kReceiving) {
      c.lazy_since = 0;
      continue;   // answered, closed or failed meanwhile
    }
    if (now - c.lazy_since < kLazyNs) {
      lazy_[keep++] = k;
      continue;
    }
    c.lazy_since = 0;
    drive(k, EPOLLIN);   // delivers what came; go_lazy() re-queues it if nothing did
    if (c.lazy_since) {   // re-queued at the end of lazy_ (past i): one entry only
      lazy_.pop_back();
      c.lazy_since = now;
      lazy_[keep++] = k;
    }
  }
  lazy_.resize(keep);
}

void BindIo::reset_lowat(Conn& c) {
  if (c.fd < 0 || !c.lowat) return;
  const int one = 1;
  setsockopt(c.fd, SOL_SOCKET, SO_RCVLOWAT, &one, sizeof one);
  c.lowat = false;
}

bool BindIo::publish(size_t k) {
  Conn& c = *conns_[k];
  if (kw_->inline_io_ || tag_bit_ != 0 || c.ssl || c.fd < 0 || !kw_->fe_send_.load(std::memory_order_relaxed) ||
      kw_->batch_labels_.load(std::memory_order_relaxed))
    return false;
  // it stays in this loop's epoll set: an edge that comes while a front-door thread holds it is
  // only noted (drive), and read once the handoff is adopted
  reset_lowat(c);   // after lazy label answers: the next binding's answer must wake the loop
  std::lock_guard<std::mutex> g(kw_->fe_mu_);
  if (kw_->fe_closed_) return false;
  c.st = kPublished;
  c.missed = false;
  kw_->fe_idle_.emplace_back(k, c.fd);
  return true;
}

void BindIo::adopt_handoffs() {
  std::vector<KubeWriter::Handoff> hs;
  {
    std::lock_guard<std::mutex> g(kw_->fe_mu_);
    if (kw_->adopt_.empty()) return;
    hs.swap(kw_->adopt_);
  }
  for (KubeWriter::Handoff& h : hs) {
    int64_t s;
    if (!free_slots_.empty()) {
      s = free_slots_.back();
      free_slots_.pop_back();
    } else {
      s = static_cast<int64_t>(slots_.size());   // sent already: always taken on
      slots_.emplace_back();
    }
    auto jb = std::make_unique<Job>();
    jb->j = std::move(h.j);
    jb->patch = std::move(h.patch);
    jb->binding = std::move(h.binding);
    if (!kw_->label_) {
      jb->left = 1;
      jb->sp = 200;
    }
    jb->reqs = kw_->label_ ? 2 : 1;   // the front door pipelined both
    req_inflight_ += jb->reqs;
    jb->seq = ++launch_seq_;
    slots_[static_cast<size_t>(s)] = std::move(jb);
    ++inflight_;
    Conn& c = *conns_[h.k];
    c.out = std::move(h.out);
    c.off = h.sent;
    c.pend.clear();
    c.head = 0;
    c.pend.push_back(Pending{s, 1});
    if (kw_->label_) c.pend.push_back(Pending{s, 0});
    c.in.clear();
    c.got_any = false;
    c.retried = false;
    c.reused = true;
    c.deadline_ns = ns_now() + timeout_ns_;
    c.st = c.off < c.out.size() ? kSending : kReceiving;
    if (h.broken) {   // a stale keep-alive connection: the whole pipeline again on a fresh one
      c.missed = false;
      fail(h.k, "connection to the API server failed");
      continue;
    }
    // the rest of a short send, or bytes whose edge came before the adoption (ignored then)
    if (c.st == kSending || c.missed) kick_.push_back(h.k);
    c.missed = false;
  }
}

// starts slot s's requests on an idle (or new) connection: the binding, then (label mode)
// the label PATCH pipelined behind it
void BindIo::launch(int64_t s) {
  Job& jb = *slots_[static_cast<size_t>(s)];
  size_t k;
  if (idle_.empty()) {   // one the front door is not using: back into this loop's epoll set
    std::pair<size_t, int> pub{0, -1};
    {
      std::lock_guard<std::mutex> g(kw_->fe_mu_);
      if (!kw_->fe_idle_.empty()) {
        pub = kw_->fe_idle_.back();
        kw_->fe_idle_.pop_back();
      }
    }
    if (pub.second >= 0) {
      Conn& pc = *conns_[pub.first];
      pc.st = kIdle;
      if (pc.missed) {   // the server closed it (or sent junk) while it was out: see to it now
        pc.missed = false;
        drive(pub.first, EPOLLIN);
      }
      if (pc.fd >= 0 && pc.st == kIdle) idle_.push_back(pub.first);
    }
  }
  if (!idle_.empty()) {
    k = idle_.back();
    idle_.pop_back();
  } else {
    k = conns_.size();
    conns_.push_back(std::make_unique<Conn>());
  }
  Conn& c = *conns_[k];
  request(&c.out, "POST", jb.j, true, kJsonE, jb.binding);
  c.pend.clear();
  c.head = 0;
  c.pend.push_back(Pending{s, 1});
  if (kw_->label_ && !jb.batch_label) {
    thread_local std::string second;
    request(&second, "PATCH", jb.j, false, kMergePatchE, jb.patch);
    c.out += second;
    c.pend.push_back(Pending{s, 0});
  }
  c.off = 0;
  c.in.clear();
  c.got_any = false;
  c.retried = false;
  c.deadline_ns = ns_now() + timeout_ns_;
  c.reused = c.fd >= 0;
  reset_lowat(c);   // idle again after lazy answers: answers wake the loop again
  if (c.fd >= 0) {
    c.st = kSending;
  } else if (!open_conn(k)) {
    close_conn(c);
    deliver_rest(c, "cannot connect to the API server");
    idle_.push_back(k);
    return;
  }
  kick_.push_back(k);
}

void BindIo::start_waiting() {
  if (!waiting_.empty() && ns_now() - auth_at_ > 1'000'000'000ull) {   // a rotated token reaches new requests
    auth_ = kw_->auth();
    auth_at_ = ns_now();
  }
  const bool label = kw_->label_, batch = label && kw_->batch_labels_.load(std::memory_order_relaxed);
  const double cap = window_ * (label ? 2 : 1);   // requests the admission window allows
  while (!waiting_.empty() && !free_slots_.empty()) {
    // labels kept waiting for room too long get it before more binds (bindings first, not only)
    if (!label_wait_.empty() && ns_now() - label_oldest_ns_ > kLabelStarveNs) break;
    const double used = static_cast<double>(req_inflight_) + static_cast<double>(labels_out_);
    int need = label && !batch ? 2 : 1;
    bool alone = batch;
    if (need == 2 && used + 2.0 * static_cast<double>(waiting_.size()) > cap) {
      // more binds waiting than the window has room for with their labels: the binding goes
      // alone and its label later, in a batch, when the window has room (kube-scheduler waits
      // on bindings, not on labels: under a saturated API server its binds keep the window's
      // whole rate). With room to spare, as nearly always, both go together as before.
      need = 1;
      alone = true;
    }
    if (used + need > cap) break;
    if (alone && !batch) kw_->stats.bindings_first.fetch_add(1, std::memory_order_relaxed);
    const int64_t s = free_slots_.back();
    free_slots_.pop_back();
    auto jb = std::make_unique<Job>();
    jb->j = std::move(waiting_.front());
    waiting_.pop_front();
    g_hops.stamp(jb->j.id, kHopLaunched);
    {
      IoTimer it{kWrBuild};
      kw_->build(jb->j, &jb->patch, &jb->binding);
    }
    if (!label) {   // the binding alone carries the annotations
      jb->left = 1;
      jb->sp = 200;
    } else if (alone) {   // the binding alone now, its label later
      jb->left = 1;
      jb->batch_label = true;
    }
    jb->reqs = need;
    req_inflight_ += need;
    jb->seq = ++launch_seq_;
    slots_[static_cast<size_t>(s)] = std::move(jb);
    ++inflight_;
    launch(s);
  }
}

void BindIo::submit(BindJob j) {
  g_hops.stamp(j.id, kHopPickup);
  kw_->stats.inflight.fetch_add(1, std::memory_order_relaxed);
  waiting_.push_back(std::move(j));
  start_waiting();
}

void BindIo::on_event(uint64_t k, uint32_t events) {
  if (k < conns_.size()) drive(k, events);
}

// a request unanswered past its deadline (a half-open connection: no answer, no reset) fails
// to the slow path with status 0, never re-sent on this connection; one scan per 100 ms
void BindIo::scan_deadlines(uint64_t now) {
  if (inflight_ + labels_out_ == 0 || now - scanned_at_ < 100'000'000ull) return;
  scanned_at_ = now;
  for (size_t k = 0; k < conns_.size(); ++k) {
    Conn& c = *conns_[k];
    if (c.npend() > 0 && c.fd >= 0 && now > c.deadline_ns) {
      timeouts_ += static_cast<uint64_t>(c.npend());
      kw_->stats.timeouts.fetch_add(static_cast<uint64_t>(c.npend()), std::memory_order_relaxed);
      c.retried = true;
      fail(k, "the API server did not answer in time");
    }
  }
}

void BindIo::queue_label(BindJob&& j, std::string&& patch) {
  int64_t ls;
  if (!lfree_.empty()) {
    ls = lfree_.back();
    lfree_.pop_back();
  } else {
    ls = static_cast<int64_t>(lslots_.size());
    lslots_.emplace_back();
  }
  auto l = std::make_unique<Label>();
  l->j = std::move(j);
  l->patch = std::move(patch);
  lslots_[static_cast<size_t>(ls)] = std::move(l);
  if (label_wait_.empty()) label_oldest_ns_ = ns_now();
  label_wait_.push_back(ls);
}

void BindIo::label_done(int64_t ls, int status, std::string body) {
  std::unique_ptr<Label> l = std::move(lslots_[static_cast<size_t>(ls)]);
  lfree_.push_back(ls);
  --labels_out_;
  if (ok2xx(status)) {
    widen();
    kw_->stats.inflight.fetch_sub(1, std::memory_order_relaxed);
    return;
  }
  if (status == 429 && l->j.throttled < kMaxThrottled) {
    throttle(l->seq);
    ++l->j.throttled;
    defer(std::move(l->j), std::move(l->patch), true, l->retry_after);
    return;
  }
  // refused by its nodeName guard cannot happen here (its binding answered 2xx): a 5xx, a
  // lost answer, a timeout: the slow path retries it
  KubeWriter::SlowJob sj;
  sj.answered = true;
  sj.j = std::move(l->j);
  sj.patch = std::move(l->patch);
  sj.sp = status;
  sj.rp = std::move(body);
  kw_->to_slow(std::move(sj));
}

// up to kLabelBatch (and `room`) waiting label PATCHes, pipelined on one idle (or new) connection
void BindIo::launch_labels(size_t room) {
  size_t k;
  if (!idle_.empty()) {
    k = idle_.back();
    idle_.pop_back();
  } else {
    k = conns_.size();
    conns_.push_back(std::make_unique<Conn>());
  }
  Conn& c = *conns_[k];
  c.out.clear();
  c.pend.clear();
  c.head = 0;
  thread_local std::string one;
  while (!label_wait_.empty() && c.pend.size() < std::min(kLabelBatch, room)) {
    const int64_t ls = label_wait_.front();
    label_wait_.pop_front();
    Label& l = *lslots_[static_cast<size_t>(ls)];
    l.seq = ++launch_seq_;
    request(&one, "PATCH", l.j, false, kMergePatchE, l.patch);
    c.out += one;
    c.pend.push_back(Pending{ls, 2});
    ++labels_out_;
  }
  label_oldest_ns_ = label_wait_.empty() ? 0 : ns_now();
  c.off = 0;
  c.in.clear();
  c.got_any = false;
  c.retried = false;
  c.deadline_ns = ns_now() + timeout_ns_;
  c.reused = c.fd >= 0;
  reset_lowat(c);   // idle again after lazy answers: answers wake the loop again
  if (c.fd >= 0) {
    c.st = kSending;
  } else if (!open_conn(k)) {
    close_conn(c);
    deliver_rest(c, "cannot connect to the API server");
    idle_.push_back(k);
    return;
  }
  kick_.push_back(k);
}

void BindIo::pump() {
  if (!deferred_.empty()) resend_due(ns_now());   // throttled binds / labels whose Retry-After passed
  // lazy label answers due by now first: their connections are free for the binds below
  if (!lazy_.empty()) drain_lazy(ns_now());
  for (int round = 0; round < 4 && (!kick_.empty() || !waiting_.empty()); ++round) {
    start_waiting();
    for (size_t i = 0; i < kick_.size(); ++i) drive(kick_[i], 0);   // fail() may append
    kick_.clear();
  }
  if (!label_wait_.empty()) {
    // labels fill the room the binds leave in the admission window
    const uint64_t now = ns_now();
    const double cap = window_ * (kw_->label_ ? 2 : 1);
    for (;;) {
      const double room = cap - static_cast<double>(req_inflight_) - static_cast<double>(labels_out_);
      if (label_wait_.empty() || room < 1 ||
          !(label_wait_.size() >= kLabelBatch || now - label_oldest_ns_ >= kLabelHoldNs))
        break;
      launch_labels(static_cast<size_t>(room));
    }
    for (size_t i = 0; i < kick_.size(); ++i) drive(kick_[i], 0);
    kick_.clear();
    // room the labels did not take goes to binds waiting behind them (kLabelStarveNs)
    if (!waiting_.empty()) {
      start_waiting();
      for (size_t i = 0; i < kick_.size(); ++i) drive(kick_[i], 0);
      kick_.clear();
    }
  }
  scan_deadlines(ns_now());
  for (size_t i = 0; i < kick_.size(); ++i) drive(kick_[i], 0);
  kick_.clear();
}

void BindIo::abandon(const char* why) {
  // answers still due: failed with `why` (binds and labels go to the slow path that way)
  for (auto& c : conns_) {
    close_conn(*c);
    deliver_rest(*c, why);
  }
  while (!label_wait_.empty()) {   // labels never sent: the slow path writes them
    const int64_t ls = label_wait_.front();
    label_wait_.pop_front();
    ++labels_out_;
    label_done(ls, 0, why);
  }
  for (size_t s = 0; s < slots_.size(); ++s) {
    if (!slots_[s]) continue;
    Job& jb = *slots_[s];
    if (jb.left > 0) {
      if (jb.sb == 0) jb.rb = why;
      if (jb.sp == 0) jb.rp = why;
    }
    KubeWriter::SlowJob sj;
    sj.j = std::move(jb.j);
    sj.patch = std::move(jb.patch);
    sj.binding = std::move(jb.binding);
    sj.rp = std::move(jb.rp);
    sj.rb = std::move(jb.rb);
    sj.sp = jb.sp;
    sj.sb = jb.sb;
    sj.answered = jb.answered;
    slots_[s].reset();
    kw_->to_slow(std::move(sj));
  }
  inflight_ = 0;
  while (!deferred_.empty()) {   // throttled, not re-sent yet: the slow path's retries finish them
    Deferred d = std::move(deferred_.front());
    deferred_.pop_front();
    KubeWriter::SlowJob sj;
    sj.answered = d.label_only;
    if (d.label_only) {
      sj.sp = 429;
      sj.patch = std::move(d.patch);
    } else {
      kw_->build(d.j, &sj.patch, &sj.binding);
      sj.sb = 429;
      sj.rb = why;
    }
    sj.j = std::move(d.j);
    kw_->to_slow(std::move(sj));
  }
  for (BindJob& j : waiting_) {
    kw_->refuse(j);
    kw_->stats.inflight.fetch_sub(1, std::memory_order_relaxed);
  }
  waiting_.clear();
}

// ------------------------------------------------------------------------------ admission
void BindIo::throttle(uint64_t seq) {
  KubeWriterStats& st = kw_->stats;
  st.throttled.fetch_add(1, std::memory_order_relaxed);
  if (seq <= cut_seq_) return;   // sent before the last cut: that cut answered it already
  window_ = std::max(1.0, window_ / 2);
  cut_seq_ = launch_seq_;
  clean_ = 0;
  st.window_cuts.fetch_add(1, std::memory_order_relaxed);
  st.window.store(static_cast<int64_t>(window_), std::memory_order_relaxed);
}

void BindIo::widen() {
  if (window_ >= max_window_) return;
  clean_ += 1;
  if (clean_ < window_) return;   // one bind wider per window of clean binds
  clean_ = 0;
  window_ = std::min(max_window_, window_ + 1);
  kw_->stats.window.store(static_cast<int64_t>(window_), std::memory_order_relaxed);
}

void BindIo::defer(BindJob&& j, std::string&& patch, bool label_only, double retry_after) {
  // the server's Retry-After (kube-apiserver: 1 s), else 5 ms x 2^k as the slow path's retries;
  // at most kMaxRetryAfterS each, so kMaxThrottled waits stay inside kube-scheduler's 30 s
  // extender timeout and the ledger's 60 s reservation TTL (the bind holds its reservation)
  const double wait_s = std::min(kMaxRetryAfterS, retry_after > 0 ? retry_after
                                                                  : 0.005 * static_cast<double>(1u << std::min(j.throttled, 12)));
  const uint64_t due = ns_now() + static_cast<uint64_t>(wait_s * 1e9);
  Deferred d{due, std::move(j), std::move(patch), label_only};
  auto at = deferred_.end();
  while (at != deferred_.begin() && std::prev(at)->due_ns > due) --at;   // due order (nearly always the end)
  deferred_.insert(at, std::move(d));
}

void BindIo::resend_due(uint64_t now) {
  while (!deferred_.empty() && deferred_.front().due_ns <= now) {
    Deferred d = std::move(deferred_.front());
    deferred_.pop_front();
    kw_->stats.throttle_resends.fetch_add(1, std::memory_order_relaxed);
    if (d.label_only) {
      queue_label(std::move(d.j), std::move(d.patch));   // batched with any other waiting label
    } else {
      waiting_.push_front(std::move(d.j));   // first in line for the window (start_waiting rebuilds it)
    }
  }
}

// ------------------------------------------------------------------------------ io thread
void KubeWriter::io_loop() {
  const int ep = epoll_create1(EPOLL_CLOEXEC);
  if (ep < 0) throw std::runtime_error("KubeWriter: epoll_create1 failed");
  {
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = UINT64_MAX;
    epoll_ctl(ep, EPOLL_CTL_ADD, efd_, &ev);
  }
  BindIo io(this, ep, 0, max_inflight_, respond_);
  {
    std::lock_guard<std::mutex> g(fe_mu_);
    io_ep_ = ep;
    fe_closed_ = false;
  }
  epoll_event evs[256];
  uint64_t stop_at = 0;
  for (;;) {
    bool stopping;
    {
      std::lock_guard<std::mutex> g(mu_);
      stopping = stop_;
      if (!stopping) {
        while (!q_.empty()) {
          stats.inflight.fetch_sub(1, std::memory_order_relaxed);   // submit() counted it; so does BindIo
          io.submit(std::move(q_.front()));
          q_.pop_front();
        }
        q_len_.store(0, std::memory_order_relaxed);
      }
    }
    if (stopping && !stop_at) {
      stop_at = ns_now() + 5'000'000'000ull;
      std::lock_guard<std::mutex> g(fe_mu_);   // no more front-door sends from here on
      fe_closed_ = true;
    }
    if (stopping) {
      io.adopt_handoffs();
      std::deque<BindJob> left;
      {
        std::lock_guard<std::mutex> g(mu_);
        left.swap(q_);
      }
      for (BindJob& j : left) {
        refuse(j);
        stats.inflight.fetch_sub(1, std::memory_order_relaxed);
      }
      if (io.inflight() == 0 || ns_now() > stop_at) break;
    }
    io.pump();
    // park: a bind submitted from here on writes efd_; one submitted before is picked up now
    io_parked_.store(true, std::memory_order_seq_cst);
    const bool queued = !stopping && q_len_.load(std::memory_order_seq_cst) > 0;
    // with answers due, wake for the deadline scan
    const uint64_t io0 = io_t0();
    const int n = epoll_wait(ep, evs, 256,
                             queued ? 0 : stopping || io.labels_waiting() ? 1 : io.inflight() ? 100 : 1000);
    io_end(kWrWait, io0);
    io_parked_.store(false, std::memory_order_relaxed);
    io.adopt_handoffs();   // before their connections' events: those are only read once adopted
    for (int e = 0; e < n; ++e) {
      if (evs[e].data.u64 == UINT64_MAX) {
        uint64_t v;
        IoTimer it{kWrEfdRead};
        (void)!::read(efd_, &v, sizeof v);
        continue;
      }
      io.on_event(evs[e].data.u64, evs[e].events);
    }
    io.pump();
  }
  // a front-door thread between taking a connection and handing it over finishes first (its
  // send uses the connection's fd and this loop's epoll set, both closed below)
  for (int i = 0; i < 100000; ++i) {
    {
      std::lock_guard<std::mutex> g(fe_mu_);
      fe_closed_ = true;
      if (fe_busy_ == 0) {
        io_ep_ = -1;
        fe_idle_.clear();
        break;
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
  io.adopt_handoffs();
  // what is still in flight after the grace period: the slow path answers it
  io.abandon("extender shutting down");
  io_done_.store(true);
  {
    std::lock_guard<std::mutex> g(mu_);   // the slow threads re-check under mu_
  }
  cv_.notify_all();
  ::close(ep);
}

std::unique_ptr<BindIo> KubeWriter::make_io(int ep, uint64_t tag_bit, Respond reply) {
  return std::make_unique<BindIo>(this, ep, tag_bit, max_inflight_, std::move(reply));
}

bool KubeWriter::send_from_caller(BindJob& j) {
  if (!fe_send_.load(std::memory_order_relaxed) || !evented_ || inline_io_ || ctx_ ||
      batch_labels_.load(std::memory_order_relaxed))
    return false;
  std::pair<size_t, int> conn;
  {
    std::lock_guard<std::mutex> g(fe_mu_);
    if (fe_closed_ || fe_idle_.empty() || io_ep_ < 0) return false;
    conn = fe_idle_.back();
    fe_idle_.pop_back();
    ++fe_busy_;   // the io thread does not close this fd until the handoff
  }
  Handoff h;
  h.k = conn.first;
  g_hops.stamp(j.id, kHopPickup);
  g_hops.stamp(j.id, kHopLaunched);   // sent by the caller: no window wait
  build(j, &h.patch, &h.binding);
  const std::string a = auth();
  compose_request(&h.out, "POST", j, true, kJsonE, h.binding, host_hdr_, a);
  if (label_) {
    thread_local std::string second;
    compose_request(&second, "PATCH", j, false, kMergePatchE, h.patch, host_hdr_, a);
    h.out += second;
  }
  ssize_t n;
  do {
    IoTimer it{kWrSend};
    n = ::send(conn.second, h.out.data(), h.out.size(), MSG_NOSIGNAL | MSG_DONTWAIT);
  } while (n < 0 && errno == EINTR);
  h.sent = n > 0 ? static_cast<size_t>(n) : 0;
  if (h.sent == h.out.size()) g_hops.stamp(j.id, kHopSent);
  h.broken = n < 0 && errno != EAGAIN && errno != EWOULDBLOCK;
  h.j = std::move(j);
  stats.inflight.fetch_add(1, std::memory_order_relaxed);
  // the connection never left the io thread's epoll set: the answer's edge may come before the
  // handoff is adopted (the io thread then notes it and reads the connection at the adoption)
  std::lock_guard<std::mutex> g(fe_mu_);
  adopt_.push_back(std::move(h));
  --fe_busy_;
  return true;
}

void KubeWriter::to_slow(SlowJob&& sj) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!slow_gone_) {
      slow_q_.push_back(std::move(sj));
      cv_.notify_one();
      return;
    }
  }
  // the slow threads have exited (the writer stopped before its inline owners): finish here
  HttpConn c(&t_, ctx_, 5), c2(&t_, ctx_, 5);
  if (sj.answered) finish_label(&c, sj.j, sj.patch, sj.sp, &sj.rp);
  else finish(&c, &c2, sj.j, sj.patch, sj.binding, sj.sp, &sj.rp, sj.sb, &sj.rb);
  stats.inflight.fetch_sub(1, std::memory_order_relaxed);
}

void KubeWriter::run_slow() {
  const int tmo = std::max(1, static_cast<int>(timeout_s_ + 0.5));
  HttpConn c(&t_, ctx_, tmo), c2(&t_, ctx_, tmo);
  for (;;) {
    SlowJob sj;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [this] { return !slow_q_.empty() || (stop_ && io_done_.load()); });
      if (slow_q_.empty()) return;
      sj = std::move(slow_q_.front());
      slow_q_.pop_front();
    }
    if (sj.answered) {   // bound and answered: only the label PATCH is left to retry
      finish_label(&c, sj.j, sj.patch, sj.sp, &sj.rp);
    } else {
      finish(&c, &c2, sj.j, sj.patch, sj.binding, sj.sp, &sj.rp, sj.sb, &sj.rb);
    }
    stats.inflight.fetch_sub(1, std::memory_order_relaxed);
  }
}

}  // namespace nanogpu
