// Evented bind writer (see kubewriter.h): one epoll thread drives the two API requests of every
// bind in flight on non-blocking keep-alive connections, plain HTTP or TLS.
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
int parse_response(const std::string& b, bool eof, int* status, std::string* body, size_t* consumed, bool* close) {
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

enum ConnState { kIdle, kConnecting, kHandshake, kSending, kReceiving };

// A bind's two requests go out pipelined on ONE connection, the binding first: one send and,
// usually, one read for both answers (HTTP/1.1 answers come back in request order; kube-
// apiserver's Go server and the bench's API server both serve pipelined requests in order).
struct Pending {
  int64_t job;   // in-flight job slot
  int which;     // 0: label PATCH, 1: binding
};

struct AConn {
  int fd = -1;
  SSL* ssl = nullptr;
  int st = kIdle;
  bool reused = false;   // the requests went out on a connection used before
  bool got_any = false;  // response bytes seen since the requests went out
  bool retried = false;  // the one fresh-connection retry is spent
  std::string out, in;
  size_t off = 0;
  Pending pend[2];       // answers still due, in request order
  int npend = 0;
  uint64_t deadline_ns = 0;   // the answers are due by then (KubeWriter timeout_s)
};

struct AJob {
  BindJob j;
  std::string patch, binding, rp, rb;
  int sp = 0, sb = 0;
  int left = 2;
  bool answered = false;   // kube-scheduler has its answer (the binding landed; the label may follow)
};

}  // namespace

void KubeWriter::io_loop() {
  const int ep = epoll_create1(EPOLL_CLOEXEC);
  if (ep < 0) throw std::runtime_error("KubeWriter: epoll_create1 failed");
  {
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = UINT64_MAX;
    epoll_ctl(ep, EPOLL_CTL_ADD, efd_, &ev);
  }
  std::vector<std::unique_ptr<AConn>> conns;   // index = epoll tag
  std::vector<size_t> idle;
  std::vector<std::unique_ptr<AJob>> slots(static_cast<size_t>(max_inflight_));
  std::vector<int64_t> free_slots;
  for (int64_t i = max_inflight_ - 1; i >= 0; --i) free_slots.push_back(i);
  std::deque<BindJob> waiting;
  sockaddr_storage addr{};
  socklen_t addr_len = 0;
  int family = AF_INET;
  std::string a = auth();
  uint64_t auth_at = ns_now();
  const std::string host_hdr = host_header(t_);

  auto resolve = [&]() -> bool {
    if (addr_len) return true;
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    if (getaddrinfo(t_.host.c_str(), std::to_string(t_.port).c_str(), &hints, &res) != 0 || !res) return false;
    std::memcpy(&addr, res->ai_addr, res->ai_addrlen);
    addr_len = res->ai_addrlen;
    family = res->ai_family;
    freeaddrinfo(res);
    return true;
  };
  auto close_conn = [&](AConn& c) {
    if (c.ssl) SSL_free(c.ssl);
    c.ssl = nullptr;
    if (c.fd >= 0) {
      epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
      ::close(c.fd);
    }
    c.fd = -1;
    c.in.clear();
    c.st = kIdle;
  };
  // a fresh non-blocking connection (connect in progress); false: cannot even start
  auto open_conn = [&](size_t k) -> bool {
    AConn& c = *conns[k];
    close_conn(c);
    if (!resolve()) return false;
    const int fd = socket(family, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    if (fd < 0) return false;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    tcp_liveness(fd, timeout_s_);
    const int cr = ::connect(fd, reinterpret_cast<sockaddr*>(&addr), addr_len);
    if (cr != 0 && errno != EINPROGRESS) {
      ::close(fd);
      return false;
    }
    c.fd = fd;
    c.st = cr == 0 ? (ctx_ ? kHandshake : kSending) : kConnecting;
    if (ctx_) {
      c.ssl = SSL_new(static_cast<SSL_CTX*>(ctx_));
      if (!c.ssl) {
        close_conn(c);
        return false;
      }
      SSL_set_fd(c.ssl, fd);
      in6_addr a6{};
      const bool ip = inet_pton(AF_INET, t_.host.c_str(), &a6) == 1 || inet_pton(AF_INET6, t_.host.c_str(), &a6) == 1;
      if (!ip) SSL_set_tlsext_host_name(c.ssl, t_.host.c_str());
      if (!t_.insecure) {
        if (ip) X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(c.ssl), t_.host.c_str());
        else SSL_set1_host(c.ssl, t_.host.c_str());
      }
    }
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP | EPOLLET;
    ev.data.u64 = k;
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
    return true;
  };
  // a request written into the connection's own buffer (its capacity is kept across binds)
  auto request = [&](std::string* r, const char* method, const BindJob& j, bool binding, std::string_view ctype,
                     const std::string& body) {
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
    if (!a.empty()) {
      *r += "Authorization: Bearer ";
      *r += a;
      *r += "\r\n";
    }
    *r += "Content-Type: ";
    *r += ctype;
    char len[24];
    *r += "\r\nContent-Length: ";
    r->append(len, static_cast<size_t>(std::to_chars(len, len + sizeof len, body.size()).ptr - len));
    *r += "\r\n\r\n";
    *r += body;
  };

  size_t inflight = 0;
  const uint64_t timeout_ns = static_cast<uint64_t>(timeout_s_ * 1e9);
  uint64_t scanned_at = ns_now();
  auto ok2xx = [](int st) { return st >= 200 && st < 300; };
  // both answers of a slot are in: commit on the happy path, else the slow path finishes it
  auto complete = [&](int64_t s) {
    std::unique_ptr<AJob> jb = std::move(slots[static_cast<size_t>(s)]);
    free_slots.push_back(s);
    --inflight;
    if (jb->answered && ok2xx(jb->sp)) {   // bound and answered earlier; the label landed too
      stats.inflight.fetch_sub(1, std::memory_order_relaxed);
      return;
    }
    const bool ok2 = ok2xx(jb->sb) && ok2xx(jb->sp);
    if (!jb->answered) stats.binding_ns.fetch_add(ns_now() - jb->j.t0_ns, std::memory_order_relaxed);
    if (ok2) {
      ledger_->commit(jb->j.uid);
      stats.ok.fetch_add(1, std::memory_order_relaxed);
      stats.inflight.fetch_sub(1, std::memory_order_relaxed);
      respond_(jb->j.id, 200, "{\"Error\":\"\"}");
      return;
    }
    SlowJob sj;
    sj.answered = jb->answered;   // then only the label is left to retry
    sj.j = std::move(jb->j);
    sj.patch = std::move(jb->patch);
    sj.binding = std::move(jb->binding);
    sj.rp = std::move(jb->rp);
    sj.rb = std::move(jb->rb);
    sj.sp = jb->sp;
    sj.sb = jb->sb;
    {
      std::lock_guard<std::mutex> g(mu_);
      slow_q_.push_back(std::move(sj));
    }
    cv_.notify_one();
  };
  // the answer to connection c's oldest pending request
  auto deliver = [&](AConn& c, int status, std::string body) {
    const Pending p = c.pend[0];
    c.pend[0] = c.pend[1];
    --c.npend;
    AJob& jb = *slots[static_cast<size_t>(p.job)];
    (p.which ? jb.sb : jb.sp) = status;
    (p.which ? jb.rb : jb.rp) = std::move(body);
    if (--jb.left == 0) {
      complete(p.job);
    } else if (p.which == 1 && ok2xx(status)) {
      // bound, with the placement annotations: kube-scheduler's bind is answered now; the
      // label PATCH behind it is the reference's selector contract only (a failure there goes
      // to the slow path's label retry, never to a rollback)
      jb.answered = true;
      stats.binding_ns.fetch_add(ns_now() - jb.j.t0_ns, std::memory_order_relaxed);
      ledger_->commit(jb.j.uid);
      stats.ok.fetch_add(1, std::memory_order_relaxed);
      respond_(jb.j.id, 200, "{\"Error\":\"\"}");
    }
  };
  // every answer still due on connection c fails with `why` (status 0: the slow path retries)
  auto deliver_rest = [&](AConn& c, const char* why) {
    while (c.npend > 0) deliver(c, 0, why);
  };
  std::vector<size_t> kick;   // connections to drive after this batch of events
  // a transport failure: one retry on a fresh connection when a reused keep-alive connection
  // failed before any answer byte (the server closed it while idle), else status 0
  auto fail = [&](size_t k, const char* why) {
    AConn& c = *conns[k];
    if (c.npend > 0 && c.reused && !c.got_any && !c.retried) {
      c.retried = true;   // nothing was answered: the whole pipeline goes out again
      c.reused = false;
      c.off = 0;
      if (open_conn(k)) {
        kick.push_back(k);
        return;
      }
    }
    close_conn(c);
    deliver_rest(c, why);
    idle.push_back(k);
  };

  // drives connection k as far as it goes without blocking (`events`: the epoll events that
  // woke it, 0 when kicked)
  auto drive = [&](size_t k, uint32_t events) {
    AConn& c = *conns[k];
    char tmp[16384];
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
            w = ::send(c.fd, c.out.data() + c.off, c.out.size() - c.off, MSG_NOSIGNAL);
            if (w < 0 && errno == EINTR) continue;
            if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return;
            if (w <= 0) return fail(k, "connection to the API server failed");
          }
          c.off += static_cast<size_t>(w);
        }
        c.st = kReceiving;
        continue;
      }
      if (c.st == kReceiving || c.st == kIdle) {
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
            r = ::recv(c.fd, tmp, sizeof tmp, 0);
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
        while (c.npend > 0) {
          int status = 0;
          std::string body;
          size_t used = 0;
          bool close = false;
          const int rc = parse_response(c.in, eof && c.npend == 1, &status, &body, &used, &close);
          if (rc < 0) return fail(k, "bad answer from the API server");
          if (rc == 0) {
            if (!eof) return;   // more bytes to come
            if (c.got_any && c.in.empty() && c.npend < 2) break;   // answered some, then closed
            return fail(k, "connection to the API server failed");
          }
          c.in.erase(0, used);
          deliver(c, status, std::move(body));
          if (close) {
            eof = true;
            break;
          }
        }
        if (c.npend > 0 || eof) {
          close_conn(c);
          deliver_rest(c, "connection to the API server closed before every answer");
        }
        c.st = kIdle;
        idle.push_back(k);
        return;
      }
      return;
    }
  };
  // starts slot s's requests on an idle (or new) connection: the binding, then (label mode)
  // the label PATCH pipelined behind it
  auto launch = [&](int64_t s) {
    AJob& jb = *slots[static_cast<size_t>(s)];
    size_t k;
    if (!idle.empty()) {
      k = idle.back();
      idle.pop_back();
    } else {
      k = conns.size();
      conns.push_back(std::make_unique<AConn>());
    }
    AConn& c = *conns[k];
    request(&c.out, "POST", jb.j, true, kJsonE, jb.binding);
    c.pend[0] = Pending{s, 1};
    c.npend = 1;
    if (label_) {
      thread_local std::string second;
      request(&second, "PATCH", jb.j, false, kMergePatchE, jb.patch);
      c.out += second;
      c.pend[1] = Pending{s, 0};
      c.npend = 2;
    }
    c.off = 0;
    c.in.clear();
    c.got_any = false;
    c.retried = false;
    c.deadline_ns = ns_now() + timeout_ns;
    c.reused = c.fd >= 0;
    if (c.fd >= 0) {
      c.st = kSending;
    } else if (!open_conn(k)) {
      close_conn(c);
      deliver_rest(c, "cannot connect to the API server");
      idle.push_back(k);
      return;
    }
    kick.push_back(k);
  };

  epoll_event evs[256];
  uint64_t stop_at = 0;
  for (;;) {
    bool stopping;
    {
      std::lock_guard<std::mutex> g(mu_);
      stopping = stop_;
      if (!stopping) {
        while (!q_.empty()) {
          waiting.push_back(std::move(q_.front()));
          q_.pop_front();
        }
        q_len_.store(0, std::memory_order_relaxed);
      }
    }
    if (stopping && !stop_at) stop_at = ns_now() + 5'000'000'000ull;
    if (stopping) {
      for (BindJob& j : waiting) {
        refuse(j);
        stats.inflight.fetch_sub(1, std::memory_order_relaxed);
      }
      waiting.clear();
      if (inflight == 0 || ns_now() > stop_at) break;
    }
    if (ns_now() - auth_at > 1'000'000'000ull) {   // a rotated token reaches new requests
      a = auth();
      auth_at = ns_now();
    }
    while (!waiting.empty() && !free_slots.empty()) {
      const int64_t s = free_slots.back();
      free_slots.pop_back();
      auto jb = std::make_unique<AJob>();
      jb->j = std::move(waiting.front());
      waiting.pop_front();
      build(jb->j, &jb->patch, &jb->binding);
      slots[static_cast<size_t>(s)] = std::move(jb);
      ++inflight;
      if (!label_) {   // the binding alone carries the annotations
        slots[static_cast<size_t>(s)]->left = 1;
        slots[static_cast<size_t>(s)]->sp = 200;
      }
      launch(s);
    }
    for (size_t i = 0; i < kick.size(); ++i) drive(kick[i], 0);   // fail() may append
    kick.clear();
    // park: a bind submitted from here on writes efd_; one submitted before is picked up now
    io_parked_.store(true, std::memory_order_seq_cst);
    const bool queued = !stopping && q_len_.load(std::memory_order_seq_cst) > 0;
    // with answers due, wake for the deadline scan
    const int n = epoll_wait(ep, evs, 256, queued ? 0 : stopping ? 10 : inflight ? 100 : 1000);
    io_parked_.store(false, std::memory_order_relaxed);
    for (int e = 0; e < n; ++e) {
      if (evs[e].data.u64 == UINT64_MAX) {
        uint64_t v;
        (void)!::read(efd_, &v, sizeof v);
        continue;
      }
      const size_t k = evs[e].data.u64;
      if (k < conns.size()) drive(k, evs[e].events);
    }
    for (size_t i = 0; i < kick.size(); ++i) drive(kick[i], 0);
    kick.clear();
    // a request unanswered past its deadline (a half-open connection: no answer, no reset)
    // fails to the slow path with status 0, never re-sent on this connection; at most one
    // scan per 100 ms
    const uint64_t now = ns_now();
    if (inflight > 0 && now - scanned_at > 100'000'000ull) {
      scanned_at = now;
      for (size_t k = 0; k < conns.size(); ++k) {
        AConn& c = *conns[k];
        if (c.npend > 0 && c.fd >= 0 && now > c.deadline_ns) {
          stats.timeouts.fetch_add(static_cast<uint64_t>(c.npend), std::memory_order_relaxed);
          c.retried = true;
          fail(k, "the API server did not answer in time");
        }
      }
      for (size_t i = 0; i < kick.size(); ++i) drive(kick[i], 0);
      kick.clear();
    }
  }
  // what is still in flight after the grace period: the slow path answers it
  for (auto& c : conns) close_conn(*c);
  for (size_t s = 0; s < slots.size(); ++s) {
    if (!slots[s]) continue;
    AJob& jb = *slots[s];
    if (jb.left > 0) {
      if (jb.sb == 0) jb.rb = "extender shutting down";
      if (jb.sp == 0) jb.rp = "extender shutting down";
    }
    SlowJob sj;
    sj.j = std::move(jb.j);
    sj.patch = std::move(jb.patch);
    sj.binding = std::move(jb.binding);
    sj.rp = std::move(jb.rp);
    sj.rb = std::move(jb.rb);
    sj.sp = jb.sp;
    sj.sb = jb.sb;
    sj.answered = jb.answered;
    {
      std::lock_guard<std::mutex> g(mu_);
      slow_q_.push_back(std::move(sj));
    }
    slots[s].reset();
  }
  io_done_.store(true);
  {
    std::lock_guard<std::mutex> g(mu_);   // the slow threads re-check under mu_
  }
  cv_.notify_all();
  ::close(ep);
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
