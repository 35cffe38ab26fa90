// Native bind writes to kube-apiserver (see kubewriter.h).
#include "nanogpu/kubewriter.h"

#include "nanogpu/bindhops.h"

#include <charconv>

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "nanogpu/json.h"

namespace nanogpu {

namespace {
constexpr const char* kAssume = "nano-gpu/assume";
constexpr const char* kAssumeTime = "nano-gpu/assume-time";
constexpr const char* kContainerPrefix = "nano-gpu/container-";
constexpr const char* kMergePatch = "application/merge-patch+json";
constexpr const char* kJson = "application/json";

uint64_t now_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count());
}
double wall_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}
double mono_s() { return static_cast<double>(now_ns()) * 1e-9; }

std::string read_token(const std::string& path, int64_t* mtime) {
  struct stat st {};
  if (stat(path.c_str(), &st) != 0) return std::string();
  *mtime = static_cast<int64_t>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
  std::ifstream f(path);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string t = ss.str();
  while (!t.empty() && (t.back() == '\n' || t.back() == '\r' || t.back() == ' ')) t.pop_back();
  return t;
}

// Status.message of an error body, else the body itself.
std::string api_message(const std::string& body) {
  json::Doc d;
  if (d.parse(body) && d.is(d.root(), json::Type::kObj)) {
    const int32_t m = d.get(d.root(), "message");
    if (d.is(m, json::Type::kStr)) return std::string(d.str(m));
  }
  return body.substr(0, 512);
}
std::string api_reason(const std::string& body) {
  json::Doc d;
  if (d.parse(body) && d.is(d.root(), json::Type::kObj)) {
    const int32_t m = d.get(d.root(), "reason");
    if (d.is(m, json::Type::kStr)) return std::string(d.str(m));
  }
  return std::string();
}
// ApiError's text in the Python client: "<status> <reason>: <message>"
std::string api_error(int status, const std::string& body) {
  if (status == 0) return body.empty() ? "connection to the API server failed" : body;
  return std::to_string(status) + " " + api_reason(body) + ": " + api_message(body);
}

std::string pod_node(const std::string& body) {
  json::Doc d;
  if (!d.parse(body) || !d.is(d.root(), json::Type::kObj)) return std::string();
  const int32_t sp = d.get(d.root(), "spec");
  if (!d.is(sp, json::Type::kObj)) return std::string();
  const int32_t n = d.get(sp, "nodeName");
  return d.is(n, json::Type::kStr) ? std::string(d.str(n)) : std::string();
}
}  // namespace

// ------------------------------------------------------------------------------ HttpConn
void* make_ssl_ctx(const KubeTarget& t) {
  if (!t.tls) return nullptr;
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) throw std::runtime_error("SSL_CTX_new failed");
  if (!t.ca_file.empty()) {
    if (SSL_CTX_load_verify_locations(ctx, t.ca_file.c_str(), nullptr) != 1) {
      SSL_CTX_free(ctx);
      throw std::runtime_error("cannot load CA file " + t.ca_file);
    }
  } else {
    SSL_CTX_set_default_verify_paths(ctx);
  }
  SSL_CTX_set_verify(ctx, t.insecure ? SSL_VERIFY_NONE : SSL_VERIFY_PEER, nullptr);
  if (!t.cert_file.empty() && !t.key_file.empty()) {
    if (SSL_CTX_use_certificate_chain_file(ctx, t.cert_file.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx, t.key_file.c_str(), SSL_FILETYPE_PEM) != 1) {
      SSL_CTX_free(ctx);
      throw std::runtime_error("cannot load the client certificate / key");
    }
  }
  return ctx;
}

void free_ssl_ctx(void* ctx) {
  if (ctx) SSL_CTX_free(static_cast<SSL_CTX*>(ctx));
}

void tcp_liveness(int fd, double timeout_s) {
  // a peer that vanished (no FIN, no RST: a rebooted node, a dropped NAT / LB entry) is
  // noticed: keepalive probes on an idle connection, and unacknowledged sends time out
  int one = 1, idle = 10, intvl = 5, cnt = 3;
  setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof one);
  setsockopt(fd, IPPROTO_TCP, TCP_KEEPIDLE, &idle, sizeof idle);
  setsockopt(fd, IPPROTO_TCP, TCP_KEEPINTVL, &intvl, sizeof intvl);
  setsockopt(fd, IPPROTO_TCP, TCP_KEEPCNT, &cnt, sizeof cnt);
  const unsigned ms = static_cast<unsigned>(std::min(timeout_s, 3600.0) * 1000.0);
  setsockopt(fd, IPPROTO_TCP, TCP_USER_TIMEOUT, &ms, sizeof ms);
}

std::string host_header(const KubeTarget& t) {
  const bool v6 = t.host.find(':') != std::string::npos && t.host.front() != '[';
  return (v6 ? "[" + t.host + "]" : t.host) + ":" + std::to_string(t.port);
}

std::string kube_token(const KubeTarget& t) {
  if (!t.token_file.empty()) {
    int64_t mtime = 0;
    std::string tok = read_token(t.token_file, &mtime);
    if (!tok.empty()) return tok;
  }
  return t.token;
}

HttpConn::~HttpConn() { close_(); }

void HttpConn::close_() {
  if (ssl_) {
    SSL_free(static_cast<SSL*>(ssl_));
    ssl_ = nullptr;
  }
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
  buf_.clear();
}

bool HttpConn::connect_() {
  close_();
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  if (getaddrinfo(t_->host.c_str(), std::to_string(t_->port).c_str(), &hints, &res) != 0 || !res) return false;
  for (addrinfo* a = res; a; a = a->ai_next) {
    const int fd = socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    // connecting and the TLS handshake are bounded at 30 s whatever the read timeout (a
    // watch's is the server's timeoutSeconds and more)
    timeval tv{std::min(timeout_s_, 30), 0};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    tcp_liveness(fd, timeout_s_);
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) {
      fd_ = fd;
      break;
    }
    ::close(fd);
  }
  freeaddrinfo(res);
  if (fd_ < 0) return false;
  if (ctx_) {
    SSL* s = SSL_new(static_cast<SSL_CTX*>(ctx_));
    if (!s) return close_(), false;
    SSL_set_fd(s, fd_);
    // in-cluster the API server is an IP (KUBERNETES_SERVICE_HOST): verify it against the
    // certificate's IP SANs; a name goes through SNI and the DNS SANs
    in6_addr a6{};
    const bool ip = inet_pton(AF_INET, t_->host.c_str(), &a6) == 1 || inet_pton(AF_INET6, t_->host.c_str(), &a6) == 1;
    if (!ip) SSL_set_tlsext_host_name(s, t_->host.c_str());
    if (!t_->insecure) {
      if (ip) X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(s), t_->host.c_str());
      else SSL_set1_host(s, t_->host.c_str());
    }
    ssl_ = s;
    if (SSL_connect(s) != 1) return close_(), false;
  }
  if (timeout_s_ > 30) {
    timeval tv{timeout_s_, 0};
    setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  }
  return true;
}

bool HttpConn::send_all(const char* p, size_t n) {
  while (n) {
    long w;
    if (ssl_) {
      const int r = SSL_write(static_cast<SSL*>(ssl_), p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
      w = r > 0 ? r : -1;
    } else {
      w = ::send(fd_, p, n, MSG_NOSIGNAL);
      if (w < 0 && errno == EINTR) continue;
    }
    if (w <= 0) return false;
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

long HttpConn::recv_some(char* p, size_t n) {
  if (ssl_) {
    const int r = SSL_read(static_cast<SSL*>(ssl_), p, static_cast<int>(n));
    return r > 0 ? r : (SSL_get_error(static_cast<SSL*>(ssl_), r) == SSL_ERROR_ZERO_RETURN ? 0 : -1);
  }
  for (;;) {
    const long r = ::recv(fd_, p, n, 0);
    if (r < 0 && errno == EINTR) continue;
    return r;
  }
}

bool HttpConn::read_head(Head* h, bool* retryable) {
  *retryable = false;
  char tmp[16384];
  size_t he;
  bool got_any = !buf_.empty();
  while ((he = buf_.find("\r\n\r\n")) == std::string::npos) {
    const long r = recv_some(tmp, sizeof tmp);
    if (r <= 0) {
      *retryable = !got_any;   // the server closed an idle keep-alive connection
      return false;
    }
    got_any = true;
    buf_.append(tmp, static_cast<size_t>(r));
  }
  const std::string head = buf_.substr(0, he);
  buf_.erase(0, he + 4);
  *h = Head();
  if (head.size() > 12) h->status = std::atoi(head.c_str() + 9);
  size_t p = head.find("\r\n");
  while (p != std::string::npos && p + 2 < head.size()) {
    const size_t e = head.find("\r\n", p + 2);
    std::string line = head.substr(p + 2, (e == std::string::npos ? head.size() : e) - p - 2);
    const size_t colon = line.find(':');
    if (colon != std::string::npos) {
      std::string k = line.substr(0, colon);
      for (char& ch : k) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
      std::string v = line.substr(colon + 1);
      while (!v.empty() && v.front() == ' ') v.erase(0, 1);
      if (k == "content-length") h->clen = std::atol(v.c_str());
      else if (k == "transfer-encoding" && v.find("chunked") != std::string::npos) h->chunked = true;
      else if (k == "connection" && (v == "close" || v == "Close")) h->close_after = true;
      else if (k == "retry-after") h->retry_after = std::atof(v.c_str());
    }
    p = e;
  }
  retry_after_ = h->retry_after;
  return true;
}

int HttpConn::read_body(const Head& h, std::string* resp) {
  char tmp[16384];
  bool close_after = h.close_after;
  resp->clear();
  if (h.chunked) {
    for (;;) {
      size_t le;
      while ((le = buf_.find("\r\n")) == std::string::npos) {
        const long r = recv_some(tmp, sizeof tmp);
        if (r <= 0) return close_(), 0;
        buf_.append(tmp, static_cast<size_t>(r));
      }
      const size_t sz = std::strtoul(buf_.c_str(), nullptr, 16);
      while (buf_.size() < le + 2 + sz + 2) {
        const long r = recv_some(tmp, sizeof tmp);
        if (r <= 0) return close_(), 0;
        buf_.append(tmp, static_cast<size_t>(r));
      }
      resp->append(buf_, le + 2, sz);
      buf_.erase(0, le + 2 + sz + 2);
      if (sz == 0) break;
    }
  } else if (h.clen >= 0) {
    while (buf_.size() < static_cast<size_t>(h.clen)) {
      const long r = recv_some(tmp, sizeof tmp);
      if (r <= 0) return close_(), 0;
      buf_.append(tmp, static_cast<size_t>(r));
    }
    resp->assign(buf_, 0, static_cast<size_t>(h.clen));
    buf_.erase(0, static_cast<size_t>(h.clen));
  } else {
    for (;;) {   // no length: the body runs to the end of the connection
      const long r = recv_some(tmp, sizeof tmp);
      if (r <= 0) break;
      buf_.append(tmp, static_cast<size_t>(r));
    }
    resp->swap(buf_);
    close_after = true;
  }
  if (close_after) close_();
  return h.status;
}

int HttpConn::receive(std::string* resp, bool* retryable) {
  Head h;
  if (!read_head(&h, retryable)) return 0;
  return read_body(h, resp);
}

int HttpConn::stream_head(std::string* body) {
  body->clear();
  if (!sent_) return 0;
  Head h;
  bool retryable = false;
  if (!read_head(&h, &retryable)) return close_(), 0;
  if (h.status != 200) return read_body(h, body);
  stream_chunked_ = h.chunked;
  stream_end_ = false;
  chunk_left_ = -1;
  return h.status;
}

long HttpConn::stream_read(std::string* out) {
  const size_t before = out->size();
  char tmp[65536];
  for (;;) {
    if (!stream_chunked_) {
      out->append(buf_);
      buf_.clear();
    } else {
      while (!stream_end_) {
        if (chunk_left_ < 0) {   // a chunk-size line next
          const size_t le = buf_.find("\r\n");
          if (le == std::string::npos) break;
          const long sz = static_cast<long>(std::strtoul(buf_.c_str(), nullptr, 16));
          buf_.erase(0, le + 2);
          if (sz == 0) {
            stream_end_ = true;
            break;
          }
          chunk_left_ = sz + 2;
        }
        const size_t take = std::min(buf_.size(), static_cast<size_t>(chunk_left_));
        const size_t data = chunk_left_ > 2 ? std::min(take, static_cast<size_t>(chunk_left_ - 2)) : 0;
        out->append(buf_, 0, data);
        buf_.erase(0, take);
        chunk_left_ -= static_cast<long>(take);
        if (chunk_left_ > 0) break;   // the rest of this chunk is still on the wire
        chunk_left_ = -1;
      }
    }
    if (out->size() > before) return static_cast<long>(out->size() - before);
    if (stream_end_) return 0;
    const long r = recv_some(tmp, sizeof tmp);
    if (r == 0 && !stream_chunked_) return 0;   // a body without framing ends with the connection
    if (r <= 0) return -1;                      // a chunked body cut short, an error, a timeout
    buf_.append(tmp, static_cast<size_t>(r));
  }
}

bool HttpConn::start(const char* method, const std::string& path, const std::string& content_type,
                     const std::string& body, const std::string& auth) {
  req_.clear();
  req_.reserve(256 + body.size());
  req_ += method;
  req_ += ' ';
  req_ += path;
  req_ += " HTTP/1.1\r\nHost: ";
  req_ += host_header(*t_);
  req_ += "\r\nUser-Agent: nano-gpu-scheduler-amd/0.1\r\nAccept: application/json\r\n";
  if (!auth.empty()) req_ += "Authorization: Bearer " + auth + "\r\n";
  if (!body.empty() || std::strcmp(method, "POST") == 0 || std::strcmp(method, "PATCH") == 0) {
    req_ += "Content-Type: " + content_type + "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  }
  req_ += "\r\n";
  req_ += body;
  reused_ = fd_ >= 0;
  sent_ = false;
  if (!reused_ && !connect_()) return false;
  sent_ = send_all(req_.data(), req_.size());
  return sent_;
}

int HttpConn::finish(std::string* resp) {
  resp->clear();
  bool retryable = false;
  if (sent_) {
    const int st = receive(resp, &retryable);
    if (st > 0) return st;
  } else {
    retryable = reused_;   // the send failed on an idle connection the server had closed
  }
  close_();
  if (!(reused_ && retryable)) {
    if (resp->empty()) *resp = sent_ || reused_ ? "connection to the API server failed"
                                                : "cannot connect to " + t_->host + ":" + std::to_string(t_->port);
    return 0;
  }
  // once more on a fresh connection
  if (!connect_()) {
    *resp = "cannot connect to " + t_->host + ":" + std::to_string(t_->port);
    return 0;
  }
  if (send_all(req_.data(), req_.size())) {
    const int st = receive(resp, &retryable);
    if (st > 0) return st;
  }
  close_();
  if (resp->empty()) *resp = "connection to the API server failed";
  return 0;
}

int HttpConn::request(const char* method, const std::string& path, const std::string& content_type,
                      const std::string& body, const std::string& auth, std::string* resp) {
  start(method, path, content_type, body, auth);
  return finish(resp);
}

// ------------------------------------------------------------------------------ KubeWriter
KubeWriter::KubeWriter(KubeTarget target, std::shared_ptr<Ledger> ledger, Respond respond, int threads, int retries,
                       bool record_events, bool evented, bool label, double timeout_s, bool inline_io, int max_binds)
    : t_(std::move(target)), ledger_(std::move(ledger)), respond_(std::move(respond)), retries_(retries),
      timeout_s_(timeout_s > 0 ? timeout_s : 30.0), events_(record_events), evented_(evented || inline_io) {
  inline_io_ = inline_io;
  label_ = label;
  ctx_ = make_ssl_ctx(t_);
  token_ = t_.token;
  if (!t_.token_file.empty()) {
    const std::string tok = read_token(t_.token_file, &token_mtime_);
    if (!tok.empty()) token_ = tok;
  }
  token_checked_ = mono_s();
  host_hdr_ = host_header(t_);
  if (evented_) {
    // the API server's address resolved here, on the thread that sets the writer up: an inline
    // BindIo runs on a front-door worker, whose epoll loop must not wait on a DNS lookup (a name
    // that does not resolve yet is looked up by the BindIo when it first connects)
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    if (getaddrinfo(t_.host.c_str(), std::to_string(t_.port).c_str(), &hints, &res) == 0 && res &&
        res->ai_addrlen <= sizeof(addr_)) {
      std::memcpy(&addr_, res->ai_addr, res->ai_addrlen);
      addr_len_ = res->ai_addrlen;
      family_ = res->ai_family;
    }
    if (res) freeaddrinfo(res);
  }
  if (threads < 1) threads = 1;
  if (evented_) {
    max_inflight_ = max_binds > 0 ? max_binds : threads * kBatch;
    stats.window.store(max_inflight_, std::memory_order_relaxed);
    if (inline_io_) {
      io_done_.store(true);   // no io thread: the owners of the BindIo drivers hand off themselves
    } else {
      efd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
      if (efd_ < 0) throw std::runtime_error("KubeWriter: eventfd failed");
      io_ = std::thread([this] {
        pthread_setname_np(pthread_self(), "ngpu-wr-io");
        io_loop();
      });
    }
    // the slow path: retries with backoff, conflict checks, rollbacks (rare; blocking is fine)
    for (int i = 0; i < 2; ++i)
      threads_.emplace_back([this, i] {
        pthread_setname_np(pthread_self(), ("ngpu-wr-slow" + std::to_string(i)).c_str());
        run_slow();
      });
    return;
  }
  for (int i = 0; i < threads; ++i)
    threads_.emplace_back([this, i] {
      pthread_setname_np(pthread_self(), ("ngpu-wr" + std::to_string(i)).c_str());
      run();
    });
}

KubeWriter::~KubeWriter() {
  stop();
  if (efd_ >= 0) ::close(efd_);
  free_ssl_ctx(ctx_);
}

void KubeWriter::refuse(BindJob& j) {
  // kube-scheduler gets an answer (and retries elsewhere); the ledger is left clean
  if (j.fresh) ledger_->release(j.uid);
  respond_(j.id, 500, "{\"Error\":\"nano-gpu: extender shutting down\"}");
}

void KubeWriter::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_all();
  if (io_.joinable()) {
    // the io thread finishes what it has in flight (bounded), hands failures to the slow path
    uint64_t one = 1;
    (void)!::write(efd_, &one, sizeof one);
    io_.join();
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  std::deque<SlowJob> late;   // handed over while the slow threads were already leaving
  {
    std::lock_guard<std::mutex> g(mu_);
    slow_gone_ = true;
    late.swap(slow_q_);
  }
  if (!late.empty()) {
    HttpConn c(&t_, ctx_, 5), c2(&t_, ctx_, 5);
    for (SlowJob& sj : late) {
      if (sj.answered) finish_label(&c, sj.j, sj.patch, sj.sp, &sj.rp);
      else finish(&c, &c2, sj.j, sj.patch, sj.binding, sj.sp, &sj.rp, sj.sb, &sj.rb);
      stats.inflight.fetch_sub(1, std::memory_order_relaxed);
    }
  }
  std::deque<BindJob> left;
  {
    std::lock_guard<std::mutex> g(mu_);
    left.swap(q_);
  }
  for (BindJob& j : left) {
    refuse(j);
    stats.inflight.fetch_sub(1, std::memory_order_relaxed);
  }
}

void KubeWriter::submit(BindJob job) {
  bool accepted = false, wake = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!stop_) {
      stats.inflight.fetch_add(1, std::memory_order_relaxed);
      const bool first = q_.empty();   // evented: the io thread drains the whole queue per wake-up
      q_.push_back(std::move(job));
      q_len_.store(q_.size(), std::memory_order_seq_cst);
      wake = first && io_parked_.load(std::memory_order_seq_cst);   // an awake io thread looks itself
      accepted = true;
      if (!evented_) cv_.notify_one();
    }
  }
  if (!accepted) {
    refuse(job);   // a bind that arrives while the writer shuts down
    return;
  }
  if (evented_ && wake) {
    uint64_t one = 1;
    (void)!::write(efd_, &one, sizeof one);
  }
}

std::string KubeWriter::auth() {
  std::lock_guard<std::mutex> g(tok_mu_);
  if (!t_.token_file.empty() && mono_s() - token_checked_ > 60.0) {
    token_checked_ = mono_s();
    int64_t mt = 0;
    struct stat st {};
    if (stat(t_.token_file.c_str(), &st) == 0) {
      mt = static_cast<int64_t>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
      if (mt != token_mtime_) {
        const std::string tok = read_token(t_.token_file, &token_mtime_);
        if (!tok.empty()) token_ = tok;
      }
    }
  }
  return token_;
}

int KubeWriter::call(HttpConn* c, const char* method, const std::string& path, const std::string& ctype,
                     const std::string& body, std::string* resp, bool retry) {
  int st = 0;
  for (int attempt = 0;; ++attempt) {
    st = c->request(method, path, ctype, body, auth(), resp);
    if (st == 401 && !t_.token_file.empty() && attempt == 0) {
      std::lock_guard<std::mutex> g(tok_mu_);   // rotated under us: re-read once
      const std::string tok = read_token(t_.token_file, &token_mtime_);
      if (!tok.empty()) token_ = tok;
      continue;
    }
    const bool transient = st >= 500 || st == 429;
    if (!retry || !transient || attempt >= retries_) return st;
    stats.retries.fetch_add(1, std::memory_order_relaxed);
    // kube-apiserver's 429 says when to come back (Retry-After, seconds); else 5 ms x 2^k
    int64_t wait_us = 5000LL << attempt;
    if (st == 429) {
      stats.throttled.fetch_add(1, std::memory_order_relaxed);
      if (c->retry_after() > 0) wait_us = std::max<int64_t>(wait_us, static_cast<int64_t>(c->retry_after() * 1e6));
    }
    // at most 2 s a wait (BindIo::kMaxRetryAfterS): kube-scheduler's bind times out at 30 s
    std::this_thread::sleep_for(std::chrono::microseconds(std::min<int64_t>(wait_us, 2'000'000)));
  }
}

// The two request bodies of one bind. The Binding carries the placement annotations
// (pu.placement_annotations), so they land on the pod atomically with spec.nodeName
// (kube-apiserver setPodHostAndAnnotations) and a refused binding writes nothing. The PATCH
// adds the assume label only, and restates spec.nodeName: kube-apiserver refuses a pod patch
// that would change it (422), so the label lands only on a pod bound to this node
// (pu.label_patch), never on one bound elsewhere or still unbound.
void KubeWriter::build(BindJob& j, std::string* patch, std::string* binding) {
  // written in place, one buffer each (no temporaries: this runs once a bind on the writer)
  std::string& p = *patch;
  p.clear();
  p.reserve(96 + j.node.size());
  p += "{\"metadata\":{\"labels\":{\"";
  p += kAssume;
  p += "\":\"true\"}},\"spec\":{\"nodeName\":";
  json::append_quoted(&p, j.node);
  p += "}}";
  std::string& b = *binding;
  b.clear();
  size_t est = 320 + j.name.size() + j.ns.size() + j.uid.size() + j.node.size();
  for (size_t k = 0; k < j.containers.size(); ++k) est += 40 + j.containers[k].size() + 4 * (k < j.plan.size() ? j.plan[k].size() : 0);
  b.reserve(est);
  b += "{\"apiVersion\":\"v1\",\"kind\":\"Binding\",\"metadata\":{\"name\":";
  json::append_quoted(&b, j.name);
  b += ",\"namespace\":";
  json::append_quoted(&b, j.ns);
  b += ",\"uid\":";
  json::append_quoted(&b, j.uid);
  b += ",\"annotations\":{";
  char num[24];
  for (size_t k = 0; k < j.containers.size() && k < j.plan.size(); ++k) {
    b += '"';
    b += kContainerPrefix;
    json::append_escaped(&b, j.containers[k]);
    b += '"';
    b += ":\"";
    for (size_t i = 0; i < j.plan[k].size(); ++i) {
      if (i) b += ',';
      b.append(num, static_cast<size_t>(std::to_chars(num, num + sizeof num, j.plan[k][i]).ptr - num));
    }
    b += "\",";
  }
  char ts[48];
  const int tl = std::snprintf(ts, sizeof ts, "%.6f", wall_s());
  b += "\"";
  b += kAssume;
  b += "\":\"true\",\"";
  b += kAssumeTime;
  b += "\":\"";
  b.append(ts, static_cast<size_t>(std::max(0, tl)));
  b += "\"}},\"target\":{\"apiVersion\":\"v1\",\"kind\":\"Node\",\"name\":";
  json::append_quoted(&b, j.node);
  b += "}}";
}

// A batch of binds taken together: every bind's binding is sent first, then the answers
// are read and each bind is finished (committed and answered, or rolled back); the label
// PATCHes of the bound pods go out after that, together.
void KubeWriter::process_batch(std::vector<BindJob>& jobs, std::vector<std::unique_ptr<HttpConn>>& conns) {
  const size_t n = jobs.size();
  std::vector<std::string> patch(n), binding(n), rp(n), rb(n);
  std::vector<int> sb(n);
  std::vector<char> bound(n, 0);
  const std::string a = auth();
  const uint64_t t1 = now_ns();
  for (size_t i = 0; i < n; ++i) {
    g_hops.stamp(jobs[i].id, kHopPickup);
    g_hops.stamp(jobs[i].id, kHopLaunched);   // blocking writer threads: no admission window
    build(jobs[i], &patch[i], &binding[i]);
    conns[2 * i + 1]->start("POST", "/api/v1/namespaces/" + jobs[i].ns + "/pods/" + jobs[i].name + "/binding", kJson,
                            binding[i], a);
    g_hops.stamp(jobs[i].id, kHopSent);
  }
  for (size_t i = 0; i < n; ++i) {
    sb[i] = conns[2 * i + 1]->finish(&rb[i]);
    g_hops.stamp(jobs[i].id, kHopAnswer);
  }
  stats.binding_ns.fetch_add(now_ns() - t1, std::memory_order_relaxed);   // in flight together
  for (size_t i = 0; i < n; ++i) bound[i] = finish_binding(conns[2 * i + 1].get(), jobs[i], binding[i], sb[i], &rb[i]);
  if (label_) {
    const uint64_t t3 = now_ns();
    for (size_t i = 0; i < n; ++i)
      if (bound[i])
        conns[2 * i]->start("PATCH", "/api/v1/namespaces/" + jobs[i].ns + "/pods/" + jobs[i].name, kMergePatch,
                            patch[i], a);
    for (size_t i = 0; i < n; ++i) {
      if (!bound[i]) continue;
      const int sp = conns[2 * i]->finish(&rp[i]);
      if (sp < 200 || sp >= 300) finish_label(conns[2 * i].get(), jobs[i], patch[i], sp, &rp[i]);
    }
    stats.patch_ns.fetch_add(now_ns() - t3, std::memory_order_relaxed);
  }
  for (size_t i = 0; i < n; ++i) stats.inflight.fetch_sub(1, std::memory_order_relaxed);
}

void KubeWriter::finish_label(HttpConn* c, const BindJob& j, const std::string& patch, int sp, std::string* rp) {
  // the pod is bound here by now: a PATCH refused by its nodeName guard (it reached the server
  // before the binding had landed) or lost in transport goes out again, with the transient
  // retries; a pod that is gone is left alone
  const uint64_t t3 = now_ns();
  if (sp != 404) sp = call(c, "PATCH", "/api/v1/namespaces/" + j.ns + "/pods/" + j.name, kMergePatch, patch, rp, true);
  stats.patch_ns.fetch_add(now_ns() - t3, std::memory_order_relaxed);
  // a pod deleted before its label landed (a label trailing its binding under a saturated
  // admission window can meet the pod's delete) needs none: not a failure
  if ((sp < 200 || sp >= 300) && sp != 404) stats.label_failures.fetch_add(1, std::memory_order_relaxed);
}

bool KubeWriter::finish_binding(HttpConn* c2, BindJob& j, const std::string& b, int sb, std::string* rb) {
  const std::string base = "/api/v1/namespaces/" + j.ns + "/pods/" + j.name;
  auto transient = [](int st) { return st == 0 || st == 401 || st == 429 || st >= 500; };
  if (transient(sb)) sb = call(c2, "POST", base + "/binding", kJson, b, rb, true);
  if (sb == 409 || transient(sb)) {
    // a retried POST whose first attempt landed (409), or an answer lost to a 5xx or the
    // transport: the pod already on this node means the bind succeeded
    std::string got;
    const int gs = call(c2, "GET", base, kJson, std::string(), &got, true);
    if (gs == 200 && pod_node(got) == j.node) sb = 201;
  }
  g_hops.stamp(j.id, kHopAnswer);   // the outcome is known (after any retry)
  if (sb >= 200 && sb < 300) {
    ledger_->commit(j.uid);
    stats.ok.fetch_add(1, std::memory_order_relaxed);
    g_hops.stamp(j.id, kHopPosted);
    respond_(j.id, 200, "{\"Error\":\"\"}");
    return true;
  }
  const std::string err = api_error(sb, *rb);
  stats.failed.fetch_add(1, std::memory_order_relaxed);
  if (j.fresh) {
    // D2: roll the reservation back and record the event. Nothing is un-annotated: the
    // Binding, which carries the annotations, was refused, and the label PATCH's nodeName
    // guard keeps it off a pod not bound here. No write of this bind landed; a pod bound
    // elsewhere keeps its own placement untouched.
    ledger_->release(j.uid);
    stats.rollbacks.fetch_add(1, std::memory_order_relaxed);
    if (events_ && sb > 0) {
      char tbuf[32];
      const std::time_t now = std::time(nullptr);
      std::tm g{};
      gmtime_r(&now, &g);
      std::strftime(tbuf, sizeof tbuf, "%Y-%m-%dT%H:%M:%SZ", &g);
      char suffix[24];
      std::snprintf(suffix, sizeof suffix, ".%016llx", static_cast<unsigned long long>(now_ns()));
      std::string ev = "{\"apiVersion\":\"v1\",\"kind\":\"Event\",\"metadata\":{\"name\":";
      json::append_quoted(&ev, j.name + suffix);
      ev += ",\"namespace\":";
      json::append_quoted(&ev, j.ns);
      ev += "},\"involvedObject\":{\"kind\":\"Pod\",\"name\":";
      json::append_quoted(&ev, j.name);
      ev += ",\"namespace\":";
      json::append_quoted(&ev, j.ns);
      ev += ",\"uid\":";
      json::append_quoted(&ev, j.uid);
      ev += "},\"reason\":\"FailedBinding\",\"message\":";
      json::append_quoted(&ev, "nano-gpu bind failed: " + err);
      ev += ",\"type\":\"Warning\",\"source\":{\"component\":\"nano-gpu-scheduler\"},\"firstTimestamp\":\"";
      ev += tbuf;
      ev += "\",\"lastTimestamp\":\"";
      ev += tbuf;
      ev += "\",\"count\":1}";
      std::string ignored;
      call(c2, "POST", "/api/v1/namespaces/" + j.ns + "/events", kJson, ev, &ignored, false);
    }
  }
  std::string body = "{\"Error\":";
  json::append_quoted(&body, err);
  body += "}";
  g_hops.stamp(j.id, kHopPosted);
  respond_(j.id, 500, body);
  return false;
}

// the slow path of the evented writer: the binding's outcome, then (bound) the label
void KubeWriter::finish(HttpConn* c, HttpConn* c2, BindJob& j, const std::string& patch, const std::string& b,
                        int sp, std::string* rp, int sb, std::string* rb) {
  if (finish_binding(c2, j, b, sb, rb) && label_ && (sp < 200 || sp >= 300)) finish_label(c, j, patch, sp, rp);
}

void KubeWriter::run() {
  std::vector<std::unique_ptr<HttpConn>> conns;
  const int tmo = std::max(1, static_cast<int>(timeout_s_ + 0.5));
  for (int i = 0; i < 2 * kBatch; ++i) conns.push_back(std::make_unique<HttpConn>(&t_, ctx_, tmo));
  std::vector<BindJob> jobs;
  for (;;) {
    jobs.clear();
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [this] { return stop_ || !q_.empty(); });
      if (stop_) return;
      while (!q_.empty() && static_cast<int>(jobs.size()) < kBatch) {
        jobs.push_back(std::move(q_.front()));
        q_.pop_front();
      }
    }
    process_batch(jobs, conns);
  }
}

}  // namespace nanogpu
