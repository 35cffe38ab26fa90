// Native kube-scheduler stand-in (see schedsim.h).
#include "nanogpu/schedsim.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cmath>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <queue>
#include <random>
#include <stdexcept>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "nanogpu/frontend.h"
#include "nanogpu/json.h"

namespace nanogpu::sim {

namespace {

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + 1e-9 * static_cast<double>(ts.tv_nsec);
}

// Pops one complete HTTP/1.1 response off the front of `buf`.
// 1 = done (status/body/close set), 0 = incomplete, -1 = malformed or unsupported.
int take_response(std::string* buf, int* status, std::string* body, bool* close) {
  size_t hdr_end = buf->find("\r\n\r\n");
  if (hdr_end == std::string::npos) return buf->size() > (64u << 10) ? -1 : 0;
  std::string_view head(buf->data(), hdr_end);
  size_t sp = head.find(' ');
  if (sp == std::string_view::npos || head.size() < sp + 4) return -1;
  *status = std::atoi(std::string(head.substr(sp + 1, 3)).c_str());
  size_t len = 0;
  *close = false;
  size_t pos = head.find("\r\n");
  while (pos != std::string_view::npos && pos < head.size()) {
    size_t next = head.find("\r\n", pos + 2);
    std::string_view line = head.substr(pos + 2, (next == std::string_view::npos ? head.size() : next) - pos - 2);
    size_t colon = line.find(':');
    if (colon != std::string_view::npos) {
      std::string key(line.substr(0, colon));
      for (char& c : key) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
      std::string_view v = line.substr(colon + 1);
      while (!v.empty() && v.front() == ' ') v.remove_prefix(1);
      if (key == "content-length") len = static_cast<size_t>(std::strtoull(std::string(v).c_str(), nullptr, 10));
      else if (key == "connection" && (v.substr(0, 5) == "close" || v.substr(0, 5) == "Close")) *close = true;
      else if (key == "transfer-encoding") return -1;   // the extender always sends a length
    }
    pos = next;
  }
  const size_t body0 = hdr_end + 4;
  if (buf->size() < body0 + len) return 0;
  body->assign(*buf, body0, len);
  buf->erase(0, body0 + len);
  return 1;
}

int open_socket(const std::string& host, int port, bool nonblock) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC | (nonblock ? SOCK_NONBLOCK : 0), 0);
  if (fd < 0) return -1;
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (::inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1 ||
      (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 && !(nonblock && errno == EINPROGRESS))) {
    ::close(fd);
    return -1;
  }
  return fd;
}

std::string post_request(std::string_view host, std::string_view path, std::string_view body) {
  std::string r;
  r.reserve(body.size() + 128);
  r.append("POST ").append(path).append(" HTTP/1.1\r\nHost: ").append(host);
  r.append("\r\nContent-Type: application/json\r\nContent-Length: ").append(std::to_string(body.size()));
  r.append("\r\n\r\n").append(body);
  return r;
}

// Blocking HTTP/1.1 client on one keep-alive connection; reconnects after any error.
class Conn {
 public:
  Conn(std::string host, int port) : host_(std::move(host)), port_(port) {}
  ~Conn() { close_fd(); }
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;

  // POST `body` to `path`; fills status and response body. false = transport error.
  bool post(std::string_view path, std::string_view body, int* status, std::string* out) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      if (fd_ < 0 && !connect_fd()) return false;
      req_ = post_request(host_, path, body);
      const double t0 = now_s();
      const bool ok = send_all(req_) && read_response(status, out);
      wire_s += now_s() - t0;
      if (ok) return true;
      close_fd();   // stale keep-alive connection: one fresh attempt
    }
    return false;
  }
  double wire_s = 0.0;   // time from the first byte sent to the whole response read

 private:
  bool connect_fd() {
    fd_ = open_socket(host_, port_, false);
    buf_.clear();
    return fd_ >= 0;
  }
  void close_fd() {
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    buf_.clear();
  }
  bool send_all(const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
      ssize_t n = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) return false;
      off += static_cast<size_t>(n);
    }
    return true;
  }
  bool fill() {
    char tmp[65536];
    for (;;) {
      ssize_t n = ::recv(fd_, tmp, sizeof tmp, 0);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) return false;
      buf_.append(tmp, static_cast<size_t>(n));
      return true;
    }
  }
  bool read_response(int* status, std::string* out) {
    bool close = false;
    int rc;
    while ((rc = take_response(&buf_, status, out, &close)) == 0)
      if (!fill()) return false;
    if (rc < 0) return false;
    if (close) close_fd();
    return true;
  }

  std::string host_;
  int port_;
  int fd_ = -1;
  std::string buf_, req_;
};

struct Ready {
  double t;
  uint64_t seq;
  size_t pod;
  bool operator>(const Ready& o) const { return t != o.t ? t > o.t : seq > o.seq; }
};

struct BindJob {
  size_t pod;
  int node;
};

}  // namespace

struct SessionState {
  std::string host;
  int port = -1;
  size_t next_start = 0;   // kube-scheduler's nextStartNodeIndex survives across cycles
  std::unique_ptr<Conn> cycle;
  std::vector<int> bind_fds;
  void reset() {
    cycle.reset();
    for (int fd : bind_fds) ::close(fd);
    bind_fds.clear();
  }
  ~SessionState() { reset(); }
};

Session::Session() : st_(std::make_unique<SessionState>()) {
  presize_fd_table();   // a long-running scheduler's client pool: no fd-table growth mid-burst
}
Session::~Session() = default;

int64_t num_feasible_nodes_to_find(int64_t all_nodes, int percentage) {
  constexpr int64_t kMinFeasible = 100, kMinPercent = 5, kBasePercent = 50;
  if (all_nodes < kMinFeasible) return all_nodes;
  int64_t pct = percentage;
  if (pct <= 0) pct = std::max(kMinPercent, kBasePercent - all_nodes / 125);
  if (pct >= 100) return all_nodes;
  return std::max(kMinFeasible, all_nodes * pct / 100);
}

SimResult drive(const SimConfig& cfg, const std::vector<SimPod>& pods, Session* session_handle) {
  SessionState* session = session_handle ? session_handle->state() : nullptr;
  presize_fd_table();
  if (session && (session->host != cfg.host || session->port != cfg.port)) {
    session->reset();
    session->host = cfg.host;
    session->port = cfg.port;
  }
  SimResult r;
  const size_t n_pods = pods.size(), n_nodes = cfg.nodes.size();
  r.node_of.assign(n_pods, std::string());
  r.last_error.assign(n_pods, std::string());
  r.bind_latencies.reserve(n_pods);
  r.e2e_latencies.reserve(n_pods);
  std::unordered_map<std::string_view, int> node_index;   // views into cfg.nodes
  for (size_t i = 0; i < n_nodes; ++i) node_index.emplace(cfg.nodes[i], static_cast<int>(i));
  // A name in a reply -> node index. The extender answers in the order the names were sent
  // (filter: the passing ones; priorities: all of them), so the next expected position of
  // the sent list is tried before the hash lookup.
  auto resolve = [&](std::string_view name, const std::vector<int>* sent, size_t* cursor) -> int {
    if (sent) {
      for (size_t k = *cursor; k < sent->size(); ++k)
        if (cfg.nodes[(*sent)[k]] == name) {
          *cursor = k + 1;
          return (*sent)[k];
        }
    }
    auto it = node_index.find(name);
    return it == node_index.end() ? -1 : it->second;
  };
  const bool fit = !cfg.capacity.empty();
  std::vector<int64_t> requested(n_nodes, 0);
  std::vector<int64_t> req_cpu(n_nodes, 0), req_mem(n_nodes, 0);   // for kube_combine
  // PodTopologySpread: pods of each owner per node, (owner << 32 | node) -> count
  std::unordered_map<uint64_t, int32_t> owner_cnt;
  auto owner_key = [](int32_t owner, int node) {
    return (static_cast<uint64_t>(static_cast<uint32_t>(owner)) << 32) | static_cast<uint32_t>(node);
  };
  for (const SimLive& l : cfg.live) {
    if (l.node < 0 || static_cast<size_t>(l.node) >= n_nodes) continue;
    requested[l.node] += l.need;
    req_cpu[l.node] += l.cpu_m;
    req_mem[l.node] += l.mem;
    if (l.owner >= 0) ++owner_cnt[owner_key(l.owner, l.node)];
  }
  size_t local_start = 0;
  size_t& next_start = session ? session->next_start : local_start;
  const int64_t want_feasible =
      cfg.sample_nodes ? num_feasible_nodes_to_find(static_cast<int64_t>(n_nodes), cfg.percentage_of_nodes_to_score)
                       : static_cast<int64_t>(n_nodes);
  // NodeResourcesLeastAllocated + NodeResourcesBalancedAllocation with the pod added
  auto plugin_score = [&](size_t n, const SimPod& p) {
    const double cf = std::min(1.0, static_cast<double>(req_cpu[n] + p.cpu_m) / static_cast<double>(cfg.node_cpu_m));
    const double mf = std::min(1.0, static_cast<double>(req_mem[n] + p.mem) / static_cast<double>(cfg.node_mem));
    const int64_t least = static_cast<int64_t>(((1.0 - cf) * 100.0 + (1.0 - mf) * 100.0) / 2.0);
    const int64_t balanced = static_cast<int64_t>((1.0 - std::fabs(cf - mf)) * 100.0);
    return least + balanced;
  };

  auto names_json = [&](const std::vector<int>& idx) {
    std::string s = "[";
    for (size_t k = 0; k < idx.size(); ++k) {
      if (k) s.push_back(',');
      json::append_quoted(&s, cfg.nodes[idx[k]]);
    }
    s.push_back(']');
    return s;
  };
  std::vector<int> all(n_nodes);
  for (size_t i = 0; i < n_nodes; ++i) all[i] = static_cast<int>(i);
  const std::string all_json = names_json(all);

  std::mutex mu;
  std::condition_variable cv;
  std::priority_queue<Ready, std::vector<Ready>, std::greater<Ready>> ready;
  std::deque<BindJob> jobs;
  bool stop = false;   // the cycle is done: the binder exits once its binds finish
  uint64_t seq = 0;
  int64_t remaining = static_cast<int64_t>(n_pods);
  std::vector<int> attempts(n_pods, 0);
  const double t_enqueue = now_s();
  for (size_t i = 0; i < n_pods; ++i) ready.push({0.0, seq++, i});

  // mu held
  auto requeue = [&](size_t i) {
    if (attempts[i] < cfg.max_attempts) {
      ready.push({now_s() + cfg.backoff_s * static_cast<double>(1u << std::min(attempts[i], 20)), seq++, i});
    } else {
      ++r.failed;
      --remaining;
    }
    cv.notify_all();
  };

  // Binding cycle: kube-scheduler starts a goroutine per bind, so a bind goes out the
  // moment its host is chosen. One epoll thread multiplexes up to `bind_threads`
  // keep-alive connections (opened on demand) instead of a thread per request.
  const int efd = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  const int ep = ::epoll_create1(EPOLL_CLOEXEC);
  if (efd < 0 || ep < 0) throw std::runtime_error("schedsim: eventfd/epoll_create1 failed");
  {
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = UINT64_MAX;
    ::epoll_ctl(ep, EPOLL_CTL_ADD, efd, &ev);
  }
  auto wake = [&] {
    uint64_t one = 1;
    (void)!::write(efd, &one, sizeof one);
  };

  // a finished bind (mu not held)
  auto complete = [&](const BindJob& job, int status, const std::string* body, const char* transport, double t0) {
    std::string err;
    const double t1 = now_s();
    if (transport) {
      err = transport;
    } else {
      json::Doc doc;
      if (!doc.parse(*body) || !doc.is(doc.root(), json::Type::kObj)) {
        err = "bind: bad response";
      } else {
        int32_t e = doc.get(doc.root(), "Error", true);
        if (doc.is(e, json::Type::kStr) && !doc.str(e).empty()) err = std::string(doc.str(e));
        else if (status != 200) err = "bind: HTTP " + std::to_string(status);
      }
    }
    std::lock_guard<std::mutex> lk(mu);
    if (!err.empty()) {
      requested[job.node] -= pods[job.pod].need;
      req_cpu[job.node] -= pods[job.pod].cpu_m;
      req_mem[job.node] -= pods[job.pod].mem;
      if (pods[job.pod].owner >= 0) --owner_cnt[owner_key(pods[job.pod].owner, job.node)];
      ++r.bind_errors;
      r.last_error[job.pod] = std::move(err);
      requeue(job.pod);
      return;
    }
    r.node_of[job.pod] = cfg.nodes[job.node];
    ++r.scheduled;
    r.bind_latencies.push_back(t1 - t0);
    r.e2e_latencies.push_back(t1 - t_enqueue);
    r.t_last_bind = std::max(r.t_last_bind, t1);
    --remaining;
    cv.notify_all();
  };

  std::thread binder([&] {
    struct MConn {
      int fd = -1;
      bool busy = false;
      bool proven = true;   // false: kept from an earlier run, no response seen yet
      BindJob job{};
      double t0 = 0.0;
      std::string out, in;
      size_t off = 0;
    };
    const size_t max_conns = static_cast<size_t>(std::max(1, cfg.bind_threads));
    std::vector<MConn> conns;
    std::vector<size_t> idle;
    std::deque<BindJob> pending;
    std::string body, resp;
    size_t busy = 0;
    bool stopping = false;
    if (session) {
      // keep-alive connections of earlier runs (kube-scheduler keeps its client's pool)
      for (int fd : session->bind_fds) {
        MConn c;
        c.fd = fd;
        c.proven = false;
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.u64 = conns.size();
        ::epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
        idle.push_back(conns.size());
        conns.push_back(std::move(c));
      }
      session->bind_fds.clear();
    }
    auto drop = [&](size_t k, const char* why) {
      MConn& c = conns[k];
      if (c.fd >= 0) {
        ::epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
        ::close(c.fd);
      }
      c.fd = -1;
      c.in.clear();
      if (c.busy) {
        c.busy = false;
        --busy;
        if (!c.proven && why) {
          pending.push_front(c.job);   // a stale kept connection: resend on a fresh one
        } else {
          complete(c.job, 0, nullptr, why, c.t0);
        }
      }
      c.proven = true;
      idle.push_back(k);
    };
    auto flush_out = [&](size_t k) {   // false = connection failed
      MConn& c = conns[k];
      while (c.off < c.out.size()) {
        ssize_t n = ::send(c.fd, c.out.data() + c.off, c.out.size() - c.off, MSG_NOSIGNAL);
        if (n > 0) {
          c.off += static_cast<size_t>(n);
          continue;
        }
        if (n < 0 && errno == EINTR) continue;
        if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOTCONN)) {
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLOUT;
          ev.data.u64 = k;
          ::epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
          return true;
        }
        return false;
      }
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = k;
      ::epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &ev);
      return true;
    };
    auto dispatch = [&] {
      while (!pending.empty() && (!idle.empty() || conns.size() < max_conns)) {
        size_t k;
        if (!idle.empty()) {
          k = idle.back();
          idle.pop_back();
        } else {
          k = conns.size();
          conns.emplace_back();
        }
        MConn& c = conns[k];
        BindJob job = pending.front();
        pending.pop_front();
        if (c.fd < 0) {
          c.fd = open_socket(cfg.host, cfg.bind_ports.empty() ? cfg.port : cfg.bind_ports[k % cfg.bind_ports.size()],
                             true);
          if (c.fd < 0) {
            c.job = job;
            c.busy = true;
            ++busy;
            c.t0 = now_s();
            drop(k, "bind: connect failed");
            continue;
          }
          epoll_event ev{};
          ev.events = EPOLLIN;
          ev.data.u64 = k;
          ::epoll_ctl(ep, EPOLL_CTL_ADD, c.fd, &ev);
        }
        const SimPod& p = pods[job.pod];
        body.assign("{\"PodName\":");
        json::append_quoted(&body, p.name);
        body.append(",\"PodNamespace\":");
        json::append_quoted(&body, p.ns);
        body.append(",\"PodUID\":");
        json::append_quoted(&body, p.uid);
        body.append(",\"Node\":");
        json::append_quoted(&body, cfg.nodes[job.node]);
        body.push_back('}');
        c.out = post_request(cfg.host, "/scheduler/bind", body);
        c.off = 0;
        c.job = job;
        c.busy = true;
        ++busy;
        c.t0 = now_s();
        if (!flush_out(k)) drop(k, "bind: transport error");
      }
    };
    epoll_event evs[128];
    for (;;) {
      if (stopping && busy == 0 && pending.empty()) break;
      int n = ::epoll_wait(ep, evs, 128, stopping ? 10 : -1);
      if (n < 0 && errno != EINTR) break;
      for (int e = 0; e < n; ++e) {
        if (evs[e].data.u64 == UINT64_MAX) {
          uint64_t v;
          (void)!::read(efd, &v, sizeof v);
          std::lock_guard<std::mutex> lk(mu);
          while (!jobs.empty()) {
            pending.push_back(jobs.front());
            jobs.pop_front();
          }
          if (stop) stopping = true;
          continue;
        }
        const size_t k = evs[e].data.u64;
        if (k >= conns.size() || conns[k].fd < 0) continue;
        MConn& c = conns[k];
        if (evs[e].events & EPOLLOUT) {
          if (!flush_out(k)) {
            drop(k, "bind: transport error");
            continue;
          }
        }
        if (evs[e].events & (EPOLLIN | EPOLLERR | EPOLLHUP)) {
          char tmp[16384];
          ssize_t got = ::recv(c.fd, tmp, sizeof tmp, 0);
          if (got <= 0) {
            if (got < 0 && (errno == EAGAIN || errno == EINTR)) continue;
            drop(k, "bind: connection closed");
            continue;
          }
          c.in.append(tmp, static_cast<size_t>(got));
          int status = 0;
          bool close = false;
          int rc = take_response(&c.in, &status, &resp, &close);
          if (rc == 0) continue;
          if (rc < 0 || !c.busy) {
            drop(k, "bind: bad response");
            continue;
          }
          c.busy = false;
          c.proven = true;
          --busy;
          complete(c.job, status, &resp, nullptr, c.t0);
          if (close) {
            drop(k, nullptr);
          } else {
            idle.push_back(k);
          }
        }
      }
      dispatch();
    }
    for (size_t k = 0; k < conns.size(); ++k) {
      if (conns[k].fd < 0) continue;
      ::epoll_ctl(ep, EPOLL_CTL_DEL, conns[k].fd, nullptr);
      if (session && !conns[k].busy && conns[k].in.empty()) session->bind_fds.push_back(conns[k].fd);
      else ::close(conns[k].fd);
    }
  });

  std::unique_ptr<Conn> own;
  Conn* cycle_conn;
  if (session) {
    if (!session->cycle) session->cycle = std::make_unique<Conn>(cfg.host, cfg.port);
    cycle_conn = session->cycle.get();
  } else {
    own = std::make_unique<Conn>(cfg.host, cfg.port);
    cycle_conn = own.get();
  }
  Conn& cycle = *cycle_conn;
  cycle.wire_s = 0.0;
  std::mt19937_64 rng(cfg.seed);
  std::string body, out, cands_json;
  std::vector<int> cands, fits, ties;
  std::vector<int64_t> spread_raw;
  int64_t spread_min = 0, spread_max = 0;
  json::Doc doc;
  for (;;) {
    size_t i;
    {
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        if (remaining <= 0) break;
        if (!ready.empty()) {
          double wait = ready.top().t - now_s();
          if (wait <= 0) break;
          cv.wait_for(lk, std::chrono::duration<double>(wait));
        } else {
          cv.wait_for(lk, std::chrono::milliseconds(50));
        }
      }
      if (remaining <= 0) break;
      i = ready.top().pod;
      ready.pop();
      ++attempts[i];
      // resource-fit pre-filter on the scheduler's own accounting (requests of pods it bound),
      // from nextStartNodeIndex until numFeasibleNodesToFind nodes passed
      cands.clear();
      if (fit && n_nodes) {
        size_t processed = 0;
        for (size_t k = 0; k < n_nodes && static_cast<int64_t>(cands.size()) < want_feasible; ++k) {
          const size_t n = (next_start + k) % n_nodes;
          ++processed;
          if (requested[n] + pods[i].need <= cfg.capacity[n]) cands.push_back(static_cast<int>(n));
        }
        next_start = (next_start + processed) % n_nodes;
      }
    }
    const double t_cycle = now_s();
    if (r.t_first_filter == 0.0) r.t_first_filter = t_cycle;
    const SimPod& p = pods[i];
    const std::string* names = &all_json;
    if (fit && cands.size() != n_nodes) {
      cands_json = names_json(cands);
      names = &cands_json;
    }
    int host = -1;
    if (!fit || !cands.empty()) {
      ++r.cycles;
      r.nodes_sent_filter += static_cast<int64_t>(fit ? cands.size() : n_nodes);
      body.assign("{\"Pod\":").append(p.json).append(",\"Nodes\":null,\"NodeNames\":").append(*names).push_back('}');
      int status = 0;
      fits.clear();
      if (cycle.post("/scheduler/filter", body, &status, &out) && doc.parse(out) &&
          doc.is(doc.root(), json::Type::kObj)) {
        int32_t nn = doc.get(doc.root(), "NodeNames", true);
        const std::vector<int>* sent = names == &all_json ? &all : &cands;
        size_t cursor = 0;
        if (doc.is(nn, json::Type::kArr))
          for (int32_t c = doc.at(nn).first; c >= 0; c = doc.at(c).next) {
            if (!doc.is(c, json::Type::kStr)) continue;
            const int n = resolve(doc.str(c), sent, &cursor);
            if (n >= 0) fits.push_back(n);
          }
      }
      if (fits.size() == 1) {
        host = fits[0];
      } else if (!fits.empty()) {
        const std::string* fj = names;
        const std::vector<int>* psent = names == &all_json ? &all : &cands;
        if (fits.size() != (fit ? cands.size() : n_nodes)) {
          cands_json = names_json(fits);
          fj = &cands_json;
          psent = &fits;
        }
        body.assign("{\"Pod\":").append(p.json).append(",\"Nodes\":null,\"NodeNames\":").append(*fj).push_back('}');
        if (cycle.post("/scheduler/priorities", body, &status, &out) && doc.parse(out) &&
            doc.is(doc.root(), json::Type::kArr)) {
          int64_t best = INT64_MIN;
          ties.clear();
          // req_cpu / req_mem also change on the binder thread (a failed bind): read under mu
          std::unique_lock<std::mutex> plk(mu, std::defer_lock);
          if (cfg.kube_combine) plk.lock();
          // PodTopologySpread (ScheduleAnyway, hostname) over the nodes priorities ran on:
          // raw = matching pods on the node x log(nodes + 2) + maxSkew - 1, then normalised
          // to 100 x (max + min - raw) / max (100 everywhere when max is 0), x weight
          const bool spread = cfg.kube_combine && p.owner >= 0 && cfg.spread_weight > 0;
          if (spread) {
            spread_raw.resize(n_nodes);
            const double w = std::log(static_cast<double>(psent->size()) + 2.0);
            spread_min = INT64_MAX;
            spread_max = 0;
            for (int node : *psent) {
              auto it = owner_cnt.find(owner_key(p.owner, node));
              const int64_t cnt = it == owner_cnt.end() ? 0 : it->second;
              const int64_t raw = static_cast<int64_t>(static_cast<double>(cnt) * w + (cfg.spread_max_skew - 1));
              spread_raw[node] = raw;
              spread_min = std::min(spread_min, raw);
              spread_max = std::max(spread_max, raw);
            }
          }
          size_t cursor = 0;
          for (int32_t c = doc.at(doc.root()).first; c >= 0; c = doc.at(c).next) {
            int32_t h = doc.get(c, "Host", true), s = doc.get(c, "Score", true);
            if (!doc.is(h, json::Type::kStr) || !doc.is(s, json::Type::kNum)) continue;
            const int node = resolve(doc.str(h), psent, &cursor);
            if (node < 0) continue;
            const std::string_view st = doc.str(s);
            int64_t score = 0;
            if (std::from_chars(st.data(), st.data() + st.size(), score).ec != std::errc())
              score = std::strtoll(std::string(st).c_str(), nullptr, 10);
            if (cfg.kube_combine)
              score = score * cfg.extender_weight * 10 + plugin_score(static_cast<size_t>(node), p);
            if (spread) {
              const int64_t s = spread_raw[node];
              score += cfg.spread_weight * (spread_max == 0 ? 100 : 100 * (spread_max + spread_min - s) / spread_max);
            }
            if (score > best) {
              best = score;
              ties.clear();
            }
            if (score == best) ties.push_back(node);
          }
          if (ties.size() == 1) host = ties[0];
          else if (!ties.empty()) host = ties[std::uniform_int_distribution<size_t>(0, ties.size() - 1)(rng)];
        }
      }
    }
    const double dt_cycle = now_s() - t_cycle;
    r.cycle_wire_s = cycle.wire_s;
    r.cycle_max_s = std::max(r.cycle_max_s, dt_cycle);
    r.cycle_sum_s += dt_cycle;
    std::lock_guard<std::mutex> lk(mu);
    if (host < 0) {
      ++r.unschedulable_attempts;
      requeue(i);
      continue;
    }
    requested[host] += p.need;
    req_cpu[host] += p.cpu_m;
    req_mem[host] += p.mem;
    if (p.owner >= 0) ++owner_cnt[owner_key(p.owner, host)];
    jobs.push_back({i, host});
    wake();
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    stop = true;
  }
  wake();
  binder.join();
  ::close(ep);
  ::close(efd);
  return r;
}

}  // namespace nanogpu::sim
