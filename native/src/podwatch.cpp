// The pod informer's watch, native side (see podwatch.h).
#include "nanogpu/podwatch.h"

#include "nanogpu/iotally.h"

#include <string.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <stdexcept>

namespace nanogpu {

namespace {
std::string_view field(const json::Doc& d, int32_t o, const char* k) {
  const int32_t v = d.is(o, json::Type::kObj) ? d.get(o, k) : -1;
  return d.is(v, json::Type::kStr) ? d.str(v) : std::string_view();
}
}  // namespace

bool filter_pod_event(PodWatchFilter& f, std::string_view line, json::Doc& d, std::string* rv) {
  rv->clear();
  // most events are dropped on a few shallow fields (type, metadata's identity, nodeName,
  // phase): parse to that depth only; what is kept is parsed in full by whoever decodes it
  if (!d.parse_shallow(line, 3) || !d.is(d.root(), json::Type::kObj))
    throw std::invalid_argument("bad watch event line");
  const int32_t t = d.get(d.root(), "type");
  const int32_t obj = d.get(d.root(), "object");
  const std::string_view type = d.is(t, json::Type::kStr) ? d.str(t) : std::string_view();
  if (!d.is(obj, json::Type::kObj) || !(type == "ADDED" || type == "MODIFIED" || type == "DELETED"))
    return true;   // ERROR, BOOKMARK: the informer's own business
  const int32_t md = d.get(obj, "metadata"), sp = d.get(obj, "spec"), st = d.get(obj, "status");
  rv->assign(field(d, md, "resourceVersion"));
  std::lock_guard<std::mutex> g(f.mu);
  // "ns/name" in the filter's own buffer (its capacity kept): built for the forwarded set only
  std::string& key = f.key_buf;
  bool have_key = false;
  auto make_key = [&] {
    if (have_key) return;
    key.assign(field(d, md, "namespace"));
    key.push_back('/');
    key.append(field(d, md, "name"));
    have_key = true;
  };
  bool seen = false;
  if (!f.forwarded.empty()) {
    make_key();
    seen = f.forwarded.count(key) > 0;
  }
  bool drop = false;
  if (!seen && type == "DELETED") {
    // Python never held it: releasing is all the controller would do (pods.py::_on_event)
    if (f.ledger->release(field(d, md, "uid")) == kOk) ++f.released;
    drop = true;
  } else if (!seen) {
    // what the controller ignores: a pending pod, or a bound, running one the ledger holds
    const std::string_view node = field(d, sp, "nodeName"), phase = field(d, st, "phase");
    const int32_t dts = d.is(md, json::Type::kObj) ? d.get(md, "deletionTimestamp") : -1;
    const bool completed = (f.release_on_terminating.load(std::memory_order_relaxed) && dts >= 0 && !d.is(dts, json::Type::kNull)) ||
                           phase == "Succeeded" || phase == "Failed";
    if (!completed && node.empty()) {
      drop = true;
    } else if (!completed) {
      drop = f.ledger->holds(field(d, md, "uid"));
      // the node agent rewrote the placement to what kubelet ran (plugin.reconcile): the
      // controller re-accounts it, so the event goes on. Looked for in the annotations'
      // text only (a depth-3 object the shallow parse spans without parsing)
      // (memmem: string_view::find stops at every '"' of the text to compare the rest)
      static constexpr char kReconciled[] = "\"nano-gpu/reconciled\"";
      const int32_t ann = d.is(md, json::Type::kObj) ? d.get(md, "annotations") : -1;
      if (drop && d.is(ann, json::Type::kObj)) {
        const std::string_view a = d.raw(ann);
        if (memmem(a.data(), a.size(), kReconciled, sizeof kReconciled - 1) != nullptr) drop = false;
      }
    }
  }
  if (drop) {
    ++f.dropped;
    return false;
  }
  make_key();
  if (type == "DELETED") f.forwarded.erase(key);
  else f.forwarded.insert(key);
  return true;
}

// ------------------------------------------------------------------------------ PodWatchStream
PodWatchStream::PodWatchStream(KubeTarget target, std::string path, std::shared_ptr<PodWatchFilter> filter,
                               int read_timeout_s)
    : t_(std::move(target)), path_(std::move(path)), f_(std::move(filter)), timeout_s_(read_timeout_s) {
  if (!f_) throw std::invalid_argument("PodWatchStream: no filter");
  ctx_ = make_ssl_ctx(t_);
  efd_ = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  if (efd_ < 0) {
    free_ssl_ctx(ctx_);
    throw std::runtime_error("PodWatchStream: eventfd failed");
  }
  th_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "ngpu-podwatch");
    run();
  });
}

PodWatchStream::~PodWatchStream() {
  stop();
  ::close(efd_);
  free_ssl_ctx(ctx_);
}

void PodWatchStream::stop() {
  {
    std::lock_guard<std::mutex> g(sock_mu_);
    stop_ = true;
    if (sock_ >= 0) ::shutdown(sock_, SHUT_RDWR);   // wakes the thread's blocking read
  }
  {
    std::lock_guard<std::mutex> g(mu_);   // ... or its wait for the event loop
  }
  drained_.notify_all();
  if (th_.joinable()) th_.join();
}

void PodWatchStream::push(std::vector<std::string>* lines, bool dropped, const std::string& tail_rv, int state,
                          int status, std::string msg) {
  std::lock_guard<std::mutex> g(mu_);
  const bool wake = !lines->empty() || state != kStreaming;
  // the resume point of the events dropped since the last kept one; handed on with the next
  // kept line or the end of the stream, no wake-up of its own (3 of 4 events are dropped)
  if (!lines->empty() || dropped) pending_.last_rv = tail_rv;
  for (auto& l : *lines) pending_.lines.push_back(std::move(l));
  lines->clear();
  if (state != kStreaming) {
    pending_.state = state;
    pending_.status = status;
    pending_.message = std::move(msg);
  }
  if (wake) {
    const uint64_t one = 1;
    (void)!::write(efd_, &one, sizeof one);
  }
}

PodWatchStream::Batch PodWatchStream::take() {
  Batch b;
  {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t v;
    (void)!::read(efd_, &v, sizeof v);
    b = std::move(pending_);
    pending_ = Batch();
    pending_.state = b.state;   // an end stays an end
  }
  drained_.notify_all();
  return b;
}

void PodWatchStream::run() {
  std::vector<std::string> kept;
  HttpConn c(&t_, ctx_, timeout_s_);
  if (!c.start("GET", path_, "", "", kube_token(t_))) {
    push(&kept, false, "", kTransportError, 0, "cannot connect to " + t_.host + ":" + std::to_string(t_.port));
    return;
  }
  {
    std::lock_guard<std::mutex> g(sock_mu_);
    if (stop_) return;
    sock_ = c.fd();
  }
  auto finish = [&](int state, int status, std::string msg) {
    {
      std::lock_guard<std::mutex> g(sock_mu_);
      sock_ = -1;   // the connection closes with `c`; stop() must not shut down a reused fd
    }
    push(&kept, false, "", state, status, std::move(msg));
  };
  std::string body;
  const int status = c.stream_head(&body);
  if (status == 0) return finish(kTransportError, 0, body.empty() ? "watch connection failed" : body);
  if (status != 200) return finish(kHttpError, status, body);
  std::string buf, rv, tail_rv;
  json::Doc d;
  for (;;) {
    const size_t had = buf.size();
    long r;
    {
      const uint64_t io0 = io_t0();
      r = c.stream_read(&buf);
      io_end(kPwRecv, io0);
    }
    if (r == 0) return finish(kEnded, 200, "");
    if (r < 0) return finish(stop_ ? kEnded : kTransportError, 0, "watch stream failed");
    bool dropped = false;
    size_t p = 0, e;
    // only the newly read bytes can hold a newline the last pass did not see
    for (size_t from = had; (e = buf.find('\n', from)) != std::string::npos; from = p) {
      std::string_view line(buf.data() + p, e - p);
      p = e + 1;
      while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.remove_suffix(1);
      if (line.empty()) continue;
      bool keep;
      try {
        IoTimer it{kPwFilter};
        keep = filter_pod_event(*f_, line, d, &rv);
      } catch (const std::invalid_argument&) {
        return finish(kTransportError, 0, "bad watch event line");
      }
      if (keep) {
        kept.emplace_back(line);
        tail_rv.clear();
      } else {
        dropped = true;
        tail_rv = rv;
      }
    }
    buf.erase(0, p);
    if (!kept.empty() || dropped) push(&kept, dropped, tail_rv, kStreaming, 0, "");
    std::unique_lock<std::mutex> lk(mu_);
    drained_.wait(lk, [&] { return pending_.lines.size() < kMaxPending || stop_.load(); });
  }
}

}  // namespace nanogpu
