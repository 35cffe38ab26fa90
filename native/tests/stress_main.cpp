// Native stress test for the sanitizer builds (ASan+UBSan, TSan): no Python involved.
//
//   * T threads reserve / commit / release pods on a shared-memory ledger while a checker
//     thread snapshots every node and asserts 0 <= free <= total on both dimensions;
//   * a second process (fork) attaches to the same /dev/shm ledger and churns too
//     (SO_REUSEPORT workers share one ledger the same way);
//   * a native front door serves filter / priorities to client threads over loopback
//     HTTP while the ledger changes underneath it;
//   * at the end every pod is released and every device must be whole again;
//   * then the native API server and the native bind writers: writer threads bind pods
//     reserved on the ledger (PATCH + binding + commit) while other threads patch the same
//     pods and a watch stream reads every event; every bind must land, no patch may be lost
//     (optimistic writes redo on conflict) and the watch must see every version;
//   * relist reconciliation (Ledger::reconcile): binder threads create, bind and delete pods,
//     some deletions in a watch gap (never released by an event), while a relister LISTs the
//     live set and reconciles; it must never release a live pod and must take back every ghost.
// Exit code 0 = pass. Usage: nanogpu-stress [threads] [iterations]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "nanogpu/apiserver.h"
#include "nanogpu/frontend.h"
#include "nanogpu/kubewriter.h"
#include "nanogpu/podwatch.h"
#include "nanogpu/ledger.h"

using namespace nanogpu;

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::_Exit(1);                                                     \
    }                                                                    \
  } while (0)

static void add_nodes(Ledger& l, int n_nodes) {
  for (int k = 0; k < n_nodes; ++k) {
    Device devs[64];
    std::memset(devs, 0, sizeof(devs));
    const int parts = (k % 2) ? 8 : 1;  // alternate SPX and CPX nodes
    const int n = 8 * parts;
    for (int i = 0; i < n; ++i) {
      devs[i].pct_total = 100;
      devs[i].mib_total = 294896 / parts;
      devs[i].gpu = static_cast<int16_t>(i / parts);
      devs[i].part = static_cast<int16_t>(i % parts);
      devs[i].numa = static_cast<int16_t>((i / parts) / 4);
      devs[i].healthy = 1;
      devs[i].xcds = static_cast<int16_t>(8 / parts);
      devs[i].cus = 256 / parts;
    }
    Topology t;
    std::memset(&t, 0, sizeof(t));
    t.n_gpus = 8;
    for (int a = 0; a < 8; ++a) {
      t.numa[a] = static_cast<int16_t>(a / 4);
      for (int b = 0; b < 8; ++b) t.link_bw[a * kMaxGpus + b] = a == b ? 0.f : 76.f;
    }
    CHECK(l.upsert_node("node-" + std::to_string(k), devs, n, t) == k);
  }
}

static void churn(Ledger& l, int n_nodes, int seed, int iters, std::atomic<int>* reserved) {
  std::mt19937_64 rng(seed);
  std::vector<std::string> live;
  Options o;
  for (int it = 0; it < iters; ++it) {
    o.policy = static_cast<Policy>(rng() % 4);
    Demand d;
    std::memset(&d, 0, sizeof(d));
    // one pod in 16 is wide (20 containers): its record spills into an overflow record
    d.n = rng() % 16 == 0 ? 20 : 1 + static_cast<int>(rng() % 3);
    static const int pcts[] = {0, 10, 25, 50, 100, 200};
    for (int c = 0; c < d.n; ++c) {
      d.c[c].pct = d.n > 16 ? 5 * static_cast<int>(rng() % 2) : pcts[rng() % 6];
      d.c[c].mib = d.n > 16 ? 0 : static_cast<int64_t>(rng() % 4) * 8192;
    }
    const int node = static_cast<int>(rng() % n_nodes);
    const std::string key = "s" + std::to_string(seed) + "-" + std::to_string(it);
    Plan p;
    const int32_t rc = l.reserve(node, key, d, o, &p);
    if (rc == kOk) {
      reserved->fetch_add(1);
      if (rng() % 4) CHECK(l.commit(key) == kOk);
      CHECK(l.set_pod_owner(key, owner_hash("owner-" + std::to_string(rng() % 8))) == kOk);
      live.push_back(key);
    }
    if (!live.empty() && rng() % 3 == 0) {
      const size_t i = rng() % live.size();
      CHECK(l.release(live[i]) == kOk);
      live.erase(live.begin() + static_cast<long>(i));
    }
  }
  for (const auto& k : live) CHECK(l.release(k) == kOk);
}

static std::string http(int port, const std::string& method, const std::string& path, const std::string& body) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  CHECK(connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0);
  const std::string req = method + " " + path + " HTTP/1.1\r\nHost: x\r\nConnection: close\r\nContent-Length: " +
                          std::to_string(body.size()) + "\r\n\r\n" + body;
  CHECK(send(fd, req.data(), req.size(), MSG_NOSIGNAL) == static_cast<ssize_t>(req.size()));
  std::string out;
  char buf[4096];
  for (;;) {
    const ssize_t r = recv(fd, buf, sizeof(buf), 0);
    if (r <= 0) break;
    out.append(buf, static_cast<size_t>(r));
  }
  close(fd);
  return out;
}

// Watch-gap deletions under concurrency (see the header comment). The "API server" is a set of
// live pod keys: a pod is created (inserted) before it is bound and deleted (erased) before its
// release event, like the real ordering.
static void relist_gap(int iters) {
  Ledger l("", 8, 65536, true);
  add_nodes(l, 4);
  std::mutex api_mu;
  std::unordered_set<std::string> api;
  std::atomic<bool> done{false};
  std::atomic<int> ghosts{0}, reconciled{0};
  std::thread relister([&] {
    while (!done.load()) {
      const double before = mono_now();
      std::vector<std::string> listed;
      {
        std::lock_guard<std::mutex> g(api_mu);
        listed.assign(api.begin(), api.end());
      }
      reconciled.fetch_add(static_cast<int>(l.reconcile(listed, before).size()));
    }
  });
  std::vector<std::thread> binders;
  for (int t = 0; t < 3; ++t)
    binders.emplace_back([&, t] {
      std::mt19937_64 rng(500 + t);
      std::vector<std::string> mine;
      Options o;
      for (int i = 0; i < iters; ++i) {
        const std::string key = "g" + std::to_string(t) + "-" + std::to_string(i);
        {
          std::lock_guard<std::mutex> g(api_mu);
          api.insert(key);
        }
        Demand d;
        std::memset(&d, 0, sizeof(d));
        d.n = 1;
        d.c[0].pct = 10;
        Plan p;
        if (l.reserve(static_cast<int32_t>(rng() % 4), key, d, o, &p) == kOk) {
          CHECK(l.commit(key) == kOk);
          mine.push_back(key);
        } else {
          std::lock_guard<std::mutex> g(api_mu);
          api.erase(key);
        }
        if (!mine.empty() && rng() % 2 == 0) {
          const size_t j = rng() % mine.size();
          const std::string k = mine[j];
          mine.erase(mine.begin() + static_cast<long>(j));
          {
            std::lock_guard<std::mutex> g(api_mu);
            api.erase(k);
          }
          if (rng() % 2) {
            const int32_t rc = l.release(k);   // the DELETED event (a relist may have been first)
            CHECK(rc == kOk || rc == kErrUnknownPod);
          } else {
            ghosts.fetch_add(1);               // deleted while the watch was down
          }
        }
      }
      // every pod still in the API server must still hold its share: reconcile never took it
      for (const auto& k : mine) {
        PodRecord rec;
        CHECK(l.lookup(k, &rec));
        {
          std::lock_guard<std::mutex> g(api_mu);
          api.erase(k);
        }
        // deleted from the API server first: a relist in between may release it before we do
        const int32_t rc = l.release(k);
        CHECK(rc == kOk || rc == kErrUnknownPod);
      }
    });
  for (auto& b : binders) b.join();
  done.store(true);
  relister.join();
  reconciled.fetch_add(static_cast<int>(l.reconcile({}, mono_now() + 1.0).size()));
  CHECK(l.n_pods() == 0);
  CHECK(reconciled.load() >= ghosts.load());
  for (int k = 0; k < 4; ++k) {
    NodeSnapshot s;
    CHECK(l.snapshot(k, &s));
    for (int i = 0; i < s.n_devs; ++i) CHECK(s.devs[i].pct_free == s.devs[i].pct_total);
  }
  std::printf("relist ok: %d ghosts, %d reconciled\n", ghosts.load(), reconciled.load());
}

// Relist reconciliation at cluster scale: `pods` committed pods on 256 nodes, a LIST that
// returns all but 1 %, reconciled while a front-door stand-in reserves and releases on the same
// ledger. Prints the best-of-3 reconcile time and the slowest reserve seen during a walk, best
// of 3 as well: a lock held across the walk stalls a reserve in every round, a preemption of the
// stand-in's thread on a busy host in one (tests/test_relist_scale.py pins both).
// Usage: nanogpu-stress relist-scale [pods]
static void relist_scale(int pods) {
  const int n_nodes = 256;
  Ledger l("", n_nodes, std::max(131072, pods + 4096), true);
  for (int k = 0; k < n_nodes; ++k) {
    Device devs[8];
    std::memset(devs, 0, sizeof(devs));
    for (int i = 0; i < 8; ++i) {
      devs[i].pct_total = 100;
      devs[i].mib_total = 294896;
      devs[i].gpu = static_cast<int16_t>(i);
      devs[i].healthy = 1;
      devs[i].xcds = 8;
      devs[i].cus = 256;
    }
    Topology t;
    std::memset(&t, 0, sizeof(t));
    t.n_gpus = 8;
    CHECK(l.upsert_node("node-" + std::to_string(k), devs, 8, t) == k);
  }
  double best_ms = 1e9, reserve_max_ms = 1e9;
  size_t released_total = 0;
  for (int round = 0; round < 3; ++round) {
    std::vector<std::string> keys;
    keys.reserve(static_cast<size_t>(pods));
    Options o;
    Demand d;
    std::memset(&d, 0, sizeof(d));
    d.n = 1;
    d.c[0].pct = 0;
    d.c[0].mib = 1;   // HBM only: 100k pods fit 256 nodes
    for (int i = 0; i < pods; ++i) {
      char uid[48];
      std::snprintf(uid, sizeof uid, "%08x-0000-4000-8000-%012d", round, i);
      keys.emplace_back(uid);
      Plan p;
      CHECK(l.reserve(i % n_nodes, keys.back(), d, o, &p) == kOk);
      CHECK(l.commit(keys.back()) == kOk);
    }
    const double before = mono_now() + 1.0;
    std::vector<std::string_view> live;
    for (int i = 0; i < pods; ++i)
      if (i % 100 != 0) live.emplace_back(keys[static_cast<size_t>(i)]);
    std::atomic<bool> walking{true};
    double worst = 0.0;
    std::thread fd([&] {   // the front door: reserve + release while the walk runs
      int n = 0;
      while (walking.load(std::memory_order_relaxed)) {
        const std::string k = "fd-" + std::to_string(n++);
        Plan p;
        const auto t0 = std::chrono::steady_clock::now();
        const int32_t rc = l.reserve(n % n_nodes, k, d, o, &p);
        worst = std::max(worst, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        if (rc == kOk) CHECK(l.release(k) == kOk);
      }
    });
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<std::string> gone = l.reconcile_views(live, before);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    walking.store(false);
    fd.join();
    CHECK(gone.size() == static_cast<size_t>((pods + 99) / 100));
    best_ms = std::min(best_ms, ms);
    reserve_max_ms = std::min(reserve_max_ms, worst);
    released_total += gone.size();
    for (const std::string_view k : live) CHECK(l.release(std::string(k)) == kOk);
    CHECK(l.n_pods() == 0);
  }
  std::printf("relist_scale {\"pods\": %d, \"reconcile_ms\": %.3f, \"reserve_max_ms\": %.3f, \"released\": %zu}\n",
              pods, best_ms, reserve_max_ms, released_total);
}

// Bind handoff slots (Ledger::put_pod_info / take_pod_info) under concurrency: writers and
// takers on colliding slots never see a torn or foreign blob.
static void handoff(int iters) {
  Ledger l("", 8, 1024, true);   // 1024 slots: keys collide on purpose
  std::atomic<int> taken{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      std::string blob;
      for (int i = 0; i < iters; ++i) {
        const std::string key = "h" + std::to_string(t) + "-" + std::to_string(i % 700);
        const std::string want(64 + (i % 200), static_cast<char>('a' + t));
        CHECK(l.put_pod_info(key, want + key));
        const std::string other = "h" + std::to_string((t + 1) % 4) + "-" + std::to_string(i % 700);
        for (const std::string* k : {&key, &other}) {
          if (!l.take_pod_info(*k, &blob)) continue;
          // a blob always ends with its own key and is one writer's byte repeated before it
          CHECK(blob.size() > k->size() && blob.compare(blob.size() - k->size(), k->size(), *k) == 0);
          const char c = blob[0];
          for (size_t j = 0; j + k->size() < blob.size(); ++j) CHECK(blob[j] == c);
          taken.fetch_add(1);
        }
      }
    });
  for (auto& t : ts) t.join();
  CHECK(taken.load() > 0);
  std::printf("handoff ok: %d taken\n", taken.load());
}

// Native API server + native bind writers under concurrency (see the header comment).
static void apiserver_and_writers(int pods, bool evented) {
  apisrv::Config cfg;
  cfg.threads = 2;
  apisrv::Server srv(cfg);
  const int port = srv.port();
  CHECK(http(port, "POST", "/api/v1/nodes", "{\"metadata\":{\"name\":\"n0\"}}").rfind("HTTP/1.1 201", 0) == 0);
  std::vector<std::string> texts;
  for (int i = 0; i < pods; ++i)
    texts.push_back("{\"metadata\":{\"name\":\"p" + std::to_string(i) + "\",\"namespace\":\"s\",\"uid\":\"w" +
                    std::to_string(i) + "\"},\"spec\":{\"containers\":[{\"name\":\"c\"}]},\"status\":{\"phase\":\"Pending\"}}");
  for (int c : srv.create_pods(texts)) CHECK(c == 201);

  // watch from the current version: every later write must arrive
  const std::string list = http(port, "GET", "/api/v1/pods", "");
  const size_t rvp = list.find("\"resourceVersion\":\"");
  CHECK(rvp != std::string::npos);
  const std::string rv0 = list.substr(rvp + 19, list.find('"', rvp + 19) - rvp - 19);
  std::atomic<int> events{0};
  std::atomic<bool> stop_watch{false};
  std::thread watcher([&] {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    CHECK(connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0);
    timeval tv{0, 200000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    const std::string req = "GET /api/v1/pods?watch=1&resourceVersion=" + rv0 + " HTTP/1.1\r\nHost: x\r\n\r\n";
    CHECK(send(fd, req.data(), req.size(), MSG_NOSIGNAL) == static_cast<ssize_t>(req.size()));
    char buf[65536];
    while (!stop_watch.load()) {
      const ssize_t r = recv(fd, buf, sizeof(buf), 0);
      if (r <= 0) continue;
      for (ssize_t i = 0; i + 7 < r; ++i)
        if (std::memcmp(buf + i, "\"type\":", 7) == 0) events.fetch_add(1);
    }
    close(fd);
  });

  auto ledger = std::make_shared<Ledger>("", 8, 4096, true);
  Device devs[8];
  std::memset(devs, 0, sizeof(devs));
  for (int i = 0; i < 8; ++i) {
    devs[i].pct_total = 100;
    devs[i].mib_total = 294896;
    devs[i].gpu = static_cast<int16_t>(i);
    devs[i].healthy = 1;
    devs[i].xcds = 8;
    devs[i].cus = 256;
  }
  Topology t;
  std::memset(&t, 0, sizeof(t));
  t.n_gpus = 8;
  const int32_t nid = ledger->upsert_node("n0", devs, 8, t);
  CHECK(nid >= 0);

  std::atomic<int> ok{0}, bad{0};
  KubeTarget tgt;
  tgt.host = "127.0.0.1";
  tgt.port = port;
  tgt.tls = false;
  // the pod informer's native watch on the same stream: every event here is one the filter
  // drops (pending pods, bound pods the ledger holds, deletions of pods Python never saw,
  // released right in the stream thread) while a consumer drains it as the event loop would
  auto filter = std::make_shared<PodWatchFilter>();
  filter->ledger = ledger;
  PodWatchStream pw(tgt, "/api/v1/pods?watch=1&resourceVersion=" + rv0, filter, 30);
  std::atomic<bool> stop_take{false};
  std::atomic<int> kept{0};
  std::thread taker([&] {
    while (!stop_take.load()) {
      kept.fetch_add(static_cast<int>(pw.take().lines.size()));
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  {
    KubeWriter kw(
        tgt, ledger,
        [&](uint64_t, int status, const std::string& body) {
          if (status == 200 && body == "{\"Error\":\"\"}") ok.fetch_add(1);
          else bad.fetch_add(1);
        },
        4, 2, false, evented);
    std::vector<std::thread> patchers;
    for (int t2 = 0; t2 < 2; ++t2)
      patchers.emplace_back([&, t2] {
        for (int i = 0; i < pods; ++i)
          CHECK(http(port, "PATCH", "/api/v1/namespaces/s/pods/p" + std::to_string(i),
                     "{\"metadata\":{\"annotations\":{\"k" + std::to_string(t2) + "\":\"v\"}}}")
                    .rfind("HTTP/1.1 200", 0) == 0);
      });
    for (int i = 0; i < pods; ++i) {
      Demand dm;
      std::memset(&dm, 0, sizeof(dm));
      dm.n = 1;
      dm.c[0].pct = 1;
      Plan plan;
      std::memset(&plan, 0, sizeof(plan));
      Options o;
      CHECK(ledger->reserve(nid, "w" + std::to_string(i), dm, o, &plan) == kOk);
      BindJob j;
      j.id = static_cast<uint64_t>(i);
      j.ns = "s";
      j.name = "p" + std::to_string(i);
      j.uid = "w" + std::to_string(i);
      j.node = "n0";
      j.containers = {"c"};
      j.plan = {{plan.idx[plan.off[0]]}};
      kw.submit(std::move(j));
    }
    for (auto& p2 : patchers) p2.join();
    for (int spin = 0; ok.load() + bad.load() < pods && spin < 3000; ++spin)
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    kw.stop();
  }
  CHECK(ok.load() == pods && bad.load() == 0);
  for (int i = 0; i < pods; ++i) {
    const std::string r = http(port, "GET", "/api/v1/namespaces/s/pods/p" + std::to_string(i), "");
    CHECK(r.find("\"nodeName\":\"n0\"") != std::string::npos);          // bound
    CHECK(r.find("\"k0\":\"v\"") != std::string::npos && r.find("\"k1\":\"v\"") != std::string::npos);   // no lost patch
    CHECK(r.find("\"nano-gpu/container-c\"") != std::string::npos);
    PodRecord rec;
    CHECK(ledger->lookup("w" + std::to_string(i), &rec));
  }
  // every write after rv0 reached the watch: 2 patches + placement PATCH + binding per pod
  for (int spin = 0; events.load() < 4 * pods && spin < 1000; ++spin)
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  stop_watch.store(true);
  watcher.join();
  CHECK(events.load() == 4 * pods);
  // deletes racing patches on the same pods (a delete re-stamps the object while a patch may
  // be building its tree outside the store lock)
  {
    std::thread patcher([&] {
      for (int i = 0; i < pods; ++i)
        http(port, "PATCH", "/api/v1/namespaces/s/pods/p" + std::to_string(i), "{\"metadata\":{\"labels\":{\"x\":\"y\"}}}");
    });
    std::thread deleter([&] {
      for (int i = 0; i < pods; ++i) {
        const std::string r = http(port, "DELETE", "/api/v1/namespaces/s/pods/p" + std::to_string(i), "");
        CHECK(r.rfind("HTTP/1.1 200", 0) == 0);
      }
    });
    patcher.join();
    deleter.join();
    CHECK(http(port, "GET", "/api/v1/namespaces/s/pods", "").find("\"items\":[]") != std::string::npos);
  }
  auto released = [&] {
    std::lock_guard<std::mutex> g(filter->mu);
    return filter->released;
  };
  for (int spin = 0; released() < static_cast<uint64_t>(pods) && spin < 2000; ++spin)
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  pw.stop();   // mid-stream: shuts the socket down under the reading thread
  stop_take.store(true);
  taker.join();
  CHECK(released() == static_cast<uint64_t>(pods) && kept.load() == 0 && ledger->n_pods() == 0);
  {
    std::lock_guard<std::mutex> g(filter->mu);
    CHECK(filter->dropped >= static_cast<uint64_t>(5 * pods));
  }
  srv.stop();
  std::printf("apiserver ok: %d pods bound by native writers, %d watch events\n", pods, events.load());
}

static std::string post(int port, const std::string& path, const std::string& body);

// A scenario step that has not finished within `secs` prints `what()` (the step's progress)
// and aborts: a hang names itself instead of running into the test's timeout.
class Watchdog {
 public:
  template <class F>
  Watchdog(const char* step, int secs, F what) : th_([this, step, secs, what] {
    // polls a flag (no mutex: a std::mutex reused at a stack address confuses TSan)
    const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(secs);
    while (!done_.load()) {
      if (std::chrono::steady_clock::now() >= end) {
        std::fprintf(stderr, "WATCHDOG: %s still running after %d s: %s\n", step, secs, what().c_str());
        std::fflush(stderr);
        std::abort();
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  }) {}
  ~Watchdog() {
    done_.store(true);
    th_.join();
  }

 private:
  std::atomic<bool> done_{false};
  std::thread th_;
};

// Inline bind writes (Frontend::set_kube_writer inline_io): client threads send filter + bind
// over HTTP to a 2-worker front door whose workers drive the binds' API requests to the native
// API server from their own epoll loops; every bind must be answered, bound and committed, and
// the front door must stop cleanly with the writer.
static void inline_binds(int pods, bool frontdoor = false) {
  apisrv::Config cfg;
  cfg.threads = 2;
  apisrv::Server srv(cfg);
  const int port = srv.port();
  CHECK(http(port, "POST", "/api/v1/nodes", "{\"metadata\":{\"name\":\"n0\"}}").rfind("HTTP/1.1 201", 0) == 0);
  std::vector<std::string> texts;
  for (int i = 0; i < pods; ++i)
    texts.push_back("{\"metadata\":{\"name\":\"q" + std::to_string(i) + "\",\"namespace\":\"s\",\"uid\":\"iq" +
                    std::to_string(i) + "\"},\"spec\":{\"containers\":[{\"name\":\"c\",\"resources\":{\"limits\":"
                    "{\"nano-gpu/gpu-percent\":\"1\"}}}]},\"status\":{\"phase\":\"Pending\"}}");
  for (int c : srv.create_pods(texts)) CHECK(c == 201);
  auto ledger = std::make_shared<Ledger>("", 8, 4096, true);
  Device devs[8];
  std::memset(devs, 0, sizeof(devs));
  for (int i = 0; i < 8; ++i) {
    devs[i].pct_total = 100;
    devs[i].mib_total = 294896;
    devs[i].gpu = static_cast<int16_t>(i);
    devs[i].healthy = 1;
    devs[i].xcds = 8;
    devs[i].cus = 256;
  }
  Topology t;
  std::memset(&t, 0, sizeof(t));
  t.n_gpus = 8;
  CHECK(ledger->upsert_node("n0", devs, 8, t) == 0);
  {
    Frontend fe(ledger, "127.0.0.1", 0, 2);
    fe.set_busy_poll_us(20);
    Options fo;
    fe.set_options(fo, true);
    KubeTarget tgt;
    tgt.host = "127.0.0.1";
    tgt.port = port;
    tgt.tls = false;
    // frontdoor: the evented writer's io thread reads the answers, the workers send the binds
    fe.set_kube_writer(tgt, 2, 2, false, true, true, 30.0, !frontdoor);
    if (frontdoor) fe.set_fe_send(true);
    std::vector<std::thread> clients;
    std::atomic<int> ok{0};
    std::atomic<int> sent[4] = {{-1}, {-1}, {-1}, {-1}};
    const KubeWriter* kw0 = fe.kube_writer();
    auto progress = [&] {
      std::string m = "answered " + std::to_string(ok.load()) + "/" + std::to_string(pods) + "; client's last bind";
      for (auto& x : sent) m += " " + std::to_string(x.load());
      if (kw0)
        m += "; writer ok " + std::to_string(kw0->stats.ok.load()) + " failed " + std::to_string(kw0->stats.failed.load()) +
             " inflight " + std::to_string(kw0->stats.inflight.load()) + " retries " + std::to_string(kw0->stats.retries.load()) +
             " timeouts " + std::to_string(kw0->stats.timeouts.load());
      return m;
    };
    Watchdog wd(frontdoor ? "frontdoor binds" : "inline binds", 45, progress);
    for (int c = 0; c < 4; ++c)
      clients.emplace_back([&, c] {
        for (int i = c; i < pods; i += 4) {
          sent[c].store(i);
          const std::string pod = texts[static_cast<size_t>(i)];
          CHECK(post(fe.port(), "/scheduler/filter", "{\"Pod\":" + pod + ",\"NodeNames\":[\"n0\"]}")
                    .rfind("HTTP/1.1 200", 0) == 0);
          const std::string r = post(fe.port(), "/scheduler/bind",
                                     "{\"PodName\":\"q" + std::to_string(i) + "\",\"PodNamespace\":\"s\",\"PodUID\":\"iq" +
                                         std::to_string(i) + "\",\"Node\":\"n0\"}");
          CHECK(r.rfind("HTTP/1.1 200", 0) == 0 && r.find("{\"Error\":\"\"}") != std::string::npos);
          ok.fetch_add(1);
        }
      });
    for (auto& c : clients) c.join();
    CHECK(ok.load() == pods);
    const KubeWriter* kw = fe.kube_writer();
    CHECK(kw && kw->stats.ok.load() == static_cast<uint64_t>(pods));
    fe.stop();
  }
  for (int i = 0; i < pods; ++i) {
    const std::string r = http(port, "GET", "/api/v1/namespaces/s/pods/q" + std::to_string(i), "");
    CHECK(r.find("\"nodeName\":\"n0\"") != std::string::npos);
    PodRecord rec;
    CHECK(ledger->lookup("iq" + std::to_string(i), &rec) && rec.state == kPodCommitted);
  }
  srv.stop();
  std::printf("%s ok: %d binds written from the front-door workers\n", frontdoor ? "frontdoor" : "inline", pods);
}

static std::string post(int port, const std::string& path, const std::string& body) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  CHECK(connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0);
  const std::string req = "POST " + path + " HTTP/1.1\r\nHost: x\r\nConnection: close\r\nContent-Length: " +
                          std::to_string(body.size()) + "\r\n\r\n" + body;
  CHECK(send(fd, req.data(), req.size(), MSG_NOSIGNAL) == static_cast<ssize_t>(req.size()));
  std::string out;
  char buf[4096];
  for (;;) {
    const ssize_t r = recv(fd, buf, sizeof(buf), 0);
    if (r <= 0) break;
    out.append(buf, static_cast<size_t>(r));
  }
  close(fd);
  return out;
}

// Responses posted from another thread (the bind writer's and Python's path) while front-door
// workers alternate between busy polling, handling batches and blocking in epoll_wait: every
// request must be answered whether the poster saw its worker parked (eventfd) or awake (the
// worker's own mailbox check). Pauses of random length let the workers park between posts.
static void mailbox_wakeups(int requests) {
  auto ledger = std::make_shared<Ledger>("", 4, 1024, true);
  Frontend fe(ledger, "127.0.0.1", 0, 2);
  fe.set_busy_poll_us(20);
  std::atomic<bool> stop{false};
  std::atomic<int> answered{0};
  std::thread py([&] {
    std::mt19937_64 rng(5);
    pollfd pf{fe.notify_fd(), POLLIN, 0};
    while (!stop.load()) {
      if (poll(&pf, 1, 20) <= 0) continue;
      std::vector<PyRequest> rs = fe.take();
      for (size_t i = 0; i < rs.size(); ++i) {
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
        const bool notify = rng() % 3 != 0;
        fe.respond(rs[i].id, 200, "application/json", "{\"ok\":" + std::to_string(i) + "}", notify);
        answered.fetch_add(1);
      }
      fe.wake_workers();
    }
  });
  std::vector<std::thread> clients;
  for (int c = 0; c < 4; ++c)
    clients.emplace_back([&, c] {
      std::mt19937_64 rng(100 + c);
      for (int i = 0; i < requests / 4; ++i) {
        if (rng() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 500));
        const std::string r = post(fe.port(), "/not-native", "{}");
        CHECK(r.rfind("HTTP/1.1 200", 0) == 0 && r.find("{\"ok\":") != std::string::npos);
      }
    });
  for (auto& c : clients) c.join();
  stop.store(true);
  py.join();
  CHECK(answered.load() == requests / 4 * 4);
  fe.stop();
  std::printf("mailbox ok: %d posted responses, %llu needed a wake-up\n", answered.load(),
              static_cast<unsigned long long>(fe.mb_wakeups.load()));
}

// Filter-path memo re-validation (Ledger::assume_many: change ring, runner-up bound, fast scan)
// and wide records (Ledger::reserve_wide) under concurrency: reader threads run assume_many over
// every node while writer threads reserve, release and account wide pods. Quiescent at the end,
// every memoised answer must equal a fresh choose() on the node's state, and every wide record
// must be free again.
static void memo_and_wide(int iters) {
  Ledger l("", 16, 65536, true);
  const int n_nodes = 6;
  add_nodes(l, n_nodes);
  std::atomic<bool> stop{false};
  Options bin;
  std::vector<std::thread> ts;
  std::vector<int32_t> ids(n_nodes);
  for (int k = 0; k < n_nodes; ++k) ids[k] = k;
  auto shape = [](std::mt19937_64& rng) {
    Demand d;
    std::memset(&d, 0, sizeof(d));
    static const int pcts[] = {5, 10, 25, 50, 100};
    d.n = 1;
    d.c[0].pct = pcts[rng() % 5];
    d.c[0].mib = static_cast<int64_t>(rng() % 3) * 16384;
    d.c[0].flags = rng() % 4 == 0 ? kFlagMemBound : 0;
    return d;
  };
  for (int r = 0; r < 2; ++r)
    ts.emplace_back([&, r] {
      std::mt19937_64 rng(100 + r);
      std::vector<int32_t> rc(n_nodes), sc(n_nodes);
      while (!stop.load()) {
        const Demand d = shape(rng);
        l.assume_many(ids.data(), n_nodes, d, bin, rc.data(), sc.data());
        for (int k = 0; k < n_nodes; ++k) CHECK(rc[k] != kErrUnknownNode);
      }
    });
  std::vector<std::thread> ws;
  for (int w = 0; w < 3; ++w)
    ws.emplace_back([&, w] {
      std::mt19937_64 rng(200 + w);
      std::vector<std::string> live;
      for (int it = 0; it < iters; ++it) {
        const std::string key = "m" + std::to_string(w) + "-" + std::to_string(it);
        const int node = static_cast<int>(rng() % n_nodes);
        if (rng() % 8 == 0) {
          // a wide pod: 70 x 1 % on the first devices, folded per device
          WidePlan wide(70);
          Demand folded;
          std::memset(&folded, 0, sizeof(folded));
          folded.n = 2;
          folded.c[0].pct = 35;
          folded.c[1].pct = 35;
          for (int c = 0; c < 70; ++c) wide[static_cast<size_t>(c)] = {c % 2};
          Plan fp;
          std::memset(&fp, 0, sizeof(fp));
          fp.n = 2;
          fp.off[0] = 0, fp.off[1] = 1, fp.off[2] = 2;
          fp.idx[0] = 0, fp.idx[1] = 1;
          WidePlan held;
          const int32_t rc = l.reserve_wide(node, key, folded, fp, wide, rng() % 2 == 0, &held);
          if (rc == kOk) {
            WidePlan got;
            CHECK(l.wide_plan(key, &got) && got == wide);
            CHECK(l.reserve_wide(node, key, folded, fp, wide, true, &held) == kOkExisting && held == wide);
            live.push_back(key);
          }
        } else {
          const Demand d = shape(rng);
          Plan p;
          if (l.reserve(node, key, d, bin, &p) == kOk) live.push_back(key);
        }
        if (!live.empty() && rng() % 3 == 0) {
          const size_t i = rng() % live.size();
          CHECK(l.release(live[i]) == kOk);
          live.erase(live.begin() + static_cast<long>(i));
        }
      }
      for (const auto& k : live) CHECK(l.release(k) == kOk);
    });
  for (auto& w : ws) w.join();
  stop.store(true);
  for (auto& t : ts) t.join();
  CHECK(l.n_pods() == 0 && l.wide_records_used() == 0);
  // quiescent: memoised (and re-validated) answers equal fresh placements
  std::mt19937_64 rng(300);
  std::vector<int32_t> rc(n_nodes), sc(n_nodes);
  for (int q = 0; q < 200; ++q) {
    const Demand d = shape(rng);
    Plan p;
    l.reserve(static_cast<int32_t>(rng() % n_nodes), "q" + std::to_string(q), d, bin, &p);
    l.assume_many(ids.data(), n_nodes, d, bin, rc.data(), sc.data());
    l.clear_cache();
    for (int k = 0; k < n_nodes; ++k) {
      const int32_t r2 = l.assume(k, d, bin, &p);
      CHECK(rc[k] == r2);
      if (r2 == kOk) CHECK(sc[k] == p.score);
    }
  }
  std::printf("memo + wide ok: %d iterations x 3 writers, 2 readers\n", iters);
}

// Nominations adopted by binds on other threads while sweepers drop them: a bind adopts its
// pod's nomination under the pod shard's lock alone (Ledger::reserve_as), a sweep releases a
// nomination under node + shard lock only while it is still one (release_if re-checks), and a
// bind to another node than the nomination releases it and reserves afresh. Whatever wins each
// race, every device is whole again once every pod is released, and no pod is counted twice.
static void nominate_adopt(int iters) {
  Ledger l("", 8, 65536, true);
  add_nodes(l, 4);
  std::mutex mu;
  std::deque<std::pair<std::string, int>> nominated;   // (key, node) waiting for a bind
  std::atomic<bool> done{false};
  std::thread nominator([&] {
    std::mt19937_64 rng(5);
    Options o;
    for (int i = 0; i < iters; ++i) {
      Demand d;
      std::memset(&d, 0, sizeof(d));
      d.n = 1;
      d.c[0].pct = 10 * (1 + static_cast<int>(rng() % 5));
      d.c[0].mib = static_cast<int64_t>(rng() % 3) * 8192;
      const int node = static_cast<int>(rng() % 4);
      const std::string key = "nom-" + std::to_string(i);
      const int32_t rc = l.nominate(node, key, d, o);
      CHECK(rc == kOk || rc == kOkExisting || rc == kErrNoFit || rc == kErrNoDevices);
      std::lock_guard<std::mutex> g(mu);
      nominated.emplace_back(key, node);
    }
    done.store(true);
  });
  std::vector<std::thread> binders;
  std::mutex live_mu;
  std::vector<std::string> live;
  for (int t = 0; t < 2; ++t)
    binders.emplace_back([&, t] {
      std::mt19937_64 rng(100 + t);
      Options o;
      for (;;) {
        std::pair<std::string, int> job;
        {
          std::lock_guard<std::mutex> g(mu);
          if (nominated.empty()) {
            if (done.load()) break;
            continue;
          }
          job = nominated.front();
          nominated.pop_front();
        }
        Demand d;
        std::memset(&d, 0, sizeof(d));
        d.n = 1;
        d.c[0].pct = 10;
        // one bind in five goes to another node than its nomination (kube-scheduler's pick)
        const int node = rng() % 5 == 0 ? (job.second + 1) % 4 : job.second;
        Plan p;
        const int32_t rc = l.reserve(node, job.first, d, o, &p);
        if (rc == kOk || rc == kOkExisting) {
          if (l.commit(job.first) == kOk) {
            std::lock_guard<std::mutex> g(live_mu);
            live.push_back(job.first);
          }
        }
        {   // an older pod deleted (the cluster stays about half full)
          std::string k;
          {
            std::lock_guard<std::mutex> g(live_mu);
            if (live.size() > 24 || (!live.empty() && rng() % 3 == 0)) {
              const size_t i = rng() % live.size();
              k = live[i];
              live.erase(live.begin() + static_cast<long>(i));
            }
          }
          if (!k.empty()) CHECK(l.release(k) == kOk);
        }
      }
    });
  std::thread sweeper([&] {   // the nomination TTL sweep, at TTL 0: every nomination is fair game
    while (!done.load()) {
      for (const std::string& k : l.expired_nominations(0.0)) l.drop_nomination(k);
    }
  });
  nominator.join();
  for (auto& b : binders) b.join();
  sweeper.join();
  for (const std::string& k : l.expired_nominations(-1.0)) CHECK(l.drop_nomination(k) == kOk);
  for (const std::string& k : live) CHECK(l.release(k) == kOk);
  for (int k = 0; k < 4; ++k) {
    NodeSnapshot s;
    CHECK(l.snapshot(k, &s));
    for (int i = 0; i < s.n_devs; ++i) {
      CHECK(s.devs[i].pct_free == s.devs[i].pct_total);
      CHECK(s.devs[i].mib_free == s.devs[i].mib_total);
    }
  }
  CHECK(l.n_pods() == 0);
  uint64_t made = 0, adopted = 0, moved = 0;
  l.nomination_counts(&made, &adopted, &moved);
  std::printf("nominate/adopt ok: %d pods, %llu nominated, %llu adopted, %llu moved\n", iters,
              static_cast<unsigned long long>(made), static_cast<unsigned long long>(adopted),
              static_cast<unsigned long long>(moved));
}

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);   // each scenario's line out as it passes (a hang names its scenario)
  if (argc > 1 && std::strcmp(argv[1], "relist-scale") == 0) {
    relist_scale(argc > 2 ? std::atoi(argv[2]) : 100000);
    return 0;
  }
  const int threads = argc > 1 ? std::atoi(argv[1]) : 4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  const int n_nodes = 6;
  const std::string path = "/dev/shm/nanogpu-stress-" + std::to_string(getpid());
  auto ledger = std::make_shared<Ledger>(path, 64, 65536, true);
  add_nodes(*ledger, n_nodes);

  // second process on the same shared ledger
  const pid_t child = fork();
  if (child == 0) {
    Ledger other(path, 64, 65536, true);
    std::atomic<int> r{0};
    churn(other, n_nodes, 9999, iters, &r);
    std::_Exit(0);
  }

  std::atomic<bool> done{false};
  std::atomic<int> reserved{0};
  // telemetry worker: HBM-hot marks flip and the streaming-owner learner scans the pod table
  // while pods are reserved, committed and released around it
  std::thread learner([&] {
    std::mt19937_64 rng(77);
    while (!done.load()) {
      CHECK(ledger->set_mem_hot(static_cast<int32_t>(rng() % n_nodes), static_cast<int>(rng() % 8),
                                rng() % 2 == 0) == kOk);
      ledger->learn_stream_owners(true);
    }
  });
  std::thread checker([&] {
    while (!done.load()) {
      for (int k = 0; k < n_nodes; ++k) {
        NodeSnapshot s;
        CHECK(ledger->snapshot(k, &s));
        for (int i = 0; i < s.n_devs; ++i) {
          CHECK(s.devs[i].pct_free >= 0 && s.devs[i].pct_free <= s.devs[i].pct_total);
          CHECK(s.devs[i].mib_free >= 0 && s.devs[i].mib_free <= s.devs[i].mib_total);
        }
      }
    }
  });

  Frontend fe(ledger, "127.0.0.1", 0, 2);
  Options fo;
  fe.set_options(fo, true);
  std::vector<std::thread> clients;
  for (int c = 0; c < 2; ++c)
    clients.emplace_back([&, c] {
      for (int i = 0; i < iters / 20; ++i) {
        const std::string body =
            "{\"Pod\":{\"metadata\":{\"uid\":\"u" + std::to_string(c * 100000 + i) +
            "\"},\"spec\":{\"containers\":[{\"name\":\"c\",\"resources\":{\"limits\":{\"nano-gpu/gpu-percent\":\"" +
            std::to_string(10 * (1 + i % 9)) + "\",\"nano-gpu/gpu-memory\":\"8Gi\"}}}]}},"
            "\"NodeNames\":[\"node-0\",\"node-1\",\"node-2\",\"node-3\",\"node-4\",\"node-5\"]}";
        const std::string r = post(fe.port(), i % 2 ? "/scheduler/priorities" : "/scheduler/filter", body);
        CHECK(r.rfind("HTTP/1.1 200", 0) == 0);
        // the options change under the workers now and then: the decisive filter (one node
        // answered) on and off, picked up by each worker's next request (no nominations: the
        // devices must all be free at the end)
        if (c == 1 && i % 7 == 3) fe.set_options(fo, true, false, (i / 7) % 2 == 0);
      }
    });

  std::vector<std::thread> ws;
  for (int t = 0; t < threads; ++t) ws.emplace_back(churn, std::ref(*ledger), n_nodes, t + 1, iters, &reserved);
  for (auto& w : ws) w.join();
  for (auto& c : clients) c.join();
  int status = 0;
  CHECK(waitpid(child, &status, 0) == child);
  CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  done.store(true);
  checker.join();
  learner.join();
  fe.stop();

  for (int k = 0; k < n_nodes; ++k) {
    NodeSnapshot s;
    CHECK(ledger->snapshot(k, &s));
    for (int i = 0; i < s.n_devs; ++i) {
      CHECK(s.devs[i].pct_free == s.devs[i].pct_total);
      CHECK(s.devs[i].mib_free == s.devs[i].mib_total);
    }
  }
  CHECK(ledger->n_pods() == 0);
  CHECK(ledger->overflow_records_used() == 0);
  const auto st = fe.filter_stats.count.load() + fe.prio_stats.count.load();
  std::printf("stress ok: %d threads x %d iters, %d reservations, %llu native verbs\n", threads, iters,
              reserved.load(), static_cast<unsigned long long>(st));
  ledger.reset();
  unlink(path.c_str());
  apiserver_and_writers(std::max(50, iters / 20), true);    // one epoll writer thread
  apiserver_and_writers(std::max(50, iters / 20), false);   // blocking writer threads
  inline_binds(std::max(100, iters / 10));
  inline_binds(std::max(100, iters / 10), true);   // sent by the workers, answers on the io thread
  relist_gap(std::max(200, iters / 4));
  handoff(std::max(500, iters));
  mailbox_wakeups(std::max(400, iters / 2));
  memo_and_wide(std::max(1000, iters));
  nominate_adopt(std::max(2000, iters));
  return 0;
}
