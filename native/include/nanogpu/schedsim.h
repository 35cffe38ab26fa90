// Native kube-scheduler stand-in for the benchmark harness.
//
// kube-scheduler is a compiled Go binary: its per-pod cost in front of an extender is a
// few microseconds of JSON work plus the extender round trips. The Python stand-in
// (nanogpu/sim/driver.py::ThreadedSchedulerDriver) spends ~150 us of interpreter time per
// pod, so at thousands of pods/s it — not the extender — set the measured rate. This is the
// same protocol loop in C++:
//   * one serial scheduling cycle on a keep-alive connection: resource-fit pre-filter
//     (NodeResourcesFit on the extended resource), POST /scheduler/filter with NodeNames
//     (nodeCacheCapable), POST /scheduler/priorities when more than one node fits, highest
//     score wins, ties broken uniformly at random;
//   * binds leave as soon as their host is chosen (kube-scheduler's asynchronous binding
//     cycle, a goroutine per pod): one epoll thread multiplexes up to `bind_threads`
//     keep-alive connections, POST /scheduler/bind;
//   * a failed attempt goes back to the queue with exponential backoff, up to max_attempts;
//   * kube-scheduler's node sampling (numFeasibleNodesToFind, generic_scheduler.go): with 100
//     nodes or more the in-tree filters stop after an adaptive share of feasible nodes
//     (50 % - nodes/125, at least 5 %, at least 100 nodes), starting where the previous cycle
//     stopped (nextStartNodeIndex), and only those reach the extender;
//   * PodTopologySpread's system default for pods owned by a ReplicaSet / StatefulSet / ...:
//     hostname, maxSkew 3, ScheduleAnyway, weight 2 (the zone constraint needs zone labels,
//     which these nodes do not carry).
// Times are steady_clock seconds (the clock of Python's time.perf_counter()).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace nanogpu::sim {

struct SimPod {
  std::string json;      // the Pod object as sent in ExtenderArgs.Pod
  std::string ns, name, uid;
  int64_t need = 0;      // Σ container gpu-percent (the pre-filter's request)
  int64_t cpu_m = 0;     // CPU (millicores) and memory (bytes) requests: kube-scheduler's own
  int64_t mem = 0;       // score plugins see these (nanogpu/sim/kubescore.py)
  int32_t owner = -1;    // controlling ReplicaSet (index), -1: none (no spread constraint)
};

// A pod already bound when a run starts (kube-scheduler's cache at a steady state).
struct SimLive {
  int32_t node = -1;
  int64_t need = 0, cpu_m = 0, mem = 0;
  int32_t owner = -1;
};

struct SimConfig {
  std::string host = "127.0.0.1";
  int port = 0;
  std::vector<std::string> nodes;
  std::vector<int64_t> capacity;   // per node; empty = no resource pre-filter
  int bind_threads = 256;   // max concurrent bind connections
  uint64_t seed = 0;
  int max_attempts = 8;
  double backoff_s = 0.001;
  // kube-scheduler score combining (nanogpu/sim/kubescore.py): total = LeastAllocated +
  // BalancedAllocation (0..100 each, on CPU/memory requests) + weight x extender score x 10,
  // random among the maxima. 0: take the extender's arg-max (random ties).
  int kube_combine = 0;
  int extender_weight = 1;
  int64_t node_cpu_m = 256000;
  int64_t node_mem = int64_t{3} << 40;
  // numFeasibleNodesToFind: 1 = on (kube-scheduler always samples; below 100 nodes it keeps
  // every node), 0 = every feasible node goes to the extender. percentage_of_nodes_to_score
  // 0 = adaptive (the KubeSchedulerConfiguration default).
  int sample_nodes = 1;
  int percentage_of_nodes_to_score = 0;
  // PodTopologySpread system default (owned pods only; needs kube_combine): weight, maxSkew
  int spread_weight = 2;
  int spread_max_skew = 3;
  std::vector<SimLive> live;   // pods bound before this run (resource fit, spread counts)
  // extender workers behind one Service: the scheduling cycle's keep-alive connection stays on
  // `port`; bind connection k goes to bind_ports[k % size] (kube-proxy spreads connections).
  // Empty: every bind to `port`.
  std::vector<int> bind_ports;
};

// kube-scheduler's numFeasibleNodesToFind (v1.18+).
int64_t num_feasible_nodes_to_find(int64_t all_nodes, int percentage);

struct SimResult {
  int64_t scheduled = 0, failed = 0, bind_errors = 0, unschedulable_attempts = 0;
  double t_first_filter = 0.0, t_last_bind = 0.0;
  double cycle_max_s = 0.0, cycle_sum_s = 0.0;
  double cycle_wire_s = 0.0;   // of which waiting on the extender (request sent -> response read)   // slowest scheduling cycle (filter -> host chosen) of one pod
  std::vector<double> bind_latencies, e2e_latencies;
  std::vector<std::string> node_of;   // per pod; "" = not scheduled
  std::vector<std::string> last_error;
  int64_t nodes_sent_filter = 0;      // node names sent to the extender's filter, summed
  int64_t cycles = 0;
};

// Keep-alive connections carried from one drive() to the next (kube-scheduler's HTTP client
// pool lives as long as the scheduler). Not thread-safe: one drive() at a time per session.
struct SessionState;
class Session {
 public:
  Session();
  ~Session();
  Session(const Session&) = delete;
  Session& operator=(const Session&) = delete;
  SessionState* state() { return st_.get(); }

 private:
  std::unique_ptr<SessionState> st_;
};

SimResult drive(const SimConfig& cfg, const std::vector<SimPod>& pods, Session* session = nullptr);

}  // namespace nanogpu::sim
