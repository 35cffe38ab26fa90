// CPU sampling profiler for the extender process (no perf on the gpurun pool): SIGPROF from a
// process CPU-time interval timer (ITIMER_PROF) lands on the thread that was running when the
// timer expired, so samples fall on threads in proportion to their CPU time. The handler
// records the interrupted instruction pointer, one frame-pointer hop up, and the thread id
// into a preallocated array (async-signal-safe: an atomic index, no allocation, no locks).
// A sample taken while the thread was in a system call lands on the libc syscall stub the
// kernel returns to (send, recv, epoll_wait, ...), so kernel time is attributed to its call
// site. nanogpu/obs.py symbolizes the PCs through /proc/self/maps and addr2line.
#include "nanogpu/sampler.h"

#include <signal.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <sys/time.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <mutex>

namespace nanogpu {
namespace sampler {

namespace {

constexpr size_t kCap = 1 << 18;   // 262k samples: over 15 minutes at the tick-bound rate
Sample g_buf[kCap];
std::atomic<size_t> g_n{0};
std::atomic<bool> g_on{false};
std::mutex g_mu;                   // start / stop
struct sigaction g_old{};

void sample_into(void* uc_);

void on_prof(int, siginfo_t*, void* uc_) {
  // the interrupted code may sit between a failed syscall and its errno check: keep its errno
  // (process_vm_readv and gettid below can set it)
  const int saved_errno = errno;
  sample_into(uc_);
  errno = saved_errno;
}

void sample_into(void* uc_) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  const size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (i >= kCap) return;
  const ucontext_t* uc = static_cast<const ucontext_t*>(uc_);
  Sample& s = g_buf[i];
  s.pc = static_cast<uint64_t>(uc->uc_mcontext.gregs[REG_RIP]);
  // the caller's return address through the frame pointer, when the frame keeps one; a read
  // is only attempted inside the interrupted thread's own stack window
  const uint64_t sp = static_cast<uint64_t>(uc->uc_mcontext.gregs[REG_RSP]);
  const uint64_t bp = static_cast<uint64_t>(uc->uc_mcontext.gregs[REG_RBP]);
  s.caller = 0;
  if (bp >= sp && bp - sp < (1u << 20) && (bp & 7) == 0) {
    // read through the kernel: a garbage frame pointer gives EFAULT instead of a fault here
    uint64_t ra = 0;
    iovec local{&ra, sizeof ra}, remote{reinterpret_cast<void*>(bp + 8), sizeof ra};
    if (process_vm_readv(getpid(), &local, 1, &remote, 1, 0) == static_cast<ssize_t>(sizeof ra)) s.caller = ra;
  }
  s.tid = static_cast<int32_t>(syscall(SYS_gettid));
}

}  // namespace

bool start(int hz) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_on.load()) return false;
  if (hz < 10) hz = 10;
  if (hz > 10000) hz = 10000;
  g_n.store(0);
  struct sigaction sa{};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old) != 0) return false;
  g_on.store(true);
  itimerval it{};
  it.it_interval.tv_usec = 1000000 / hz;
  it.it_value = it.it_interval;
  if (setitimer(ITIMER_PROF, &it, nullptr) != 0) {
    g_on.store(false);
    sigaction(SIGPROF, &g_old, nullptr);
    return false;
  }
  return true;
}

std::vector<Sample> stop() {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_on.load()) return {};
  itimerval off{};
  setitimer(ITIMER_PROF, &off, nullptr);
  g_on.store(false);
  // a handler already running finishes its one slot; SIGPROF keeps our handler (ignoring the
  // signal instead could kill the process if a late one came in with the default action)
  const size_t n = std::min(g_n.load(), kCap);
  return std::vector<Sample>(g_buf, g_buf + n);
}

}  // namespace sampler
}  // namespace nanogpu
