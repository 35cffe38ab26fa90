// Cost of one empty poll of a TCP socket: epoll_wait(timeout 0) on an epoll holding it and 8
// other fds, against recv(MSG_DONTWAIT). Build: g++ -O2 -o poll_cost tools/poll_cost.cpp
// (profiles/extender_cpu_r04.md, "The verdict's three suggestions")
#include <sys/epoll.h>
#include <sys/socket.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <arpa/inet.h>
#include <unistd.h>
#include <cstdio>
#include <chrono>
int main() {
  int l = socket(AF_INET, SOCK_STREAM, 0); sockaddr_in a{}; a.sin_family = AF_INET; a.sin_addr.s_addr = htonl(0x7f000001);
  bind(l, (sockaddr*)&a, sizeof a); listen(l, 1); socklen_t n = sizeof a; getsockname(l, (sockaddr*)&a, &n);
  int c = socket(AF_INET, SOCK_STREAM, 0); connect(c, (sockaddr*)&a, sizeof a); int s = accept(l, nullptr, nullptr);
  int ep = epoll_create1(0); epoll_event ev{}; ev.events = EPOLLIN; epoll_ctl(ep, EPOLL_CTL_ADD, s, &ev);
  for (int k = 0; k < 8; ++k) { int e = epoll_create1(0); epoll_ctl(ep, EPOLL_CTL_ADD, e, &ev); }  // other fds
  const int N = 2000000; epoll_event out[128]; char buf[65536];
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) epoll_wait(ep, out, 128, 0);
    auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; ++i) recv(s, buf, sizeof buf, MSG_DONTWAIT);
    auto t2 = std::chrono::steady_clock::now();
    printf("empty epoll_wait(0) %.0f ns  empty recv(MSG_DONTWAIT) %.0f ns\n",
           std::chrono::duration<double, std::nano>(t1 - t0).count() / N,
           std::chrono::duration<double, std::nano>(t2 - t1).count() / N);
  }
}
