// CPU sampling profiler (sampler.cpp): SIGPROF on process CPU time, leaf PC + caller + tid.
#pragma once

#include <cstdint>
#include <vector>

namespace nanogpu {
namespace sampler {

struct Sample {
  uint64_t pc;
  uint64_t caller;   // 0: the frame kept no frame pointer
  int32_t tid;
};

// Starts sampling at `hz` samples per second of process CPU time; false if already running.
bool start(int hz);
// Stops and returns the samples taken since start().
std::vector<Sample> stop();

}  // namespace sampler
}  // namespace nanogpu
