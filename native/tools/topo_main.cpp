// nanogpu-topo: prints the node's AMD GPU topology (KFD/DRM sysfs + libamd_smi) as JSON.
// Used by the node agent image, which does not need Python to publish the annotation.
//   nanogpu-topo [--root DIR] [--no-amdsmi]
#include <cstdio>
#include <cstring>
#include <string>

#include "nanogpu/topo.h"

int main(int argc, char** argv) {
  std::string root;
  bool smi = true;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--root") && i + 1 < argc) {
      root = argv[++i];
    } else if (!std::strcmp(argv[i], "--no-amdsmi")) {
      smi = false;
    } else {
      std::fprintf(stderr, "usage: %s [--root DIR] [--no-amdsmi]\n", argv[0]);
      return 2;
    }
  }
  const nanogpu::HostTopology t = nanogpu::discover(root, smi);
  std::printf("%s\n", nanogpu::to_json(t).c_str());
  return t.gpus.empty() ? 1 : 0;
}
