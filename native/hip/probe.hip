// nanogpu._probe — MI355X (gfx950) calibration kernels for the node agent.
//
// The reference scheduler never touches a GPU; it trusts an external NVIDIA device plugin
// to realise "gpu-percent" (reference README.md:9, 30-34). On MI355X the agent realises a
// fractional grant spatially: a container with p% of a device gets a CU mask covering
// ceil(p/100 * CUs) compute units, XCD-aligned where possible (each XCD has its own 4 MiB
// L2, so a grant that owns whole XCDs keeps its L2 to itself). These kernels measure the
// facts that mapping needs, on the real device:
//   * cu_census   — which XCD / SE / CU each CU-mask bit enables (s_getreg XCC_ID, HW_ID);
//   * mfma_burn   — bf16 MFMA throughput of a masked stream (isolation check: TFLOP/s
//                   must scale with the CUs granted);
//   * hbm_copy    — streaming HBM3E bandwidth (16 B/lane, grid >> 256 WGs);
//   * peer_bandwidth — per-pair xGMI rate: copy kernel pulling over peer access, and SDMA
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_));      \
  } while (0)

namespace {

// ---------------------------------------------------------------------------- kernels

// Streaming copy: each thread keeps kCopyUnroll 16-B loads in flight before its stores
// (one pass, no grid-stride loop: the grid is n / 4096 workgroups, >> 256 CUs), with
// non-temporal hints so the once-touched stream does not evict L2/MALL.
using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int kCopyUnroll = 4;
constexpr int kCopyBlock = 256;

__global__ __launch_bounds__(kCopyBlock) void hbm_copy(const float4* __restrict__ src,
                                                       float4* __restrict__ dst, size_t n) {
  const size_t base = static_cast<size_t>(blockIdx.x) * (kCopyBlock * kCopyUnroll) + threadIdx.x;
  if (base + (kCopyUnroll - 1) * kCopyBlock < n) {
    const f32x4* s4 = reinterpret_cast<const f32x4*>(src) + base;
    f32x4* d4 = reinterpret_cast<f32x4*>(dst) + base;
    f32x4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) v[u] = __builtin_nontemporal_load(s4 + u * kCopyBlock);
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) __builtin_nontemporal_store(v[u], d4 + u * kCopyBlock);
  } else {
    for (int u = 0; u < kCopyUnroll; ++u)
      if (base + u * kCopyBlock < n) dst[base + u * kCopyBlock] = src[base + u * kCopyBlock];
  }
}

inline unsigned copy_grid(size_t n) {
  return static_cast<unsigned>((n + kCopyBlock * kCopyUnroll - 1) / (kCopyBlock * kCopyUnroll));
}

// One record per workgroup: {xcc_id, hw_id, block}. A bounded sleep keeps each workgroup
// resident long enough that the dispatcher spreads the grid over every enabled CU.
__global__ __launch_bounds__(64) void cu_census(uint32_t* out, int sleep_iters) {
  if (threadIdx.x != 0) return;
  uint32_t xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  for (int i = 0; i < sleep_iters; ++i) __builtin_amdgcn_s_sleep(16);
  out[3 * blockIdx.x + 0] = xcc;
  out[3 * blockIdx.x + 1] = hwid;
  out[3 * blockIdx.x + 2] = blockIdx.x;
}

using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

// MFMA-bound burn: 4 independent 32x32x16 bf16 accumulator chains per wave hide the
// dependent-accumulator latency; each MFMA is 2*32*32*16 = 32768 FLOP.
__global__ __launch_bounds__(256) void mfma_burn(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(0.001f * static_cast<float>((lane + j) & 7));
    b[j] = static_cast<__bf16>(0.002f * static_cast<float>((lane * 3 + j) & 7));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 12345.678f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // keeps the chains live
}

// One wave computes C[32x32] = A[32x16] * B[16x32] with a single bf16 MFMA: the numerics
// self-test of the burn kernel's instruction (operand/accumulator lane maps per
// cdna_hip_programming.md §3: lane l holds A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31];
// C row = (reg&3) + 8(reg>>2) + 4(l>>5), col = l&31).
__global__ __launch_bounds__(64) void mfma_tile(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                float* __restrict__ C) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[r * 16 + 8 * h + j];
    b[j] = B[(8 * h + j) * 32 + r];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) C[((reg & 3) + 8 * (reg >> 2) + 4 * h) * 32 + r] = c[reg];
}

// ---------------------------------------------------------------------------- host helpers

uint16_t f32_to_bf16_bits(float f) {  // round to nearest even
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return static_cast<uint16_t>(u >> 16);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

std::vector<float> gemm_tile(const std::vector<float>& a, const std::vector<float>& b) {
  if (a.size() != 32 * 16 || b.size() != 16 * 32) throw std::invalid_argument("gemm_tile: A is 32x16, B is 16x32");
  std::vector<uint16_t> ha(a.size()), hb(b.size());
  for (size_t i = 0; i < a.size(); ++i) ha[i] = f32_to_bf16_bits(a[i]);
  for (size_t i = 0; i < b.size(); ++i) hb[i] = f32_to_bf16_bits(b[i]);
  uint16_t *da = nullptr, *db = nullptr;
  float* dc = nullptr;
  HIP_OK(hipMalloc(&da, ha.size() * 2));
  HIP_OK(hipMalloc(&db, hb.size() * 2));
  HIP_OK(hipMalloc(&dc, 32 * 32 * 4));
  HIP_OK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(mfma_tile, dim3(1), dim3(64), 0, 0, reinterpret_cast<const __bf16*>(da),
                     reinterpret_cast<const __bf16*>(db), dc);
  HIP_OK(hipGetLastError());
  std::vector<float> c(32 * 32);
  HIP_OK(hipMemcpy(c.data(), dc, c.size() * 4, hipMemcpyDeviceToHost));
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dc);
  return c;
}

struct Stream {
  hipStream_t s = nullptr;
  explicit Stream(const std::vector<uint32_t>& mask) {
    if (mask.empty())
      HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    else
      HIP_OK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
  }
  ~Stream() {
    if (s) (void)hipStreamDestroy(s);
  }
};

struct Events {
  hipEvent_t a = nullptr, b = nullptr;
  Events() {
    HIP_OK(hipEventCreate(&a));
    HIP_OK(hipEventCreate(&b));
  }
  ~Events() {
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
  }
  float ms() {
    HIP_OK(hipEventSynchronize(b));
    float t = 0.f;
    HIP_OK(hipEventElapsedTime(&t, a, b));
    return t;
  }
};

template <class T>
struct DevBuf {
  T* p = nullptr;
  explicit DevBuf(size_t n) { HIP_OK(hipMalloc(&p, n * sizeof(T))); }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

int cu_count(int dev) {
  int n = 0;
  HIP_OK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  return n;
}

py::dict device_props(int dev) {
  hipDeviceProp_t p;
  HIP_OK(hipGetDeviceProperties(&p, dev));
  py::dict d;
  d["name"] = std::string(p.name);
  d["gcn_arch"] = std::string(p.gcnArchName);
  d["cus"] = p.multiProcessorCount;
  d["total_mem_bytes"] = static_cast<uint64_t>(p.totalGlobalMem);
  d["l2_bytes"] = p.l2CacheSize;
  d["lds_per_block_bytes"] = static_cast<uint64_t>(p.sharedMemPerBlock);
  d["max_shared_per_cu_bytes"] = static_cast<uint64_t>(p.maxSharedMemoryPerMultiProcessor);
  d["warp_size"] = p.warpSize;
  d["clock_khz"] = p.clockRate;
  d["mem_clock_khz"] = p.memoryClockRate;
  d["mem_bus_width"] = p.memoryBusWidth;
  d["pci_bus"] = p.pciBusID;
  d["pci_device"] = p.pciDeviceID;
  d["pci_domain"] = p.pciDomainID;
  d["multi_gpu_board"] = p.isMultiGpuBoard;
  int count = 0;
  HIP_OK(hipGetDeviceCount(&count));
  d["device_count"] = count;
  return d;
}

bool copy_check(int dev, size_t n_floats) {
  HIP_OK(hipSetDevice(dev));
  const size_t n4 = (n_floats + 3) / 4;
  std::vector<float> h(n4 * 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<float>((i * 2654435761u) % 1000003u);
  DevBuf<float4> a(n4), b(n4);
  HIP_OK(hipMemcpy(a.p, h.data(), n4 * 16, hipMemcpyHostToDevice));
  HIP_OK(hipMemset(b.p, 0, n4 * 16));
  hipLaunchKernelGGL(hbm_copy, dim3(copy_grid(n4)), dim3(kCopyBlock), 0, 0, a.p, b.p, n4);
  HIP_OK(hipGetLastError());
  std::vector<float> out(n4 * 4);
  HIP_OK(hipMemcpy(out.data(), b.p, n4 * 16, hipMemcpyDeviceToHost));
  return std::memcmp(out.data(), h.data(), n4 * 16) == 0;
}

double hbm_bandwidth(int dev, size_t bytes, int iters) {
  HIP_OK(hipSetDevice(dev));
  const size_t n = bytes / sizeof(float4);
  if (n == 0 || iters <= 0) throw std::invalid_argument("hbm_bandwidth: bytes/iters must be positive");
  DevBuf<float4> a(n), b(n);
  HIP_OK(hipMemset(a.p, 0, n * sizeof(float4)));
  Stream st({});
  Events ev;
  const dim3 grid(copy_grid(n));
  hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, st.s, a.p, b.p, n);  // warm-up
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev.a, st.s));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, st.s, a.p, b.p, n);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev.b, st.s));
  const double ms = ev.ms();
  return 2.0 * static_cast<double>(n * sizeof(float4)) * iters / (ms * 1e-3) / 1e9;  // GB/s, read+write
}

py::list census(int dev, const std::vector<uint32_t>& mask, int blocks, int sleep_iters) {
  HIP_OK(hipSetDevice(dev));
  if (blocks <= 0 || blocks > (1 << 20)) throw std::invalid_argument("census: bad block count");
  DevBuf<uint32_t> out(static_cast<size_t>(blocks) * 3);
  HIP_OK(hipMemset(out.p, 0xff, static_cast<size_t>(blocks) * 3 * sizeof(uint32_t)));
  Stream st(mask);
  hipLaunchKernelGGL(cu_census, dim3(blocks), dim3(64), 0, st.s, out.p, sleep_iters);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(st.s));
  std::vector<uint32_t> h(static_cast<size_t>(blocks) * 3);
  HIP_OK(hipMemcpy(h.data(), out.p, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  py::list res;
  for (int i = 0; i < blocks; ++i) res.append(py::make_tuple(h[3 * i], h[3 * i + 1]));
  return res;
}

double mfma_ms_impl(int dev, const std::vector<uint32_t>& mask, int blocks, int iters);
inline double mfma_ms(int dev, const std::vector<uint32_t>& mask, int blocks, int iters) {
  return mfma_ms_impl(dev, mask, blocks, iters);
}

py::dict mfma_throughput(int dev, const std::vector<uint32_t>& mask, int blocks, int iters) {
  double ms = 0.0;
  {
    py::gil_scoped_release nogil;  // device work without the GIL; py objects built after
    ms = mfma_ms(dev, mask, blocks, iters);
  }
  const double flop = 4.0 * 32768.0 * iters * (static_cast<double>(blocks) * 256 / 64);
  py::dict d;
  d["ms"] = ms;
  d["tflops"] = flop / (ms * 1e-3) / 1e12;
  d["blocks"] = blocks;
  d["iters"] = iters;
  return d;
}

double mfma_ms_impl(int dev, const std::vector<uint32_t>& mask, int blocks, int iters) {
  HIP_OK(hipSetDevice(dev));
  if (blocks <= 0 || iters <= 0) throw std::invalid_argument("mfma_throughput: bad shape");
  DevBuf<float> out(static_cast<size_t>(blocks) * 256);
  Stream st(mask);
  Events ev;
  hipLaunchKernelGGL(mfma_burn, dim3(blocks), dim3(256), 0, st.s, out.p, 8);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev.a, st.s));
  hipLaunchKernelGGL(mfma_burn, dim3(blocks), dim3(256), 0, st.s, out.p, iters);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(ev.b, st.s));
  return ev.ms();
}

// Co-located tenants: one MFMA burn per CU mask, each on its own CU-masked stream, all
// launched back to back so they run concurrently. Returns per-tenant TFLOP/s, timed with
// each stream's own events: with disjoint XCD-symmetric masks every tenant must get
// throughput proportional to its CUs regardless of its neighbours (the agent's spatial
// share, nanogpu/agent/cumask.py).
std::vector<double> mfma_colocated(int dev, const std::vector<std::vector<uint32_t>>& masks,
                                   const std::vector<int>& blocks, int iters) {
  HIP_OK(hipSetDevice(dev));
  if (masks.empty() || masks.size() != blocks.size() || iters <= 0)
    throw std::invalid_argument("mfma_colocated: one block count per mask, iters > 0");
  const size_t n = masks.size();
  std::vector<std::unique_ptr<Stream>> streams;
  std::vector<std::unique_ptr<Events>> evs;
  std::vector<std::unique_ptr<DevBuf<float>>> outs;
  for (size_t i = 0; i < n; ++i) {
    if (blocks[i] <= 0) throw std::invalid_argument("mfma_colocated: bad block count");
    streams.emplace_back(new Stream(masks[i]));
    evs.emplace_back(new Events());
    outs.emplace_back(new DevBuf<float>(static_cast<size_t>(blocks[i]) * 256));
    hipLaunchKernelGGL(mfma_burn, dim3(blocks[i]), dim3(256), 0, streams[i]->s, outs[i]->p, 8);  // warm-up
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipDeviceSynchronize());
  for (size_t i = 0; i < n; ++i) {
    HIP_OK(hipEventRecord(evs[i]->a, streams[i]->s));
    hipLaunchKernelGGL(mfma_burn, dim3(blocks[i]), dim3(256), 0, streams[i]->s, outs[i]->p, iters);
    HIP_OK(hipEventRecord(evs[i]->b, streams[i]->s));
  }
  HIP_OK(hipGetLastError());
  std::vector<double> tf(n);
  for (size_t i = 0; i < n; ++i) {
    const double ms = evs[i]->ms();
    tf[i] = 4.0 * 32768.0 * iters * (static_cast<double>(blocks[i]) * 4) / (ms * 1e-3) / 1e12;
  }
  return tf;
}

// Co-located streaming tenants: one HBM copy per CU mask, each on its own CU-masked stream,
// launched together. Returns per-tenant GB/s (read + write) over each tenant's own events.
// CU masks partition the compute units, not the memory system: this measures how the HBM3E
// bandwidth splits between memory-bound neighbours (profiles/gpu_calibration.md).
// `iters_each` (optional, one per mask) lets a neighbour outlast the tenant being measured.
std::vector<double> hbm_colocated(int dev, const std::vector<std::vector<uint32_t>>& masks, size_t bytes,
                                  int iters, std::vector<int> iters_each) {
  HIP_OK(hipSetDevice(dev));
  const size_t n = bytes / sizeof(float4);
  if (masks.empty() || n == 0 || iters <= 0) throw std::invalid_argument("hbm_colocated: masks, bytes, iters");
  const size_t k = masks.size();
  if (iters_each.empty()) iters_each.assign(k, iters);
  if (iters_each.size() != k) throw std::invalid_argument("hbm_colocated: one iteration count per mask");
  for (int it : iters_each)
    if (it <= 0 || it > 1000) throw std::invalid_argument("hbm_colocated: iterations in 1..1000");
  std::vector<std::unique_ptr<Stream>> streams;
  std::vector<std::unique_ptr<Events>> evs;
  std::vector<std::unique_ptr<DevBuf<float4>>> src, dst;
  const dim3 grid(copy_grid(n));
  for (size_t i = 0; i < k; ++i) {
    streams.emplace_back(new Stream(masks[i]));
    evs.emplace_back(new Events());
    src.emplace_back(new DevBuf<float4>(n));
    dst.emplace_back(new DevBuf<float4>(n));
    HIP_OK(hipMemset(src[i]->p, 0, n * sizeof(float4)));
    hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, streams[i]->s, src[i]->p, dst[i]->p, n);  // warm-up
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipDeviceSynchronize());
  for (size_t i = 0; i < k; ++i) {
    HIP_OK(hipEventRecord(evs[i]->a, streams[i]->s));
    for (int it = 0; it < iters_each[i]; ++it)
      hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, streams[i]->s, src[i]->p, dst[i]->p, n);
    HIP_OK(hipEventRecord(evs[i]->b, streams[i]->s));
  }
  HIP_OK(hipGetLastError());
  std::vector<double> gbs(k);
  for (size_t i = 0; i < k; ++i)
    gbs[i] = 2.0 * static_cast<double>(n * sizeof(float4)) * iters_each[i] / (evs[i]->ms() * 1e-3) / 1e9;
  return gbs;
}

// A streaming tenant next to a compute-bound one: an HBM copy on `hbm_mask` and an MFMA
// burn on `mfma_mask`, launched together on their own CU-masked streams. The burn is sized
// (`mfma_iters`) to outlast the copy, so the copy's rate is measured entirely beside it.
// Returns {copy GB/s, burn TFLOP/s}: what a memory-bound pod gets when the scheduler pairs
// it with a compute-bound neighbour (kFlagMemBound) instead of another streaming one.
std::vector<double> mixed_colocated(int dev, const std::vector<uint32_t>& hbm_mask,
                                    const std::vector<uint32_t>& mfma_mask, size_t bytes, int iters,
                                    int mfma_blocks, int mfma_iters) {
  HIP_OK(hipSetDevice(dev));
  const size_t n = bytes / sizeof(float4);
  if (n == 0 || iters <= 0 || mfma_blocks <= 0 || mfma_iters <= 0)
    throw std::invalid_argument("mixed_colocated: bytes, iters and the burn shape must be positive");
  Stream sc(hbm_mask), sm(mfma_mask);
  Events ec, em;
  DevBuf<float4> src(n), dst(n);
  DevBuf<float> out(static_cast<size_t>(mfma_blocks) * 256);
  HIP_OK(hipMemset(src.p, 0, n * sizeof(float4)));
  const dim3 grid(copy_grid(n));
  hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, sc.s, src.p, dst.p, n);    // warm-up
  hipLaunchKernelGGL(mfma_burn, dim3(mfma_blocks), dim3(256), 0, sm.s, out.p, 8);
  HIP_OK(hipGetLastError());
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipEventRecord(em.a, sm.s));
  hipLaunchKernelGGL(mfma_burn, dim3(mfma_blocks), dim3(256), 0, sm.s, out.p, mfma_iters);
  HIP_OK(hipEventRecord(em.b, sm.s));
  HIP_OK(hipEventRecord(ec.a, sc.s));
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, sc.s, src.p, dst.p, n);
  HIP_OK(hipEventRecord(ec.b, sc.s));
  HIP_OK(hipGetLastError());
  const double gbs = 2.0 * static_cast<double>(n * sizeof(float4)) * iters / (ec.ms() * 1e-3) / 1e9;
  const double tf = 4.0 * 32768.0 * mfma_iters * (static_cast<double>(mfma_blocks) * 4) / (em.ms() * 1e-3) / 1e12;
  return {gbs, tf};
}

struct PeerRate {
  double pull_gbs;   // copy kernel on `dst` reading `src`'s HBM over xGMI (one link, one direction)
  double dma_gbs;    // hipMemcpyPeerAsync (SDMA engines) over the same link
  bool peer_access;
};

// A peer transfer that did not finish by its deadline (a wedged link or peer). Its stream,
// events and buffers are abandoned, never freed: hipFree / hipStreamDestroy would wait on the
// work that never completes.
struct PeerTimeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

using Clock = std::chrono::steady_clock;

// Polls `e` until it completes (true) or `deadline` passes (false); never blocks in the runtime.
bool wait_event(hipEvent_t e, Clock::time_point deadline) {
  for (;;) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) HIP_OK(q);
    if (Clock::now() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Per-pair link rate for the topology scorer. The copy kernel runs on the destination GPU and
// loads straight from the peer's memory (peer access enabled), so every byte crosses the one
// xGMI link between the pair in one direction; its grid (n / 4096 WGs, >> 256 CUs) keeps
// enough loads in flight to saturate the link rather than one SDMA engine. Every wait polls an
// event against `deadline_s` (from the call): a transfer that never completes throws
// PeerTimeout instead of blocking the rank (and, through the next collective, the whole job).
PeerRate peer_bandwidth(int src, int dst, size_t bytes, int iters, double deadline_s) {
  int n_dev = 0;
  HIP_OK(hipGetDeviceCount(&n_dev));
  if (src < 0 || dst < 0 || src >= n_dev || dst >= n_dev || src == dst)
    throw std::invalid_argument("peer_bandwidth: need two distinct visible devices");
  const size_t n = bytes / sizeof(float4);
  if (n == 0 || iters <= 0) throw std::invalid_argument("peer_bandwidth: bytes/iters must be positive");
  const Clock::time_point deadline =
      Clock::now() + std::chrono::microseconds(static_cast<int64_t>((deadline_s > 0 ? deadline_s : 30.0) * 1e6));
  PeerRate r{0.0, 0.0, false};
  int prev = 0;   // the caller's current device comes back on return (torch tracks it)
  HIP_OK(hipGetDevice(&prev));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  int can = 0;
  HIP_OK(hipDeviceCanAccessPeer(&can, dst, src));
  HIP_OK(hipSetDevice(dst));
  if (can) {
    hipError_t e = hipDeviceEnablePeerAccess(src, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_OK(e);
    (void)hipGetLastError();
    r.peer_access = true;
  }
  // owned until a timeout abandons them
  hipStream_t ss = nullptr, st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float4 *a = nullptr, *b = nullptr;
  bool abandoned = false;
  auto cleanup = [&] {
    if (abandoned) return;
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (ss) (void)hipStreamDestroy(ss);
    if (st) (void)hipStreamDestroy(st);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
  };
  auto timed = [&](const char* what, auto&& enqueue) -> double {   // seconds of `enqueue`'s work
    HIP_OK(hipEventRecord(e0, st));
    enqueue();
    HIP_OK(hipEventRecord(e1, st));
    if (!wait_event(e1, deadline)) {
      abandoned = true;
      throw PeerTimeout(std::string("peer_bandwidth ") + std::to_string(src) + "->" + std::to_string(dst) + ": " +
                        what + " did not finish within " + std::to_string(deadline_s) + " s");
    }
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e-3;
  };
  try {
    HIP_OK(hipSetDevice(src));
    HIP_OK(hipMalloc(&a, n * sizeof(float4)));
    HIP_OK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
    HIP_OK(hipMemsetAsync(a, 0, n * sizeof(float4), ss));
    hipEvent_t fill = nullptr;
    HIP_OK(hipEventCreateWithFlags(&fill, hipEventDisableTiming));
    HIP_OK(hipEventRecord(fill, ss));
    const bool filled = wait_event(fill, deadline);
    (void)hipEventDestroy(fill);
    if (!filled) {
      abandoned = true;
      throw PeerTimeout("peer_bandwidth: the source fill on GPU " + std::to_string(src) + " did not finish");
    }
    HIP_OK(hipSetDevice(dst));
    HIP_OK(hipMalloc(&b, n * sizeof(float4)));
    HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    const double nb = static_cast<double>(n * sizeof(float4));
    timed("SDMA warm-up", [&] { HIP_OK(hipMemcpyPeerAsync(b, dst, a, src, n * sizeof(float4), st)); });
    r.dma_gbs = nb * iters / timed("SDMA copies", [&] {
      for (int i = 0; i < iters; ++i) HIP_OK(hipMemcpyPeerAsync(b, dst, a, src, n * sizeof(float4), st));
    }) / 1e9;
    if (r.peer_access) {
      const dim3 grid(copy_grid(n));
      timed("pull warm-up", [&] {
        hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, st, a, b, n);
        HIP_OK(hipGetLastError());
      });
      r.pull_gbs = nb * iters / timed("pull copies", [&] {
        for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(hbm_copy, grid, dim3(kCopyBlock), 0, st, a, b, n);
        HIP_OK(hipGetLastError());
      }) / 1e9;
    }
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
  return r;
}

}  // namespace

PYBIND11_MODULE(_probe, m) {
  m.doc() = "MI355X calibration kernels (gfx950): CU census, MFMA burn, HBM and xGMI bandwidth";
  m.def("device_count", []() {
    int n = 0;
    HIP_OK(hipGetDeviceCount(&n));
    return n;
  });
  m.def("device_props", &device_props, py::arg("device") = 0);
  m.def("hbm_bandwidth", &hbm_bandwidth, py::arg("device") = 0, py::arg("bytes") = size_t(1) << 30,
        py::arg("iters") = 10, py::call_guard<py::gil_scoped_release>(),
        "Streaming copy bandwidth in GB/s (read + write bytes).");
  m.def("cu_census", &census, py::arg("device") = 0, py::arg("cu_mask") = std::vector<uint32_t>{},
        py::arg("blocks") = 2048, py::arg("sleep_iters") = 64,
        "Per-workgroup (xcc_id, hw_id) for a launch on a CU-masked stream.");
  m.def("mfma_throughput", &mfma_throughput, py::arg("device") = 0,
        py::arg("cu_mask") = std::vector<uint32_t>{}, py::arg("blocks") = 2048, py::arg("iters") = 2048,
        "bf16 MFMA TFLOP/s on a CU-masked stream.");
  m.def("gemm_tile", &gemm_tile, py::arg("a"), py::arg("b"),
        "C[32x32] = bf16(A[32x16]) @ bf16(B[16x32]) with one v_mfma_f32_32x32x16_bf16 (fp32 accumulate).");
  m.def("copy_check", &copy_check, py::arg("device") = 0, py::arg("n_floats") = size_t(1) << 24,
        py::call_guard<py::gil_scoped_release>(), "hbm_copy kernel result == source, bit for bit.");
  m.def("mixed_colocated", &mixed_colocated, py::arg("device"), py::arg("hbm_mask"), py::arg("mfma_mask"),
        py::arg("bytes") = size_t(1) << 30, py::arg("iters") = 10, py::arg("mfma_blocks") = 1536,
        py::arg("mfma_iters") = 4096, py::call_guard<py::gil_scoped_release>(),
        "{copy GB/s, MFMA TFLOP/s} for a streaming tenant beside a compute-bound one.");
  m.def("hbm_colocated", &hbm_colocated, py::arg("device"), py::arg("cu_masks"), py::arg("bytes") = size_t(1) << 30,
        py::arg("iters") = 10, py::arg("iters_each") = std::vector<int>{}, py::call_guard<py::gil_scoped_release>(),
        "Per-tenant HBM copy GB/s for concurrent tenants on CU-masked streams.");
  m.def("mfma_colocated", &mfma_colocated, py::arg("device"), py::arg("cu_masks"), py::arg("blocks"),
        py::arg("iters") = 2048, py::call_guard<py::gil_scoped_release>(),
        "Concurrent MFMA burns on CU-masked streams; per-stream TFLOP/s.");
  m.def(
      "peer_bandwidth",
      [](int src, int dst, size_t bytes, int iters, double deadline_s) {
        PeerRate r;
        {
          py::gil_scoped_release nogil;
          r = peer_bandwidth(src, dst, bytes, iters, deadline_s);
        }
        py::dict d;
        d["pull_gbs"] = r.pull_gbs;
        d["dma_gbs"] = r.dma_gbs;
        d["peer_access"] = r.peer_access;
        d["gbs"] = std::max(r.pull_gbs, r.dma_gbs);
        return d;
      },
      py::arg("src"), py::arg("dst"), py::arg("bytes") = size_t(256) << 20, py::arg("iters") = 10,
      py::arg("deadline_s") = 30.0,
      "One-direction xGMI rate src -> dst in GB/s: copy kernel pulling over peer access, and SDMA. "
      "Raises TimeoutError when the transfers do not finish within deadline_s (the work is abandoned).");
  py::register_exception<PeerTimeout>(m, "PeerTimeout", PyExc_TimeoutError);
}
