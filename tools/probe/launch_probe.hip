// Fixed cost of the small per-window kernels (cfg2's window
// is init + pair + chain + reduce, ~53 us, of which the chain streams ~26 us).
// How long does a near-empty kernel take on the queue, after a 128-MB write
// kernel, with and without a device- or system-scope fence, and with a
// store to pinned host memory?  Run under rocprofv3 --kernel-trace --stats.
//   hipcc -O3 --offload-arch=gfx950 launch_probe.hip -o launch_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_big(u32x4* __restrict__ out, size_t n, unsigned v) {
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
    u32x4 x = {v, v + 1, v + 2, static_cast<unsigned>(i)};
    __builtin_nontemporal_store(x, out + i);
  }
}

__global__ __launch_bounds__(256) void k_empty(unsigned long long* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 1000000) p[0] = 1;
}

__global__ __launch_bounds__(256) void k_small_dev(unsigned long long* p) {
  p[blockIdx.x * 256 + threadIdx.x] += 1;
}

__global__ __launch_bounds__(256) void k_fence_dev(unsigned long long* p) {
  p[blockIdx.x * 256 + threadIdx.x] += 1;
  __syncthreads();
  if (threadIdx.x == 0) __threadfence();
}

__global__ __launch_bounds__(256) void k_fence_sys(unsigned long long* p) {
  p[blockIdx.x * 256 + threadIdx.x] += 1;
  __syncthreads();
  if (threadIdx.x == 0) __threadfence_system();
}

// stats rows in pinned host memory, system-scope stores, one fence per block
// and a release store of a flag (the signalled-window reduce's shape)
__global__ __launch_bounds__(256) void k_host_sys(unsigned long long* p, unsigned long long* host) {
  p[blockIdx.x * 256 + threadIdx.x] += 1;
  if (threadIdx.x < 8)
    __hip_atomic_store(host + blockIdx.x * 8 + threadIdx.x, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(host + 4096, 2ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// the same without the fence: relaxed system-scope stores only, the flag
// ordered after the rows by waiting for the stores (no cache writeback)
__global__ __launch_bounds__(256) void k_host_nofence(unsigned long long* p, unsigned long long* host) {
  p[blockIdx.x * 256 + threadIdx.x] += 1;
  if (threadIdx.x < 8)
    __hip_atomic_store(host + blockIdx.x * 8 + threadIdx.x, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    __hip_atomic_store(host + 4096, 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main() {
  const size_t n = (128u << 20) / 16;
  u32x4* big;
  unsigned long long* small;
  unsigned long long* host;
  CK(hipMalloc(&big, n * 16));
  CK(hipMalloc(&small, 64 * 256 * 8));
  CK(hipMemset(small, 0, 64 * 256 * 8));
  CK(hipHostMalloc(&host, 8192 * 8, hipHostMallocCoherent | hipHostMallocMapped));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int reps = 40;
  for (int r = 0; r < reps; ++r) {
    // small kernels back to back (no heavy predecessor)
    k_empty<<<7, 256, 0, s>>>(nullptr);
    k_empty<<<7, 256, 0, s>>>(nullptr);
    k_small_dev<<<7, 256, 0, s>>>(small);
    // each variant right after a 128-MB write
    k_big<<<4096, 256, 0, s>>>(big, n, r);
    k_empty<<<7, 256, 0, s>>>(nullptr);
    k_big<<<4096, 256, 0, s>>>(big, n, r);
    k_fence_dev<<<7, 256, 0, s>>>(small);
    k_big<<<4096, 256, 0, s>>>(big, n, r);
    k_fence_sys<<<7, 256, 0, s>>>(small);
    k_big<<<4096, 256, 0, s>>>(big, n, r);
    k_host_sys<<<7, 256, 0, s>>>(small, host);
    k_big<<<4096, 256, 0, s>>>(big, n, r);
    k_host_nofence<<<7, 256, 0, s>>>(small, host);
    CK(hipGetLastError());
  }
  CK(hipStreamSynchronize(s));
  // without the profiler: 200 empty kernels between two events
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 200; ++i) k_empty<<<7, 256, 0, s>>>(nullptr);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("empty kernels back to back: %.2f us each\n", ms * 1000 / 200);
  }
  // any-order launches: a 128-MB write, then an empty kernel without the
  // barrier bit (does it start before the write ends?)
  for (int r = 0; r < 20; ++r) {
    k_big<<<4096, 256, 0, s>>>(big, n, r);
    hipExtLaunchKernelGGL(k_small_dev, dim3(7), dim3(256), 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, small);
    k_empty<<<7, 256, 0, s>>>(nullptr);
  }
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));
  // a graph of 4 small kernels (the cfg2 window's count), replayed
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  k_small_dev<<<7, 256, 0, s>>>(small);
  k_empty<<<7, 256, 0, s>>>(nullptr);
  k_fence_dev<<<7, 256, 0, s>>>(small);
  k_empty<<<7, 256, 0, s>>>(nullptr);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 50; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("graph of 4 small kernels: %.2f us per replay\n", ms * 1000 / 50);
  }
  std::printf("launch_probe done: %d reps, host flag %llu\n", reps, host[4096]);
  return 0;
}
