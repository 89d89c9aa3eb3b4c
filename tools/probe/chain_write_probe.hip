// chain_write_probe.hip -- is k_pull_chain's write pattern itself slower
// than a plain write stream on MI355X?  (profiles/r04: the bulk chain launch
// writes 3.6 GB of rows at 4.5 TB/s, the one-shot 8-KB probe reaches ~6.)
// Each one-wave workgroup writes L segments, segment k of S_k bytes at
// region_k + w * S_k (the chain's level streams: a run's rows, its children's,
// ...), 16 B per lane, 1 KB per store instruction, the data from LDS as the
// chain's stage stream reads it.  Variants: the segments' sizes and count,
// non-temporal or plain stores, LDS per wave (residency), and one contiguous
// segment per wave (the one-shot probe) for reference.
//   hipcc -O3 --offload-arch=gfx950 chain_write_probe.hip -o cwp && ./cwp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Seg {
  unsigned long long base[6];  // region of segment k (bytes)
  unsigned size[6];            // bytes per wave (multiple of 1 KB)
  int n;
};

template <bool kNT>
__global__ __launch_bounds__(64) void k_segs(char* __restrict__ out, Seg sg) {
  extern __shared__ u32x4 lds[];  // >= 64 x 16 B used; the rest pads residency
  const unsigned lane = threadIdx.x;
  lds[lane] = u32x4{lane, blockIdx.x, 1u, 2u};
  __syncthreads();
  const unsigned long long w = blockIdx.x;
  for (int k = 0; k < sg.n; ++k) {
    u32x4* o = reinterpret_cast<u32x4*>(out + sg.base[k] + w * sg.size[k]);
    const unsigned units = sg.size[k] / 16;
    for (unsigned i0 = 0; i0 < units; i0 += 8 * 64) {
      u32x4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = lds[(lane + u) & 63];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const unsigned i = i0 + u * 64 + lane;
        if (i < units) {
          if constexpr (kNT)
            __builtin_nontemporal_store(x[u], o + i);
          else
            o[i] = x[u];
        }
      }
    }
  }
}

int main(int argc, char** argv) {
  const size_t total = (argc > 1 ? std::atoll(argv[1]) : 3600) * (1ull << 20);  // bytes per launch
  char* buf = nullptr;
  CK(hipMalloc(&buf, total + (64ull << 20)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, std::vector<unsigned> sizes, bool nt, size_t lds) {
    Seg sg{};
    sg.n = static_cast<int>(sizes.size());
    unsigned per = 0;
    for (unsigned s : sizes) per += s;
    const unsigned waves = static_cast<unsigned>(total / per);
    unsigned long long off = 0;
    for (int k = 0; k < sg.n; ++k) {
      sg.base[k] = off;
      sg.size[k] = sizes[k];
      off += static_cast<unsigned long long>(sizes[k]) * waves;
      off = (off + 4095) & ~4095ull;
    }
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipEventRecord(a));
      if (nt)
        hipLaunchKernelGGL(k_segs<true>, dim3(waves), dim3(64), lds, 0, buf, sg);
      else
        hipLaunchKernelGGL(k_segs<false>, dim3(waves), dim3(64), lds, 0, buf, sg);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep && ms < best) best = ms;
    }
    const double bytes = static_cast<double>(per) * waves;
    std::printf("%-34s nt=%d lds=%6zu waves=%7u per-wave=%6u B: %7.1f us  %.2f TB/s\n", name, nt ? 1 : 0, lds, waves,
                per, best * 1e3, bytes / (best * 1e-3) / 1e12);
    std::fflush(stdout);
  };
  for (bool nt : {true, false})
    for (size_t lds : {1024ul, 9472ul, 20480ul}) {
      run("chain 2.6K,5.3K,10.6K,21K,2K", {2688, 5376, 10752, 21504, 2048}, nt, lds);
      run("one segment 42K", {42368}, nt, lds);
      run("one segment 8K", {8192}, nt, lds);
      run("chain small 1K,2K,4K,8K,1K", {1024, 2048, 4096, 8192, 1024}, nt, lds);
    }
  return 0;
}
