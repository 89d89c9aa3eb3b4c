// HBM write / copy ceilings on one MI355X (the pull kernels
// write ~4.3 GB of rows per cfg3 step and read less; which rate binds?).
// Each kernel streams 16-B units, grid-stride, one block of 256 threads per
// 1 KB x 8 units; dynamic LDS pads the blocks to a given count per CU.
//   hipcc -O3 --offload-arch=gfx950 hbm_write_probe.hip -o probe && ./probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool kNT>
__global__ __launch_bounds__(256) void k_fill(u32x4* __restrict__ out, size_t n, unsigned v) {
  extern __shared__ unsigned pad[];
  if (n == 0) pad[threadIdx.x] = v;  // (keeps the dynamic LDS)
  const size_t stride = static_cast<size_t>(gridDim.x) * 256 * 8;
  for (size_t i0 = static_cast<size_t>(blockIdx.x) * 256 * 8 + threadIdx.x; i0 < n; i0 += stride) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t i = i0 + u * 256;
      if (i < n) {
        u32x4 x = {v, v + 1, v + 2, static_cast<unsigned>(i)};
        if constexpr (kNT)
          __builtin_nontemporal_store(x, out + i);
        else
          out[i] = x;
      }
    }
  }
}

template <bool kNT>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
  extern __shared__ unsigned pad[];
  if (n == 0) pad[threadIdx.x] = 0;
  const size_t stride = static_cast<size_t>(gridDim.x) * 256 * 8;
  for (size_t i0 = static_cast<size_t>(blockIdx.x) * 256 * 8 + threadIdx.x; i0 < n; i0 += stride) {
    u32x4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t i = i0 + u * 256;
      x[u] = i < n ? in[i] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t i = i0 + u * 256;
      if (i < n) {
        if constexpr (kNT)
          __builtin_nontemporal_store(x[u], out + i);
        else
          out[i] = x[u];
      }
    }
  }
}

// Store patterns of one-shot grids (one 8-KB piece per wave, as the pull
// kernels write their chunks): kPat 0 = each store instruction covers 1 KB
// contiguous (lane l: unit u*64 + l), 1 = each lane stores 4 consecutive
// units (a store covers 64 B-strided lanes: 4 stores = 4 KB), 2 = 8-KB piece
// per wave, the wave's pieces in dispatch order but waves of a block 32 KB
// apart (XCD-interleaved pieces).
template <int kPat, bool kNT>
__global__ __launch_bounds__(64) void k_fill_wave(u32x4* __restrict__ out, size_t n, unsigned v) {
  const size_t w = blockIdx.x;
  const size_t base = w * 512;  // units (8 KB)
  u32x4 x = {v, v + 1, v + 2, static_cast<unsigned>(w)};
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    size_t i;
    if constexpr (kPat == 0) i = base + u * 64 + threadIdx.x;
    else i = base + threadIdx.x * 8 + u;
    if (i < n) {
      if constexpr (kNT) __builtin_nontemporal_store(x, out + i);
      else out[i] = x;
    }
  }
}

// One-shot waves writing kKB contiguous KB each (1-KB stores, 8 in flight),
// optionally reading one unit per kMix units first (the chain kernels' mix:
// ~1 byte read per 8 written).
template <int kKB, int kMix, bool kNT>
__global__ __launch_bounds__(64) void k_fill_piece(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n,
                                                   unsigned v) {
  const size_t base = static_cast<size_t>(blockIdx.x) * (kKB * 64);  // units of 16 B
  u32x4 acc = {v, v, v, v};
  for (int b = 0; b < kKB; b += 8) {
    u32x4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t i = base + static_cast<size_t>(b + u) * 64 + threadIdx.x;
      x[u] = acc;
      if (kMix && ((b + u) % kMix) == 0 && i < n) x[u] = in[i];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t i = base + static_cast<size_t>(b + u) * 64 + threadIdx.x;
      if (i < n) {
        if constexpr (kNT) __builtin_nontemporal_store(x[u], out + i);
        else out[i] = x[u];
      }
    }
  }
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? std::atoll(argv[1]) : 2048) << 20;
  const size_t n = bytes / 16;
  u32x4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    return best;
  };
  std::printf("buffer %zu MB, %d CUs\n", bytes >> 20, cus);
  for (int bpc : {4, 8}) {
    const size_t lds = 160 * 1024 / bpc - 1024;  // bpc blocks fit per CU
    for (int waves_mult : {1, 4}) {
      const unsigned grid = cus * bpc * waves_mult;
      const float f0 = timeit([&] { hipLaunchKernelGGL(k_fill<false>, dim3(grid), dim3(256), lds, 0, a, n, 7u); });
      const float f1 = timeit([&] { hipLaunchKernelGGL(k_fill<true>, dim3(grid), dim3(256), lds, 0, a, n, 7u); });
      const float c0 = timeit([&] { hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(256), lds, 0, b, a, n); });
      const float c1 = timeit([&] { hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), lds, 0, b, a, n); });
      std::printf("blocks/CU %d grid %6u: fill %.2f TB/s, fill-nt %.2f TB/s, copy %.2f TB/s (w %.2f), copy-nt %.2f TB/s\n",
                  bpc, grid, bytes / f0 / 1e9, bytes / f1 / 1e9, 2 * bytes / c0 / 1e9, bytes / c0 / 1e9,
                  2 * bytes / c1 / 1e9);
    }
  }
  {
    const unsigned grid = static_cast<unsigned>((n + 511) / 512);
    const float p0 = timeit([&] { hipLaunchKernelGGL((k_fill_wave<0, false>), dim3(grid), dim3(64), 0, 0, a, n, 5u); });
    const float p0n = timeit([&] { hipLaunchKernelGGL((k_fill_wave<0, true>), dim3(grid), dim3(64), 0, 0, a, n, 5u); });
    const float p1 = timeit([&] { hipLaunchKernelGGL((k_fill_wave<1, false>), dim3(grid), dim3(64), 0, 0, a, n, 5u); });
    const float p1n = timeit([&] { hipLaunchKernelGGL((k_fill_wave<1, true>), dim3(grid), dim3(64), 0, 0, a, n, 5u); });
    std::printf("one-shot 8-KB waves (%u): 1-KB stores %.2f / nt %.2f TB/s; 64-B lanes %.2f / nt %.2f TB/s\n", grid,
                bytes / p0 / 1e9, bytes / p0n / 1e9, bytes / p1 / 1e9, bytes / p1n / 1e9);
  }
  {
    auto piece = [&](auto kern, int kb) {
      const unsigned grid = static_cast<unsigned>((n + kb * 64 - 1) / (kb * 64));
      return timeit([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, b, a, n, 9u); });
    };
    std::printf("one-shot waves, contiguous piece per wave, nt / default stores (TB/s of writes):\n");
    std::printf("  8 KB   %.2f / %.2f\n", bytes / piece(k_fill_piece<8, 0, true>, 8) / 1e9,
                bytes / piece(k_fill_piece<8, 0, false>, 8) / 1e9);
    std::printf("  32 KB  %.2f / %.2f\n", bytes / piece(k_fill_piece<32, 0, true>, 32) / 1e9,
                bytes / piece(k_fill_piece<32, 0, false>, 32) / 1e9);
    std::printf("  128 KB %.2f / %.2f\n", bytes / piece(k_fill_piece<128, 0, true>, 128) / 1e9,
                bytes / piece(k_fill_piece<128, 0, false>, 128) / 1e9);
    const float m8 = piece(k_fill_piece<32, 8, true>, 32);
    std::printf("  32 KB, 1 of 8 units read first (nt): %.2f TB/s written + %.2f read\n", bytes / m8 / 1e9,
                bytes / 8 / m8 / 1e9);
  }
  const float ms = timeit([&] { CK(hipMemsetAsync(a, 3, bytes, 0)); });
  std::printf("hipMemsetAsync: %.2f TB/s\n", bytes / ms / 1e9);
  return 0;
}
