// FETCH_SIZE calibration by load width (MI355X_MICROARCH.md §HBM: "FETCH_SIZE
// reports exactly 1/2 of the bytes of a wide coalesced streaming read ...
// other access widths are uncalibrated").  Each kernel reads the same 2 GiB
// buffer once, coalesced, with 16-, 8-, 4- or 1-byte loads per lane (and the
// 4-byte LDS-DMA form the pull kernels stage metadata with), and writes one
// word per block; rocprofv3 --pmc FETCH_SIZE over this program gives the
// counter's bytes per true byte for each width:
//   hipcc -O3 --offload-arch=gfx950 fetch_probe.hip -o fetch_probe
//   rocprofv3 --pmc FETCH_SIZE -f csv -d out -o run -- ./fetch_probe
#include <hip/hip_runtime.h>

#include <cstdint>
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

template <class T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ in, size_t n, unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
    const T v = in[i];
    if constexpr (sizeof(T) == 16) {
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    } else {
      acc ^= static_cast<unsigned>(v) ^ static_cast<unsigned>(static_cast<uint64_t>(v) >> 32);
    }
  }
  __shared__ unsigned red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int k = 0; k < 256; ++k) t ^= red[k];
    out[blockIdx.x] = t;
  }
}

// 4-byte LDS-DMA (global_load_lds_dword): the metadata staging form
__global__ __launch_bounds__(256) void k_read_lds4(const unsigned* __restrict__ in, size_t n,
                                                   unsigned* __restrict__ out) {
  __shared__ unsigned buf[256];
  unsigned acc = 0;
  for (size_t i0 = static_cast<size_t>(blockIdx.x) * 256; i0 < n; i0 += static_cast<size_t>(gridDim.x) * 256) {
    __builtin_amdgcn_global_load_lds(in + i0 + threadIdx.x, buf + (threadIdx.x & ~63u), 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    acc ^= buf[threadIdx.x];
    __syncthreads();
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// scattered 8-byte loads, one per `stride` bytes (a line each): what a
// request for a partly used line is tallied as
__global__ __launch_bounds__(256) void k_gather8(const uint64_t* __restrict__ in, size_t n, size_t stride_words,
                                                 unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
    const uint64_t v = in[i * stride_words];
    acc ^= static_cast<unsigned>(v);
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  const size_t bytes = 2ull << 30;
  void* in = nullptr;
  unsigned* out = nullptr;
  CK(hipMalloc(&in, bytes));
  CK(hipMemset(in, 1, bytes));
  const unsigned grid = 4096;
  CK(hipMalloc(&out, grid * 4));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_read<u32x4>, dim3(grid), dim3(256), 0, 0, static_cast<const u32x4*>(in), bytes / 16, out);
    hipLaunchKernelGGL(k_read<uint64_t>, dim3(grid), dim3(256), 0, 0, static_cast<const uint64_t*>(in), bytes / 8, out);
    hipLaunchKernelGGL(k_read<unsigned>, dim3(grid), dim3(256), 0, 0, static_cast<const unsigned*>(in), bytes / 4, out);
    hipLaunchKernelGGL(k_read<uint8_t>, dim3(grid), dim3(256), 0, 0, static_cast<const uint8_t*>(in), bytes, out);
    hipLaunchKernelGGL(k_read_lds4, dim3(grid), dim3(256), 0, 0, static_cast<const unsigned*>(in), bytes / 4, out);
    // one 8-B word per 64 B, per 128 B and per 256 B (2 GiB / stride loads)
    for (size_t st : {8, 16, 32})
      hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(256), 0, 0, static_cast<const uint64_t*>(in), bytes / (st * 8), st,
                         out);
  }
  CK(hipDeviceSynchronize());
  std::printf("fetch_probe: %zu bytes read per kernel (16/8/4/1-byte loads, 4-byte LDS-DMA; then one 8-B load "
              "per 64/128/256 B), 2 reps\n", bytes);
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
