// The s_memrealtime frequency on this MI355X: hipDeviceAttributeWallClockRate
// against two stamps 200 ms apart on the host clock.
//   hipcc -O3 --offload-arch=gfx950 clock_probe.hip -o clock_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k_stamp(unsigned long long* out) {
  if (threadIdx.x == 0) *out = __builtin_amdgcn_s_memrealtime();
}

int main() {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess) return 1;
  unsigned long long* d;
  unsigned long long h[2];
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  k_stamp<<<1, 64>>>(d);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const auto t0 = std::chrono::steady_clock::now();
  k_stamp<<<1, 64>>>(d);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  k_stamp<<<1, 64>>>(d + 1);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const auto t1 = std::chrono::steady_clock::now();
  if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const double host_s = std::chrono::duration<double>(t1 - t0).count();
  std::printf("wall clock rate attribute: %d kHz; s_memrealtime: %llu ticks in %.6f s of host time = %.3f MHz\n", khz,
              h[1] - h[0], host_s, (h[1] - h[0]) / host_s / 1e6);
  return 0;
}
