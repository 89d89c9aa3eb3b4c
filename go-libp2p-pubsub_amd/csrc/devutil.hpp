// devutil.hpp -- device helpers shared by the gfx950 kernels (kernels.hip,
// flood.hip): wave reductions, the hop record, and the device-coherent (sc1)
// accesses of in-launch hand-offs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace psamd {
namespace dev {

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = static_cast<uint32_t>(v), hi = static_cast<uint32_t>(v >> 32);
  lo = __shfl_xor(lo, m, 64);
  hi = __shfl_xor(hi, m, 64);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_u64(v, m);
  return v;
}

__device__ __forceinline__ uint32_t popc4(uint4 v) {
  return __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
}

// Parity mode: the delivery round of every newly set bit of word cw.
__device__ __forceinline__ void record_word(uint16_t* hop_rec, uint64_t cw, uint64_t m, uint32_t round) {
  uint16_t* h = hop_rec + cw * 64;
  while (m) {
    const int q = __ffsll(static_cast<long long>(m)) - 1;
    h[q] = hop_round(round);
    m &= m - 1;
  }
}

// One wave's counters for one round (pull-style byte model).
struct PullCtr {
  uint64_t deliv = 0, dup = 0;
  uint32_t sw = 0, kids = 0, reached = 0, parents = 0, pwords = 0;
};

// Counter slot k of the pull model from the seven wave sums (deliveries,
// seen words, nodes visited, nodes reached, parents, parent words, duplicates).
__device__ __forceinline__ uint64_t pull_ctr_pick(const uint64_t* t, uint32_t k) {
  switch (k) {
    case kCtrDeliveries: return t[0];
    case kCtrEntries: return t[4];
    case kCtrEntryWords: return t[5];
    case kCtrChildren: return t[2];
    case kCtrMeshChildren: return t[3];  // pull mode: nodes reached (generation writes)
    case kCtrSeenWrites: return t[1];
    case kCtrDuplicates: return t[6];
    default: return 0;
  }
}

// ---- device-coherent accesses (sc1) -----------------------------------------
// Bytes handed from one wave to another inside a launch are stored
// write-through and loaded past the L1 (MI355X_MICROARCH.md §Workgroup
// dispatch ... Valid forms; cdna_hip_programming.md §6 Guideline 16): 16-B
// rows by buffer ops with the sc1 cache bit, bytes and words by relaxed
// agent-scope atomics (global_store_byte / global_load_dword ... sc1).
constexpr int kAuxSC1 = 16;                  // buffer-op cache bits: sc1
constexpr int kRsrcWord3 = 0x00020000;       // raw buffer, 32-bit data format (gfx9 family)
constexpr uint32_t kOutOfRange = 0x80000000u;  // buffer offset past any range: load 0, store dropped

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, static_cast<int>(bytes), kRsrcWord3);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 ld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSC1);
  return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint64_t ld8_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxSC1);
  return static_cast<uint64_t>(v.y) << 32 | v.x;
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& v) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, kAuxSC1);
}
__device__ __forceinline__ void st8_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, uint64_t v) {
  const u32x2 x = {static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, kAuxSC1);
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint8_t* p, uint8_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dev
}  // namespace psamd
