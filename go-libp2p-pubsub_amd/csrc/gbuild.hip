// gbuild.hip -- gfx950 kernels of the GPU node-space rebuild (gbuild.hpp).
// Integer work over peer-indexed arrays: coalesced, HBM/latency-bound; the
// one scan over the peers (the child lists' offsets) is hipcub's.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "gbuild.hpp"
#include "kernels.hpp"

namespace psamd {

namespace {

constexpr uint32_t kB = 256;
constexpr uint32_t kNoneP = 0xFFFFFFFFu;


uint32_t blocks(uint64_t n) { return static_cast<uint32_t>(std::max<uint64_t>(1, (n + kB - 1) / kB)); }

__global__ __launch_bounds__(kB) void k_scatter_pairs(const uint32_t* __restrict__ pairs, uint32_t n,
                                                      uint32_t* __restrict__ par, uint8_t* __restrict__ orph) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pairs[2 * i], v = pairs[2 * i + 1];
  par[p] = v >= kOrphanCode ? kNoneP : v;
  orph[p] = v == kOrphanCode;
}

__global__ __launch_bounds__(kB) void k_node_flags(const uint32_t* __restrict__ node_peer,
                                                   const uint32_t* __restrict__ row_ptr,
                                                   const uint8_t* __restrict__ live, uint32_t n_nodes,
                                                   uint8_t* __restrict__ flags) {
  const uint32_t u = blockIdx.x * kB + threadIdx.x;
  if (u >= n_nodes) return;
  uint8_t f = live[node_peer[u]] ? kNodeLive : 0;
  if (row_ptr[u + 1] > row_ptr[u]) f |= kNodeInternal;
  flags[u] = f;
}

__global__ __launch_bounds__(kB) void k_root_flags(const uint32_t* __restrict__ roots, uint32_t n,
                                                   uint8_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i < n) flags[roots[i]] |= kNodeLive;  // roots forward (they are not recipients)
}

// out[i] = 1 iff peers[i] holds a node of the topic placed at [nbase, nbase +
// n_nodes) by the last build (local[] may hold stale ids: node_peer confirms)
// (the upward walk of an unreached peer: at most the depth of its cut
// subtree, <= n_peers hops; the build bounds attached depths by 255)
__global__ __launch_bounds__(kB) void k_reach_query(const uint32_t* __restrict__ peers, uint32_t n,
                                                    uint32_t n_peers, const uint32_t* __restrict__ par,
                                                    const uint8_t* __restrict__ orph, uint32_t root,
                                                    uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = peers[i];
  uint8_t r = 0;
  if (p < n_peers) {
    // up the topic's upstream array: the root (the peer holds a node of the
    // node space: the message reached it), or the first peer without an
    // upstream (below_orphan, tree.cpp: 2 if it is an Orphan)
    uint32_t q = p;
    r = 1;
    for (uint32_t h = 0; h < n_peers && q != root; ++h) {
      const uint32_t up = par[q];
      if (up >= n_peers) {
        r = orph[q] ? 2 : 0;
        break;
      }
      q = up;
    }
  }
  out[i] = r;
}

// ---- by-parent CSR BFS rebuild -----------

__global__ __launch_bounds__(kB) void k_clear(ClearRegions r) {
  for (uint32_t k = 0; k < r.n; ++k)
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kB + threadIdx.x; i < r.words[k];
         i += static_cast<uint64_t>(gridDim.x) * kB)
      r.p[k][i] = 0;
}

// cnt[v] += 1 for every peer p whose upstream v is a peer (histogram of the
// parent array)
__global__ __launch_bounds__(kB) void k_kid_count(const uint32_t* __restrict__ par, uint32_t n,
                                                  uint32_t* __restrict__ cnt) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= n) return;
  const uint32_t v = par[p];
  if (v < n) atomicAdd(cnt + v, 1u);
}

// kids[koff[v] + i] = the i-th arriving child of v (order fixed below)
__global__ __launch_bounds__(kB) void k_kid_scatter(const uint32_t* __restrict__ par, uint32_t n,
                                                    const uint32_t* __restrict__ koff, uint32_t* __restrict__ fill,
                                                    uint32_t* __restrict__ kids) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= n) return;
  const uint32_t v = par[p];
  if (v < n) kids[koff[v] + atomicAdd(fill + v, 1u)] = p;
}

// Siblings in peer order (a deterministic BFS numbering): a parent's list of
// at most kKidSmall children sorted by its own thread; longer lists are
// queued for k_kid_sort_big.
constexpr uint32_t kKidSmall = 32;
constexpr uint32_t kKidBig = 4096;  // the LDS sort's capacity (longer lists keep their arrival order)
__global__ __launch_bounds__(kB) void k_kid_sort(const uint32_t* __restrict__ koff, const uint32_t* __restrict__ cnt,
                                                 uint32_t n, uint32_t* __restrict__ kids, uint32_t* __restrict__ big,
                                                 uint32_t* __restrict__ n_big) {
  const uint32_t v = blockIdx.x * kB + threadIdx.x;
  if (v >= n) return;
  const uint32_t c = cnt[v];
  if (c < 2) return;
  if (c > kKidSmall) {
    big[atomicAdd(n_big, 1u)] = v;
    return;
  }
  uint32_t* k = kids + koff[v];
  for (uint32_t i = 1; i < c; ++i) {
    const uint32_t x = k[i];
    uint32_t j = i;
    for (; j > 0 && k[j - 1] > x; --j) k[j] = k[j - 1];
    k[j] = x;
  }
}

// One block per queued long list (grid-stride): a bitonic sort in LDS
__global__ __launch_bounds__(kB) void k_kid_sort_big(const uint32_t* __restrict__ koff,
                                                     const uint32_t* __restrict__ cnt, uint32_t* __restrict__ kids,
                                                     const uint32_t* __restrict__ big,
                                                     const uint32_t* __restrict__ n_big) {
  __shared__ uint32_t x[kKidBig];
  const uint32_t nb = *n_big;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t v = big[b];
    const uint32_t c = cnt[v];
    if (c > kKidBig) continue;
    uint32_t* k = kids + koff[v];
    uint32_t m = 1;
    while (m < c) m <<= 1;
    for (uint32_t i = threadIdx.x; i < m; i += kB) x[i] = i < c ? k[i] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t size = 2; size <= m; size <<= 1)
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t i = threadIdx.x; i < m; i += kB) {
          const uint32_t j = i ^ stride;
          if (j > i) {
            const bool up = (i & size) == 0;
            const uint32_t a = x[i], bb = x[j];
            if ((a > bb) == up) {
              x[i] = bb;
              x[j] = a;
            }
          }
        }
        __syncthreads();
      }
    for (uint32_t i = threadIdx.x; i < c; i += kB) k[i] = x[i];
    __syncthreads();
  }
}

// The placement of a child node c (topic-relative index cr >= 1, level d)
// of parent node pu: node arrays, the peer -> node map, its flags (live;
// internal when the peer has children) and its CSR column (edge cr - 1 of
// the topic: BFS numbering makes col the identity shifted by one).
__device__ __forceinline__ bool place_child(const PlaceArgs& P, uint32_t nbase, uint32_t ebase, uint32_t cr,
                                            uint32_t pu, uint32_t peer) {
  const uint32_t c = nbase + cr;
  P.node_peer[c] = peer;
  P.node_topic[c] = P.topic;
  P.local[peer] = c;
  P.node_parent[c] = pu;
  P.col[ebase + cr - 1] = c;
  const uint32_t dg = P.cnt[peer];
  P.ndeg[c] = dg;
  P.nkat[c] = P.koff[peer];
  P.flags[c] = (P.live[peer] ? kNodeLive : 0) | (dg ? kNodeInternal : 0);
  return dg != 0;
}

// A parent node's CSR row and first child (topic-relative child start cs)
__device__ __forceinline__ void place_row(const PlaceArgs& P, uint32_t nbase, uint32_t ebase, uint32_t u,
                                          uint32_t cs) {
  P.row_ptr[u] = ebase + cs - 1;
  P.first[u] = nbase + cs;
}

// The end of a level pass: the next level's start, the topic's node and edge
// end (the next active topic's bases, and the CSR's closing entry)
__device__ __forceinline__ void place_close(const PlaceArgs& P, uint32_t nbase, uint32_t ebase, uint32_t d,
                                            uint32_t next_lo) {
  P.lvl[d + 1] = next_lo;
  P.tb[2 * P.a + 2] = nbase + next_lo;
  P.tb[2 * P.a + 3] = ebase + next_lo - 1;
  P.row_ptr[nbase + next_lo] = ebase + next_lo - 1;
  if (next_lo > P.lvl[d]) P.gst[kGstDepth] = d;
  __threadfence();
  P.gst[kGstDone] = d;
}

// The root and the small top levels of one topic in ONE block: each level d
// = 1 .. d_limit - 1 whose parents number at most kBuildTopLevel, from the
// parents' fan-out scanned in LDS, children flattened in parent order (a
// binary search finds each child's parent).  Stops at the first larger level
// (the look-back launches take over) or when the tree ends.
constexpr uint32_t kSmallB = kBuildTopLevel;
constexpr uint32_t kSmallPer = 1;  // parents per thread

__device__ __forceinline__ uint32_t load_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kSmallB) void k_place_top(PlaceArgs P, uint32_t d_limit) {
  __shared__ uint32_t off[kBuildTopLevel + 1];
  __shared__ uint32_t wsum[kSmallB / 64];
  __shared__ uint32_t red[kSmallB / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nbase = P.tb[2 * P.a], ebase = P.tb[2 * P.a + 1];
  if (tid == 0) {
    const uint32_t r = P.root;
    P.node_peer[nbase] = r;
    P.node_topic[nbase] = P.topic;
    P.local[r] = nbase;
    P.node_parent[nbase] = kNoneP;
    const bool internal = P.cnt[r] != 0;
    P.ndeg[nbase] = P.cnt[r];
    P.nkat[nbase] = P.koff[r];
    P.flags[nbase] = kNodeLive | (internal ? kNodeInternal : 0);  // roots forward (they are not recipients)
    P.lvl[0] = 0;
    P.lvl[1] = 1;
    P.lvl[256] = internal ? 1u : 0u;
    P.gst[kGstDepth] = 0;
    P.gst[kGstMaxDeg] = P.cnt[r];
    P.gst[kGstDone] = 0;
    P.tb[2 * P.a + 2] = nbase + 1;
    P.tb[2 * P.a + 3] = ebase;
    P.row_ptr[nbase + 1] = ebase;
  }
  __threadfence_block();
  __syncthreads();
  uint32_t plo = 0, lo = 1, mdeg = 0;
  for (uint32_t d = 1; d < d_limit; ++d) {
    const uint32_t np = lo - plo;
    if (np == 0 || np > kBuildTopLevel) break;
    // exclusive scan of the parents' fan-out: kSmallPer per thread, then waves
    uint32_t v[kSmallPer];
    uint32_t run = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSmallPer; ++k) {
      const uint32_t j = tid * kSmallPer + k;
      v[k] = j < np ? load_agent(P.ndeg + nbase + plo + j) : 0u;
      run += v[k];
    }
    uint32_t incl = run;
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
      const uint32_t o = static_cast<uint32_t>(__shfl_up(static_cast<int>(incl), sh, 64));
      if (lane >= static_cast<uint32_t>(sh)) incl += o;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (uint32_t q = 0; q < kSmallB / 64; ++q) {
      base += q < w ? wsum[q] : 0u;
      total += wsum[q];
    }
    uint32_t acc = base + incl - run;
#pragma unroll
    for (uint32_t k = 0; k < kSmallPer; ++k) {
      const uint32_t j = tid * kSmallPer + k;
      if (j < np) {
        off[j] = acc;  // exclusive
        place_row(P, nbase, ebase, nbase + plo + j, lo + acc);
        mdeg = max(mdeg, v[k]);
      }
      acc += v[k];
    }
    if (tid == 0) off[np] = total;
    __syncthreads();
    uint32_t n_int = 0;
    for (uint32_t k = tid; k < total; k += kSmallB) {
      uint32_t a = 0, b = np - 1;  // the last parent whose exclusive offset <= k
      while (a < b) {
        const uint32_t mid = (a + b + 1) >> 1;
        if (off[mid] <= k)
          a = mid;
        else
          b = mid - 1;
      }
      const uint32_t peer = P.kids[load_agent(P.nkat + nbase + plo + a) + (k - off[a])];
      n_int += place_child(P, nbase, ebase, lo + k, nbase + plo + a, peer) ? 1u : 0u;
    }
    n_int = __reduce_add_sync(~0ull, n_int);
    if (lane == 0) red[w] = n_int;
    __threadfence_block();
    __syncthreads();
    if (tid == 0) {
      uint32_t t = 0;
      for (uint32_t q = 0; q < kSmallB / 64; ++q) t += red[q];
      P.lvl[256 + d] = t;
      place_close(P, nbase, ebase, d, lo + total);
    }
    __syncthreads();
    plo = lo;
    lo += total;
  }
  mdeg = __reduce_max_sync(~0ull, mdeg);
  if (lane == 0 && mdeg) atomicMax(P.gst + kGstMaxDeg, mdeg);
}

// Level d (the children of level d - 1's nodes) in ONE launch, parent-centric
// (tile b = one block owns the parents 256 b .. 256 b + 255 of the level,
// scans their fan-out and takes its prefix from the tiles before it by a
// decoupled look-back -- status[b], zeroed per launch -- so the children of
// the tile's parents are one contiguous node range).  The level's size comes
// from the level table the previous launch closed; the grid is the host's
// estimate: a level with more tiles than blocks flags kBuildErrGrid and the
// build is redone with full grids.  A level the top kernel already placed is
// skipped; a launch whose parent level is not placed flags kBuildErrOrder.
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbFlags = 3ull << 62;
constexpr uint32_t kLbSpin = 1u << 24;

__global__ __launch_bounds__(kB) void k_place_lb(PlaceArgs P, uint32_t d, uint64_t* __restrict__ status) {
  __shared__ uint32_t incl_s[kB];
  __shared__ uint32_t peer_s[kB];
  __shared__ uint32_t wsum[kB / 64];
  __shared__ uint32_t prefix_s;
  const uint32_t done = P.gst[kGstDone];
  if (done >= d) return;  // (placed by the top kernel)
  if (done + 1 != d) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(P.err, kBuildErrOrder);
    return;
  }
  const uint32_t plo = P.lvl[d - 1], lo = P.lvl[d], np = lo - plo;
  const uint32_t nbase = P.tb[2 * P.a], ebase = P.tb[2 * P.a + 1];
  if (np == 0) {  // the tree ended above: close the level
    if (blockIdx.x == 0 && threadIdx.x == 0) place_close(P, nbase, ebase, d, lo);
    return;
  }
  const uint32_t ntiles = lb_tiles(np);
  if (ntiles > gridDim.x) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(P.err, kBuildErrGrid);
    return;
  }
  // the tile from a ticket (status[-1], zeroed with the status words): a
  // tile only ever waits on tiles whose blocks already run, whatever order
  // the dispatcher starts blocks in
  __shared__ uint32_t tile_s;
  if (threadIdx.x == 0) tile_s = atomicAdd(reinterpret_cast<unsigned int*>(status - 1), 1u);
  __syncthreads();
  const uint32_t tile = tile_s;
  if (tile >= ntiles) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t j0 = tile * kB + tid;
  const uint32_t u = nbase + plo + j0;
  const bool valid = j0 < np;
  const uint32_t dg = valid ? P.ndeg[u] : 0u;
  peer_s[tid] = valid ? P.nkat[u] : 0u;  // (the parent's first child in kids)
  uint32_t inc = dg;
#pragma unroll
  for (int sh = 1; sh < 64; sh <<= 1) {
    const uint32_t o = static_cast<uint32_t>(__shfl_up(static_cast<int>(inc), sh, 64));
    if (lane >= static_cast<uint32_t>(sh)) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = 0, agg = 0;
#pragma unroll
  for (uint32_t q = 0; q < kB / 64; ++q) {
    base += q < w ? wsum[q] : 0u;
    agg += wsum[q];
  }
  incl_s[tid] = base + inc;
  if (w == 0) {
    uint32_t prefix = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(status, kLbIncl | agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(status + tile, kLbAgg | agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t spins = 0;
      int32_t j = static_cast<int32_t>(tile) - 1;
      for (;;) {
        const int32_t idx = j - static_cast<int32_t>(lane);
        const uint64_t v = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                    : kLbIncl;
        if (__any((v & kLbFlags) == 0)) {
          if (++spins > kLbSpin) {
            if (lane == 0) atomicOr(P.err, kBuildErrStall);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const uint64_t incl_mask = __ballot((v & kLbFlags) == kLbIncl);
        const uint32_t stop = incl_mask ? static_cast<uint32_t>(__builtin_ctzll(incl_mask)) : 63u;
        uint32_t part = lane <= stop ? static_cast<uint32_t>(v) : 0u;
#pragma unroll
        for (int sh = 32; sh >= 1; sh >>= 1) part += static_cast<uint32_t>(__shfl_xor(static_cast<int>(part), sh, 64));
        prefix += part;
        if (incl_mask) break;
        j -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(status + tile, kLbIncl | (prefix + agg), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) prefix_s = prefix;
  }
  __syncthreads();
  const uint32_t prefix = prefix_s;
  if (valid) place_row(P, nbase, ebase, u, lo + prefix + incl_s[tid] - dg);
  uint32_t n_int = 0;
  for (uint32_t k = tid; k < agg; k += kB) {
    uint32_t a = 0, b = kB - 1;  // the first parent whose inclusive sum exceeds k
    while (a < b) {
      const uint32_t mid = (a + b) >> 1;
      if (incl_s[mid] > k)
        b = mid;
      else
        a = mid + 1;
    }
    const uint32_t rank = k - (a ? incl_s[a - 1] : 0u);
    const uint32_t peer = P.kids[peer_s[a] + rank];
    n_int += place_child(P, nbase, ebase, lo + prefix + k, nbase + plo + tile * kB + a, peer) ? 1u : 0u;
  }
  n_int = __reduce_add_sync(~0ull, n_int);
  uint32_t mdeg = __reduce_max_sync(~0ull, dg);
  if (lane == 0) {
    if (n_int) atomicAdd(P.lvl + 256 + d, n_int);
    if (mdeg) atomicMax(P.gst + kGstMaxDeg, mdeg);
  }
  if (tile == ntiles - 1 && tid == 0) place_close(P, nbase, ebase, d, lo + prefix + agg);
}

}  // namespace


hipError_t launch_clear(const ClearRegions& r, hipStream_t s) {
  if (r.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_clear, dim3(1024), dim3(kB), 0, s, r);
  return hipGetLastError();
}

hipError_t build_kids(const uint32_t* par, uint32_t n, uint32_t* cnt, uint32_t* koff, uint32_t* fill, uint32_t* kids,
                      uint32_t* big, uint32_t* n_big, void* temp, size_t temp_bytes, hipStream_t s) {
  hipLaunchKernelGGL(k_kid_count, dim3(blocks(n)), dim3(kB), 0, s, par, n, cnt);
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, cnt, koff, n + 1, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_kid_scatter, dim3(blocks(n)), dim3(kB), 0, s, par, n, koff, fill, kids);
  hipLaunchKernelGGL(k_kid_sort, dim3(blocks(n)), dim3(kB), 0, s, koff, cnt, n, kids, big, n_big);
  hipLaunchKernelGGL(k_kid_sort_big, dim3(64), dim3(kB), 0, s, koff, cnt, kids, big, n_big);
  return hipGetLastError();
}

hipError_t launch_place_top(const PlaceArgs& P, uint32_t d_limit, hipStream_t s) {
  hipLaunchKernelGGL(k_place_top, dim3(1), dim3(kSmallB), 0, s, P, d_limit);
  return hipGetLastError();
}

hipError_t launch_place_lb(const PlaceArgs& P, uint32_t d, uint32_t grid, uint64_t* status, hipStream_t s) {
  hipLaunchKernelGGL(k_place_lb, dim3(std::max<uint32_t>(grid, 1)), dim3(kB), 0, s, P, d, status);
  return hipGetLastError();
}

hipError_t launch_reach_query(const uint32_t* peers, uint32_t n, uint32_t n_peers, const uint32_t* par,
                              const uint8_t* orph, uint32_t root, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_reach_query, dim3(blocks(n)), dim3(kB), 0, s, peers, n, n_peers, par, orph, root, out);
  return hipGetLastError();
}

hipError_t launch_scatter_pairs(const uint32_t* pairs, uint32_t n, uint32_t* par, uint8_t* orph, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_pairs, dim3(blocks(n)), dim3(kB), 0, s, pairs, n, par, orph);
  return hipGetLastError();
}

hipError_t scan_u32(void* temp, size_t* temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                    hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, out, n, s);
}

hipError_t launch_node_flags(const uint32_t* node_peer, const uint32_t* row_ptr,
                             const uint8_t* live, uint32_t n_nodes, const uint32_t* roots,
                             uint32_t n_roots, uint8_t* flags, hipStream_t s) {
  if (n_nodes)
    hipLaunchKernelGGL(k_node_flags, dim3(blocks(n_nodes)), dim3(kB), 0, s, node_peer, row_ptr, live,
                       n_nodes, flags);
  if (n_roots)
    hipLaunchKernelGGL(k_root_flags, dim3(blocks(n_roots)), dim3(kB), 0, s, roots, n_roots, flags);
  return hipGetLastError();
}

}  // namespace psamd
