// gbuild.hip -- gfx950 kernels of the GPU node-space rebuild (gbuild.hpp).
// Integer work over peer-indexed arrays: coalesced, HBM/latency-bound; the
// sort and the scan are hipcub's (rocPRIM) device primitives.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "gbuild.hpp"
#include "kernels.hpp"

namespace psamd {

namespace {

constexpr uint32_t kB = 256;
constexpr uint32_t kNoneP = 0xFFFFFFFFu;

constexpr uint32_t kStatBlocks = 1024;  // grid of the reducing kernels

uint32_t blocks(uint64_t n) { return static_cast<uint32_t>(std::max<uint64_t>(1, (n + kB - 1) / kB)); }

__global__ __launch_bounds__(kB) void k_scatter_pairs(const uint32_t* __restrict__ pairs, uint32_t n,
                                                      uint32_t* __restrict__ par, uint8_t* __restrict__ orph) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pairs[2 * i], v = pairs[2 * i + 1];
  par[p] = v >= kOrphanCode ? kNoneP : v;
  orph[p] = v == kOrphanCode;
}

// anc = upstream (root: itself), dep = 1 (root: 0)
__global__ __launch_bounds__(kB) void k_depth_init(const uint32_t* __restrict__ par, uint32_t n,
                                                   uint32_t root, uint32_t* __restrict__ anc,
                                                   uint32_t* __restrict__ dep) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= n) return;
  anc[p] = p == root ? root : par[p];
  dep[p] = p == root ? 0u : 1u;
}

// One pointer-jumping step: dep += dep[anc], anc = anc[anc]; the root is a
// fixed point, kNone (not subscribed / cut) absorbs.
__global__ __launch_bounds__(kB) void k_depth_jump(const uint32_t* __restrict__ ai,
                                                   const uint32_t* __restrict__ di,
                                                   uint32_t* __restrict__ ao, uint32_t* __restrict__ dout,
                                                   uint32_t n, uint32_t root) {
  const uint32_t p = blockIdx.x * kB + threadIdx.x;
  if (p >= n) return;
  const uint32_t a = ai[p];
  if (a == kNoneP || a == root) {
    ao[p] = a;
    dout[p] = di[p];
    return;
  }
  ao[p] = ai[a];
  dout[p] = di[p] + di[a];
}

// Block-wide max / sum through LDS: one global atomic per block (thousands of
// same-address atomics, one per wave, serialise in one L2 channel).
template <bool kMax>
__device__ uint32_t block_reduce(uint32_t v, uint32_t* lds) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint32_t o = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), s, 64));
    v = kMax ? max(v, o) : v + o;
  }
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  v = lds[0];
  for (uint32_t w = 1; w < kB / 64; ++w) v = kMax ? max(v, lds[w]) : v + lds[w];
  __syncthreads();
  return v;
}

// Keys of the reachable peers (grid-stride): kf.make(depth, parent, peer),
// ~0 otherwise.  gstat[0] += reachable, gstat[1] = max depth,
// gstat[3] += peers whose ancestor is neither the root nor cut (the jump
// steps did not cover their depth: the caller repeats with more steps).
__global__ __launch_bounds__(kB) void k_depth_keys(const uint32_t* __restrict__ anc,
                                                   const uint32_t* __restrict__ dep,
                                                   const uint32_t* __restrict__ par, uint32_t n,
                                                   uint32_t root, uint64_t* __restrict__ keys,
                                                   uint32_t* __restrict__ gstat, BuildKey kf) {
  __shared__ uint32_t lds[kB / 64];
  uint32_t cnt = 0, far = 0, m = 0;
  for (uint32_t p = blockIdx.x * kB + threadIdx.x; p < n; p += gridDim.x * kB) {
    const uint32_t a = anc[p];
    uint64_t k = ~0ull;
    if (a == root) {
      const uint32_t d = dep[p];
      const uint32_t pp = p == root ? 0u : par[p];
      k = kf.make(min(d, kBuildMaxDepth), pp, p);
      ++cnt;
      m = max(m, d);
    } else if (a != kNoneP) {
      ++far;
    }
    keys[p] = k;
  }
  cnt = block_reduce<false>(cnt, lds);
  m = block_reduce<true>(m, lds);
  far = block_reduce<false>(far, lds);
  if (threadIdx.x == 0) {
    if (cnt) atomicAdd(gstat + 0, cnt);
    if (m) atomicMax(gstat + 1, m);
    if (far) atomicAdd(gstat + 3, far);
  }
}

__global__ __launch_bounds__(kB) void k_fill_col(const uint32_t* __restrict__ row_ptr,
                                                 const uint32_t* __restrict__ first, uint32_t n_nodes,
                                                 uint32_t* __restrict__ col) {
  const uint32_t u = blockIdx.x * kB + threadIdx.x;
  if (u >= n_nodes) return;
  const uint32_t b = row_ptr[u], e = row_ptr[u + 1];
  for (uint32_t k = b; k < e; ++k) col[k] = first[u] + (k - b);
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

// Level starts of a topic's (depth, parent, peer)-sorted keys (first R valid).
__global__ __launch_bounds__(kB) void k_level_starts(const uint64_t* __restrict__ keys, uint32_t R,
                                                     uint32_t* __restrict__ lvl_start, BuildKey kf) {
  const uint32_t u = blockIdx.x * kB + threadIdx.x;
  if (u >= R) return;
  const uint32_t d = kf.depth(keys[u]);
  if (u == 0 || kf.depth(keys[u - 1]) != d) lvl_start[d] = u;
}

// Internal nodes per level and the largest fan-out of a topic placed at
// [nbase, nbase + R) with level starts lvl_start[0..depth] (topic-relative):
// a per-block LDS histogram over the levels, flushed with one atomic per
// non-empty bin (a tree has a few dozen levels: per-node global atomics on
// them serialise).
__global__ __launch_bounds__(kB) void k_level_internal(const uint32_t* __restrict__ deg, uint32_t nbase,
                                                       uint32_t R, const uint32_t* __restrict__ lvl_start,
                                                       uint32_t depth, uint32_t* __restrict__ lvl_internal,
                                                       uint32_t* __restrict__ max_deg) {
  __shared__ uint32_t hist[kBuildMaxDepth + 1];
  __shared__ uint32_t starts[kBuildMaxDepth + 2];
  __shared__ uint32_t lds[kB / 64];
  for (uint32_t d = threadIdx.x; d <= kBuildMaxDepth; d += kB) hist[d] = 0;
  for (uint32_t d = threadIdx.x; d <= depth; d += kB) starts[d] = lvl_start[d];
  __syncthreads();
  uint32_t m = 0;
  for (uint32_t u = blockIdx.x * kB + threadIdx.x; u < R; u += gridDim.x * kB) {
    const uint32_t dg = deg[nbase + u];
    if (!dg) continue;
    m = max(m, dg);
    uint32_t lo = 0, hi = depth;  // last level whose start <= u
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) / 2;
      if (starts[mid] <= u)
        lo = mid;
      else
        hi = mid - 1;
    }
    atomicAdd(hist + lo, 1u);
  }
  m = block_reduce<true>(m, lds);  // includes the barrier after the histogram
  for (uint32_t d = threadIdx.x; d <= depth; d += kB)
    if (hist[d]) atomicAdd(lvl_internal + d, hist[d]);
  if (threadIdx.x == 0 && m) atomicMax(max_deg, m);
}

// Fan-out and first child of every parent peer in one topic's (depth, parent,
// peer)-sorted keys (first R valid; keys[0] is the root): cnt[parent] += 1,
// firstidx[parent] = min index.  Siblings are contiguous and sorted by peer.
__global__ __launch_bounds__(kB) void k_child_stats(const uint64_t* __restrict__ keys, uint32_t R,
                                                    uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ firstidx, BuildKey kf) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i == 0 || i >= R) return;
  const uint32_t pp = kf.parent(keys[i]);
  atomicAdd(cnt + pp, 1u);
  atomicMin(firstidx + pp, i);
}

__global__ void k_place_root(const uint64_t* __restrict__ keys, uint32_t nbase, uint16_t topic,
                             const uint32_t* __restrict__ cnt, uint32_t* __restrict__ node_peer,
                             uint16_t* __restrict__ node_topic, uint32_t* __restrict__ local,
                             uint32_t* __restrict__ node_parent, uint32_t* __restrict__ deg, BuildKey kf) {
  if (threadIdx.x) return;
  const uint32_t peer = kf.peer(keys[0]);
  node_peer[nbase] = peer;
  node_topic[nbase] = topic;
  local[peer] = nbase;
  node_parent[nbase] = kNoneP;
  deg[nbase] = cnt[peer];
}

// BFS placement of level d (keys [lo, hi), nodes nbase + [lo, hi)) without a
// sort: the children of parent node u form one group at nbase + lo +
// childoff[u - prev0] (exclusive scan of the parents' fan-out, in parent node
// order), each child at its rank among its siblings (index - first index).
__global__ __launch_bounds__(kB) void k_place_level(
    const uint64_t* __restrict__ keys, uint32_t lo, uint32_t hi, uint32_t nbase, uint32_t prev0,
    const uint32_t* __restrict__ childoff, const uint32_t* __restrict__ cnt,
    const uint32_t* __restrict__ firstidx, uint16_t topic, uint32_t* __restrict__ node_peer,
    uint16_t* __restrict__ node_topic, uint32_t* __restrict__ local, uint32_t* __restrict__ node_parent,
    uint32_t* __restrict__ deg, uint32_t* __restrict__ first, BuildKey kf) {
  const uint32_t i = lo + blockIdx.x * kB + threadIdx.x;
  if (i >= hi) return;
  const uint64_t k = keys[i];
  const uint32_t peer = kf.peer(k);
  const uint32_t pp = kf.parent(k);
  const uint32_t pu = local[pp];
  const uint32_t f = firstidx[pp];
  const uint32_t node = nbase + lo + childoff[pu - prev0] + (i - f);
  node_peer[node] = peer;
  node_topic[node] = topic;
  local[peer] = node;
  node_parent[node] = pu;
  deg[node] = cnt[peer];
  if (i == f) first[pu] = node;
}

// BFS placement of level d in ONE launch, parent-centric: tile b (one
// block) owns the parent nodes pbase + [256 b, 256 b + 256) of level d - 1,
// scans their fan-out in the block and takes its prefix from the tiles before
// it by a decoupled look-back (status[b]: kLbAgg | the tile's sum once known,
// kLbIncl | the inclusive prefix once its own prefix is; tiles start in
// order, so a tile only ever waits on tiles already running).  The children
// of the tile's parents are then one contiguous range: child k of the tile's
// flattened child list is node cbase + prefix + k, its parent the tile's
// parent whose inclusive sum first exceeds k, its peer the key at
// firstidx[parent peer] + its sibling rank.  (The previous form: a device scan
// of the parents' fan-out -- two launches -- then a child-parallel placement;
// three launches per level.)  A look-back that spins past kLbSpin polls
// flags the build as failed (*err), and the caller builds on the host.
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbFlags = 3ull << 62;
constexpr uint32_t kLbSpin = 1u << 24;

__global__ __launch_bounds__(kB) void k_place_level_lb(
    const uint64_t* __restrict__ keys, uint32_t np, uint32_t pbase, uint32_t cbase,
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ firstidx, uint16_t topic,
    uint32_t* __restrict__ node_peer, uint16_t* __restrict__ node_topic, uint32_t* __restrict__ local,
    uint32_t* __restrict__ node_parent, uint32_t* __restrict__ deg, uint32_t* __restrict__ first,
    uint64_t* __restrict__ status, uint32_t* __restrict__ err, BuildKey kf) {
  __shared__ uint32_t incl_s[kB];
  __shared__ uint32_t peer_s[kB];
  __shared__ uint32_t wsum[kB / 64];
  __shared__ uint32_t prefix_s;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t tile = blockIdx.x;
  const uint32_t j0 = tile * kB + tid;
  const uint32_t u = pbase + j0;
  const bool valid = j0 < np;
  const uint32_t dg = valid ? deg[u] : 0u;
  peer_s[tid] = valid ? node_peer[u] : 0u;
  // block inclusive scan of the fan-out
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
    // the look-back, one wave: 64 predecessors per step (lane i reads tile
    // j - i), summed up to the nearest inclusive one
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
                                    : kLbIncl;  // (before tile 0: an inclusive zero)
        if (__any((v & kLbFlags) == 0)) {  // a predecessor has not published yet
          if (++spins > kLbSpin) {
            if (lane == 0) atomicOr(err, 1u);
            break;
          }
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
  // the tile's children, flattened: child k's parent is the first q with
  // incl_s[q] > k (binary search over the tile's 256 parents)
  for (uint32_t k = tid; k < agg; k += kB) {
    uint32_t lo = 0, hi = kB - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (incl_s[mid] > k)
        hi = mid;
      else
        lo = mid + 1;
    }
    const uint32_t q = lo;
    const uint32_t rank = k - (q ? incl_s[q - 1] : 0u);  // (k minus the parent's exclusive sum)
    const uint32_t pu = pbase + tile * kB + q;
    const uint32_t pp = peer_s[q];
    const uint32_t peer = kf.peer(keys[firstidx[pp] + rank]);
    const uint32_t node = cbase + prefix + k;
    node_peer[node] = peer;
    node_topic[node] = topic;
    local[peer] = node;
    node_parent[node] = pu;
    deg[node] = cnt[peer];
    if (rank == 0) first[pu] = node;
  }
}

// The small top levels of one topic in ONE block (one launch for what would be
// 3 launches per level): root, then each level 1 .. d_end - 1 (at most
// kBuildSmallLevel nodes and parents) with the parents' fan-out scanned in
// LDS.  Nodes placed by other waves of the block are read back through L1-
// bypassing loads after the barrier.
constexpr uint32_t kSmallB = 1024;
constexpr uint32_t kSmallPer = kBuildSmallLevel / kSmallB;

__device__ __forceinline__ uint32_t load_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kSmallB) void k_place_small(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ lvl, uint32_t d_end, uint32_t depth, uint32_t n_nodes,
    uint32_t nbase, uint16_t topic, const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ firstidx,
    uint32_t* __restrict__ node_peer, uint16_t* __restrict__ node_topic, uint32_t* local,
    uint32_t* __restrict__ node_parent, uint32_t* deg, uint32_t* __restrict__ first, BuildKey kf) {
  __shared__ uint32_t off[kBuildSmallLevel];
  __shared__ uint32_t wsum[kSmallB / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) {
    const uint32_t peer = kf.peer(keys[0]);
    node_peer[nbase] = peer;
    node_topic[nbase] = topic;
    local[peer] = nbase;
    node_parent[nbase] = kNoneP;
    deg[nbase] = cnt[peer];
  }
  __threadfence_block();
  __syncthreads();
  for (uint32_t d = 1; d < d_end; ++d) {
    const uint32_t plo = lvl[d - 1], lo = lvl[d];
    const uint32_t hi = d == depth ? n_nodes : lvl[d + 1];
    const uint32_t np = lo - plo;
    // exclusive scan of the parents' fan-out: kSmallPer per thread, then waves
    uint32_t v[kSmallPer];
    uint32_t run = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSmallPer; ++k) {
      const uint32_t j = tid * kSmallPer + k;
      v[k] = j < np ? load_agent(deg + nbase + plo + j) : 0u;
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
    uint32_t base = 0;
    for (uint32_t q = 0; q < w; ++q) base += wsum[q];
    uint32_t acc = base + incl - run;
#pragma unroll
    for (uint32_t k = 0; k < kSmallPer; ++k) {
      const uint32_t j = tid * kSmallPer + k;
      if (j < np) off[j] = acc;
      acc += v[k];
    }
    __syncthreads();
    for (uint32_t i = lo + tid; i < hi; i += kSmallB) {
      const uint64_t kk = keys[i];
      const uint32_t peer = kf.peer(kk);
      const uint32_t pp = kf.parent(kk);
      const uint32_t pu = load_agent(local + pp);
      const uint32_t f = firstidx[pp];
      const uint32_t node = nbase + lo + off[pu - nbase - plo] + (i - f);
      node_peer[node] = peer;
      node_topic[node] = topic;
      local[peer] = node;
      node_parent[node] = pu;
      deg[node] = cnt[peer];
      if (i == f) first[pu] = node;
    }
    __threadfence_block();
    __syncthreads();
  }
}

// out[i] = 1 iff peers[i] holds a node of the topic placed at [nbase, nbase +
// n_nodes) by the last build (local[] may hold stale ids: node_peer confirms)
// (the upward walk of an unreached peer: at most the depth of its cut
// subtree, <= n_peers hops; the build bounds attached depths by 255)
__global__ __launch_bounds__(kB) void k_reach_query(const uint32_t* __restrict__ peers, uint32_t n,
                                                    uint32_t n_peers, const uint32_t* __restrict__ local,
                                                    const uint32_t* __restrict__ node_peer, uint32_t nbase,
                                                    uint32_t n_nodes, const uint32_t* __restrict__ par,
                                                    const uint8_t* __restrict__ orph, uint32_t root,
                                                    uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = peers[i];
  uint8_t r = 0;
  if (p < n_peers) {
    const uint32_t u = local[p];
    r = u >= nbase && u - nbase < n_nodes && node_peer[u] == p;
    if (!r) {  // below_orphan (tree.cpp): the first peer without an upstream
      uint32_t q = p;
      for (uint32_t h = 0; h < n_peers && q != root; ++h) {
        const uint32_t up = par[q];
        if (up >= n_peers) {
          r = orph[q] ? 2 : 0;
          break;
        }
        q = up;
      }
    }
  }
  out[i] = r;
}

}  // namespace

hipError_t launch_reach_query(const uint32_t* peers, uint32_t n, uint32_t n_peers, const uint32_t* local,
                              const uint32_t* node_peer, uint32_t nbase, uint32_t n_nodes, const uint32_t* par,
                              const uint8_t* orph, uint32_t root, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_reach_query, dim3(blocks(n)), dim3(kB), 0, s, peers, n, n_peers, local, node_peer,
                     nbase, n_nodes, par, orph, root, out);
  return hipGetLastError();
}

hipError_t launch_child_stats(const uint64_t* keys, uint32_t R, uint32_t* cnt, uint32_t* firstidx,
                              BuildKey kf, hipStream_t s) {
  if (R < 2) return hipSuccess;
  hipLaunchKernelGGL(k_child_stats, dim3(blocks(R)), dim3(kB), 0, s, keys, R, cnt, firstidx, kf);
  return hipGetLastError();
}

hipError_t launch_place_root(const uint64_t* keys, uint32_t nbase, uint16_t topic, const uint32_t* cnt,
                             uint32_t* node_peer, uint16_t* node_topic, uint32_t* local,
                             uint32_t* node_parent, uint32_t* deg, BuildKey kf, hipStream_t s) {
  hipLaunchKernelGGL(k_place_root, dim3(1), dim3(64), 0, s, keys, nbase, topic, cnt, node_peer, node_topic,
                     local, node_parent, deg, kf);
  return hipGetLastError();
}

hipError_t launch_place_small(const uint64_t* keys, const uint32_t* lvl, uint32_t d_end, uint32_t depth, uint32_t n_nodes,
                              uint32_t nbase, uint16_t topic, const uint32_t* cnt, const uint32_t* firstidx,
                              uint32_t* node_peer, uint16_t* node_topic, uint32_t* local,
                              uint32_t* node_parent, uint32_t* deg, uint32_t* first, BuildKey kf, hipStream_t s) {
  if (d_end > depth + 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_place_small, dim3(1), dim3(kSmallB), 0, s, keys, lvl, d_end, depth, n_nodes, nbase, topic, cnt,
                     firstidx, node_peer, node_topic, local, node_parent, deg, first, kf);
  return hipGetLastError();
}

hipError_t launch_place_level(const uint64_t* keys, uint32_t lo, uint32_t hi, uint32_t nbase, uint32_t prev0,
                              const uint32_t* childoff, const uint32_t* cnt, const uint32_t* firstidx,
                              uint16_t topic, uint32_t* node_peer, uint16_t* node_topic, uint32_t* local,
                              uint32_t* node_parent, uint32_t* deg, uint32_t* first, BuildKey kf, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(k_place_level, dim3(blocks(hi - lo)), dim3(kB), 0, s, keys, lo, hi, nbase, prev0,
                     childoff, cnt, firstidx, topic, node_peer, node_topic, local, node_parent, deg, first, kf);
  return hipGetLastError();
}

hipError_t launch_place_level_lb(const uint64_t* keys, uint32_t np, uint32_t pbase, uint32_t cbase,
                                 const uint32_t* cnt, const uint32_t* firstidx, uint16_t topic, uint32_t* node_peer,
                                 uint16_t* node_topic, uint32_t* local, uint32_t* node_parent, uint32_t* deg,
                                 uint32_t* first, uint64_t* status, uint32_t* err, BuildKey kf, hipStream_t s) {
  if (np == 0) return hipSuccess;
  hipLaunchKernelGGL(k_place_level_lb, dim3(lb_tiles(np)), dim3(kB), 0, s, keys, np, pbase, cbase, cnt, firstidx,
                     topic, node_peer, node_topic, local, node_parent, deg, first, status, err, kf);
  return hipGetLastError();
}

hipError_t launch_level_starts(const uint64_t* keys, uint32_t R, uint32_t* lvl_start, BuildKey kf, hipStream_t s) {
  if (R == 0) return hipSuccess;
  hipLaunchKernelGGL(k_level_starts, dim3(blocks(R)), dim3(kB), 0, s, keys, R, lvl_start, kf);
  return hipGetLastError();
}

hipError_t launch_level_internal(const uint32_t* deg, uint32_t nbase, uint32_t R,
                                 const uint32_t* lvl_start, uint32_t depth, uint32_t* lvl_internal,
                                 uint32_t* max_deg, hipStream_t s) {
  if (R == 0) return hipSuccess;
  if (depth > kBuildMaxDepth) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_level_internal, dim3(std::min(blocks(R), kStatBlocks)), dim3(kB), 0, s, deg, nbase,
                     R, lvl_start, depth,
                     lvl_internal, max_deg);
  return hipGetLastError();
}

hipError_t launch_scatter_pairs(const uint32_t* pairs, uint32_t n, uint32_t* par, uint8_t* orph, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_pairs, dim3(blocks(n)), dim3(kB), 0, s, pairs, n, par, orph);
  return hipGetLastError();
}

hipError_t launch_depth_keys(const uint32_t* par, uint32_t n, uint32_t root, uint32_t jumps,
                             uint32_t* anc0, uint32_t* anc1, uint32_t* dep0, uint32_t* dep1,
                             uint64_t* keys, uint32_t* gstat, BuildKey kf, hipStream_t s) {
  hipLaunchKernelGGL(k_depth_init, dim3(blocks(n)), dim3(kB), 0, s, par, n, root, anc0, dep0);
  // after j jumps every peer's ancestor is 2^j levels up (or the root / cut)
  uint32_t *ai = anc0, *ao = anc1, *di = dep0, *dout = dep1;
  for (uint32_t j = 0; j < jumps; ++j) {
    hipLaunchKernelGGL(k_depth_jump, dim3(blocks(n)), dim3(kB), 0, s, ai, di, ao, dout, n, root);
    std::swap(ai, ao);
    std::swap(di, dout);
  }
  hipLaunchKernelGGL(k_depth_keys, dim3(std::min(blocks(n), kStatBlocks)), dim3(kB), 0, s, ai, di, par, n,
                     root, keys, gstat, kf);
  return hipGetLastError();
}

hipError_t sort_keys(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, uint32_t n,
                     BuildKey kf, bool peer_bits, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, in, out, n, peer_bits ? 0 : static_cast<int>(kf.b),
                                           static_cast<int>(kf.sort_bits()), s);
}

hipError_t scan_u32(void* temp, size_t* temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                    hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, out, n, s);
}

hipError_t launch_fill_col(const uint32_t* row_ptr, const uint32_t* first, uint32_t n_nodes,
                           uint32_t* col, hipStream_t s) {
  if (n_nodes == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_col, dim3(blocks(n_nodes)), dim3(kB), 0, s, row_ptr, first, n_nodes, col);
  return hipGetLastError();
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
