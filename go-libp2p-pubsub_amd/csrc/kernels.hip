// kernels.hip -- gfx950 kernels of the subtree-dissemination hot path.
//
// One synchronous round = k_expand over the compacted frontier, then the
// ballot/prefix-scan compaction (k_flag_count + k_flag_compact) of the nodes
// that received something and have children.  Messages travel as bits: node
// u's row of W 64-bit words holds, for the window's messages of u's topic,
//   seen[u]    the messages u has already delivered (dedup record),
//   arrival[u] the messages that reached u in the previous round.
// A frontier node p forwards arrival[p] to every child c:
//   new = arrival[p] & ~seen[c]   (drop already-seen message ids)
// restricted to live (subscribed) children; seen[c] |= new; arrival'[c] = new.
// Reference: subtree.forwardMessage (subtree.go:319-354) and
// client.processMessages (client.go:100-132).  Design: DESIGN.md §5.
#include "kernels.hpp"

namespace psamd {

namespace {

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

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Block-wide exclusive scan of one u32 per thread (kBlock threads); returns
// the exclusive prefix and writes the block total to *total.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[kBlock / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kBlock / 64; ++i) {
    if (i < wid) off += wsum[i];
    tot += wsum[i];
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v) {
  uint32_t tot;
  (void)block_excl_scan(v, &tot);
  return tot;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ---------------------------------------------------------------- seeds ---
// Topic.PublishMessage (pubsub.go:111-120): the root "has" its own messages
// (it is not a recipient) and forwards them in the next round.
__global__ __launch_bounds__(kBlock) void k_seed(const SeedDev* __restrict__ seeds, uint32_t lo,
                                                 uint32_t hi, uint64_t* __restrict__ arrivals,
                                                 uint64_t* __restrict__ seen,
                                                 uint8_t* __restrict__ next_flag) {
  const uint32_t i = lo + blockIdx.x * kBlock + threadIdx.x;
  if (i >= hi) return;
  const SeedDev s = seeds[i];
  arrivals[s.woff] |= s.mask;
  seen[s.woff] |= s.mask;
  next_flag[s.node] = 1;
}

// --------------------------------------------------------------- expand ---
// One wave per frontier node p (grid-stride).  The wave flattens p's
// (child j, word w) pairs, deg*W of them, over its 64 lanes: for W >= 64 one
// iteration touches 512 contiguous bytes of the children's seen rows (BFS
// numbering puts siblings next to each other).  Tree topics own each child
// row exclusively (one parent), so the test-and-set is a plain RMW; mesh
// topics use returning 64-bit atomicOr so exactly one parent wins each bit.
template <bool kRecord>
__global__ __launch_bounds__(kBlock) void k_expand(ExpandArgs a, uint32_t round) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave =
      __builtin_amdgcn_readfirstlane((blockIdx.x * kBlock + threadIdx.x) >> 6);
  const uint32_t n_waves = (gridDim.x * kBlock) >> 6;
  const uint32_t n = *a.n_front;

  uint64_t c_deliv = 0, c_dup = 0, c_items = 0, c_seen_w = 0, c_arr_w = 0;
  uint32_t c_ent = 0, c_ent_words = 0, c_kids = 0;

  for (uint32_t e = wave; e < n; e += n_waves) {
    const uint32_t p = __builtin_amdgcn_readfirstlane(a.frontier[e]);
    const uint32_t t = __builtin_amdgcn_readfirstlane(a.node_topic[p]);
    const TopicDev T = a.topics[t];
    const uint32_t rs = __builtin_amdgcn_readfirstlane(a.row_ptr[p]);
    const uint32_t deg = __builtin_amdgcn_readfirstlane(a.row_ptr[p + 1]) - rs;
    const uint32_t W = T.W;
    if (W == 0) continue;  // idle topic in this window (never seeded)
    const uint64_t pw = T.wbase + static_cast<uint64_t>(p - T.nbase) * W;
    const uint64_t cbase = T.wbase - static_cast<uint64_t>(T.nbase) * W;
    const bool mesh = (T.flags & kTopicMesh) != 0;
    c_ent += 1;
    c_ent_words += W;
    c_kids += deg;
    // children in chunks of <= 2^16/W so that it * W < 2^32 and the
    // multiply-high split below is exact (one chunk for any tree)
    const uint32_t chunk = W >= 65536 ? 1u : (65536u / W);
    for (uint32_t j0 = 0; j0 < deg; j0 += chunk) {
    const uint32_t items = min(chunk, deg - j0) * W;
    for (uint32_t it = lane; it < items; it += 64) {
      const uint32_t j = j0 + static_cast<uint32_t>((static_cast<uint64_t>(it) * T.magic) >> 32);
      const uint32_t w = it - (j - j0) * W;
      const uint32_t c = a.col[rs + j];
      const uint8_t f = a.node_flags[c];
      const uint64_t m = a.a_cur[pw + w];
      if (!(f & kNodeLive) || m == 0) continue;
      const uint64_t cw = cbase + static_cast<uint64_t>(c) * W + w;
      const bool internal = (f & kNodeInternal) != 0;
      uint64_t old, nm;
      if (mesh) {
        old = atomicOr(reinterpret_cast<unsigned long long*>(a.seen + cw),
                       static_cast<unsigned long long>(m));
        nm = m & ~old;
        if (nm && internal)
          atomicOr(reinterpret_cast<unsigned long long*>(a.a_next + cw),
                   static_cast<unsigned long long>(nm));
      } else {
        old = a.seen[cw];
        nm = m & ~old;
        if (nm) {
          a.seen[cw] = old | nm;
          if (internal) a.a_next[cw] = nm;
        }
      }
      c_items += 1;
      c_dup += __popcll(m & old);
      if (nm) {
        c_deliv += __popcll(nm);
        c_seen_w += 1;
        if (internal) {
          c_arr_w += 1;
          a.next_flag[c] = 1;
        }
        if constexpr (kRecord) {
          uint8_t* h = a.hop_rec + cw * 64;
          uint64_t b = nm;
          while (b) {
            const int k = __ffsll(static_cast<long long>(b)) - 1;
            h[k] = static_cast<uint8_t>(round);
            b &= b - 1;
          }
        }
      }
    }
    }
    // consume-and-clear: arrival rows are zero outside the frontier
    for (uint32_t w = lane; w < W; w += 64) a.a_cur[pw + w] = 0;
  }

  c_deliv = wave_sum_u64(c_deliv);
  c_dup = wave_sum_u64(c_dup);
  c_items = wave_sum_u64(c_items);
  c_seen_w = wave_sum_u64(c_seen_w);
  c_arr_w = wave_sum_u64(c_arr_w);
  if (lane == 0) {
    uint64_t* out = a.partials + static_cast<uint64_t>(wave) * kNumCtr;
    out[kCtrDeliveries] = c_deliv;
    out[kCtrDuplicates] = c_dup;
    out[kCtrEntries] = c_ent;
    out[kCtrEntryWords] = c_ent_words;
    out[kCtrChildren] = c_kids;
    out[kCtrItemReads] = c_items;
    out[kCtrSeenWrites] = c_seen_w;
    out[kCtrArrivalWrites] = c_arr_w;
  }
}

// ------------------------------------------------------------ compaction ---
// Pass 1: per-block count of flagged nodes (16 one-byte flags per lane, one
// 16-B load).  Block 0 also folds the expand kernel's per-wave counters into
// this round's statistics.
__global__ __launch_bounds__(kBlock) void k_flag_count(const uint8_t* __restrict__ flags,
                                                       uint32_t n_pad,
                                                       uint32_t* __restrict__ wg_count,
                                                       const uint64_t* __restrict__ partials,
                                                       uint32_t n_waves,
                                                       uint64_t* __restrict__ round_stats) {
  const uint32_t base = blockIdx.x * kFlagsPerBlock + threadIdx.x * kFlagsPerThread;
  uint32_t c = 0;
  if (base < n_pad) {
    const uint4 v = *reinterpret_cast<const uint4*>(flags + base);
    c = __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  }
  c = block_sum_u32(c);
  if (threadIdx.x == 0) wg_count[blockIdx.x] = c;
  if (blockIdx.x == 0 && round_stats != nullptr) {
    __shared__ uint64_t red[kNumCtr][kBlock / 64];
    uint64_t acc[kNumCtr];
#pragma unroll
    for (int k = 0; k < kNumCtr; ++k) acc[k] = 0;
    for (uint32_t w = threadIdx.x; w < n_waves; w += kBlock)
#pragma unroll
      for (int k = 0; k < kNumCtr; ++k) acc[k] += partials[static_cast<uint64_t>(w) * kNumCtr + k];
#pragma unroll
    for (int k = 0; k < kNumCtr; ++k) {
      uint64_t s = wave_sum_u64(acc[k]);
      if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = s;
    }
    __syncthreads();
    if (threadIdx.x < kNumCtr) {
      uint64_t s = 0;
      for (int i = 0; i < kBlock / 64; ++i) s += red[threadIdx.x][i];
      round_stats[threadIdx.x] = s;
    }
  }
}

// Pass 2: ordered compaction.  Each block sums the counts of the blocks
// before it, scans its lanes' counts, writes the flagged node ids in node
// order (so the next frontier is sorted: siblings stay adjacent) and clears
// the flags.  The last block publishes the frontier length.
__global__ __launch_bounds__(kBlock) void k_flag_compact(uint8_t* __restrict__ flags,
                                                         uint32_t n_pad,
                                                         const uint32_t* __restrict__ wg_count,
                                                         uint32_t* __restrict__ frontier,
                                                         uint32_t* __restrict__ n_front) {
  uint32_t pre = 0;
  for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kBlock) pre += wg_count[i];
  pre = block_sum_u32(pre);
  const uint32_t base = blockIdx.x * kFlagsPerBlock + threadIdx.x * kFlagsPerThread;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (base < n_pad) v = *reinterpret_cast<const uint4*>(flags + base);
  const uint32_t c = __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  uint32_t total;
  uint32_t pos = pre + block_excl_scan(c, &total);
  if (c) {
    const uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t wv = words[q];
      while (wv) {
        const int bit = __ffs(wv) - 1;
        frontier[pos++] = base + q * 4 + (bit >> 3);
        wv &= wv - 1;
      }
    }
    *reinterpret_cast<uint4*>(flags + base) = make_uint4(0, 0, 0, 0);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_front = pre + total;
}

// ---------------------------------------------------------------- digest ---
__global__ __launch_bounds__(kBlock) void k_digest(const uint64_t* __restrict__ seen,
                                                   const uint32_t* __restrict__ node_peer,
                                                   const uint16_t* __restrict__ node_topic,
                                                   const TopicDev* __restrict__ topics,
                                                   uint32_t n_nodes, uint64_t* out) {
  uint64_t acc = 0;
  for (uint32_t u = blockIdx.x * kBlock + threadIdx.x; u < n_nodes; u += gridDim.x * kBlock) {
    const uint32_t t = node_topic[u];
    const TopicDev T = topics[t];
    if (T.W == 0) continue;
    const uint64_t row = T.wbase + static_cast<uint64_t>(u - T.nbase) * T.W;
    const uint64_t key0 = (static_cast<uint64_t>(node_peer[u]) << 32) | (static_cast<uint64_t>(t) << 16);
    for (uint32_t w = 0; w < T.W; ++w) acc += mix64((key0 | w) ^ mix64(seen[row + w]));
  }
  acc = wave_sum_u64(acc);
  if ((threadIdx.x & 63) == 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(out), static_cast<unsigned long long>(acc));
}

}  // namespace

hipError_t launch_seed(const SeedDev* seeds, uint32_t lo, uint32_t hi, uint64_t* arrivals,
                       uint64_t* seen, uint8_t* next_flag, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  const uint32_t grid = (hi - lo + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_seed, dim3(grid), dim3(kBlock), 0, s, seeds, lo, hi, arrivals, seen,
                     next_flag);
  return hipGetLastError();
}

hipError_t launch_expand(const ExpandArgs& a, uint32_t round, bool record, uint32_t grid,
                         hipStream_t s) {
  if (record)
    hipLaunchKernelGGL(k_expand<true>, dim3(grid), dim3(kBlock), 0, s, a, round);
  else
    hipLaunchKernelGGL(k_expand<false>, dim3(grid), dim3(kBlock), 0, s, a, round);
  return hipGetLastError();
}

hipError_t launch_flag_count(const uint8_t* flags, uint32_t n_pad, uint32_t* wg_count,
                             const uint64_t* partials, uint32_t n_waves, uint64_t* round_stats,
                             hipStream_t s) {
  const uint32_t grid = (n_pad + kFlagsPerBlock - 1) / kFlagsPerBlock;
  hipLaunchKernelGGL(k_flag_count, dim3(grid), dim3(kBlock), 0, s, flags, n_pad, wg_count,
                     partials, n_waves, round_stats);
  return hipGetLastError();
}

hipError_t launch_flag_compact(uint8_t* flags, uint32_t n_pad, const uint32_t* wg_count,
                               uint32_t* frontier, uint32_t* n_front, hipStream_t s) {
  const uint32_t grid = (n_pad + kFlagsPerBlock - 1) / kFlagsPerBlock;
  hipLaunchKernelGGL(k_flag_compact, dim3(grid), dim3(kBlock), 0, s, flags, n_pad, wg_count,
                     frontier, n_front);
  return hipGetLastError();
}

hipError_t launch_digest(const uint64_t* seen, const uint32_t* node_peer,
                         const uint16_t* node_topic, const TopicDev* topics, uint32_t n_nodes,
                         uint64_t* out, hipStream_t s) {
  uint32_t grid = (n_nodes + kBlock - 1) / kBlock;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(k_digest, dim3(grid), dim3(kBlock), 0, s, seen, node_peer, node_topic,
                     topics, n_nodes, out);
  return hipGetLastError();
}

}  // namespace psamd
