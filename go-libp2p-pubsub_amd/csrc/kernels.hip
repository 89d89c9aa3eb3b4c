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

// ----------------------------------------------------------- window init ---
// Per window: zero every topic root's rows (seen and both arrival buffers;
// the root is node 0 of its topic) and stamp its generation; mesh topics get
// all their rows zeroed (they do not use generations).  Grid: x = chunk, y =
// topic.
__global__ __launch_bounds__(kBlock) void k_window_init(const TopicDev* __restrict__ topics,
                                                        uint64_t* __restrict__ seen,
                                                        uint64_t* __restrict__ a0,
                                                        uint64_t* __restrict__ a1,
                                                        uint8_t* __restrict__ gen,
                                                        uint32_t gen_cur) {
  const TopicDev T = topics[blockIdx.y];
  if (T.W == 0 || T.n_nodes == 0) return;
  const bool mesh = (T.flags & kTopicMesh) != 0;
  const uint64_t n_words = mesh ? static_cast<uint64_t>(T.n_nodes) * T.W : T.W;
  if (!mesh && blockIdx.x != 0) return;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n_words;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    seen[T.wbase + i] = 0;
    a0[T.wbase + i] = 0;
    a1[T.wbase + i] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) gen[T.nbase] = static_cast<uint8_t>(gen_cur);
}

// ---------------------------------------------------------------- seeds ---
// Topic.PublishMessage (pubsub.go:111-120): the root "has" its own messages
// (it is not a recipient) and forwards them in the next round.
__global__ __launch_bounds__(kBlock) void k_seed(const SeedDev* __restrict__ seeds, uint32_t lo,
                                                 uint32_t hi, uint64_t* __restrict__ arrivals,
                                                 uint64_t* __restrict__ seen,
                                                 uint8_t* __restrict__ next_flag,
                                                 uint8_t* __restrict__ blk_flag) {
  const uint32_t i = lo + blockIdx.x * kBlock + threadIdx.x;
  if (i >= hi) return;
  const SeedDev s = seeds[i];
  arrivals[s.woff] |= s.mask;
  seen[s.woff] |= s.mask;
  next_flag[s.node] = 1;
  blk_flag[s.node >> kFlagBlockShift] = 1;
}

// --------------------------------------------------------------- expand ---
// Tree topics: every child has exactly one parent, so p's wave owns the
// child's rows this round.  The seen test is lazy: a child whose generation
// byte is not the window's has seen nothing yet (its row is stale from an
// older window), so it is tested against 0 and its whole row is written; a
// current child is tested against its stored row.  Arrival rows of internal
// children are written whole (zeros included), so they need no clearing.
// Mesh topics: returning 64-bit atomicOr decides which parent wins each bit;
// arrival rows are OR-accumulated and consumed-and-cleared.

// per-lane counters of one launch (a lane handles < 2^26 words per launch)
struct ExpandCtr {
  uint32_t deliv = 0, dup = 0, sr = 0, sw = 0, aw = 0;
};

// Test-and-set of one (child, word): returns the newly delivered bits.
template <bool kRecord>
__device__ __forceinline__ uint64_t deliver_word(const ExpandArgs& a, bool mesh, bool stale,
                                                 bool internal, uint64_t cw, uint64_t m,
                                                 uint32_t round, ExpandCtr& k) {
  uint64_t old = 0, nm;
  if (mesh) {
    if (m == 0) return 0;
    old = atomicOr(reinterpret_cast<unsigned long long*>(a.seen + cw),
                   static_cast<unsigned long long>(m));
    nm = m & ~old;
    k.sr += 1;
    k.sw += 1;
    if (nm && internal) {
      atomicOr(reinterpret_cast<unsigned long long*>(a.a_next + cw),
               static_cast<unsigned long long>(nm));
      k.aw += 1;
    }
  } else {
    if (!stale && m) {
      old = a.seen[cw];
      k.sr += 1;
    }
    nm = m & ~old;
    if (stale || nm) {
      a.seen[cw] = old | nm;
      k.sw += 1;
    }
    if (internal) {
      a.a_next[cw] = nm;
      k.aw += 1;
    }
  }
  k.dup += __popcll(m & old);
  k.deliv += __popcll(nm);
  if constexpr (kRecord) {
    uint8_t* h = a.hop_rec + cw * 64;
    uint64_t b = nm;
    while (b) {
      const int q = __ffsll(static_cast<long long>(b)) - 1;
      h[q] = static_cast<uint8_t>(round);
      b &= b - 1;
    }
  }
  return nm;
}

__device__ __forceinline__ void mark_next(const ExpandArgs& a, uint32_t c) {
  a.next_flag[c] = 1;
  a.blk_flag[c >> kFlagBlockShift] = 1;
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

// Frontier entries are dealt to waves round-robin (entry e -> wave e mod
// n_waves).  A wave prefetches the metadata of its next 64 entries into lane
// registers (frontier id, topic, row range, first child) and broadcasts them
// with readlane, so the dependent-load chain is paid once per 64 entries.
//  W >= 64: word blocks outer, children inner: a child is wave-uniform
//    (flags and generation by readlane), each lane owns one word, so every
//    child costs one 512-B contiguous store burst per array.
//  W <  64: lanes split into 64/Wp groups of Wp = pow2ceil(W) lanes, one
//    child per group per pass.
// One lane per child raises the child's frontier flag.
template <bool kRecord>
__global__ __launch_bounds__(kBlock) void k_expand(ExpandArgs a, uint32_t round) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave =
      __builtin_amdgcn_readfirstlane((blockIdx.x * kBlock + threadIdx.x) >> 6);
  const uint32_t n_waves = (gridDim.x * kBlock) >> 6;
  const uint32_t n = *a.n_front;
  const uint32_t cur = a.gen_cur & 0xFF;

  ExpandCtr k;
  uint32_t c_ent = 0, c_ent_words = 0, c_kids = 0, c_mesh_kids = 0, c_clear = 0;

  for (uint64_t e0 = wave; e0 < n; e0 += 64ull * n_waves) {
    const uint64_t el = e0 + static_cast<uint64_t>(lane) * n_waves;
    uint32_t bp = 0, bt = 0, brs = 0, bdeg = 0, bc0 = 0;
    if (el < n) {
      bp = a.frontier[el];
      bt = a.node_topic[bp];
      brs = a.row_ptr[bp];
      bdeg = a.row_ptr[bp + 1] - brs;
      if (bdeg) bc0 = a.col[brs];
    }
    const uint32_t nb = static_cast<uint32_t>(__popcll(__ballot(el < n)));
    for (uint32_t q = 0; q < nb; ++q) {
      const uint32_t p = rl(bp, q), t = rl(bt, q), rs = rl(brs, q), deg = rl(bdeg, q);
      const uint32_t c0 = rl(bc0, q);
      const TopicDev T = a.topics[t];
      const uint32_t W = T.W;
      if (W == 0) continue;  // idle topic in this window (never seeded)
      const bool mesh = (T.flags & kTopicMesh) != 0;
      const uint64_t pw = T.wbase + static_cast<uint64_t>(p - T.nbase) * W;
      const uint64_t cbase = T.wbase - static_cast<uint64_t>(T.nbase) * W;
      c_ent += 1;
      c_ent_words += W;
      c_kids += deg;
      if (mesh) c_mesh_kids += deg;
      for (uint32_t j0 = 0; j0 < deg; j0 += 64) {
        const uint32_t cd = min(64u, deg - j0);
        // lane j < cd: child j0+j (BFS trees: contiguous from c0)
        uint32_t cj = 0, fj = 0, gj = 0;
        if (lane < cd) {
          cj = mesh ? a.col[rs + j0 + lane] : c0 + j0 + lane;
          fj = a.node_flags[cj];
          gj = mesh ? 0u : a.gen[cj];
        }
        if (W >= 64) {
          for (uint32_t wb = 0; wb < W; wb += 64) {
            const uint32_t w = wb + lane;
            const bool active = w < W;
            const uint64_t m = active ? a.a_cur[pw + w] : 0ull;
            for (uint32_t jj = 0; jj < cd; ++jj) {
              const uint32_t f = rl(fj, jj);
              if (!(f & kNodeLive)) continue;
              const uint32_t c = rl(cj, jj);
              const bool stale = !mesh && rl(gj, jj) != cur;
              const bool internal = (f & kNodeInternal) != 0;
              uint64_t nm = 0;
              if (active)
                nm = deliver_word<kRecord>(a, mesh, stale, internal,
                                           cbase + static_cast<uint64_t>(c) * W + w, m, round, k);
              if (internal && __ballot(nm != 0) && lane == 0) mark_next(a, c);
            }
          }
        } else {
          const uint32_t sh = 32u - __clz(W - 1u);  // Wp = 1 << sh >= W
          const uint32_t wp = 1u << sh;
          const uint32_t w = lane & (wp - 1u);
          const uint32_t jl = lane >> sh;
          const uint32_t groups = 64u >> sh;
          const uint64_t gmask = (wp == 64u ? ~0ull : ((1ull << wp) - 1ull)) << (jl << sh);
          const uint64_t m = w < W ? a.a_cur[pw + w] : 0ull;
          for (uint32_t jb = 0; jb < cd; jb += groups) {
            const uint32_t jj = jb + jl;
            const uint32_t c = static_cast<uint32_t>(__shfl(static_cast<int>(cj), static_cast<int>(jj), 64));
            const uint32_t f = static_cast<uint32_t>(__shfl(static_cast<int>(fj), static_cast<int>(jj), 64));
            const uint32_t g = static_cast<uint32_t>(__shfl(static_cast<int>(gj), static_cast<int>(jj), 64));
            const bool live = (w < W) && (jj < cd) && (f & kNodeLive);
            uint64_t nm = 0;
            if (live)
              nm = deliver_word<kRecord>(a, mesh, !mesh && g != cur, (f & kNodeInternal) != 0,
                                         cbase + static_cast<uint64_t>(c) * W + w, m, round, k);
            const uint64_t bal = __ballot(nm != 0);
            if (live && w == 0 && (f & kNodeInternal) && (bal & gmask)) mark_next(a, c);
          }
        }
        // this chunk's live tree children hold current rows now
        if (!mesh && lane < cd && (fj & kNodeLive)) a.gen[cj] = static_cast<uint8_t>(cur);
      }
      if (mesh || p == T.nbase) {
        // consume-and-clear: mesh rows are OR-accumulated, root rows are seeded
        for (uint32_t w = lane; w < W; w += 64) a.a_cur[pw + w] = 0;
        c_clear += W;
      }
    }
  }

  const uint64_t s_deliv = wave_sum_u64(k.deliv);
  const uint64_t s_dup = wave_sum_u64(k.dup);
  const uint64_t s_sr = wave_sum_u64(k.sr);
  const uint64_t s_sw = wave_sum_u64(k.sw);
  const uint64_t s_aw = wave_sum_u64(k.aw);
  if (lane == 0) {
    uint64_t* out = a.partials + static_cast<uint64_t>(wave) * kNumCtr;
    out[kCtrDeliveries] = s_deliv;
    out[kCtrDuplicates] = s_dup;
    out[kCtrEntries] = c_ent;
    out[kCtrEntryWords] = c_ent_words;
    out[kCtrChildren] = c_kids;
    out[kCtrMeshChildren] = c_mesh_kids;
    out[kCtrSeenReads] = s_sr;
    out[kCtrSeenWrites] = s_sw;
    out[kCtrArrivalWrites] = s_aw;
    out[kCtrClearWords] = c_clear;
  }
}

// ------------------------------------------------------------ compaction ---
// Pass 1: per-block count of flagged nodes (16 one-byte flags per lane, one
// 16-B load); blocks whose blk_flag byte is clear exit at once.  Block 0 also
// folds the expand kernel's per-wave counters into this round's statistics.
__global__ __launch_bounds__(kBlock) void k_flag_count(const uint8_t* __restrict__ flags,
                                                       const uint8_t* __restrict__ blk_flag,
                                                       uint32_t n_pad,
                                                       uint32_t* __restrict__ wg_count,
                                                       const uint64_t* __restrict__ partials,
                                                       uint32_t n_waves,
                                                       uint64_t* __restrict__ round_stats) {
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
  if (blk_flag[blockIdx.x] == 0) {
    if (threadIdx.x == 0) wg_count[blockIdx.x] = 0;
    return;
  }
  const uint32_t base = blockIdx.x * kFlagsPerBlock + threadIdx.x * kFlagsPerThread;
  uint32_t c = 0;
  if (base < n_pad) {
    const uint4 v = *reinterpret_cast<const uint4*>(flags + base);
    c = __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  }
  c = block_sum_u32(c);
  if (threadIdx.x == 0) wg_count[blockIdx.x] = c;
}

// Pass 2: ordered compaction.  Each non-empty block sums the counts of the
// blocks before it, scans its lanes' counts, writes the flagged node ids in
// node order (so the next frontier is sorted: siblings stay adjacent) and
// clears its flags.  The last block publishes the frontier length.
__global__ __launch_bounds__(kBlock) void k_flag_compact(uint8_t* __restrict__ flags,
                                                         uint8_t* __restrict__ blk_flag,
                                                         uint32_t n_pad,
                                                         const uint32_t* __restrict__ wg_count,
                                                         uint32_t* __restrict__ frontier,
                                                         uint32_t* __restrict__ n_front) {
  const bool last = blockIdx.x == gridDim.x - 1;
  const bool busy = blk_flag[blockIdx.x] != 0;
  if (!busy && !last) return;
  uint32_t pre = 0;
  for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kBlock) pre += wg_count[i];
  pre = block_sum_u32(pre);
  const uint32_t base = blockIdx.x * kFlagsPerBlock + threadIdx.x * kFlagsPerThread;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (busy && base < n_pad) v = *reinterpret_cast<const uint4*>(flags + base);
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
  if (busy && threadIdx.x == 0) blk_flag[blockIdx.x] = 0;
  if (last && threadIdx.x == 0) *n_front = pre + total;
}

// ---------------------------------------------------------------- digest ---
// Order-independent digest of the window's delivered state: a tree node whose
// generation is not the window's holds nothing (its row is stale).
__global__ __launch_bounds__(kBlock) void k_digest(const uint64_t* __restrict__ seen,
                                                   const uint8_t* __restrict__ gen,
                                                   uint32_t gen_cur,
                                                   const uint32_t* __restrict__ node_peer,
                                                   const uint16_t* __restrict__ node_topic,
                                                   const TopicDev* __restrict__ topics,
                                                   uint32_t n_nodes, uint64_t* out) {
  uint64_t acc = 0;
  for (uint32_t u = blockIdx.x * kBlock + threadIdx.x; u < n_nodes; u += gridDim.x * kBlock) {
    const uint32_t t = node_topic[u];
    const TopicDev T = topics[t];
    if (T.W == 0) continue;
    const bool valid = (T.flags & kTopicMesh) || gen[u] == static_cast<uint8_t>(gen_cur);
    const uint64_t row = T.wbase + static_cast<uint64_t>(u - T.nbase) * T.W;
    const uint64_t key0 = (static_cast<uint64_t>(node_peer[u]) << 32) | (static_cast<uint64_t>(t) << 16);
    for (uint32_t w = 0; w < T.W; ++w)
      acc += mix64((key0 | w) ^ mix64(valid ? seen[row + w] : 0ull));
  }
  acc = wave_sum_u64(acc);
  if ((threadIdx.x & 63) == 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(out), static_cast<unsigned long long>(acc));
}

}  // namespace

hipError_t launch_window_init(const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur,
                              bool any_mesh, hipStream_t s) {
  if (n_topics == 0) return hipSuccess;
  const dim3 grid(any_mesh ? 64 : 1, n_topics);
  hipLaunchKernelGGL(k_window_init, grid, dim3(kBlock), 0, s, topics, seen, a0, a1, gen, gen_cur);
  return hipGetLastError();
}

hipError_t launch_seed(const SeedDev* seeds, uint32_t lo, uint32_t hi, uint64_t* arrivals,
                       uint64_t* seen, uint8_t* next_flag, uint8_t* blk_flag, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  const uint32_t grid = (hi - lo + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_seed, dim3(grid), dim3(kBlock), 0, s, seeds, lo, hi, arrivals, seen,
                     next_flag, blk_flag);
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

hipError_t launch_flag_count(const uint8_t* flags, const uint8_t* blk_flag, uint32_t n_pad,
                             uint32_t* wg_count, const uint64_t* partials, uint32_t n_waves,
                             uint64_t* round_stats, hipStream_t s) {
  const uint32_t grid = (n_pad + kFlagsPerBlock - 1) / kFlagsPerBlock;
  hipLaunchKernelGGL(k_flag_count, dim3(grid), dim3(kBlock), 0, s, flags, blk_flag, n_pad,
                     wg_count, partials, n_waves, round_stats);
  return hipGetLastError();
}

hipError_t launch_flag_compact(uint8_t* flags, uint8_t* blk_flag, uint32_t n_pad,
                               const uint32_t* wg_count, uint32_t* frontier, uint32_t* n_front,
                               hipStream_t s) {
  const uint32_t grid = (n_pad + kFlagsPerBlock - 1) / kFlagsPerBlock;
  hipLaunchKernelGGL(k_flag_compact, dim3(grid), dim3(kBlock), 0, s, flags, blk_flag, n_pad,
                     wg_count, frontier, n_front);
  return hipGetLastError();
}

hipError_t launch_digest(const uint64_t* seen, const uint8_t* gen, uint32_t gen_cur,
                         const uint32_t* node_peer, const uint16_t* node_topic,
                         const TopicDev* topics, uint32_t n_nodes, uint64_t* out, hipStream_t s) {
  uint32_t grid = (n_nodes + kBlock - 1) / kBlock;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(k_digest, dim3(grid), dim3(kBlock), 0, s, seen, gen, gen_cur, node_peer,
                     node_topic, topics, n_nodes, out);
  return hipGetLastError();
}

}  // namespace psamd
