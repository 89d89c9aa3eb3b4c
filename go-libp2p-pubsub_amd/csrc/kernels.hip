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
#include <algorithm>

#include "devutil.hpp"
#include "kernels.hpp"

namespace psamd {

namespace {

using namespace dev;

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
                                                        uint32_t gen_cur, WindowStart ws) {
  // folded-in work (one launch instead of three): the staged copies and the
  // partial-slot clear, grid-stride over every block
  const uint32_t nb = gridDim.x * gridDim.y;
  const uint32_t bid = blockIdx.y * gridDim.x + blockIdx.x;
  for (uint32_t k = 0; k < ws.copy.n; ++k)
    for (uint32_t i = bid * kBlock + threadIdx.x; i < ws.copy.words[k]; i += nb * kBlock)
      ws.copy.dst[k][i] = ws.copy.src[k][i];
  for (uint64_t i = static_cast<uint64_t>(bid) * kBlock + threadIdx.x; i < ws.zero_words;
       i += static_cast<uint64_t>(nb) * kBlock)
    ws.zero[i] = 0;
  const TopicDev T = topics[blockIdx.y];
  if (T.W == 0 || T.n_nodes == 0) return;
  const bool mesh = (T.flags & kTopicMesh) != 0;
  const uint64_t n_words = mesh ? static_cast<uint64_t>(T.n_nodes) * T.W : T.root_words;
  if (!mesh && (blockIdx.x != 0 || !(T.flags & kTopicRootLocal))) return;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n_words;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    seen[T.wbase + i] = 0;
    a0[T.wbase + i] = 0;
    a1[T.wbase + i] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (T.flags & kTopicRootLocal))
    gen[T.nbase] = static_cast<uint8_t>(gen_cur);
  if (ws.seeds && !mesh) {
    // Topic.PublishMessage (pubsub.go:111-120), round 0: this block zeroed
    // the root's row above; the barrier orders the seeds after it
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < T.seed_n; i += kBlock) {
      const SeedDev sd = ws.seeds[T.seed_lo + i];
      a0[sd.woff] = sd.assign ? sd.mask : a0[sd.woff] | sd.mask;
      seen[sd.woff] = sd.assign ? sd.mask : seen[sd.woff] | sd.mask;
    }
  }
}

// Nodes fed by a parent on another rank: rows zeroed, so the apply kernel can
// test-and-set them with atomics.  Compaction mode stamps their generation
// here (their rows are current from the start); level mode leaves that to
// the apply kernel, which stamps a node when something reaches it, so that
// "generation current" keeps meaning "reached this window".
__global__ __launch_bounds__(kBlock) void k_init_nodes(const uint32_t* __restrict__ nodes,
                                                       uint32_t n,
                                                       const uint16_t* __restrict__ node_topic,
                                                       const TopicDev* __restrict__ topics,
                                                       uint64_t* __restrict__ seen,
                                                       uint64_t* __restrict__ a0,
                                                       uint64_t* __restrict__ a1,
                                                       uint8_t* __restrict__ gen, uint32_t gen_cur,
                                                       bool stamp) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * kBlock + threadIdx.x) >> 6;
  const uint32_t n_waves = (gridDim.x * kBlock) >> 6;
  for (uint32_t i = wave; i < n; i += n_waves) {
    const uint32_t u = nodes[i];
    const TopicDev T = topics[node_topic[u]];
    if (T.W == 0) continue;
    const uint64_t row = T.wbase + static_cast<uint64_t>(u - T.nbase) * T.W;
    for (uint32_t w = lane; w < T.W; w += 64) {
      seen[row + w] = 0;
      a0[row + w] = 0;
      a1[row + w] = 0;
    }
    if (lane == 0 && stamp) gen[u] = static_cast<uint8_t>(gen_cur);
  }
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
  arrivals[s.woff] = s.assign ? s.mask : arrivals[s.woff] | s.mask;
  seen[s.woff] = s.assign ? s.mask : seen[s.woff] | s.mask;
  if (next_flag == nullptr) return;  // level mode: the root is scheduled statically
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
    uint16_t* h = a.hop_rec + cw * 64;
    uint64_t b = nm;
    while (b) {
      const int q = __ffsll(static_cast<long long>(b)) - 1;
      h[q] = hop_round(round);
      b &= b - 1;
    }
  }
  return nm;
}

// A child whose row is stale (nothing seen this window): every arriving bit is
// new, the whole row is written, no load -- so no vmcnt wait in the burst.
template <bool kRecord>
__device__ __forceinline__ void deliver_fresh(const ExpandArgs& a, bool internal, uint64_t cw,
                                              uint64_t m, uint32_t round, ExpandCtr& k) {
  a.seen[cw] = m;
  k.sw += 1;
  if (internal) {
    a.a_next[cw] = m;
    k.aw += 1;
  }
  k.deliv += __popcll(m);
  if constexpr (kRecord) {
    uint16_t* h = a.hop_rec + cw * 64;
    uint64_t b = m;
    while (b) {
      const int q = __ffsll(static_cast<long long>(b)) - 1;
      h[q] = hop_round(round);
      b &= b - 1;
    }
  }
}

// Two adjacent words of a fresh row (16-B aligned): one dwordx4 store each.
template <bool kRecord>
__device__ __forceinline__ void deliver_fresh2(const ExpandArgs& a, bool internal, uint64_t cw,
                                               uint4 v, uint32_t round, ExpandCtr& k) {
  *reinterpret_cast<uint4*>(a.seen + cw) = v;
  k.sw += 2;
  if (internal) {
    *reinterpret_cast<uint4*>(a.a_next + cw) = v;
    k.aw += 2;
  }
  k.deliv += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  if constexpr (kRecord) {
    for (int h = 0; h < 2; ++h) {
      uint16_t* rec = a.hop_rec + (cw + h) * 64;
      uint64_t b = h ? (static_cast<uint64_t>(v.w) << 32 | v.z) : (static_cast<uint64_t>(v.y) << 32 | v.x);
      while (b) {
        const int q = __ffsll(static_cast<long long>(b)) - 1;
        rec[q] = hop_round(round);
        b &= b - 1;
      }
    }
  }
}

__device__ __forceinline__ void mark_next(const ExpandArgs& a, uint32_t c) {
  a.next_flag[c] = 1;
  a.blk_flag[c >> kFlagBlockShift] = 1;
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(lane)));
}

__device__ __forceinline__ uint32_t pow2_shift(uint32_t W) { return 32u - __clz(W - 1u); }

// LDS-DMA: lane i copies N bytes from its own global address into
// lds_base + i * N (lds_base wave-uniform); no VGPR destination.
#define PSAMD_LDS_DMA(g, lds_base, N)                                            \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g), \
                                   (__attribute__((address_space(3))) void*)(lds_base), N, 0, 0)

// Per-wave LDS slice of the staged path: arrival words of a sub-batch of
// entries, plus the flag and generation bytes of their children.
constexpr uint32_t kStageWords = 704;  // 5.5 KiB
constexpr uint32_t kStageBytes = 512;  // 2 x 512 B of child flag / generation dwords
struct __attribute__((aligned(16))) WaveStage {
  uint64_t words[kStageWords];
  uint8_t flags[kStageBytes];
  uint8_t gens[kStageBytes];
};

struct EntryCtr {
  uint32_t ent = 0, ent_words = 0, kids = 0, mesh_kids = 0, clear = 0;
};

// Direct path: one entry with its loads inline (mesh topics, rows wider than
// the stage, fan-out above 64).
template <bool kRecord>
__device__ void expand_direct(const ExpandArgs& a, uint32_t p, uint32_t rs, uint32_t deg,
                              uint32_t c0, uint32_t W, uint32_t nbase, uint32_t tflags,
                              uint64_t wbase, uint32_t lane, uint32_t cur, uint32_t round,
                              ExpandCtr& k, EntryCtr& ec) {
  const bool mesh = (tflags & kTopicMesh) != 0;
  const bool split = (tflags & kEntrySplit) != 0;  // some children live on other ranks
  const bool listed = mesh || split;
  const bool is_root = p == nbase && (tflags & kTopicRootLocal);
  // single-start tree topic: arrival rows live in `seen` (roots: seeded rows)
  const bool single = (tflags & kTopicSingleStart) && !mesh;
  const uint64_t* src = (single && !is_root) ? a.seen : a.a_cur;
  const uint64_t pw = wbase + static_cast<uint64_t>(p - nbase) * W;
  const uint64_t cbase = wbase - static_cast<uint64_t>(nbase) * W;
  ec.ent += 1;
  ec.ent_words += W;
  ec.kids += deg;
  if (mesh) ec.mesh_kids += deg;
  for (uint32_t j0 = 0; j0 < deg; j0 += 64) {
    const uint32_t cd = min(64u, deg - j0);
    uint32_t cj = 0, fj = 0, gj = 0;
    if (lane < cd) {
      cj = listed ? a.col[rs + j0 + lane] : c0 + j0 + lane;
      if (!(cj & kRemoteBit)) {  // a remote child is not live here: routed below
        fj = a.node_flags[cj];
        gj = mesh ? 0u : a.gen[cj];
      }
    }
    if (split) {
      // children owned by other ranks: the whole arrival row goes into the
      // owner's send region (one reservation per child)
      for (uint32_t jj = 0; jj < cd; ++jj) {
        const uint32_t c = rl(cj, jj);
        if (!(c & kRemoteBit)) continue;
        const uint32_t dest = (c >> kRemoteRankShift) & 0xFu;
        uint8_t* region = a.send + a.send_off[dest];
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(reinterpret_cast<uint32_t*>(region), W);
        base = static_cast<uint32_t>(__shfl(static_cast<int>(base), 0, 64));
        XItem* out = reinterpret_cast<XItem*>(region + kRegionHeader) + base;
        for (uint32_t w = lane; w < W; w += 64) {
          XItem it;
          it.node = c & kRemoteIdMask;
          it.word = w;
          it.mask = src[pw + w];
          out[w] = it;
        }
      }
    }
    if (W >= 64) {
      for (uint32_t wb = 0; wb < W; wb += 64) {
        const uint32_t w = wb + lane;
        const bool active = w < W;
        const uint64_t m = active ? src[pw + w] : 0ull;
        for (uint32_t jj = 0; jj < cd; ++jj) {
          const uint32_t f = rl(fj, jj);
          if (!(f & kNodeLive)) continue;
          const uint32_t c = rl(cj, jj);
          const bool stale = !mesh && rl(gj, jj) != cur;
          const bool internal = (f & kNodeInternal) != 0;
          uint64_t nm = 0;
          if (active)
            nm = deliver_word<kRecord>(a, mesh, stale, internal && !single,
                                       cbase + static_cast<uint64_t>(c) * W + w, m, round, k);
          if (internal && __ballot(nm != 0) && lane == 0) mark_next(a, c);
        }
      }
    } else {
      const uint32_t sh = pow2_shift(W);
      const uint32_t wp = 1u << sh;
      const uint32_t w = lane & (wp - 1u);
      const uint32_t jl = lane >> sh;
      const uint32_t groups = 64u >> sh;
      const uint64_t gmask = (wp == 64u ? ~0ull : ((1ull << wp) - 1ull)) << (jl << sh);
      const uint64_t m = w < W ? src[pw + w] : 0ull;
      for (uint32_t jb = 0; jb < cd; jb += groups) {
        const uint32_t jj = jb + jl;
        const uint32_t c = static_cast<uint32_t>(__shfl(static_cast<int>(cj), static_cast<int>(jj), 64));
        const uint32_t f = static_cast<uint32_t>(__shfl(static_cast<int>(fj), static_cast<int>(jj), 64));
        const uint32_t g = static_cast<uint32_t>(__shfl(static_cast<int>(gj), static_cast<int>(jj), 64));
        const bool live = (w < W) && (jj < cd) && (f & kNodeLive);
        uint64_t nm = 0;
        if (live)
          nm = deliver_word<kRecord>(a, mesh, !mesh && g != cur,
                                     (f & kNodeInternal) != 0 && !single,
                                     cbase + static_cast<uint64_t>(c) * W + w, m, round, k);
        const uint64_t bal = __ballot(nm != 0);
        if (live && w == 0 && (f & kNodeInternal) && (bal & gmask)) mark_next(a, c);
      }
    }
    if (!mesh && lane < cd && (fj & kNodeLive))
      a.gen[cj] = static_cast<uint8_t>(cur);
  }
  if (mesh || is_root) {
    // consume-and-clear: mesh rows are OR-accumulated, root rows are seeded
    for (uint32_t w = lane; w < W; w += 64) a.a_cur[pw + w] = 0;
    ec.clear += W;
  }
}

// One tree entry whose row is wider than the stage (W > kStageWords, so W is
// even and 16-B aligned): the row goes through the stage in slices of
// kStageWords words, each slice stored to every live child before the next
// is loaded.  The children's flag and generation bytes are read once, before
// any store, so every slice sees the same staleness.
template <bool kRecord>
__device__ void expand_wide(const ExpandArgs& a, WaveStage& ws, uint32_t p, uint32_t deg,
                            uint32_t c0, uint32_t W, uint32_t nbase, uint32_t fl, uint64_t wbase,
                            uint32_t lane, uint32_t cur, uint32_t round, ExpandCtr& k,
                            EntryCtr& ec) {
  const bool is_root = p == nbase && (fl & kTopicRootLocal);
  const bool from_seen = (fl & kTopicSingleStart) && !is_root;
  const bool keep = !(fl & kTopicSingleStart);
  const uint64_t pw = wbase + static_cast<uint64_t>(p - nbase) * W;
  const uint64_t cbase = wbase - static_cast<uint64_t>(nbase) * W;
  const uint32_t* row = reinterpret_cast<const uint32_t*>((from_seen ? a.seen : a.a_cur) + pw);
  uint32_t fj = 0, gj = 0;
  if (lane < deg) {  // deg <= 64
    fj = a.node_flags[c0 + lane];
    gj = a.gen[c0 + lane];
  }
  ec.ent += 1;
  ec.ent_words += W;
  ec.kids += deg;
  uint64_t got = 0;  // bit j: child j received something
  for (uint32_t w0 = 0; w0 < W; w0 += kStageWords) {
    const uint32_t len = min(kStageWords, W - w0);  // even
    uint32_t* dst = reinterpret_cast<uint32_t*>(ws.words);
    for (uint32_t d = 0; d < 2 * len; d += 256)
      if (d + 4 * lane < 2 * len) PSAMD_LDS_DMA(row + 2 * w0 + d + 4 * lane, dst + d, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t jj = 0; jj < deg; ++jj) {
      const uint32_t f = rl(fj, jj);
      if (!(f & kNodeLive)) continue;
      const bool stale = rl(gj, jj) != cur;
      const bool store = (f & kNodeInternal) && keep;
      const uint64_t crow = cbase + static_cast<uint64_t>(c0 + jj) * W + w0;
      bool any = false;
      if (stale) {
        for (uint32_t wb = 0; wb < len; wb += 128) {
          const uint32_t w = wb + 2 * lane;
          if (w < len) {
            const uint4 v = *reinterpret_cast<const uint4*>(ws.words + w);
            deliver_fresh2<kRecord>(a, store, crow + w, v, round, k);
            any |= (v.x | v.y | v.z | v.w) != 0;
          }
        }
      } else {
        for (uint32_t wb = 0; wb < len; wb += 64) {
          const uint32_t w = wb + lane;
          if (w < len) {
            const uint64_t nm =
                deliver_word<kRecord>(a, false, false, store, crow + w, ws.words[w], round, k);
            any |= nm != 0;
          }
        }
      }
      if (__ballot(any)) got |= 1ull << jj;
    }
  }
  if (lane < deg && (fj & kNodeInternal) && ((got >> lane) & 1ull)) mark_next(a, c0 + lane);
  if (lane < deg && (fj & kNodeLive))
    a.gen[c0 + lane] = static_cast<uint8_t>(cur);
  if (is_root) {  // seeded with |=: consume-and-clear
    for (uint32_t w = lane; w < W; w += 64) a.a_cur[pw + w] = 0;
    ec.clear += W;
  }
}

// Frontier entries are dealt to waves round-robin (entry e -> wave e mod
// n_waves).  A wave loads the metadata of its next 64 entries into lane
// registers (frontier id, row range, first child, topic fields) and
// broadcasts them with readlane.  Tree entries then go through the staged
// path in sub-batches that fit the wave's LDS slice:
//   phase A  LDS-DMA of every arrival row and of the children's flag and
//            generation bytes (BFS numbering: contiguous), one vmcnt(0) wait;
//   phase B  stores only: W >= 64 child-outer / word-block-inner (512-B
//            contiguous bursts, child wave-uniform), W < 64 Wp-lane groups.
// The waves therefore wait once per sub-batch, not once per word block.
// kDirect = false: the staged path only (entries that need the direct path
// are left to the second instance); kDirect = true: the direct path only.
// Separate instances keep the hot staged kernel's register budget small.
template <bool kRecord, bool kDirect>
__global__ __launch_bounds__(kBlock) void k_expand(ExpandArgs a, uint32_t round) {
  __shared__ WaveStage stage_lds[kDirect ? 1 : kBlock / 64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave =
      __builtin_amdgcn_readfirstlane((blockIdx.x * kBlock + threadIdx.x) >> 6);
  WaveStage& ws = stage_lds[kDirect ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];
  const uint32_t n_waves = (gridDim.x * kBlock) >> 6;
  const uint32_t n = *a.n_front;
  const uint32_t cur = a.gen_cur & 0xFF;

  ExpandCtr k;
  EntryCtr ec;

  for (uint64_t e0 = wave; e0 < n; e0 += 64ull * n_waves) {
    const uint64_t el = e0 + static_cast<uint64_t>(lane) * n_waves;
    uint32_t bp = 0, brs = 0, bdeg = 0, bc0 = 0, bW = 0, bnb = 0, bfl = 0, bwl = 0, bwh = 0;
    if (el < n) {
      bp = a.frontier[el];
      const uint32_t t = a.node_topic[bp];
      brs = a.row_ptr[bp];
      bdeg = a.row_ptr[bp + 1] - brs;
      const TopicDev T = a.topics[t];
      bW = T.W;
      bnb = T.nbase;
      bfl = T.flags | ((a.node_flags[bp] & kNodeSplit) ? kEntrySplit : 0u);
      bwl = static_cast<uint32_t>(T.wbase);
      bwh = static_cast<uint32_t>(T.wbase >> 32);
      if (bdeg && T.W) bc0 = a.col[brs];
    }
    const uint32_t nb = static_cast<uint32_t>(__popcll(__ballot(el < n)));
    uint32_t q = 0;
    while (q < nb) {
      const uint32_t W0 = rl(bW, q), d0 = rl(bdeg, q), f0 = rl(bfl, q);
      if (W0 == 0) {
        ++q;
        continue;
      }
      const bool direct = (f0 & (kTopicMesh | kEntrySplit)) || d0 > 64;
      if (direct || kDirect) {
        if (direct && kDirect)
          expand_direct<kRecord>(a, rl(bp, q), rl(brs, q), d0, rl(bc0, q), W0, rl(bnb, q), f0,
                                 (static_cast<uint64_t>(rl(bwh, q)) << 32) | rl(bwl, q), lane,
                                 cur, round, k, ec);
        ++q;
        continue;
      }
      if (W0 > kStageWords) {  // wide row: staged slice by slice
        expand_wide<kRecord>(a, ws, rl(bp, q), d0, rl(bc0, q), W0, rl(bnb, q), f0,
                                     (static_cast<uint64_t>(rl(bwh, q)) << 32) | rl(bwl, q), lane,
                                     cur, round, k, ec);
        ++q;
        continue;
      }
      // sub-batch [q, q + nq) that fits the stage; a child's flag and
      // generation bytes are staged as the dwords enclosing [c0, c0 + deg)
      // (sub-dword LDS-DMA does not pack lanes byte by byte)
      uint32_t nq = 0, sw = 0, sd = 0;
      while (q + nq < nb) {
        const uint32_t Wn = rl(bW, q + nq), dn = rl(bdeg, q + nq), fn = rl(bfl, q + nq);
        const uint32_t cn = rl(bc0, q + nq);
        const uint32_t bn = 4u * (((cn + dn + 3u) >> 2) - (cn >> 2));
        if ((fn & (kTopicMesh | kEntrySplit)) || Wn > kStageWords || dn > 64) break;
        if (sw + Wn + (Wn & 1u) > kStageWords || sd + bn > kStageBytes) break;
        sw += Wn + (Wn & 1u);
        sd += bn;
        ++nq;
      }
      // phase A: LDS-DMA of arrival rows and child flag / generation bytes
      {
        uint32_t off = 0, doff = 0;
        for (uint32_t i = q; i < q + nq; ++i) {
          const uint32_t W = rl(bW, i), deg = rl(bdeg, i);
          if (W == 0) continue;
          const uint32_t p = rl(bp, i), nbase = rl(bnb, i), c0 = rl(bc0, i);
          const uint64_t wbase = (static_cast<uint64_t>(rl(bwh, i)) << 32) | rl(bwl, i);
          const uint32_t fl = rl(bfl, i);
          const bool from_seen = (fl & kTopicSingleStart) && !(p == nbase && (fl & kTopicRootLocal));
          const uint32_t* row = reinterpret_cast<const uint32_t*>(
              (from_seen ? a.seen : a.a_cur) + wbase + static_cast<uint64_t>(p - nbase) * W);
          uint32_t* dst = reinterpret_cast<uint32_t*>(ws.words + off);
          if ((W & 1u) == 0) {
            // even W: the row and its stage slot are 16-B aligned (topic
            // blocks start on 128-B lines, slots keep even offsets): one
            // dwordx4 DMA per lane, 1 KiB per wave instruction
            for (uint32_t d = 0; d < 2 * W; d += 256)
              if (d + 4 * lane < 2 * W) PSAMD_LDS_DMA(row + d + 4 * lane, dst + d, 16);
          } else {
            for (uint32_t d = 0; d < 2 * W; d += 64)
              if (d + lane < 2 * W) PSAMD_LDS_DMA(row + d + lane, dst + d, 4);
          }
          const uint32_t nd = ((c0 + deg + 3u) >> 2) - (c0 >> 2);
          if (lane < nd) {
            PSAMD_LDS_DMA(reinterpret_cast<const uint32_t*>(a.node_flags) + (c0 >> 2) + lane,
                          ws.flags + doff, 4);
            PSAMD_LDS_DMA(reinterpret_cast<const uint32_t*>(a.gen) + (c0 >> 2) + lane,
                          ws.gens + doff, 4);
          }
          off += W + (W & 1u);  // keep every staged row 16-B aligned
          doff += 4u * nd;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // phase B: stores
      {
        uint32_t off = 0, doff = 0;
        for (uint32_t i = q; i < q + nq; ++i) {
          const uint32_t W = rl(bW, i), deg = rl(bdeg, i);
          if (W == 0) continue;
          const uint32_t p = rl(bp, i), nbase = rl(bnb, i), c0 = rl(bc0, i);
          const uint64_t wbase = (static_cast<uint64_t>(rl(bwh, i)) << 32) | rl(bwl, i);
          const uint64_t cbase = wbase - static_cast<uint64_t>(nbase) * W;
          const uint32_t nd = ((c0 + deg + 3u) >> 2) - (c0 >> 2);
          const uint32_t fo = doff + (c0 & 3u);  // byte of child 0
          // single-start topics keep no arrival rows (see kTopicSingleStart)
          const bool keep = !(rl(bfl, i) & kTopicSingleStart);
          ec.ent += 1;
          ec.ent_words += W;
          ec.kids += deg;
          if (W >= 64) {
            for (uint32_t jj = 0; jj < deg; ++jj) {
              const uint32_t f = ws.flags[fo + jj];
              if (!(f & kNodeLive)) continue;
              const bool stale = ws.gens[fo + jj] != cur;
              const bool internal = (f & kNodeInternal) != 0;
              const bool store = internal && keep;
              const uint32_t c = c0 + jj;
              const uint64_t row = cbase + static_cast<uint64_t>(c) * W;
              bool any = false;
              if (stale) {
                // W even, row and stage offset even: two words per lane,
                // 1 KiB per store instruction
                for (uint32_t wb = 0; wb < W; wb += 128) {
                  const uint32_t w = wb + 2 * lane;
                  if (w < W) {
                    const uint4 v = *reinterpret_cast<const uint4*>(ws.words + off + w);
                    deliver_fresh2<kRecord>(a, store, row + w, v, round, k);
                    any |= (v.x | v.y | v.z | v.w) != 0;
                  }
                }
              } else {
                for (uint32_t wb = 0; wb < W; wb += 64) {
                  const uint32_t w = wb + lane;
                  if (w < W) {
                    const uint64_t nm = deliver_word<kRecord>(a, false, false, store, row + w,
                                                              ws.words[off + w], round, k);
                    any |= nm != 0;
                  }
                }
              }
              if (internal && __ballot(any) && lane == 0) mark_next(a, c);
            }
          } else {
            const uint32_t sh = pow2_shift(W);
            const uint32_t wp = 1u << sh;
            const uint32_t w = lane & (wp - 1u);
            const uint32_t jl = lane >> sh;
            const uint32_t groups = 64u >> sh;
            const uint64_t gmask = (wp == 64u ? ~0ull : ((1ull << wp) - 1ull)) << (jl << sh);
            const uint64_t m = w < W ? ws.words[off + w] : 0ull;
            for (uint32_t jb = 0; jb < deg; jb += groups) {
              const uint32_t jj = jb + jl;
              const bool valid = (w < W) && (jj < deg);
              const uint32_t f = valid ? ws.flags[fo + jj] : 0u;
              const bool live = valid && (f & kNodeLive);
              const bool stale = ws.gens[fo + jj] != cur;
              const uint32_t c = c0 + jj;
              const uint64_t cw = cbase + static_cast<uint64_t>(c) * W + w;
              uint64_t nm = 0;
              if (__ballot(live && !stale) == 0) {  // burst: every live child fresh
                if (live) {
                  deliver_fresh<kRecord>(a, keep && (f & kNodeInternal), cw, m, round, k);
                  nm = m;
                }
              } else if (live) {
                nm = deliver_word<kRecord>(a, false, stale, keep && (f & kNodeInternal), cw, m,
                                           round, k);
              }
              const uint64_t bal = __ballot(nm != 0);
              if (live && w == 0 && (f & kNodeInternal) && (bal & gmask)) mark_next(a, c);
            }
          }
          // live children hold current rows now
          if (lane < deg && (ws.flags[fo + lane] & kNodeLive))
            a.gen[c0 + lane] = static_cast<uint8_t>(cur);
          if (p == nbase && (rl(bfl, i) & kTopicRootLocal)) {  // seeded with |=: consume-and-clear
            const uint64_t pw = wbase + static_cast<uint64_t>(p - nbase) * W;
            for (uint32_t w = lane; w < W; w += 64) a.a_cur[pw + w] = 0;
            ec.clear += W;
          }
          off += W + (W & 1u);
          doff += 4u * nd;
        }
      }
      q += nq;
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
    out[kCtrEntries] = ec.ent;
    out[kCtrEntryWords] = ec.ent_words;
    out[kCtrChildren] = ec.kids;
    out[kCtrMeshChildren] = ec.mesh_kids;
    out[kCtrSeenReads] = s_sr;
    out[kCtrSeenWrites] = s_sw;
    out[kCtrArrivalWrites] = s_aw;
    out[kCtrClearWords] = ec.clear;
  }
}

// ------------------------------------------------------------------ pull ---
// Level mode, pull direction, one launch per round (multi-GPU windows, whose
// rounds are separated by the frontier exchange; PSAMD_FLOOD=0 on one GPU).
// In a single-start tree window a node of BFS level d receives, in round
// s + d, exactly its parent's row -- if the parent was reached this window
// (generation current) and the node is live -- and it is fresh (it has seen
// nothing this window), so the seen test-and-set is new = row(parent) & ~0
// and the whole row is written.  A wave owns a contiguous run of next-level
// nodes, whose rows form one contiguous output stream:
//   phase 1  resolves each node's source into a wave-private LDS table: its
//            parent if the parent is in the frontier (generation current) and
//            the node is live, else none; the node's generation is stamped;
//   phase 2  streams the run's rows in order with 16-B stores (8-B for odd
//            W), each lane's load taken from its node's parent row (siblings
//            read the same parent row: L2 hits).  Loads are unconditional (a
//            skipped node reads its own row) so the unrolled body keeps
//            several in flight.
// Counters: deliveries, seen writes, nodes visited, nodes reached, parents
// expanded (a reached parent counts at its first child) and their row words.
struct PullVec {
  bool go;
  uint4 v;
};

// Counters of the pull kernels, two forms: PullCtr (devutil.hpp) counts per
// lane, as k_pull's block reduction wants; WaveCtr keeps one per-lane
// delivery sum and counts everything else wave-uniformly (ballots: scalar
// registers), which k_pull_pair's persistent waves carry across chunks for
// two rounds without the vector registers per-lane counters would take.
struct WaveCtr {
  uint32_t deliv = 0;                      // per lane, folded into dsum per sub-run
  uint32_t kids = 0, reached = 0, parents = 0;  // wave-uniform
  uint64_t sw = 0, pwords = 0;             // wave-uniform: words written, parent words read
  uint64_t dsum = 0;                       // wave-uniform: folded deliveries
};
// The per-lane delivery count into the 64-bit wave total: after each sub-run
// of at most kPairKids rows (<= 2^24 bits), so neither the lane counts nor
// the sum over a wide run's children (f * W * 64 bits) wrap.
__device__ __forceinline__ void ctr_fold(WaveCtr& c) {
  c.dsum += __builtin_amdgcn_readfirstlane(__reduce_add_sync(~0ull, c.deliv));  // (a sub-run: < 2^32)
  c.deliv = 0;
}
// One batch of (up to 64) nodes: visited (in), reached (ok), a reached
// parent's first child (par); W_sw row words written per reached node,
// W_pw parent row words read per counted parent.
__device__ __forceinline__ void ctr_nodes(PullCtr& c, bool in, bool ok, bool par, uint32_t, uint32_t W_pw) {
  c.kids += in;
  c.reached += ok;
  if (par) {
    c.parents += 1;
    c.pwords += W_pw;
  }
}
__device__ __forceinline__ void ctr_nodes(WaveCtr& c, bool in, bool ok, bool par, uint32_t W_sw, uint32_t W_pw) {
  c.kids += __popcll(__ballot(in));
  const uint32_t r = __popcll(__ballot(ok));
  c.reached += r;
  c.sw += static_cast<uint64_t>(r) * W_sw;
  const uint32_t p = __popcll(__ballot(par));
  c.parents += p;
  c.pwords += static_cast<uint64_t>(p) * W_pw;
}
// One lane's stored unit: its delivered bits, and (PullCtr) its words.
__device__ __forceinline__ void ctr_unit(PullCtr& c, bool own, uint32_t pop, uint32_t words) {
  c.deliv += own ? pop : 0u;
  c.sw += own ? words : 0u;
}
__device__ __forceinline__ void ctr_unit(WaveCtr& c, bool own, uint32_t pop, uint32_t) { c.deliv += own ? pop : 0u; }

// Chunk constants: row of node u = base + u * W (a start group's block row
// for kTopicGroups topics).
struct PullTopic {
  uint64_t base;
  uint32_t W, nbase, root;
};

// Phase 1 for the nodes [nb, nb + nk) of one level: src[j] = the address of
// the row node nb + j copies (its parent's row: the root's arrival row, a
// seen row, or -- multi-GPU -- a ghost row in the receive buffer), or 0.  The
// parents of a run are consecutive node ids [p_lo, p_hi] (BFS numbering):
// their generation bytes are staged into LDS by loads issued together with
// the nodes' own metadata, so phase 1 costs one memory round trip.
template <class Ctr>
__device__ __forceinline__ void pull_resolve(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t nk,
                                             uint32_t p_lo, uint32_t p_hi, uint64_t* src, uint8_t* genl,
                                             uint32_t lane, uint32_t cur, Ctr& c, uint32_t gin,
                                             uint32_t stage_cap = kPullMaxKids) {
  uint32_t g0 = 0;
  const bool staged = p_lo != kNoneNode && p_hi - p_lo < stage_cap;  // genl holds stage_cap + 8 bytes
  if (staged) {
    g0 = p_lo & ~3u;
    const uint32_t nd = ((p_hi + 4u) & ~3u) - g0;  // bytes, whole dwords
    const uint32_t* gsrc = reinterpret_cast<const uint32_t*>(a.gen + g0);
    for (uint32_t d = lane; 4 * d < nd; d += 64) reinterpret_cast<uint32_t*>(genl)[d] = gsrc[d];
  }
  for (uint32_t j0 = 0; j0 < nk; j0 += 64) {
    const uint32_t j = j0 + lane;
    const bool in = j < nk;
    uint32_t p = kNoneNode, f = 0;
    if (in) {
      p = a.node_parent[nb + j];
      f = a.node_flags[nb + j];
    }
    bool up = false;  // the parent was reached this window
    uint64_t row = 0;
    uint32_t pid = p;  // the parent's identity for the once-per-parent count
    if (in && p != kNoneNode) {
      up = (staged ? genl[p - g0] : a.gen[p]) == cur;
      row = reinterpret_cast<uint64_t>((p == P.root ? a.a_cur : a.seen) + P.base + static_cast<uint64_t>(p) * P.W);
    } else if (in && gin != kNoneNode) {  // parent on another rank: its record arrived this round
      const uint32_t g = a.ghost_ref[nb + j];
      if (g != kNoneNode) {
        const GhostSeg* S = a.gsegs + gin;
        const uint64_t* rec = a.recv + S->rbase[g >> kRemoteRankShift] +
                              static_cast<uint64_t>(g & kRemoteIdMask) * S->rw;
        up = rec[0] != 0;  // an unreached parent's record starts with a zero word
        row = reinterpret_cast<uint64_t>(rec);
        pid = 0x80000000u | g;
      }
    }
    uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(pid), 1, 64));
    if (lane == 0) {
      prev = kNoneNode;
      const uint32_t q = nb + j0;
      if (q > P.nbase) {
        prev = a.node_parent[q - 1];
        if (prev == kNoneNode && gin != kNoneNode && a.ghost_ref[q - 1] != kNoneNode)
          prev = 0x80000000u | a.ghost_ref[q - 1];
      }
    }
    const bool ok = up && (f & kNodeLive);
    if (in) src[j] = ok ? row : 0ull;
    if (ok) a.gen[nb + j] = static_cast<uint8_t>(cur);
    ctr_nodes(c, in, ok, up && pid != prev, P.W, P.W);
  }
}

// row store of the pull stream: plain, or non-temporal (`nt`: rows nobody
// re-reads soon)
template <bool kNT>
__device__ __forceinline__ void store_row16(uint64_t* p, const uint4& v) {
  if constexpr (kNT) {
    u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}
template <bool kNT>
__device__ __forceinline__ void store_row8(uint64_t* p, uint64_t v) {
  if constexpr (kNT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Phase 2: the rows of nodes [nb, nb + nk) as one output stream, each lane's
// load from the row its node copies (src[], kNoneNode = skip).  8 loads in
// flight, then 8 stores, unconditional and branch-free (a skipped lane writes
// its own row back unchanged, a lane past the run's end stores the run's last
// pair again with the value its owner stores), so the compiler counts vmcnt
// exactly instead of draining at branches.  kLds (k_pull_pair): every word
// also goes to lrows[i], the run's rows in LDS for its children.
template <bool kRecord, bool kNT, bool kLds = false, class Ctr = PullCtr>
__device__ __forceinline__ void pull_stream(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t nk,
                                            const uint64_t* src, uint32_t lane, uint32_t round, Ctr& c,
                                            uint64_t* lrows = nullptr) {
  constexpr uint32_t kU = 8;
  const uint32_t W = P.W;
  const uint64_t base = P.base;
  const uint32_t total = nk * W;
  uint64_t* const out = a.seen + base + static_cast<uint64_t>(nb) * W;
  const float rw = 1.0f / static_cast<float>(W);
  // row kk = i / W and word r of the run, branch-free (float estimate off by
  // at most one; i < 2^24)
  auto split = [&](uint32_t i, int32_t& kk, int32_t& r) {
    kk = static_cast<int32_t>(static_cast<float>(i) * rw);
    r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(W);
    const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(W);
    kk += hi - lo;
    r += (lo - hi) * static_cast<int32_t>(W);
  };
  if (!(W & 1u)) {
    // even W: every row 16-B aligned, a 2-word pair never straddles rows
    auto one = [&](uint32_t i) {
      int32_t kk, r;
      split(i, kk, r);
      const uint64_t row = src[kk];
      const bool go = row != 0;
      const uint64_t* s = go ? reinterpret_cast<const uint64_t*>(row) + r : out + i;
      return PullVec{go, *reinterpret_cast<const uint4*>(s)};
    };
    // the stream starts h words before the run, at a 128-B line, so every
    // 1-KB wave store covers whole lines (lanes before the run store its
    // first pair again, with the value its owner stores)
    const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;
    for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 128) {
      PullVec x[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t i = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
        x[u] = one(i < 0 ? 0u : (static_cast<uint32_t>(i) < total ? static_cast<uint32_t>(i) : total - 2));
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
        const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
        const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 2);
        if constexpr (kRecord) {
          if (x[u].go && inr) {
            *reinterpret_cast<uint4*>(out + i) = x[u].v;
            const uint64_t cw = (out - a.seen) + i;
            record_word(a.hop_rec, cw, static_cast<uint64_t>(x[u].v.y) << 32 | x[u].v.x, round);
            record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(x[u].v.w) << 32 | x[u].v.z, round);
          }
        } else {
          store_row16<kNT>(out + i, x[u].v);
        }
        if constexpr (kLds) *reinterpret_cast<uint4*>(lrows + i) = x[u].v;  // (i clamped: its owner's value)
        const bool own = x[u].go && inr;
        ctr_unit(c, own, popc4(x[u].v), 2u);
      }
    }
  } else {
    // odd W: one word (8 B) per lane, the same pipeline
    const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;  // line-aligned start
    for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 64) {
      uint64_t m[kU];
      bool go[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
        // before the run: its first word again; past the end: its last word again
        const uint32_t ic = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 1);
        int32_t kk, r;
        split(ic, kk, r);
        const uint64_t row = src[kk];
        go[u] = row != 0;
        const uint64_t* s = go[u] ? reinterpret_cast<const uint64_t*>(row) + r : out + ic;
        m[u] = *s;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
        const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
        const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 1);
        if constexpr (kRecord) {
          if (go[u] && inr) {
            out[i] = m[u];
            record_word(a.hop_rec, (out - a.seen) + i, m[u], round);
          }
        } else {
          store_row8<kNT>(out + i, m[u]);
        }
        if constexpr (kLds) lrows[i] = m[u];
        const bool own = go[u] && inr;
        ctr_unit(c, own, __popcll(m[u]), 1u);
      }
    }
  }
}

// Multi-GPU: the chunk's nodes that are ghost parents next round ship their
// rows now, as records in the send buffer (GhostSeg gout: record k to rank b
// at sbase[b] + k * W), from the rows they copied (src[]: L2-resident, just
// read): one pass over the records, 16-B units for even W.  An unreached
// node's record gets a zero first word.  Replaces a separate pack launch that
// re-read the rows from HBM.
__device__ __forceinline__ void pull_ship(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t e_lo,
                                          uint32_t e_hi, uint32_t gout, const uint64_t* src, uint32_t lane) {
  const GhostSeg* S = a.gsegs + gout;
  const bool pairs = !(P.W & 1u);
  const uint32_t per = pairs ? P.W >> 1 : P.W;
  const uint32_t total = (e_hi - e_lo) * per;
  for (uint32_t i = lane; i < total; i += 64) {
    const uint32_t k = i / per, r = i - k * per;
    const ShipEntry E = a.ship[e_lo + k];
    const uint64_t row = src[E.node - nb];
    uint64_t* rec = a.send + S->sbase[E.dst >> kRemoteRankShift] +
                    static_cast<uint64_t>(E.dst & kRemoteIdMask) * P.W;
    if (row == 0) {
      if (r == 0) rec[0] = 0;
      continue;
    }
    const uint32_t w = pairs ? 2 * r : r;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(row) + w;
    if (pairs)
      *reinterpret_cast<uint4*>(rec + w) = *reinterpret_cast<const uint4*>(s);
    else
      rec[w] = *s;
  }
}

// The block's counters of one launch into partial slot `slot` (blocks share
// a slot: slots are zeroed per window).
__device__ __forceinline__ void pull_flush(const PullCtr& c, uint64_t* partials, uint64_t slot, uint32_t lane,
                                           uint32_t wid) {
  __shared__ uint64_t red[kBlock / 64][7];
  const uint64_t v7[7] = {wave_sum_u64(c.deliv),   wave_sum_u64(c.sw),      wave_sum_u64(c.kids),
                          wave_sum_u64(c.reached), wave_sum_u64(c.parents), wave_sum_u64(c.pwords),
                          wave_sum_u64(c.dup)};
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) red[wid][q] = v7[q];
  __syncthreads();
  if (threadIdx.x < kNumCtr) {
    uint64_t t[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < kBlock / 64; ++w)
#pragma unroll
      for (int q = 0; q < 7; ++q) t[q] += red[w][q];
    const uint64_t v = pull_ctr_pick(t, threadIdx.x);
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(partials + slot * kNumCtr + threadIdx.x),
                     static_cast<unsigned long long>(v));
  }
}

template <bool kRecord, bool kNT>
__global__ __launch_bounds__(kBlock) void k_pull(PullArgs a, const PullChunk* __restrict__ chunks,
                                                 uint32_t n_chunks, uint32_t round) {
  __shared__ uint64_t src_lds[kBlock / 64][kPullMaxKids];
  __shared__ uint32_t gen_lds[kBlock / 64][kPullMaxKids / 4 + 2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * (kBlock / 64) + wid;
  uint64_t* src = src_lds[wid];
  uint8_t* genl = reinterpret_cast<uint8_t*>(gen_lds[wid]);
  const uint32_t cur = a.gen_cur & 0xFF;
  PullCtr c;
  if (wave < n_chunks) {  // one chunk per wave
    const PullChunk ch = chunks[wave];
    const TopicDev T = a.topics[ch.topic];
    PullTopic P;
    P.W = ch.W;
    P.nbase = T.nbase;
    P.base = (static_cast<uint64_t>(ch.row0_hi) << 32 | ch.row0_lo) - static_cast<uint64_t>(T.nbase) * ch.W;
    P.root = (T.flags & kTopicRootLocal) ? T.nbase : kNoneNode;
    const uint32_t n1 = ch.node_end - ch.node_begin;
    // LDS ops of a wave are processed in order: the table written in phase 1
    // is visible to the reads that follow
    pull_resolve(a, P, ch.node_begin, n1, ch.p_lo, ch.p_hi, src, genl, lane, cur, c, ch.gin);
    pull_stream<kRecord, kNT>(a, P, ch.node_begin, n1, src, lane, round, c);
    if (ch.e_hi > ch.e_lo) pull_ship(a, P, ch.node_begin, ch.e_lo, ch.e_hi, ch.gout, src, lane);
  }
  pull_flush(c, a.partials, blockIdx.x % a.slot_mod, lane, wid);
}

// k_pull_pair: rounds q and q + 1 in one launch (one rank).
// A wave writes a run of level-d nodes as k_pull does (phase A: round q, the
// parents' rows from HBM, reach decided from this window's generation
// bytes), keeping the rows it writes in LDS, and then every child of the run
// (phase B: round q + 1, level d + 1 -- the children of a BFS-numbered run
// are consecutive ids): a child copies its parent's row as round q left it,
// read from LDS instead of HBM, if the parent was reached and the child is
// live, and stamps its generation.  No other wave writes those parents or
// reads those children, so the launch needs no cross-wave ordering.
//
// Phase B, one sub-run of at most kPairKids children: resolve into ctab (the
// LDS word offset of the parent's row, or kPairWords: a zero pair, so an
// unreached child's row is written with zeros -- stale under its old
// generation byte, so never read), then one line-aligned output stream with
// the phase-A pipeline.
// The first sub-run's parent ids and flags arrive prefetched (pf_p, pf_f:
// loaded with phase A's metadata, one memory round trip for both).
template <bool kRecord, bool kNT, uint32_t kWords>
__device__ __forceinline__ void pair_kids(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t n1,
                                          uint32_t c_lo, uint32_t c_hi, const uint64_t* reach,
                                          const uint64_t* lrows, uint32_t* ctab, uint32_t lane, uint32_t round,
                                          const uint32_t* pf_p, const uint32_t* pf_f, WaveCtr& c) {
  constexpr uint32_t kU = 8;
  constexpr uint32_t kZero = kWords;
  const uint32_t W = P.W;
  const uint32_t cur = a.gen_cur & 0xFF;
  const float rw = 1.0f / static_cast<float>(W);
  auto split = [&](uint32_t i, int32_t& kk, int32_t& r) {
    kk = static_cast<int32_t>(static_cast<float>(i) * rw);
    r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(W);
    const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(W);
    kk += hi - lo;
    r += (lo - hi) * static_cast<int32_t>(W);
  };
  for (uint32_t k0 = c_lo; k0 < c_hi; k0 += kPairKids) {
    const uint32_t nk = min(kPairKids, c_hi - k0);
#pragma unroll
    for (uint32_t s = 0; s < kPairKids / 64; ++s) {
      const uint32_t j0 = s * 64;
      if (j0 >= nk) break;
      const uint32_t j = j0 + lane;
      const bool in = j < nk;
      uint32_t p = kNoneNode, f = 0;
      if (k0 == c_lo) {
        p = in ? pf_p[s] : kNoneNode;
        f = pf_f[s];
      } else if (in) {
        p = a.node_parent[k0 + j];
        f = a.node_flags[k0 + j];
      }
      const uint32_t kp = p - nb;  // the parent's place in the run
      const bool up = in && kp < n1 && ((a.all_current & 1u) || ((reach[kp >> 6] >> (kp & 63)) & 1ull));
      const bool ok = up && (f & kNodeLive);
      if (in) ctab[j] = ok ? kp * W : kZero;
      if (ok) a.gen[k0 + j] = static_cast<uint8_t>(cur);
      uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(p), 1, 64));
      if (lane == 0) prev = k0 + j0 > P.nbase ? a.node_parent[k0 + j0 - 1] : kNoneNode;
      ctr_nodes(c, in, ok, up && p != prev, W, 0u);  // (parent rows from LDS: no parent words read)
    }
    const uint32_t total = nk * W;
    uint64_t* const out = a.seen + P.base + static_cast<uint64_t>(k0) * W;
    const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;
    if (!(W & 1u)) {
      for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 128) {
        uint4 x[kU];
        bool go[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
          const uint32_t i = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 2);
          int32_t kk, r;
          split(i, kk, r);
          const uint32_t off = ctab[kk];
          go[u] = off != kZero;
          x[u] = *reinterpret_cast<const uint4*>(lrows + (go[u] ? off + r : kZero));
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
          const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
          const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 2);
          if constexpr (kRecord) {
            if (go[u] && inr) {
              *reinterpret_cast<uint4*>(out + i) = x[u];
              const uint64_t cw = (out - a.seen) + i;
              record_word(a.hop_rec, cw, static_cast<uint64_t>(x[u].y) << 32 | x[u].x, round);
              record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(x[u].w) << 32 | x[u].z, round);
            }
          } else {
            store_row16<kNT>(out + i, x[u]);
          }
          const bool own = go[u] && inr;
          ctr_unit(c, own, popc4(x[u]), 2u);
        }
      }
    } else {
      for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 64) {
        uint64_t m[kU];
        bool go[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
          const uint32_t i = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 1);
          int32_t kk, r;
          split(i, kk, r);
          const uint32_t off = ctab[kk];
          go[u] = off != kZero;
          m[u] = lrows[go[u] ? off + r : kZero];
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
          const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
          const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 1);
          if constexpr (kRecord) {
            if (go[u] && inr) {
              out[i] = m[u];
              record_word(a.hop_rec, (out - a.seen) + i, m[u], round);
            }
          } else {
            store_row8<kNT>(out + i, m[u]);
          }
          const bool own = go[u] && inr;
          ctr_unit(c, own, __popcll(m[u]), 1u);
        }
      }
    }
    ctr_fold(c);
  }
}

__device__ __forceinline__ void ctr_add(WaveCtr& d, const WaveCtr& s) {
  d.deliv += s.deliv;  // (one phase-A run: <= kPairWords * 64 bits, folded below)
  d.dsum += s.dsum;
  d.sw += s.sw;
  d.kids += s.kids;
  d.reached += s.reached;
  d.parents += s.parents;
  d.pwords += s.pwords;
}

// Counters of a wave (two rounds) added with its own atomics: no block
// reduction, so no barrier.
__device__ __forceinline__ void pull_flush_wave(const WaveCtr& c, uint64_t* partials, uint64_t slot, uint32_t lane) {
  const uint64_t v7[7] = {c.dsum + __reduce_add_sync(~0ull, c.deliv), c.sw, c.kids, c.reached, c.parents,
                          c.pwords, 0ull};
  if (lane < kNumCtr) {
    const uint64_t v = pull_ctr_pick(v7, lane);
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(partials + slot * kNumCtr + lane),
                     static_cast<unsigned long long>(v));
  }
}

// One wave per workgroup, one chunk per wave (grid = n_chunks; the loop
// only guards a smaller grid).  A chunk's two phases take longer when its
// run has more children: one-wave workgroups never wait for siblings (a
// 4-wave block's barrier held its LDS behind the slowest chunk: cfg3 (18,19)
// 583 -> 549 us).  Persistent waves looping over chunks measured slower at
// every grid tried (resident grid 700 us, 8192 waves 588 us, one chunk per
// wave 543 us): a wave's chunks run back to back, each paying its round
// trips, where fresh waves overlap them.
template <bool kRecord, bool kNT2>
__global__ __launch_bounds__(64) void k_pull_pair(PullArgs a, const PullChunk* __restrict__ chunks,
                                                  uint32_t n_chunks, uint32_t round) {
  __shared__ uint64_t rows[kPairWords + 2];  // + the zero pair
  __shared__ uint64_t src[kPairPar];         // phase A sources, then phase B's ctab
  __shared__ uint32_t gen_lds[kPairPar / 4 + 2];
  __shared__ uint64_t reach[kPairPar / 64];
  static_assert(kPairKids * 4 <= kPairPar * 8, "ctab fits the source table");
  const uint32_t lane = threadIdx.x;
  uint8_t* genl = reinterpret_cast<uint8_t*>(gen_lds);
  const uint32_t cur = a.gen_cur & 0xFF;
  if (lane < 2) rows[kPairWords + lane] = 0;
  WaveCtr c, c2;
  for (uint32_t ci = blockIdx.x; ci < n_chunks; ci += gridDim.x) {
    const PullChunk ch = chunks[ci];
    const TopicDev T = a.topics[ch.topic];
    PullTopic P;
    P.W = ch.W;
    P.nbase = T.nbase;
    P.base = (static_cast<uint64_t>(ch.row0_hi) << 32 | ch.row0_lo) - static_cast<uint64_t>(T.nbase) * ch.W;
    P.root = (T.flags & kTopicRootLocal) ? T.nbase : kNoneNode;
    const uint32_t n1 = ch.node_end - ch.node_begin;  // <= kPairPar, n1 * W <= kPairWords (host plan)
    const bool late = ch.c_lo == kNoneNode;           // a level-1 run of round q + 1
    // the first children's metadata, issued ahead of phase A's own
    uint32_t pf_p[kPairKids / 64], pf_f[kPairKids / 64];
    const uint32_t nk0 = late ? 0u : min(kPairKids, ch.c_hi - ch.c_lo);
#pragma unroll
    for (uint32_t s = 0; s < kPairKids / 64; ++s) {
      const uint32_t j = s * 64 + lane;
      pf_p[s] = j < nk0 ? a.node_parent[ch.c_lo + j] : kNoneNode;
      pf_f[s] = j < nk0 ? a.node_flags[ch.c_lo + j] : 0u;
    }
    WaveCtr ca;
    pull_resolve(a, P, ch.node_begin, n1, ch.p_lo, ch.p_hi, src, genl, lane, cur, ca, ch.gin, kPairPar);
    for (uint32_t j0 = 0; j0 < n1; j0 += 64) {
      const uint64_t b = __ballot(j0 + lane < n1 && src[j0 + lane] != 0);
      if (lane == 0) reach[j0 >> 6] = b;
    }
    pull_stream<kRecord, true, true>(a, P, ch.node_begin, n1, src, lane, round + (late ? 1 : 0), ca, rows);
    ctr_fold(ca);
    // src (u64 sources) and ctab (u32 offsets) share the LDS table: no memory
    // access may move across the switch from one view to the other
    asm volatile("" ::: "memory");
    if (late) {
      ctr_add(c2, ca);
    } else {
      ctr_add(c, ca);
      if (ch.c_hi > ch.c_lo)
        pair_kids<kRecord, kNT2, kPairWords>(a, P, ch.node_begin, n1, ch.c_lo, ch.c_hi, reach, rows,
                                             reinterpret_cast<uint32_t*>(src), lane, round + 1, pf_p, pf_f, c2);
    }
    asm volatile("" ::: "memory");
  }
  pull_flush_wave(c, a.partials, blockIdx.x % a.slot_mod, lane);
  pull_flush_wave(c2, a.partials2, blockIdx.x % a.slot_mod, lane);
}

// Children ranges of the pair chunks (GPU or host node space alike).
__global__ __launch_bounds__(kBlock) void k_pair_kids(PullChunk* __restrict__ chunks, uint32_t n,
                                                      const uint32_t* __restrict__ row_ptr,
                                                      const uint32_t* __restrict__ col) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  PullChunk& c = chunks[i];
  if (c.c_lo == kNoneNode) return;
  const uint32_t rb = row_ptr[c.node_begin], re = row_ptr[c.node_end];
  c.c_lo = re > rb ? col[rb] : 0u;
  c.c_hi = re > rb ? col[re - 1] + 1u : 0u;
}

// Multi-GPU level mode: the topic roots' records of a round (the roots are
// seeded, so always reached).  Thread i of the flattened stream copies unit i
// of one record -- a 16-B word pair for even W, one word for odd W: segment
// (one root, constant W) by a short scan, entry = offset / units per row.
__global__ __launch_bounds__(kBlock) void k_pack(const ShipEntry* __restrict__ ship,
                                                 const PackSeg* __restrict__ segs, uint32_t n_segs,
                                                 uint64_t total, const GhostSeg* __restrict__ gsegs,
                                                 const uint64_t* __restrict__ seen, uint64_t* __restrict__ send) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < total;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    uint32_t k = 0;
    while (k + 1 < n_segs && segs[k + 1].unit0 <= i) ++k;
    const PackSeg S = segs[k];
    const bool pairs = !(S.W & 1u);
    const uint32_t per = pairs ? S.W >> 1 : S.W;  // units per row
    const uint32_t o = static_cast<uint32_t>(i - S.unit0);
    const uint32_t e = S.e0 + o / per;
    const uint32_t w = (o - (e - S.e0) * per) << (pairs ? 1 : 0);
    const ShipEntry E = ship[e];
    uint64_t* rec = send + gsegs[S.gseg].sbase[E.dst >> kRemoteRankShift] +
                    static_cast<uint64_t>(E.dst & kRemoteIdMask) * S.W;
    const uint64_t* row = seen + S.row + w;
    if (pairs)
      *reinterpret_cast<uint4*>(rec + w) = *reinterpret_cast<const uint4*>(row);
    else
      rec[w] = *row;
  }
}

// GPU-built node spaces have no host mirror of node_parent: the chunks'
// parent ranges (k_pull's generation staging) are filled in on the device.
__global__ __launch_bounds__(kBlock) void k_chunk_parents(PullChunk* __restrict__ chunks, uint32_t n,
                                                          const uint32_t* __restrict__ node_parent) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  PullChunk& c = chunks[i];
  if (c.node_end <= c.node_begin) return;
  c.p_lo = node_parent[c.node_begin];
  c.p_hi = node_parent[c.node_end - 1];
}

__global__ __launch_bounds__(kBlock) void k_stage_copy(StageCopy c) {
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x, nth = gridDim.x * kBlock;
  for (uint32_t k = 0; k < c.n; ++k)
    for (uint32_t i = tid; i < c.words[k]; i += nth) c.dst[k][i] = c.src[k][i];
}

// ----------------------------------------------------------------- apply ---
// Deliveries received from other ranks: test-and-set into the owned node's
// row (atomic: its row was zeroed at window init), arrival row written whole
// (the sender ships every word of the parent's arrival row).
template <bool kRecord>
__global__ __launch_bounds__(kBlock) void k_apply(ApplyArgs a, uint32_t round) {
  const uint64_t total = a.cap_pre[a.world];
  uint64_t deliv = 0, dup = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < total;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    uint32_t src = 0;
    while (i >= a.cap_pre[src + 1]) ++src;
    const uint8_t* region = a.recv + a.recv_off[src];
    const uint64_t k = i - a.cap_pre[src];
    if (k >= *reinterpret_cast<const uint32_t*>(region)) continue;
    const XItem it = reinterpret_cast<const XItem*>(region + kRegionHeader)[k];
    const uint8_t f = a.node_flags[it.node];
    if (!(f & kNodeLive) || it.mask == 0) {
      if ((f & kNodeLive) && (f & kNodeInternal)) {
        const TopicDev T = a.topics[a.node_topic[it.node]];
        if (!(T.flags & kTopicSingleStart))
          a.a_next[T.wbase + static_cast<uint64_t>(it.node - T.nbase) * T.W + it.word] = 0;
      }
      continue;
    }
    const TopicDev T = a.topics[a.node_topic[it.node]];
    const uint64_t cw = T.wbase + static_cast<uint64_t>(it.node - T.nbase) * T.W + it.word;
    const uint64_t old = atomicOr(reinterpret_cast<unsigned long long*>(a.seen + cw),
                                  static_cast<unsigned long long>(it.mask));
    const uint64_t nm = it.mask & ~old;
    if (a.gen != nullptr && nm) a.gen[it.node] = static_cast<uint8_t>(a.gen_cur);  // reached
    if ((f & kNodeInternal) && !(T.flags & kTopicSingleStart)) a.a_next[cw] = nm;
    dup += __popcll(it.mask & old);
    if (nm) {
      deliv += __popcll(nm);
      if ((f & kNodeInternal) && a.next_flag != nullptr) {
        a.next_flag[it.node] = 1;
        a.blk_flag[it.node >> kFlagBlockShift] = 1;
      }
      if constexpr (kRecord) {
        uint16_t* h = a.hop_rec + cw * 64;
        uint64_t b = nm;
        while (b) {
          const int q = __ffsll(static_cast<long long>(b)) - 1;
          h[q] = hop_round(round);
          b &= b - 1;
        }
      }
    }
  }
  deliv = wave_sum_u64(deliv);
  dup = wave_sum_u64(dup);
  if ((threadIdx.x & 63) == 0 && (deliv || dup)) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a.stats + kCtrDeliveries), deliv);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.stats + kCtrDuplicates), dup);
  }
}

// ------------------------------------------------------------ compaction ---
// One block folds the partial counter slots w0, w0 + stride, ... (< w1) into
// one round's statistics.
__device__ __forceinline__ void block_reduce_ctrs(const uint64_t* __restrict__ partials,
                                                  uint32_t w0, uint32_t w1, uint32_t stride,
                                                  uint64_t* __restrict__ out) {
  __shared__ uint64_t red[kNumCtr][kBlock / 64];
  uint64_t acc[kNumCtr];
#pragma unroll
  for (int k = 0; k < kNumCtr; ++k) acc[k] = 0;
  for (uint32_t w = w0 + threadIdx.x * stride; w < w1; w += kBlock * stride)
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
    out[threadIdx.x] = s;
  }
}

// Level mode: one block per round q (block 0: the unused row 0) folds the
// round's partial slots (desc[3q..3q+2] = first slot, end slot, stride) as
// one coalesced stream of counters (kAct threads, each on one counter index)
// and writes the round's statistics row.  Pull launches share at most
// kPullSlots slots per round between their blocks, so the streams are short.
__global__ __launch_bounds__(kBlock) void k_reduce_rounds(const uint64_t* __restrict__ partials,
                                                          const uint32_t* __restrict__ desc,
                                                          uint64_t* __restrict__ round_stats,
                                                          uint64_t* __restrict__ host_stats) {
  constexpr uint32_t kAct = (kBlock / kNumCtr) * kNumCtr;
  __shared__ uint64_t red[kBlock];
  const uint32_t q = blockIdx.x;
  const uint32_t first = desc[3 * q], end = desc[3 * q + 1], stride = desc[3 * q + 2];
  uint64_t acc = 0;
  if (stride && threadIdx.x < kAct) {
    const uint32_t e1 = end * kNumCtr;
    uint32_t i = first * kNumCtr + threadIdx.x;
    if (stride == 1) {
      uint64_t x[4] = {0, 0, 0, 0};
      for (; i + 3 * kAct < e1; i += 4 * kAct)
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] += partials[i + u * kAct];
      for (; i < e1; i += kAct) x[0] += partials[i];
      acc = x[0] + x[1] + x[2] + x[3];
    } else {
      for (; i < e1; i += kAct)
        if ((i / kNumCtr - first) % stride == 0) acc += partials[i];
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < kNumCtr) {
    uint64_t t = 0;
    for (uint32_t k = threadIdx.x; k < kAct; k += kNumCtr) t += red[k];
    round_stats[static_cast<uint64_t>(q) * kNumCtr + threadIdx.x] = t;
    if (host_stats) {  // fine-grained pinned host rows: visible to the host once the kernel ends
      __hip_atomic_store(host_stats + static_cast<uint64_t>(q) * kNumCtr + threadIdx.x, t, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
    }
  }
}

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
  if (blockIdx.x == 0 && round_stats != nullptr) block_reduce_ctrs(partials, 0, n_waves, 1, round_stats);
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
                                                   const GroupDev* __restrict__ groups,
                                                   uint32_t n_nodes, uint64_t* out) {
  uint64_t acc = 0;
  for (uint32_t u = blockIdx.x * kBlock + threadIdx.x; u < n_nodes; u += gridDim.x * kBlock) {
    const uint32_t t = node_topic[u];
    const TopicDev T = topics[t];
    if (T.W == 0) continue;
    const bool valid = (T.flags & kTopicMesh) || gen[u] == static_cast<uint8_t>(gen_cur);
    const uint64_t key0 = (static_cast<uint64_t>(node_peer[u]) << 32) | (static_cast<uint64_t>(t) << 16);
    if (T.flags & kTopicGroups) {  // virtual word w of the row from its group's block
      for (uint32_t g = 0; g < T.group_n; ++g) {
        const GroupDev G = groups[T.group_lo + g];
        const uint64_t blk = T.wbase + static_cast<uint64_t>(T.n_nodes) * G.w0 + static_cast<uint64_t>(u - T.nbase) * G.wn;
        for (uint32_t r = 0; r < G.wn && G.w0 + r < T.w_msgs; ++r)
          acc += mix64((key0 | (G.w0 + r)) ^ mix64(valid ? seen[blk + r] : 0ull));
      }
      continue;
    }
    const uint64_t row = T.wbase + static_cast<uint64_t>(u - T.nbase) * T.W;
    for (uint32_t w = 0; w < T.w_msgs; ++w)
      acc += mix64((key0 | w) ^ mix64(valid ? seen[row + w] : 0ull));
  }
  acc = wave_sum_u64(acc);
  if ((threadIdx.x & 63) == 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(out), static_cast<unsigned long long>(acc));
}

}  // namespace

hipError_t launch_window_init(const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur,
                              bool any_mesh, const WindowStart& ws, hipStream_t s) {
  if (n_topics == 0) return hipSuccess;
  const dim3 grid(any_mesh ? 64 : 1, n_topics);
  hipLaunchKernelGGL(k_window_init, grid, dim3(kBlock), 0, s, topics, seen, a0, a1, gen, gen_cur, ws);
  return hipGetLastError();
}

hipError_t launch_init_nodes(const uint32_t* nodes, uint32_t n, const uint16_t* node_topic,
                             const TopicDev* topics, uint64_t* seen, uint64_t* a0, uint64_t* a1,
                             uint8_t* gen, uint32_t gen_cur, bool stamp, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>(1024, (n + 3) / 4);
  hipLaunchKernelGGL(k_init_nodes, dim3(grid), dim3(kBlock), 0, s, nodes, n, node_topic, topics,
                     seen, a0, a1, gen, gen_cur, stamp);
  return hipGetLastError();
}

hipError_t launch_apply(const ApplyArgs& a, uint32_t round, bool record, hipStream_t s) {
  const uint64_t total = a.cap_pre[a.world];
  if (total == 0) return hipSuccess;
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(2048, (total + kBlock - 1) / kBlock));
  if (record)
    hipLaunchKernelGGL(k_apply<true>, dim3(grid), dim3(kBlock), 0, s, a, round);
  else
    hipLaunchKernelGGL(k_apply<false>, dim3(grid), dim3(kBlock), 0, s, a, round);
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

hipError_t launch_expand(const ExpandArgs& a, uint32_t round, bool record, uint32_t grid, hipStream_t s) {
  if (record)
    hipLaunchKernelGGL((k_expand<true, false>), dim3(grid), dim3(kBlock), 0, s, a, round);
  else
    hipLaunchKernelGGL((k_expand<false, false>), dim3(grid), dim3(kBlock), 0, s, a, round);
  return hipGetLastError();
}

hipError_t launch_expand_direct(const ExpandArgs& a, uint32_t round, bool record, uint32_t grid,
                                hipStream_t s) {
  if (record)
    hipLaunchKernelGGL((k_expand<true, true>), dim3(grid), dim3(kBlock), 0, s, a, round);
  else
    hipLaunchKernelGGL((k_expand<false, true>), dim3(grid), dim3(kBlock), 0, s, a, round);
  return hipGetLastError();
}

hipError_t launch_pull(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks,
                       uint32_t grid, uint32_t round, bool record, bool nt, bool cap, hipStream_t s) {
  if (n_chunks == 0 || grid == 0) return hipSuccess;
  // cap: the large (nt) rounds run at most 5 blocks per CU -- 10 KB of LDS
  // left unused per block caps residency (8 blocks: 6 % slower on cfg3's big
  // rounds on one rank); small rounds keep full residency, they need the
  // waves in flight
  const size_t kBigRoundLdsPad = cap ? 10240 : 0;
  if (record)  // parity runs: one variant
    hipLaunchKernelGGL((k_pull<true, false>), dim3(grid), dim3(kBlock), 0, s, a, chunks, n_chunks, round);
  else if (nt)
    hipLaunchKernelGGL((k_pull<false, true>), dim3(grid), dim3(kBlock), kBigRoundLdsPad, s, a, chunks, n_chunks,
                       round);
  else
    hipLaunchKernelGGL((k_pull<false, false>), dim3(grid), dim3(kBlock), 0, s, a, chunks, n_chunks, round);
  return hipGetLastError();
}

hipError_t launch_pull_pair(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks, uint32_t grid,
                            uint32_t round, bool record, bool nt2, hipStream_t s) {
  if (n_chunks == 0 || grid == 0) return hipSuccess;
  grid = grid < n_chunks ? grid : n_chunks;
  if (record)
    hipLaunchKernelGGL((k_pull_pair<true, false>), dim3(grid), dim3(64), 0, s, a, chunks, n_chunks, round);
  else if (nt2)
    hipLaunchKernelGGL((k_pull_pair<false, true>), dim3(grid), dim3(64), 0, s, a, chunks, n_chunks, round);
  else
    hipLaunchKernelGGL((k_pull_pair<false, false>), dim3(grid), dim3(64), 0, s, a, chunks, n_chunks, round);
  return hipGetLastError();
}

hipError_t launch_pair_kids(PullChunk* chunks, uint32_t n, const uint32_t* row_ptr, const uint32_t* col,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_kids, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chunks, n, row_ptr, col);
  return hipGetLastError();
}

hipError_t launch_pack(const ShipEntry* ship, const PackSeg* segs, uint32_t n_segs, uint64_t total_units,
                       const GhostSeg* gsegs, const uint64_t* seen, uint64_t* send, hipStream_t s) {
  if (total_units == 0 || n_segs == 0) return hipSuccess;
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(4096, (total_units + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_pack, dim3(grid), dim3(kBlock), 0, s, ship, segs, n_segs, total_units, gsegs, seen, send);
  return hipGetLastError();
}

hipError_t launch_chunk_parents(PullChunk* chunks, uint32_t n, const uint32_t* node_parent, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_chunk_parents, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chunks, n, node_parent);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_copy_regions(CopyRegions c) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x, nth = gridDim.x * kBlock;
  for (uint32_t k = 0; k < c.n; ++k)
    for (uint64_t i = tid; i < c.units[k]; i += nth) c.dst[k][i] = c.src[k][i];
}

hipError_t launch_copy_regions(const CopyRegions& c, hipStream_t s) {
  uint64_t most = 0;
  for (uint32_t k = 0; k < c.n; ++k) most = c.units[k] > most ? c.units[k] : most;
  if (most == 0) return hipSuccess;
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(2048, (most + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_copy_regions, dim3(grid), dim3(kBlock), 0, s, c);
  return hipGetLastError();
}

hipError_t launch_stage_copy(const StageCopy& c, hipStream_t s) {
  uint32_t most = 0;
  for (uint32_t k = 0; k < c.n; ++k) most = c.words[k] > most ? c.words[k] : most;
  if (most == 0) return hipSuccess;
  uint32_t grid = (most + kBlock - 1) / kBlock;
  grid = grid > 64 ? 64 : grid;
  hipLaunchKernelGGL(k_stage_copy, dim3(grid), dim3(kBlock), 0, s, c);
  return hipGetLastError();
}

hipError_t launch_reduce_rounds(const uint64_t* partials, const uint32_t* desc, uint32_t n_rounds,
                                uint64_t* round_stats, uint64_t* host_stats, hipStream_t s) {
  if (n_rounds == 0) return hipSuccess;
  hipLaunchKernelGGL(k_reduce_rounds, dim3(n_rounds + 1), dim3(kBlock), 0, s, partials, desc, round_stats,
                     host_stats);
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
                         const TopicDev* topics, const GroupDev* groups, uint32_t n_nodes, uint64_t* out,
                         hipStream_t s) {
  uint32_t grid = (n_nodes + kBlock - 1) / kBlock;
  if (grid > 4096) grid = 4096;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(k_digest, dim3(grid), dim3(kBlock), 0, s, seen, gen, gen_cur, node_peer,
                     node_topic, topics, groups, n_nodes, out);
  return hipGetLastError();
}

}  // namespace psamd
