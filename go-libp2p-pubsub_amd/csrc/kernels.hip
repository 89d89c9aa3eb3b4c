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
// Mesh children test-and-set with atomics; a tree child's test is settled
// without a load (deliver_tree), and on one rank a tree row of 64..704 words
// moves only its arrival extent -- the one start-group block a node receives
// per round (ExpandArgs::ext_cur).
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
// (block (bx, by) of a gx x gy grid: k_window_init's own, or the init part
// of k_window_turn)
__device__ __forceinline__ void window_init_block(const TopicDev* __restrict__ topics, uint64_t* __restrict__ seen,
                                                  uint64_t* __restrict__ a0, uint64_t* __restrict__ a1,
                                                  uint8_t* __restrict__ gen, uint32_t gen_cur, const WindowStart& ws,
                                                  uint32_t bx, uint32_t by, uint32_t gx, uint32_t gy) {
  // folded-in work (one launch instead of three): the staged copies and the
  // partial-slot clear, grid-stride over every block
  const uint32_t nb = gx * gy;
  const uint32_t bid = by * gx + bx;
  for (uint32_t k = 0; k < ws.copy.n; ++k)
    for (uint32_t i = bid * kBlock + threadIdx.x; i < ws.copy.words[k]; i += nb * kBlock)
      ws.copy.dst[k][i] = ws.copy.src[k][i];
  for (uint64_t i = static_cast<uint64_t>(bid) * kBlock + threadIdx.x; i < ws.zero_words;
       i += static_cast<uint64_t>(nb) * kBlock)
    ws.zero[i] = 0;
  if (ws.t0 && bid == 0 && threadIdx.x == 0) *ws.t0 = __builtin_amdgcn_s_memrealtime();
  const TopicDev T = topics[by];
  if (T.W == 0 || T.n_nodes == 0) return;
  const bool mesh = (T.flags & kTopicMesh) != 0;
  const uint64_t n_words = mesh ? static_cast<uint64_t>(T.n_nodes) * T.W : T.root_words;
  if (!mesh && (bx != 0 || !(T.flags & kTopicRootLocal))) return;
  // (a tree root's row: block 0 alone, every word -- striding by the grid's
  // gx blocks left words 256 .. of rows wider than 256 words stale: a window
  // with fewer messages than the one before kept the old ones' bits there)
  const uint64_t step = static_cast<uint64_t>(mesh ? gx : 1u) * kBlock;
  for (uint64_t i = static_cast<uint64_t>(bx) * kBlock + threadIdx.x; i < n_words; i += step) {
    seen[T.wbase + i] = 0;
    a0[T.wbase + i] = 0;
    a1[T.wbase + i] = 0;
  }
  if (bx == 0 && threadIdx.x == 0 && (T.flags & kTopicRootLocal))
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

__global__ __launch_bounds__(kBlock) void k_window_init(const TopicDev* __restrict__ topics,
                                                        uint64_t* __restrict__ seen,
                                                        uint64_t* __restrict__ a0,
                                                        uint64_t* __restrict__ a1,
                                                        uint8_t* __restrict__ gen,
                                                        uint32_t gen_cur, WindowStart ws) {
  window_init_block(topics, seen, a0, a1, gen, gen_cur, ws, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y);
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

// A tree child whose row is current: stored, not tested.  A tree node has
// one parent, which forwards each start group's block once, and the blocks
// are word-disjoint (plan_window_layout), so every word that carries bits now
// is still zero in the child's seen row -- its first visit wrote the whole
// row, later visits only their own block's words.  (Meshes keep the atomic
// test-and-set, expand_direct; level mode relies on the same property.)
template <bool kRecord>
__device__ __forceinline__ uint64_t deliver_tree(const ExpandArgs& a, bool internal, uint64_t cw, uint64_t m,
                                                 uint32_t round, ExpandCtr& k) {
  if (m) {
    a.seen[cw] = m;
    k.sw += 1;
  }
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
  return m;
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

// Arrival extents (ExpandArgs::ext_cur / ext_next) apply to rows of a
// multi-start tree topic of 64..kStageWords words: a node at depth d receives
// only start group r - d in round r, one block of its row, so its parent
// writes (and it later reads) only that block's words.  Producer and
// consumer decide by the topic alone, so they always agree.
__device__ __forceinline__ bool ext_rows(const ExpandArgs& a, uint32_t W, uint32_t tflags) {
  return a.ext_cur != nullptr && W >= 64 && W <= kStageWords && !(tflags & (kTopicSingleStart | kTopicMesh));
}
constexpr uint32_t ext_whole(uint32_t W) { return W << 16; }
// the extent a consumer uses: ext_cur[p], or the whole row if that is not a
// sub-range of it (a guard: the stage is sized by it)
__device__ __forceinline__ uint32_t ext_of(const ExpandArgs& a, uint32_t p, uint32_t W) {
  const uint32_t x = a.ext_cur[p];
  return (x >> 16) <= W && (x & 0xFFFFu) <= (x >> 16) ? x : ext_whole(W);
}

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
  // arrival extent: words outside [xlo, xhi) of p's row are stale (read as 0)
  const bool ext = ext_rows(a, W, tflags);
  const uint32_t xe = ext && !is_root ? ext_of(a, p, W) : ext_whole(W);
  const uint32_t xlo = xe & 0xFFFFu, xhi = xe >> 16;
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
        const uint64_t m = active && w >= xlo && w < xhi ? src[pw + w] : 0ull;
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
          if (internal && __ballot(nm != 0) && lane == 0) {
            mark_next(a, c);
            if (ext) a.ext_next[c] = xe;
          }
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
                deliver_tree<kRecord>(a, store, crow + w, ws.words[w], round, k);
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

// Short tree entries: staged, not a topic root, and forwarding fewer than
// kFlatWords words -- a row under 64 words, or the arrival extent of a 64..704
// word row (one start-group block).  A 64-entry batch of them is one flattened
// index space instead of one entry at a time under scalar control (each cost
// ~224 scalar instructions of readlane broadcasts, address arithmetic and
// per-child loops: profiles/r05/expand/):
//   K1  (entry, child) pairs: the children's flag and generation bytes into
//       LDS slots (at most kFlatKids per batch; a batch with more flattens a
//       prefix of its entries and leaves the rest to the entry loop);
//   W   (entry, child, word) triples: item x of entry i is child j, word
//       lo_i + w with (j, w) = divmod(x - pre_i, L_i), pre_i a wave prefix of
//       deg_i * L_i; a lane finds its entry by a 6-step binary search of the
//       prefix ends (__shfl), loads the parent's word and stores as
//       deliver_fresh / deliver_tree do -- consecutive lanes write consecutive
//       words of one child row;
//   F   a stale child of an extent row: its seen row outside the extent is
//       zeroed (the lazy initialisation), one child at a time, 1 KiB per store;
//   K2  (entry, child) pairs: generation stamps, mark_next and the child's
//       extent, after every word pass (a child's row may straddle passes, and
//       every pass must see its pre-window generation).
// A non-root tree entry's staged extent is already the nonzero range of its
// words (its parent computed it from the same words, which a tree child
// receives unchanged), so the extent is forwarded as it is.
constexpr uint32_t kFlatWords = 64;
constexpr uint32_t kFlatKids = kStageBytes;  // child slots: ws.flags / ws.gens
#ifndef PSAMD_FLAT_UNROLL
#define PSAMD_FLAT_UNROLL 2
#endif
constexpr uint32_t kFlatUnroll = PSAMD_FLAT_UNROLL;  // (A/B builds: tools/build_variant.sh -DPSAMD_FLAT_UNROLL=n)

__device__ __forceinline__ bool flat_on(const ExpandArgs& a) { return (a.opts & kExpandNoNarrow) == 0; }

// Of the wave's 64 nondecreasing `end` values, the first lane whose end
// exceeds x (x < the last end).
__device__ __forceinline__ uint32_t owner_of(uint32_t end, uint32_t x) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 32; step; step >>= 1) {
    const uint32_t e = static_cast<uint32_t>(__shfl(static_cast<int>(end), static_cast<int>(lo + step - 1), 64));
    lo += e <= x ? step : 0u;
  }
  return lo;
}

__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, uint32_t lane) {
  return static_cast<uint32_t>(__shfl(static_cast<int>(v), static_cast<int>(lane), 64));
}

// One flat entry's fields, read by its items' lanes from LDS (kept there,
// not in registers for shuffles: the hot kernel's 80 VGPRs also hold the
// batch for the entry loop).
struct __attribute__((aligned(16))) FlatEnt {
  uint32_t pre;       // first W-pass item
  uint32_t lk;        // range words L | keep << 31
  uint32_t sl, sh;    // the staged words' address
  uint32_t cl, ch;    // child 0's first range word (seen / arrival word index)
  uint32_t W;         // row words
  uint32_t kpre;      // first child slot
  uint32_t c0;        // first child
  uint32_t xe;        // extent rows: lo | hi << 16 (the children's arrival extent); 0 otherwise
  uint32_t pad[2];
};
static_assert(sizeof(FlatEnt) == 48, "FlatEnt: three 16-B LDS reads");
constexpr uint32_t kFlatEntOff = 16;  // FlatEnt table in ws.words, after the `any` bytes
static_assert((kFlatEntOff + 64 * sizeof(FlatEnt) / 8) <= kStageWords, "FlatEnt table fits the stage");

// flat: this lane's entry takes the flat path; xe = its staged words (lo | hi
// << 16); ext: its children get arrival extents.  Returns whether the entry
// was handled (false: left to the entry loop, the child slots ran out).
__device__ __forceinline__ bool expand_flat(const ExpandArgs& a, WaveStage& ws, bool flat, uint32_t W, uint32_t xe,
                                            bool ext, uint32_t deg, uint32_t c0, uint64_t src, uint64_t crow,
                                            bool keep, uint32_t lane, uint32_t cur, ExpandCtr& k, EntryCtr& ec) {
  if (!__ballot(flat)) return false;
  // the child slots: a prefix of the flat entries whose children fit
  {
    const uint32_t kd = flat ? deg : 0u;
    const uint32_t kin = wave_incl_scan(kd);
    flat = flat && kin <= kFlatKids;
  }
  const uint64_t fmask = __ballot(flat);
  if (!fmask) return false;
  uint8_t* const fl = ws.flags;  // per child slot: node flag byte
  uint8_t* const gn = ws.gens;   // ... generation byte (before this round's stamps)
  uint8_t* const any = reinterpret_cast<uint8_t*>(ws.words);  // per entry lane: a word of its range is nonzero
  FlatEnt* const fe = reinterpret_cast<FlatEnt*>(ws.words + kFlatEntOff);
  const uint32_t lo = xe & 0xFFFFu, L = flat ? (xe >> 16) - lo : 0u;
  const uint32_t kids = flat ? deg : 0u;
  const uint32_t kend = wave_incl_scan(kids);
  const uint32_t ktotal = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(kend), 63));
  const uint32_t items = L * kids;
  const uint32_t end = wave_incl_scan(items);
  const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(end), 63));
  {
    FlatEnt e;
    e.pre = end - items;
    e.lk = L | (keep ? 0x80000000u : 0u);
    e.sl = static_cast<uint32_t>(src);
    e.sh = static_cast<uint32_t>(src >> 32);
    const uint64_t crow_lo = crow + lo;  // child 0's first word of the range
    e.cl = static_cast<uint32_t>(crow_lo);
    e.ch = static_cast<uint32_t>(crow_lo >> 32);
    e.W = W;
    e.kpre = kend - kids;
    e.c0 = c0;
    e.xe = ext ? xe : 0u;
    e.pad[0] = e.pad[1] = 0;
    fe[lane] = e;
    any[lane] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // K1: the children's bytes
  for (uint32_t b = 0; b < ktotal; b += 64) {
    const uint32_t x = b + lane;
    const bool valid = x < ktotal;  // (every lane takes part in the search's shuffles)
    const uint32_t o = owner_of(kend, valid ? x : ktotal - 1);
    if (valid) {
      const uint32_t c = fe[o].c0 + x - fe[o].kpre;
      fl[x] = a.node_flags[c];
      gn[x] = a.gen[c];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // W: the words of the ranges, kFlatUnroll passes per step -- every pass's
  // loads are issued before any pass's stores, so the parent words'
  // load-to-use latency is paid once per step
  for (uint32_t b = 0; b < total; b += 64 * kFlatUnroll) {
    uint64_t m[kFlatUnroll], cw[kFlatUnroll];
    uint32_t info[kFlatUnroll];  // flag | gen << 8 | keep << 16 | child 0 << 17 | owner << 24
#pragma unroll
    for (uint32_t u = 0; u < kFlatUnroll; ++u) {
      const uint32_t x = b + u * 64 + lane;
      const bool valid = x < total;
      const uint32_t o = owner_of(end, valid ? x : total - 1);
      m[u] = 0;
      info[u] = 0;
      cw[u] = 0;
      if (valid) {
        const FlatEnt& e = fe[o];
        const uint32_t Lo = e.lk & 0x7FFFFFFFu;
        const uint32_t r = x - e.pre;
        // j = r / Lo, w = r % Lo (float estimate, off by at most one; r < 2^24)
        int32_t j = static_cast<int32_t>(static_cast<float>(r) * (1.0f / static_cast<float>(Lo)));
        int32_t w = static_cast<int32_t>(r) - j * static_cast<int32_t>(Lo);
        const int32_t under = w < 0, over = w >= static_cast<int32_t>(Lo);
        j += over - under;
        w += (under - over) * static_cast<int32_t>(Lo);
        const uint32_t slot = e.kpre + j;
        const uint64_t* sp = reinterpret_cast<const uint64_t*>((static_cast<uint64_t>(e.sh) << 32) | e.sl);
        cw[u] = ((static_cast<uint64_t>(e.ch) << 32) | e.cl) + static_cast<uint64_t>(j) * e.W + w;
        m[u] = sp[w];
        info[u] = fl[slot] | static_cast<uint32_t>(gn[slot]) << 8 | (e.lk >> 31) << 16 | (j == 0 ? 1u : 0u) << 17 |
                  o << 24;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kFlatUnroll; ++u) {
      const uint32_t f = info[u];
      if (f & kNodeLive) {  // (valid items only: info is 0 elsewhere)
        if (((f >> 8) & 0xFFu) != cur || m[u]) {
          a.seen[cw[u]] = m[u];
          k.sw += 1;
        }
        if ((f & kNodeInternal) && (f & (1u << 16))) {
          a.a_next[cw[u]] = m[u];
          k.aw += 1;
        }
        k.deliv += __popcll(m[u]);
      }
      if ((f & (1u << 17)) && m[u]) any[f >> 24] = 1;
    }
  }
  // F: stale children of extent rows -- zeros outside the range
  for (uint32_t b = 0; b < ktotal; b += 64) {
    const uint32_t x = b + lane;
    const bool valid = x < ktotal;
    const uint32_t o = owner_of(kend, valid ? x : ktotal - 1);
    const bool fill = valid && fe[o].xe != 0 && (fl[x] & kNodeLive) && gn[x] != cur;
    uint64_t todo = __ballot(fill);
    while (todo) {
      const uint32_t v = static_cast<uint32_t>(__ffsll(static_cast<long long>(todo))) - 1u;
      todo &= todo - 1;
      const uint32_t ov = shfl_u32(o, v), xv = b + v;
      const FlatEnt& e = fe[ov];
      const uint32_t Wv = e.W, lov = e.xe & 0xFFFFu, hiv = e.xe >> 16;
      const uint64_t row =
          ((static_cast<uint64_t>(e.ch) << 32) | e.cl) - lov + static_cast<uint64_t>(xv - e.kpre) * Wv;
      for (uint32_t wb = 0; wb < Wv; wb += 128) {
        const uint32_t w = wb + 2 * lane;  // (W, lo and hi even; rows 16-B aligned)
        if (w < Wv && (w < lov || w >= hiv)) {
          *reinterpret_cast<uint4*>(a.seen + row + w) = make_uint4(0u, 0u, 0u, 0u);
          k.sw += 2;
        }
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // K2: generation stamps, the next frontier and its extents
  for (uint32_t b = 0; b < ktotal; b += 64) {
    const uint32_t x = b + lane;
    const bool valid = x < ktotal;
    const uint32_t o = owner_of(kend, valid ? x : ktotal - 1);
    const uint32_t f = valid ? fl[x] : 0u;
    if (f & kNodeLive) {
      const FlatEnt& e = fe[o];
      const uint32_t c = e.c0 + x - e.kpre;
      a.gen[c] = static_cast<uint8_t>(cur);
      if ((f & kNodeInternal) && any[o]) {
        mark_next(a, c);
        if (e.xe) a.ext_next[c] = e.xe;
      }
    }
  }
  ec.ent += static_cast<uint32_t>(__popcll(fmask));
  ec.ent_words += static_cast<uint32_t>(wave_sum_u64(L));
  ec.kids += ktotal;
  return flat;
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
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void k_expand(ExpandArgs a,
                                                                                            uint32_t round) {
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

  // v: the wave's slot in the sweep, numbered XCD-major (blocks are dealt
  // to the 8 XCDs round-robin; the blocks of one XCD take consecutive
  // slots): neighbouring entries -- their metadata, flag and generation
  // lines -- meet in one L2 (k_expand read traffic 1.42x -> 1.18x of its
  // algorithmic reads at equal speed, profiles/r05/expand/NOTES.md)
  const uint32_t v = __builtin_amdgcn_readfirstlane(
      (gridDim.x & 7u) ? wave
                       : ((blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)) * (kBlock / 64) +
                             (threadIdx.x >> 6));
  for (uint64_t e0 = v; e0 < n; e0 += 64ull * n_waves) {
    const uint64_t el = e0 + static_cast<uint64_t>(lane) * n_waves;
    uint32_t bp = 0, brs = 0, bdeg = 0, bc0 = 0, bW = 0, bnb = 0, bfl = 0, bwl = 0, bwh = 0, bex = 0;
    // per lane, so the staged phases broadcast them instead of recomputing
    // them in scalar registers: the staged row's address, the children's
    // row base, the flag dwords
    uint32_t brl = 0, brh = 0, bcl = 0, bch = 0, bnd = 0, bst = 0;
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
      // the staged words [lo, hi) of the entry's row (lo | hi << 16)
      bex = ext_rows(a, T.W, T.flags) && !(bp == T.nbase && (T.flags & kTopicRootLocal)) ? ext_of(a, bp, T.W)
                                                                                          : ext_whole(T.W);
    }
    const uint32_t nb = static_cast<uint32_t>(__popcll(__ballot(el < n)));
    const bool is_root = bp == bnb && (bfl & kTopicRootLocal);
    const bool staged = el < n && bW > 0 && !(bfl & (kTopicMesh | kEntrySplit)) && bW <= kStageWords && bdeg <= 64;
    if constexpr (!kRecord && !kDirect) {
      if (flat_on(a)) {
        // (before the entry loop's per-lane values are computed: fewer live registers)
        const bool short_row = staged && !is_root && (bex >> 16) - (bex & 0xFFFFu) < kFlatWords;
        const uint64_t wbase = (static_cast<uint64_t>(bwh) << 32) | bwl;
        const uint64_t src = reinterpret_cast<uint64_t>(((bfl & kTopicSingleStart) ? a.seen : a.a_cur) + wbase +
                                                        static_cast<uint64_t>(bp - bnb) * bW + (bex & 0xFFFFu));
        const uint64_t crow = wbase + static_cast<uint64_t>(bc0 - bnb) * bW;
        if (expand_flat(a, ws, short_row, bW, bex, short_row && ext_rows(a, bW, bfl), bdeg, bc0, src, crow,
                        !(bfl & kTopicSingleStart), lane, cur, k, ec))
          bW = 0;  // (the entry loop below skips it)
      }
    }
    if (el < n && bW) {
      // per lane, so the staged phases broadcast them instead of recomputing
      // them in scalar registers: the staged row's address, the children's
      // row base, the flag dwords
      const uint64_t wbase = (static_cast<uint64_t>(bwh) << 32) | bwl;
      const bool from_seen = (bfl & kTopicSingleStart) && !is_root;
      const uint64_t rp = reinterpret_cast<uint64_t>((from_seen ? a.seen : a.a_cur) + wbase +
                                                     static_cast<uint64_t>(bp - bnb) * bW + (bex & 0xFFFFu));
      brl = static_cast<uint32_t>(rp);
      brh = static_cast<uint32_t>(rp >> 32);
      // the children's rows: child c0's row, the others follow at stride W
      const uint64_t cb = wbase + static_cast<uint64_t>(bc0 - bnb) * bW;
      bcl = static_cast<uint32_t>(cb);
      bch = static_cast<uint32_t>(cb >> 32);
      bnd = ((bc0 + bdeg + 3u) >> 2) - (bc0 >> 2);
      // stage needs (staged words, even | flag dwords << 16), or ~0: not staged
      const uint32_t Ls = (bex >> 16) - (bex & 0xFFFFu);
      bst = staged ? (Ls + (Ls & 1u)) | (4u * bnd) << 16 : ~0u;
    }
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
        const uint32_t sn = rl(bst, q + nq);
        if (sn == ~0u) break;
        const uint32_t Ln = sn & 0xFFFFu, bn = sn >> 16;  // staged words (even), flag bytes
        if (sw + Ln > kStageWords || sd + bn > kStageBytes) break;
        sw += Ln;
        sd += bn;
        ++nq;
      }
      // phase A: LDS-DMA of arrival rows and child flag / generation bytes
      {
        uint32_t off = 0, doff = 0;
        for (uint32_t i = q; i < q + nq; ++i) {
          const uint32_t W = rl(bW, i);
          if (W == 0) continue;
          const uint32_t c0 = rl(bc0, i);
          // the row's words [lo, lo + L): its arrival extent (even bounds) or all of it
          const uint32_t xe = rl(bex, i), lo = xe & 0xFFFFu, L = (xe >> 16) - lo;
          const uint32_t* row =
              reinterpret_cast<const uint32_t*>((static_cast<uint64_t>(rl(brh, i)) << 32) | rl(brl, i));
          uint32_t* dst = reinterpret_cast<uint32_t*>(ws.words + off);
          if ((W & 1u) == 0) {
            // even W: the row and its stage slot are 16-B aligned (topic
            // blocks start on 128-B lines, slots keep even offsets): one
            // dwordx4 DMA per lane, 1 KiB per wave instruction
            for (uint32_t d = 0; d < 2 * L; d += 256)
              if (d + 4 * lane < 2 * L) PSAMD_LDS_DMA(row + d + 4 * lane, dst + d, 16);
          } else {
            for (uint32_t d = 0; d < 2 * L; d += 64)
              if (d + lane < 2 * L) PSAMD_LDS_DMA(row + d + lane, dst + d, 4);
          }
          const uint32_t nd = rl(bnd, i);
          if (lane < nd) {
            PSAMD_LDS_DMA(reinterpret_cast<const uint32_t*>(a.node_flags) + (c0 >> 2) + lane,
                          ws.flags + doff, 4);
            PSAMD_LDS_DMA(reinterpret_cast<const uint32_t*>(a.gen) + (c0 >> 2) + lane,
                          ws.gens + doff, 4);
          }
          off += L + (L & 1u);  // keep every staged row 16-B aligned
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
          const uint32_t c0 = rl(bc0, i);
          const uint64_t crow0 = (static_cast<uint64_t>(rl(bch, i)) << 32) | rl(bcl, i);  // child c0's row
          const uint32_t nd = rl(bnd, i);
          const uint32_t fo = doff + (c0 & 3u);  // byte of child 0
          // single-start topics keep no arrival rows (see kTopicSingleStart)
          const bool keep = !(rl(bfl, i) & kTopicSingleStart);
          const uint32_t xe = rl(bex, i), lo = xe & 0xFFFFu, hi = xe >> 16;  // staged words
          ec.ent += 1;
          ec.ent_words += hi - lo;
          ec.kids += deg;
          if (W >= 64) {
            // extent rows: the children's rows change only in [tlo, thi), the
            // staged words' nonzero range (even bounds); their arrival rows
            // are written there alone and it becomes their extent
            const bool ext = ext_rows(a, W, rl(bfl, i));
            uint32_t tlo = lo, thi = hi;
            if (ext) {
              tlo = hi;
              thi = lo;
              for (uint32_t wb = lo; wb < hi; wb += 64) {
                const uint32_t w = wb + lane;
                const uint64_t nz = __ballot(w < hi && ws.words[off + w - lo] != 0);
                if (nz) {
                  tlo = min(tlo, wb + static_cast<uint32_t>(__ffsll(static_cast<long long>(nz))) - 1u);
                  thi = wb + 64u - static_cast<uint32_t>(__clzll(static_cast<long long>(nz)));
                }
              }
              if (tlo >= thi) {
                tlo = thi = lo;
              } else {
                tlo &= ~1u;
                thi = (thi + 1u) & ~1u;
              }
            }
            for (uint32_t jj = 0; jj < deg; ++jj) {
              const uint32_t f = ws.flags[fo + jj];
              if (!(f & kNodeLive)) continue;
              const bool stale = ws.gens[fo + jj] != cur;
              const bool internal = (f & kNodeInternal) != 0;
              const bool store = internal && keep;
              const uint32_t c = c0 + jj;
              const uint64_t row = crow0 + static_cast<uint64_t>(jj) * W;
              bool any = false;
              if (stale) {
                // the whole seen row (zeros outside the staged words); W
                // even, row and stage offset even: two words per lane, 1 KiB
                // per store instruction
                for (uint32_t wb = 0; wb < W; wb += 128) {
                  const uint32_t w = wb + 2 * lane;
                  if (w < W) {
                    const bool in = w >= tlo && w < thi;
                    const uint4 v = in ? *reinterpret_cast<const uint4*>(ws.words + off + w - lo)
                                       : make_uint4(0u, 0u, 0u, 0u);
                    deliver_fresh2<kRecord>(a, store && (in || !ext), row + w, v, round, k);
                    any |= (v.x | v.y | v.z | v.w) != 0;
                  }
                }
              } else {
                for (uint32_t wb = tlo; wb < thi; wb += 64) {
                  const uint32_t w = wb + lane;
                  if (w < thi) {
                    const uint64_t nm = deliver_tree<kRecord>(a, store, row + w, ws.words[off + w - lo], round, k);
                    any |= nm != 0;
                  }
                }
              }
              if (internal && __ballot(any) && lane == 0) {
                mark_next(a, c);
                if (ext) a.ext_next[c] = tlo | thi << 16;
              }
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
              const uint64_t cw = crow0 + static_cast<uint64_t>(jj) * W + w;
              uint64_t nm = 0;
              if (__ballot(live && !stale) == 0) {  // burst: every live child fresh
                if (live) {
                  deliver_fresh<kRecord>(a, keep && (f & kNodeInternal), cw, m, round, k);
                  nm = m;
                }
              } else if (live) {
                if (stale) {
                  deliver_fresh<kRecord>(a, keep && (f & kNodeInternal), cw, m, round, k);
                  nm = m;
                } else {
                  nm = deliver_tree<kRecord>(a, keep && (f & kNodeInternal), cw, m, round, k);
                }
              }
              const uint64_t bal = __ballot(nm != 0);
              if (live && w == 0 && (f & kNodeInternal) && (bal & gmask)) mark_next(a, c);
            }
          }
          // live children hold current rows now
          if (lane < deg && (ws.flags[fo + lane] & kNodeLive))
            a.gen[c0 + lane] = static_cast<uint8_t>(cur);
          if (rl(bp, i) == rl(bnb, i) && (rl(bfl, i) & kTopicRootLocal)) {  // seeded with |=: consume-and-clear
            const uint64_t pw = (static_cast<uint64_t>(rl(bwh, i)) << 32) | rl(bwl, i);  // (the root: node nbase)
            for (uint32_t w = lane; w < W; w += 64) a.a_cur[pw + w] = 0;
            ec.clear += W;
          }
          off += (hi - lo) + ((hi - lo) & 1u);  // (as phase A)
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
// (block q of nq: k_reduce_rounds' own, or the reduce part of k_window_turn)
__device__ __forceinline__ void reduce_rounds_block(const uint64_t* __restrict__ partials,
                                                    const uint32_t* __restrict__ desc,
                                                    uint64_t* __restrict__ round_stats,
                                                    uint64_t* __restrict__ host_stats, const WindowSignal& sig,
                                                    uint32_t q, uint32_t nq) {
  constexpr uint32_t kAct = (kBlock / kNumCtr) * kNumCtr;
  __shared__ uint64_t red[kBlock];
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
    if (round_stats) round_stats[static_cast<uint64_t>(q) * kNumCtr + threadIdx.x] = t;
    if (host_stats) {  // fine-grained pinned host rows: visible to the host once the kernel ends
      __hip_atomic_store(host_stats + static_cast<uint64_t>(q) * kNumCtr + threadIdx.x, t, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      if (!sig.flag) __threadfence_system();  // (a signalled window fences once, below)
    }
  }
  // a signalled window: the last block to finish stamps the end and raises
  // the flag (after every block's rows; the counter re-zeroes itself)
  if (sig.flag) __syncthreads();  // (the block's row stores precede its fence)
  if (sig.flag && threadIdx.x == 0) {
    __threadfence_system();
    if (atomicAdd(sig.ctr, 1u) == nq - 1) {
      sig.flag[2] = __builtin_amdgcn_s_memrealtime();
      __threadfence_system();
      __hip_atomic_store(sig.flag, sig.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      atomicExch(sig.ctr, 0u);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_reduce_rounds(const uint64_t* __restrict__ partials,
                                                          const uint32_t* __restrict__ desc,
                                                          uint64_t* __restrict__ round_stats,
                                                          uint64_t* __restrict__ host_stats,
                                                          WindowSignal sig) {
  reduce_rounds_block(partials, desc, round_stats, host_stats, sig, blockIdx.x, gridDim.x);
}

// The previous window's reduce (blocks 0 .. n_rounds) beside this window's
// init (the blocks after them, as the gx x gy grid of k_window_init).
__global__ __launch_bounds__(kBlock) void k_window_turn(ReduceArgs rd, const TopicDev* __restrict__ topics,
                                                        uint64_t* __restrict__ seen, uint64_t* __restrict__ a0,
                                                        uint64_t* __restrict__ a1, uint8_t* __restrict__ gen,
                                                        uint32_t gen_cur, WindowStart ws, uint32_t gx, uint32_t gy) {
  const uint32_t nq = rd.n_rounds + 1;
  if (blockIdx.x < nq) {
    reduce_rounds_block(rd.partials, rd.desc, rd.round_stats, rd.host_stats, rd.sig, blockIdx.x, nq);
  } else {
    const uint32_t b = blockIdx.x - nq;
    window_init_block(topics, seen, a0, a1, gen, gen_cur, ws, b % gx, b / gx, gx, gy);
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
    if (T.flags & kTopicPacked) {  // group g's virtual word r: its bits b0 + 64 r .. of the packed row
      for (uint32_t g = 0; g < T.group_n; ++g) {
        const GroupDev G = groups[T.group_lo + g];
        for (uint32_t r = 0; r < G.wn; ++r) {
          uint64_t x = 0;
          if (valid && 64 * r < G.n) {
            const uint32_t b = G.b0 + 64 * r, take = min(64u, G.n - 64 * r);
            const uint64_t lo = seen[row + (b >> 6)] >> (b & 63);
            const uint64_t hi = (b & 63) && (b >> 6) + 1 < T.W ? seen[row + (b >> 6) + 1] << (64 - (b & 63)) : 0ull;
            x = (lo | hi) & (take == 64 ? ~0ull : (1ull << take) - 1);
          }
          acc += mix64((key0 | (G.w0 + r)) ^ mix64(x));
        }
      }
      continue;
    }
    for (uint32_t w = 0; w < T.w_msgs; ++w)
      acc += mix64((key0 | w) ^ mix64(valid ? seen[row + w] : 0ull));
  }
  acc = wave_sum_u64(acc);
  if ((threadIdx.x & 63) == 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(out), static_cast<unsigned long long>(acc));
}

}  // namespace

namespace {
__global__ void k_window_done(uint64_t* sig, uint64_t seq) {
  if (threadIdx.x) return;
  sig[2] = __builtin_amdgcn_s_memrealtime();
  __threadfence_system();
  __hip_atomic_store(sig, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

hipError_t launch_window_done(uint64_t* sig, uint64_t seq, hipStream_t s) {
  hipLaunchKernelGGL(k_window_done, dim3(1), dim3(64), 0, s, sig, seq);
  return hipGetLastError();
}

// tree topics need block x = 0 only; the other blocks share the staged
// copies and the partial-slot clear (>= 256 blocks in all)
static uint32_t window_init_gx(uint32_t n_topics, bool any_mesh) {
  return any_mesh ? 64u : std::max<uint32_t>(1, (256 + n_topics - 1) / n_topics);
}

hipError_t launch_window_init(const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur,
                              bool any_mesh, const WindowStart& ws, hipStream_t s) {
  if (n_topics == 0) return hipSuccess;
  const dim3 grid(window_init_gx(n_topics, any_mesh), n_topics);
  hipLaunchKernelGGL(k_window_init, grid, dim3(kBlock), 0, s, topics, seen, a0, a1, gen, gen_cur, ws);
  return hipGetLastError();
}

hipError_t launch_window_turn(const ReduceArgs& rd, const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur, bool any_mesh,
                              const WindowStart& ws, hipStream_t s) {
  if (rd.n_rounds == 0 || n_topics == 0) return hipErrorInvalidValue;  // (the caller launches them apart)
  const uint32_t gx = window_init_gx(n_topics, any_mesh);
  const uint32_t grid = rd.n_rounds + 1 + gx * n_topics;
  hipLaunchKernelGGL(k_window_turn, dim3(grid), dim3(kBlock), 0, s, rd, topics, seen, a0, a1, gen, gen_cur, ws, gx,
                     n_topics);
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

// One lane: the flag store.  The launches before it on the stream ended with
// their release (rows and records written back past the XCDs' L2s); the
// store itself is a vector atomic at system scope.
__global__ void k_flag_set(uint64_t* flag, uint64_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lane q polls rank q's flag; the wave leaves when every lane is satisfied or
// the clock runs out (every wave reaches the exit: a dead peer cannot hang
// the GPU, it fails the window through *err).
__global__ void k_flag_wait(FlagWait w, uint32_t* err, uint64_t timeout_ticks) {
  const uint32_t q = threadIdx.x;
  const uint64_t* f = q < static_cast<uint32_t>(kMaxRanks) ? w.flag[q] : nullptr;
  const uint64_t want = f ? w.value[q] : 0;
  bool done = f == nullptr;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    if (!done) done = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >= want;
    if (__all(done)) break;
    const uint64_t waited = wall_clock64() - t0;
    // past 1 ms, an earlier wait that timed out ends this one too (the
    // window fails once, instead of one timeout per round)
    if (waited > timeout_ticks ||
        (waited > 100000u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)) {
      if (!done) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

hipError_t launch_flag_set(uint64_t* flag, uint64_t value, hipStream_t s) {
  hipLaunchKernelGGL(k_flag_set, dim3(1), dim3(64), 0, s, flag, value);
  return hipGetLastError();
}

hipError_t launch_flag_wait(const FlagWait& w, uint32_t* err, uint64_t timeout_ticks, hipStream_t s) {
  hipLaunchKernelGGL(k_flag_wait, dim3(1), dim3(64), 0, s, w, err, timeout_ticks);
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

__global__ __launch_bounds__(kBlock) void k_level_reach(const ReachPiece* __restrict__ pieces,
                                                        const uint8_t* __restrict__ gen, uint32_t gen_cur,
                                                        const uint8_t* __restrict__ node_flags,
                                                        const TopicDev* __restrict__ topics,
                                                        const uint64_t* __restrict__ seen, uint32_t eager,
                                                        unsigned long long* __restrict__ out) {
  __shared__ uint32_t red[2][kBlock / 64];
  const ReachPiece P = pieces[blockIdx.x];
  const TopicDev T = topics[P.topic];
  const uint32_t cur = gen_cur & 0xFF;
  uint32_t r = 0, f = 0;
  if (eager) {
    for (uint32_t u = P.lo + threadIdx.x; u < P.hi; u += kBlock) {
      const bool reached = u == T.nbase || seen[T.wbase + static_cast<uint64_t>(u - T.nbase) * T.W] != 0;
      const bool internal = (node_flags[u] & kNodeInternal) != 0;
      r += reached ? 1u : 0u;
      f += (internal && reached) ? 1u : 0u;
    }
  } else {
    // 16 nodes per lane and load: the generation and flag bytes as dwordx4
    // (16-B aligned units over the piece, bytes outside it masked off; both
    // arrays are padded past n_pad)
    const uint32_t b0 = P.lo & ~15u;
    for (uint32_t b = b0 + 16 * threadIdx.x; b < P.hi; b += 16 * kBlock) {
      const uint4 g = *reinterpret_cast<const uint4*>(gen + b);
      const uint4 fl = *reinterpret_cast<const uint4*>(node_flags + b);
      const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, fw[4] = {fl.x, fl.y, fl.z, fl.w};
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t u = b + k;
        const bool in = u >= P.lo && u < P.hi;
        const bool reached = in && (u == T.nbase || ((gw[k >> 2] >> (8 * (k & 3))) & 0xFFu) == cur);
        const bool internal = ((fw[k >> 2] >> (8 * (k & 3))) & kNodeInternal) != 0;
        r += reached ? 1u : 0u;
        f += (internal && reached) ? 1u : 0u;
      }
    }
  }
  r = __reduce_add_sync(~0ull, r);
  f = __reduce_add_sync(~0ull, f);
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = r;
    red[1][wid] = f;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kBlock / 64; ++w) t += red[threadIdx.x][w];
    if (t) atomicAdd(out + 2 * P.seg + threadIdx.x, static_cast<unsigned long long>(t));
  }
}

hipError_t launch_level_reach(const ReachPiece* pieces, uint32_t n, const uint8_t* gen, uint32_t gen_cur,
                              const uint8_t* node_flags, const TopicDev* topics, const uint64_t* seen, bool eager,
                              uint64_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_level_reach, dim3(n), dim3(kBlock), 0, s, pieces, gen, gen_cur, node_flags, topics, seen,
                     eager ? 1u : 0u, reinterpret_cast<unsigned long long*>(out));
  return hipGetLastError();
}

hipError_t launch_reduce_rounds(const uint64_t* partials, const uint32_t* desc, uint32_t n_rounds,
                                uint64_t* round_stats, uint64_t* host_stats, const WindowSignal& sig, hipStream_t s) {
  if (n_rounds == 0) return sig.flag ? launch_window_done(sig.flag, sig.seq, s) : hipSuccess;
  hipLaunchKernelGGL(k_reduce_rounds, dim3(n_rounds + 1), dim3(kBlock), 0, s, partials, desc, round_stats,
                     host_stats, sig);
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
