// engine.cpp -- host runtime and C ABI of the MI355X subtree-dissemination
// engine (include/psengine.h).  Owns all device memory, builds the fused CSR
// node space from the per-topic trees, plans propagation windows and drives
// the synchronous rounds of kernels.hip on one HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "dist.hpp"
#include "gbuild.hpp"
#include "kernels.hpp"
#include "psengine.h"
#include "tree.hpp"

using namespace psamd;

namespace {

constexpr uint32_t kMaxRoundsCap = 4096;  // round buffers' minimum size (deeper windows grow them)
constexpr uint32_t kMaxStartRound = 200;
constexpr uint32_t kDefaultWindow = 65536;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // Grow-only allocation; returns true when a fresh allocation was made.
  hipError_t ensure(size_t n, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    if (n == 0) n = 16;
    if (n <= bytes) return hipSuccess;
    release();
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    bytes = n;
    if (fresh) *fresh = true;
    return hipSuccess;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

enum class Kind { None, Join, Parent, Children };

struct TopicHost {
  bool exists = false;
  Kind kind = Kind::None;
  uint32_t root = 0, width = 2, max_width = 5;
  SubscriptionTree tree;
  std::vector<uint32_t> parent;  // Kind::Parent
  std::vector<uint32_t> rp, cl;  // Kind::Children
  // node space (set by build_graph)
  uint32_t nbase = 0, n_nodes = 0, depth = 0;
  bool mesh = false;
  bool root_local = true;                // this rank owns the root
  uint32_t max_deg = 0;
  std::vector<uint32_t> level_internal;  // BFS level -> owned nodes with children
  std::vector<uint32_t> level_off;       // single rank: BFS level -> first node (topic-relative)
  // GPU rebuild: the upstream of every peer as last shipped to the device
  std::vector<uint32_t> par_mirror;
  bool par_dev_valid = false;  // the device parent array holds par_mirror
  bool par_full_dirty = true;  // Kind::Parent: re-diff the whole array
  // cross-rank edges by the parent's BFS level: (level, from rank, to rank, count)
  struct Cross {
    uint32_t level, from, to, count;
  };
  std::vector<Cross> cross;
  // multi-GPU level mode: ghost parents.  gcnt[(d * world + a)
  // * world + b] = parents at level d - 1 owned by rank a with a child at
  // level d owned by rank b (a != b); each such row crosses once per round.
  // This rank's parents to ship: send_node[i] (local node), send_dst[i]
  // (dest rank << 27 | index among the a -> b ghosts of the level), grouped
  // by level: send_lvl[d] .. send_lvl[d + 1].
  std::vector<uint32_t> gcnt, send_node, send_dst, send_lvl;
};

struct RunMsg {
  uint32_t topic;
  uint32_t start;
};

// Messages of one topic in one window: a slice of the run's topic-sorted
// message index array (bit li of the topic block = message idx[li]).
struct WinSlice {
  const uint32_t* idx = nullptr;
  uint32_t n = 0;
};

// One start round of a topic's window and its word block [w0, w0 + wn) of
// every row: a tree node at level d receives the block in round start + d.
// A topic whose window messages share one start round has one group, the
// whole row.
struct StartGroup {
  uint32_t start, w0, wn;
};

// Word offset of virtual word w of row u (relative to the topic's first
// node): node-major rows, or a kTopicGroups topic's group-major blocks.
uint64_t phys_word(const TopicDev& d, const std::vector<StartGroup>& G, uint64_t u, uint32_t w) {
  if (!(d.flags & kTopicGroups)) return d.wbase + u * d.W + w;
  for (const StartGroup& g : G)
    if (w < g.w0 + g.wn) return d.wbase + static_cast<uint64_t>(d.n_nodes) * g.w0 + u * g.wn + (w - g.w0);
  return d.wbase;  // (w < W always)
}

uint32_t ceil_div(uint64_t a, uint64_t b) { return static_cast<uint32_t>((a + b - 1) / b); }

}  // namespace

struct ps_engine {
  ps_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev_run0 = nullptr, ev_run1 = nullptr;
  std::vector<hipEvent_t> ev_k;  // pairs around expand launches
  uint32_t n_cus = 256, expand_grid = 2048;
  std::vector<uint64_t> pull_bytes;    // row bytes written per round (pull chunks)
  bool host_timing = false;      // PSAMD_HOST_TIMING=1: host phase times to stderr
  uint32_t small_place = 512;    // top levels up to this many nodes placed by one block
  // GPU rebuild of the node space: on by default for one
  // rank and tree topics (PSAMD_GPU_BUILD=0: host build)
  bool gpu_build_on = true;
  bool gpu_graph = false;     // the current node space was built on the GPU
  bool mirrors_valid = true;  // host copies of node_peer / flags / CSR are current
  std::vector<uint32_t> pairs_host, gstat_host, lvl_host, roots_host;
  std::vector<size_t> pair_off;
  DevBuf d_tpar, d_anc0, d_anc1, d_dep0, d_dep1, d_keys0, d_skeys, d_local, d_deg, d_first, d_lvl,
      d_gstat, d_cub, d_pairs, d_live, d_roots, d_cnt, d_fidx, d_childoff;
  std::chrono::steady_clock::time_point t_run0;
  // k_flood: a single-rank level window in one persistent
  // launch; PSAMD_FLOOD=0 runs one k_pull launch per round instead
  bool flood_on = true;
  bool flood_broken = false;  // a dependency wait timed out once: per-level launches from then on
  uint32_t flood_grid = 0;    // resident blocks (0: k_flood unavailable)
  uint32_t flood_words = kFloodWords;  // row words per task (PSAMD_FLOOD_WORDS)
  uint32_t pull_words = kPullWords;    // row words per k_pull chunk (512..4096 measured: 1024 best)
  uint64_t flood_top_bytes = 16ull << 20;  // k_flood runs the leading rounds writing at most this many row bytes
  uint32_t flood_epoch = 0;   // granule tag of the last launch (granules are never reset)
  uint32_t flood_spin_ticks = 200000000u;  // dependency-wait bound: 2 s of s_memrealtime (100 MHz); PSAMD_FLOOD_SPIN_TICKS
  std::vector<uint64_t> flood_key;
  std::vector<FloodTask> flood_tasks;
  std::vector<FloodSeg> flood_segs;
  std::vector<uint32_t> flood_slot0, flood_nslot;  // per round: partial counter slots
  uint32_t flood_slots = 1;   // slots of a window (slot 0: the timeout word)
  DevBuf d_flood_tasks, d_flood_segs, d_flood_gran;
  bool flood_profile = false;  // PSAMD_FLOOD_PROFILE=1: per-wave phase times of k_flood to stderr (sync runs)
  DevBuf d_flood_prof;
  uint32_t flood_prof_waves = 0;

  std::vector<TopicHost> topics;
  std::vector<uint8_t> live;
  bool graph_dirty = true, flags_dirty = true;
  uint64_t graph_epoch = 0, flags_epoch = 0;  // bumped by every upload

  // level mode, per-round counter slots and their reduce descriptors
  std::vector<uint32_t> woff_host, desc_host;
  DevBuf d_woff;
  // level mode, pull direction: per-round chunks of next-level nodes
  std::vector<uint64_t> pull_key;
  std::vector<PullChunk> pull_host;
  std::vector<uint32_t> pull_off;
  DevBuf d_pull;
  // k_pull_pair: rounds q and q + 1 in one launch, one rank
  // (PSAMD_PULL_PAIR=0: one k_pull launch per round)
  bool pair_on = true;
  std::vector<uint64_t> pp_key;
  std::vector<PullChunk> pp_host;
  std::vector<uint32_t> pp_lo, pp_hi;  // round q: chunks of the pair launch starting at q
  std::vector<uint8_t> pp_kind;        // per round of the cached plan: PS_K_*
  std::vector<uint8_t> round_kind;     // per round of the current window: PS_K_* (empty: k_expand)
  DevBuf d_pp;

  // fused node space (host mirror)
  uint32_t n_nodes = 0, n_pad = 16;
  std::vector<uint32_t> node_peer, row_ptr, col;
  std::vector<uint32_t> node_parent;  // node-space parent on this rank (kNone: root / remote)
  std::vector<uint16_t> node_topic;
  std::vector<uint8_t> node_flags;

  DevBuf d_row_ptr, d_col, d_node_topic, d_node_flags, d_node_peer, d_node_parent;
  DevBuf d_seen, d_arr0, d_arr1, d_hop, d_flags, d_blk, d_gen, d_frontier, d_nfront, d_wgcount,
      d_partials, d_stats, d_topics, d_seeds, d_digest, d_groups;
  uint32_t gen_cur = 0;  // window generation stamped into d_gen (1..255)
  DevBuf d_remote_fed, d_send, d_recv, d_apply_stats;
  // multi-GPU level mode: ghost parents
  std::vector<uint32_t> ghost_ref;  // per node: remote parent's rank << 27 | ghost index, or kNone
  std::vector<uint64_t> ghost_key;  // (graph, start rounds, row widths) the plan below was built for
  struct GhostRound {
    std::vector<uint64_t> s_off, s_len, r_off, r_len;  // transport regions, bytes
    uint32_t pack0 = 0, pack1 = 0;                     // pack entries of the round
    uint32_t seg0 = 0, seg1 = 0;                       // their (topic) segments
    bool any = false;                                  // some rank ships rows this round
  };
  std::vector<GhostRound> ghost_rounds;
  std::vector<PackEntry> pack_host;
  std::vector<PackSeg> pack_seg_host;
  std::vector<uint64_t> ghost_off_host;  // per node: flag byte << 40 | row word, in the recv buffer
  DevBuf d_pack, d_pack_seg, d_ghost_off;
  uint64_t ghost_send_max = 0, ghost_recv_max = 0;
  uint32_t n_remote_fed = 0;
  std::vector<uint32_t> remote_fed;  // owned nodes whose parent is on another rank

  // multi-GPU: this engine owns a hash-partitioned share of every topic
  int32_t rank = 0, world = 1;
  uint32_t partition = PS_PART_PEER, split_depth = 0;
  std::unique_ptr<Transport> transport;

  // publishes not yet run
  std::vector<RunMsg> pending;
  bool pending_nonzero_start = false;  // some pending message starts after round 0
  bool run_zero_start = true;          // every message of the current run starts in round 0
  uint32_t next_msg = 0;

  // results of the last run
  uint32_t last_first = 0, last_n = 0;
  bool have_hops = false;
  std::vector<uint8_t> hops;  // [msg][peer]
  std::vector<RunMsg> last_msgs;        // messages of the last run, publish order
  std::vector<uint32_t> run_sorted;     // run message indices grouped by topic
  std::vector<uint32_t> run_topic_off;  // topic -> first position in run_sorted
  std::vector<uint32_t> run_rank;       // message -> position within its topic
  std::vector<uint32_t> last_lo, last_cnt;  // topic -> last window's rank range
  // topic -> the last window's row bit of each window message (empty: bit li
  // = the message's window slot; else the start-group layout, StartGroup)
  std::vector<std::vector<uint32_t>> last_pos;
  std::vector<std::vector<StartGroup>> last_groups;  // topic -> the last window's start groups
  std::vector<TopicDev> last_topics;
  bool have_window = false;
  std::map<uint32_t, std::vector<uint32_t>> peer_node;  // topic -> peer -> node (ps_read_peer_messages)
  std::vector<uint64_t> peer_node_epoch;                 // graph_epoch each map was built for

  // asynchronous runs (ps_run_async / ps_wait): the last window of a run may
  // leave its stats on the stream (pinned readback) so that the host plans
  // the next run while this one's kernels execute
  struct Inflight {
    ps_stats st{};
    bool deferred = false;
    uint32_t r = 0, launches = 0;
    uint32_t mode = PS_MODE_COMPACT, flood_rounds = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the window's kernels
    uint64_t* hs = nullptr;  // pinned: (PS_MAX_ROUNDS + 1) x kNumCtr counters
    uint64_t* hs_dev = nullptr;  // hs, device-mapped (k_reduce_rounds writes it)
    uint64_t* ha = nullptr;  // pinned: apply counters of a multi-GPU window
    uint32_t planned0 = 0;
    int32_t world = 1;
    std::vector<uint8_t> kinds;  // round_kind of the window
  };
  Inflight infl[2];
  uint32_t infl_head = 0, infl_count = 0;

  // per-window uploads (topic table, seeds, reduce descriptors) go through
  // pinned staging: a copy from pageable memory blocks the host until the
  // stream has drained, so the next batch's launches would only be issued
  // once the previous batch had finished (a ~35 us bubble per pipelined
  // step).  Two slots alternate; a slot is rewritten only after the copies
  // of its previous use have completed: slot i belongs to asynchronous run
  // slot i (synchronous runs use slot 0 with nothing in flight).
  struct Staging {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;  // the slot's device-mapped address
    size_t cap = 0;
  };
  Staging stg[2];
  bool defer_phase = false;  // the current phase may defer its last window's stats
  bool defer_last = false;   // ... and this window is that last window
  Inflight* defer_into = nullptr;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return PS_E_DEVICE;
  }
};

#define HIP_TRY(expr, what)                     \
  do {                                          \
    hipError_t _e = (expr);                     \
    if (_e != hipSuccess) return e->hip_fail(_e, what); \
  } while (0)

namespace {

bool topic_ok(ps_engine* e, uint32_t topic) {
  return topic < e->topics.size() && e->topics[topic].exists;
}

// Child lists of one topic in peer space, insertion order.
void peer_children(const ps_engine* e, const TopicHost& T, std::vector<uint32_t>& rp,
                   std::vector<uint32_t>& cl) {
  const uint32_t n = e->cfg.n_peers;
  if (T.kind == Kind::Children) {
    rp = T.rp;
    cl = T.cl;
    return;
  }
  rp.assign(n + 1, 0);
  if (T.kind == Kind::Parent) {
    for (uint32_t c = 0; c < n; ++c)
      if (T.parent[c] != kNone && c != T.root) rp[T.parent[c] + 1]++;
    for (uint32_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
    cl.assign(rp[n], 0);
    std::vector<uint32_t> fill(rp.begin(), rp.end() - 1);
    for (uint32_t c = 0; c < n; ++c)
      if (T.parent[c] != kNone && c != T.root) cl[fill[T.parent[c]]++] = c;
    return;
  }
  // Kind::Join: attached children (subscribed and not failed) in map order
  for (uint32_t p = 0; p < n; ++p) {
    uint32_t k = 0;
    for (const auto& r : T.tree.children(p))
      if (T.tree.state(r.id) == PeerState::In) ++k;
    rp[p + 1] = k;
  }
  for (uint32_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
  cl.assign(rp[n], 0);
  for (uint32_t p = 0; p < n; ++p) {
    uint32_t o = rp[p];
    for (const auto& r : T.tree.children(p))
      if (T.tree.state(r.id) == PeerState::In) cl[o++] = r.id;
  }
}

// Ownership of one topic's nodes (positions in its BFS order) among `world`
// ranks.  PS_PART_PEER: owner = splitmix64(peer) mod world.
// PS_PART_SUBTREE: nodes at BFS level >= L belong to the owner of their
// ancestor at level L; the level-L subtrees are dealt largest first to the
// least-loaded rank; the few nodes above L hash by peer.  L = split_depth, or
// (0) the first level holding >= 64*world nodes, so only edges out of levels
// < L cross ranks.
void partition_topic(const std::vector<uint32_t>& order, const std::vector<uint32_t>& bfs_parent,
                     const std::vector<uint32_t>& level, uint32_t topic, int32_t world,
                     uint32_t part, uint32_t split_depth, std::vector<int32_t>& owner) {
  const size_t n = order.size();
  owner.assign(n, 0);
  if (world <= 1) return;
  auto mix = [](uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  uint32_t L = split_depth;
  if (part == PS_PART_SUBTREE && L == 0) {
    std::vector<uint64_t> cnt;
    for (size_t u = 0; u < n; ++u) {
      if (level[u] >= cnt.size()) cnt.resize(level[u] + 1, 0);
      cnt[level[u]]++;
    }
    L = static_cast<uint32_t>(cnt.size() ? cnt.size() - 1 : 0);
    for (uint32_t d = 0; d < cnt.size(); ++d)
      if (cnt[d] >= 64ull * world) {
        L = d;
        break;
      }
  }
  std::vector<uint32_t> anc(n, kNone);
  const bool subtree = part == PS_PART_SUBTREE && L > 0;
  // subtree mode: the level-L subtrees go to ranks largest first, each to the
  // least-loaded rank (LPT), so every rank holds the same share of this
  // topic's nodes whatever the topic's message weight (hashing the subtree
  // roots left 14 % imbalance at 8 ranks on cfg3)
  std::vector<uint64_t> size(subtree ? n : 0, 0);
  // subtree mode: the levels above L (< 64 * world nodes each) stay whole
  // with the root's owner, so edges cross ranks only from level L - 1 into
  // the level-L subtrees: one exchange round per topic
  const int32_t top_owner = n ? static_cast<int32_t>(mix(order[0]) % static_cast<uint64_t>(world)) : 0;
  uint64_t n_top = 0;
  for (size_t u = 0; u < n; ++u) {
    if (subtree && level[u] >= L) {
      anc[u] = level[u] == L ? static_cast<uint32_t>(u) : anc[bfs_parent[u]];
      size[anc[u]]++;
    } else if (subtree) {
      owner[u] = top_owner;
      ++n_top;
    } else {
      owner[u] = static_cast<int32_t>(mix(order[u]) % static_cast<uint64_t>(world));
    }
  }
  if (!subtree) return;
  std::vector<uint32_t> roots;
  for (size_t u = 0; u < n; ++u)
    if (level[u] == L) roots.push_back(static_cast<uint32_t>(u));
  std::sort(roots.begin(), roots.end(), [&](uint32_t a, uint32_t b) {
    return size[a] != size[b] ? size[a] > size[b] : order[a] < order[b];
  });
  std::vector<uint64_t> load(world, 0);
  load[top_owner] = n_top;  // the dealing evens out the top levels too
  for (uint32_t u : roots) {
    int32_t best = 0;
    for (int32_t q = 1; q < world; ++q)
      if (load[q] < load[best]) best = q;
    owner[u] = best;
    load[best] += size[u];
  }
  (void)topic;
  for (size_t u = 0; u < n; ++u)
    if (level[u] > L) owner[u] = owner[anc[u]];
}

// Builds this rank's node space: per topic, the owned nodes among those
// reachable from the root, in global BFS order (siblings contiguous, the root
// first when owned), CSR over node ids; a child owned by another rank is
// encoded kRemoteBit | rank << 27 | its id at that rank.
int build_graph(ps_engine* e) {
  const uint32_t n = e->cfg.n_peers;
  const int32_t world = e->world, me = e->rank;
  e->node_peer.clear();
  e->node_parent.clear();
  e->node_topic.clear();
  e->row_ptr.assign(1, 0);
  e->col.clear();
  e->remote_fed.clear();
  e->ghost_ref.clear();
  std::vector<uint32_t> ghost_of;  // per global BFS position: owner << 27 | ghost index, or kNone
  std::vector<uint32_t> local(n, kNone);  // peer -> BFS position
  std::vector<uint32_t> rp, cl, order, indeg, bfs_parent, level, loc;
  std::vector<int32_t> owner;
  // node-space base of every topic at every rank (multi-GPU: a remote child
  // is addressed by its fused node id at its owner)
  const uint32_t ntop = static_cast<uint32_t>(e->topics.size());
  std::vector<uint64_t> base_at(static_cast<size_t>(ntop) * std::max(world, 1), 0);
  auto topic_bfs = [&](TopicHost& T, uint32_t t) -> int {
    peer_children(e, T, rp, cl);
    order.assign(1, T.root);
    bfs_parent.assign(1, kNone);
    level.assign(1, 0);
    local[T.root] = 0;
    for (size_t qi = 0; qi < order.size(); ++qi) {
      const uint32_t p = order[qi];
      for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
        const uint32_t c = cl[k];
        if (c >= n) return e->fail(PS_E_INVAL, "child id out of range");
        if (local[c] == kNone) {
          local[c] = static_cast<uint32_t>(order.size());
          order.push_back(c);
          bfs_parent.push_back(static_cast<uint32_t>(qi));
          level.push_back(level[qi] + 1);
        }
      }
    }
    partition_topic(order, bfs_parent, level, t, world, e->partition, e->split_depth, owner);
    return PS_OK;
  };
  if (world > 1) {
    std::vector<uint64_t> run(world, 0);
    for (uint32_t t = 0; t < ntop; ++t) {
      for (int32_t q = 0; q < world; ++q) base_at[static_cast<size_t>(t) * world + q] = run[q];
      TopicHost& T = e->topics[t];
      if (!T.exists) continue;
      int rc = topic_bfs(T, t);
      if (rc) return rc;
      for (size_t u = 0; u < order.size(); ++u) run[owner[u]]++;
      for (uint32_t p : order) local[p] = kNone;
    }
  }
  uint64_t n_total = 0;
  for (uint32_t t = 0; t < e->topics.size(); ++t) {
    TopicHost& T = e->topics[t];
    T.nbase = static_cast<uint32_t>(n_total);
    T.n_nodes = 0;
    T.depth = 0;
    T.mesh = false;
    T.root_local = true;
    T.max_deg = 0;
    T.cross.clear();
    T.level_internal.clear();
    if (!T.exists) continue;
    {
      int rc = topic_bfs(T, t);
      if (rc) return rc;
    }
    for (uint32_t p : order) T.max_deg = std::max(T.max_deg, rp[p + 1] - rp[p]);
    const uint32_t N = static_cast<uint32_t>(order.size());
    T.depth = level.back();
    indeg.assign(N, 0);
    for (uint32_t u = 0; u < N; ++u)
      for (uint32_t k = rp[order[u]]; k < rp[order[u] + 1]; ++k) indeg[local[cl[k]]]++;
    for (uint32_t u = 0; u < N; ++u)
      if (indeg[u] > (u == 0 ? 0u : 1u)) T.mesh = true;
    if (T.mesh && world > 1) return e->fail(PS_E_STATE, "multi-GPU engines support tree topics only");
    // local ids at every rank: rank of each position among its owner's nodes
    loc.assign(N, 0);
    {
      std::vector<uint32_t> next(std::max(world, 1), 0);
      for (uint32_t u = 0; u < N; ++u) loc[u] = next[owner[u]]++;
    }
    T.root_local = owner[0] == me;
    // ghost parents: per parent in BFS order, one row per remote rank that
    // owns one of its children (children are consecutive BFS positions)
    T.gcnt.assign(world > 1 ? static_cast<size_t>(T.depth + 2) * world * world : 0, 0);
    T.send_node.clear();
    T.send_dst.clear();
    T.send_lvl.assign(T.depth + 3, 0);
    if (world > 1) {
      ghost_of.assign(N, kNone);
      for (uint32_t u = 0; u < N; ++u) {
        const uint32_t p = order[u];
        uint32_t mask = 0;
        for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
          const uint32_t v = local[cl[k]];
          if (owner[v] != owner[u]) mask |= 1u << owner[v];
        }
        const uint32_t d = level[u] + 1;
        for (int32_t b = 0; mask; ++b, mask >>= 1) {
          if (!(mask & 1u)) continue;
          const uint32_t gk = T.gcnt[(static_cast<size_t>(d) * world + owner[u]) * world + b]++;
          if (gk > kRemoteIdMask) return e->fail(PS_E_NOMEM, "ghost rows of one level exceed 2^27");
          if (owner[u] == me) {
            T.send_node.push_back(T.nbase + loc[u]);
            T.send_dst.push_back(static_cast<uint32_t>(b) << kRemoteRankShift | gk);
            T.send_lvl[d + 1] = static_cast<uint32_t>(T.send_node.size());
          }
          if (b == me)
            for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
              const uint32_t v = local[cl[k]];
              if (owner[v] == me) ghost_of[v] = static_cast<uint32_t>(owner[u]) << kRemoteRankShift | gk;
            }
        }
      }
      for (uint32_t d = 1; d < T.send_lvl.size(); ++d) T.send_lvl[d] = std::max(T.send_lvl[d], T.send_lvl[d - 1]);
    }
    T.level_internal.assign(T.depth + 1, 0);
    // owned nodes are numbered in BFS order: each level is a contiguous range
    T.level_off.assign(T.depth + 2, 0);
    for (uint32_t u = 0; u < N; ++u)
      if (owner[u] == me) T.level_off[level[u] + 1]++;
    for (uint32_t d = 0; d <= T.depth; ++d) T.level_off[d + 1] += T.level_off[d];
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> cross;
    uint32_t n_own = 0;
    for (uint32_t u = 0; u < N; ++u) {
      const uint32_t p = order[u];
      const uint32_t deg = rp[p + 1] - rp[p];
      for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
        const uint32_t v = local[cl[k]];
        if (owner[v] != owner[u]) cross[{level[u], static_cast<uint32_t>(owner[u]), static_cast<uint32_t>(owner[v])}]++;
      }
      if (owner[u] != me) continue;
      ++n_own;
      e->node_peer.push_back(p);
      if (world > 1) e->ghost_ref.push_back(u ? ghost_of[u] : kNone);
      e->node_parent.push_back(u && owner[bfs_parent[u]] == me ? T.nbase + loc[bfs_parent[u]] : kNone);
      e->node_topic.push_back(static_cast<uint16_t>(t));
      for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
        const uint32_t v = local[cl[k]];
        if (owner[v] == me) {
          e->col.push_back(T.nbase + loc[v]);
        } else {
          const uint64_t id = base_at[static_cast<size_t>(t) * world + owner[v]] + loc[v];
          if (id > kRemoteIdMask) return e->fail(PS_E_NOMEM, "rank node space exceeds 2^27");
          e->col.push_back(kRemoteBit | (static_cast<uint32_t>(owner[v]) << kRemoteRankShift) |
                           static_cast<uint32_t>(id));
        }
      }
      e->row_ptr.push_back(static_cast<uint32_t>(e->col.size()));
      if (deg) T.level_internal[level[u]]++;
      if (u && owner[bfs_parent[u]] != me) e->remote_fed.push_back(T.nbase + loc[u]);
      if (e->col.size() >= 0xFFFFFFF0ull) return e->fail(PS_E_NOMEM, "edge space exceeds 2^32");
    }
    for (const auto& kv : cross)
      T.cross.push_back({std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), kv.second});
    T.n_nodes = n_own;
    for (uint32_t p : order) local[p] = kNone;
    n_total += n_own;
    if (n_total >= 0xFFFFFFF0ull) return e->fail(PS_E_NOMEM, "node space exceeds 2^32 nodes");
  }
  e->n_nodes = static_cast<uint32_t>(n_total);
  e->n_pad = ((e->n_nodes + 15) / 16) * 16;
  if (e->n_pad == 0) e->n_pad = 16;
  return PS_OK;
}

void build_flags(ps_engine* e) {
  e->node_flags.assign(e->n_nodes, 0);
  for (uint32_t u = 0; u < e->n_nodes; ++u) {
    const uint32_t p = e->node_peer[u];
    uint8_t f = e->live[p] ? kNodeLive : 0;
    if (e->row_ptr[u + 1] > e->row_ptr[u]) f |= kNodeInternal;
    for (uint32_t k = e->row_ptr[u]; k < e->row_ptr[u + 1]; ++k)
      if (e->col[k] & kRemoteBit) {
        f |= kNodeSplit;
        break;
      }
    e->node_flags[u] = f;
  }
  for (const auto& T : e->topics)
    if (T.exists && T.n_nodes && T.root_local) e->node_flags[T.nbase] |= kNodeLive;  // roots forward
}

// Host copies of the node space when it was built on the GPU (record-mode
// readback, ps_read_delivered, the push kernel's level schedule).
int ensure_mirrors(ps_engine* e) {
  if (e->mirrors_valid) return PS_OK;
  const size_t nn = e->n_nodes;
  e->node_peer.resize(nn);
  e->node_parent.resize(nn);
  e->node_topic.resize(nn);
  e->node_flags.resize(nn);
  e->row_ptr.resize(nn + 1);
  hipStream_t s = e->stream;
  HIP_TRY(hipMemcpyAsync(e->row_ptr.data(), e->d_row_ptr.p, (nn + 1) * 4, hipMemcpyDeviceToHost, s), "read row_ptr");
  HIP_TRY(hipStreamSynchronize(s), "sync");
  e->col.resize(e->row_ptr[nn]);
  if (nn) {
    HIP_TRY(hipMemcpyAsync(e->node_peer.data(), e->d_node_peer.p, nn * 4, hipMemcpyDeviceToHost, s), "read node_peer");
    HIP_TRY(hipMemcpyAsync(e->node_parent.data(), e->d_node_parent.p, nn * 4, hipMemcpyDeviceToHost, s),
            "read node_parent");
    HIP_TRY(hipMemcpyAsync(e->node_topic.data(), e->d_node_topic.p, nn * 2, hipMemcpyDeviceToHost, s), "read node_topic");
    HIP_TRY(hipMemcpyAsync(e->node_flags.data(), e->d_node_flags.p, nn, hipMemcpyDeviceToHost, s), "read node_flags");
  }
  if (!e->col.empty())
    HIP_TRY(hipMemcpyAsync(e->col.data(), e->d_col.p, e->col.size() * 4, hipMemcpyDeviceToHost, s), "read col");
  HIP_TRY(hipStreamSynchronize(s), "sync");
  e->mirrors_valid = true;
  return PS_OK;
}

bool can_gpu_build(const ps_engine* e) {
  if (!e->gpu_build_on || e->world != 1 || e->cfg.n_peers >= (1u << kBuildPeerBits)) return false;
  bool any = false;
  for (const auto& T : e->topics) {
    if (!T.exists) continue;
    if (T.kind != Kind::Join && T.kind != Kind::Parent) return false;
    any = true;
  }
  return any;
}

// GPU rebuild of the node space (gbuild.hip): ship the
// changed upstream entries, then per topic depth (pointer jumping) -> sort
// of (depth, parent, peer) -> node ids, parents, fan-out; one scan for the
// CSR, flags from the live mask.  Two small readbacks: reachable counts and
// depths (to lay out the topics), then the level tables.  *fallback: a tree
// deeper than the sort key allows -- the caller builds on the host.
int gpu_build_graph(ps_engine* e, bool* fallback) {
  *fallback = false;
  const auto tb0 = std::chrono::steady_clock::now();
  const uint32_t n = e->cfg.n_peers;
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  hipStream_t s = e->stream;
  HIP_TRY(e->d_tpar.ensure(static_cast<size_t>(nt) * n * 4), "alloc parents");
  // 1. parent deltas of every topic, one upload
  auto& pairs = e->pairs_host;
  pairs.clear();
  e->pair_off.assign(nt + 1, 0);
  std::vector<uint32_t> cand;
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    e->pair_off[t] = pairs.size() / 2;
    if (!T.exists) continue;
    uint32_t* par_t = e->d_tpar.as<uint32_t>() + static_cast<size_t>(t) * n;
    bool full = false;
    if (!T.par_dev_valid) {
      HIP_TRY(hipMemsetAsync(par_t, 0xFF, static_cast<size_t>(n) * 4, s), "clear parents");
      T.par_mirror.assign(n, kNone);
      T.par_dev_valid = true;
      full = true;
    }
    auto diff = [&](uint32_t p, uint32_t v) {
      if (T.par_mirror[p] != v) {
        T.par_mirror[p] = v;
        pairs.push_back(p);
        pairs.push_back(v);
      }
    };
    if (T.kind == Kind::Join) {
      T.tree.take_touched(cand);
      if (full)
        for (uint32_t p = 0; p < n; ++p) diff(p, T.tree.in_parent(p));
      else
        for (size_t i = 0; i < cand.size(); ++i) {
          if (i + 16 < cand.size()) {  // touched peers are scattered: fetch ahead
            T.tree.prefetch_peer(cand[i + 16]);
            __builtin_prefetch(&T.par_mirror[cand[i + 16]]);
          }
          diff(cand[i], T.tree.in_parent(cand[i]));
        }
    } else if (T.par_full_dirty || full) {
      for (uint32_t p = 0; p < n; ++p) diff(p, p == T.root ? kNone : T.parent[p]);
      T.par_full_dirty = false;
    }
  }
  e->pair_off[nt] = pairs.size() / 2;
  if (!pairs.empty()) {
    HIP_TRY(e->d_pairs.ensure(pairs.size() * 4), "alloc deltas");
    HIP_TRY(hipMemcpyAsync(e->d_pairs.p, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice, s),
            "upload deltas");
    for (uint32_t t = 0; t < nt; ++t)
      HIP_TRY(launch_scatter_pairs(e->d_pairs.as<uint32_t>() + 2 * e->pair_off[t],
                                   static_cast<uint32_t>(e->pair_off[t + 1] - e->pair_off[t]),
                                   e->d_tpar.as<uint32_t>() + static_cast<size_t>(t) * n, s),
              "scatter deltas");
  }
  using clk = std::chrono::steady_clock;
  const auto tb1 = clk::now();
  // 2. depth keys and sort per topic
  HIP_TRY(e->d_anc0.ensure(static_cast<size_t>(n) * 4), "alloc scratch");
  HIP_TRY(e->d_anc1.ensure(static_cast<size_t>(n) * 4), "alloc scratch");
  HIP_TRY(e->d_dep0.ensure(static_cast<size_t>(n) * 4), "alloc scratch");
  HIP_TRY(e->d_dep1.ensure(static_cast<size_t>(n) * 4), "alloc scratch");
  HIP_TRY(e->d_keys0.ensure(static_cast<size_t>(n) * 8), "alloc keys");
  HIP_TRY(e->d_skeys.ensure(static_cast<size_t>(nt) * n * 8), "alloc sorted keys");
  HIP_TRY(e->d_gstat.ensure(static_cast<size_t>(nt) * 4 * 4), "alloc build stats");
  HIP_TRY(e->d_lvl.ensure(static_cast<size_t>(nt) * 512 * 4), "alloc level tables");
  size_t cub_bytes = 0, scan_bytes = 0;
  HIP_TRY(sort_keys(nullptr, &cub_bytes, nullptr, nullptr, n, s), "sort size");
  HIP_TRY(e->d_cub.ensure(std::max<size_t>(cub_bytes, 16)), "alloc sort temp");
  // [t][reach, max depth, max fan-out, unresolved]
  uint32_t* gstat = e->d_gstat.as<uint32_t>();
  auto& gs = e->gstat_host;
  auto& lh = e->lvl_host;
  // pointer jumping sized from the last build's depth (x4 headroom); a topic
  // that grew deeper reports unresolved peers and is redone with full jumps
  std::vector<uint32_t> jumps(nt, depth_jumps_full(n));
  for (uint32_t t = 0; t < nt; ++t) {
    const uint32_t d = e->topics[t].depth;
    if (d) jumps[t] = std::min(jumps[t], depth_jumps_full(4 * d));
  }
  for (int pass = 0; pass < 2; ++pass) {
    HIP_TRY(hipMemsetAsync(e->d_gstat.p, 0, static_cast<size_t>(nt) * 4 * 4, s), "clear build stats");
    HIP_TRY(hipMemsetAsync(e->d_lvl.p, 0, static_cast<size_t>(nt) * 512 * 4, s), "clear level tables");
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (!T.exists) continue;
      HIP_TRY(launch_depth_keys(e->d_tpar.as<uint32_t>() + static_cast<size_t>(t) * n, n, T.root, jumps[t],
                                e->d_anc0.as<uint32_t>(), e->d_anc1.as<uint32_t>(),
                                e->d_dep0.as<uint32_t>(), e->d_dep1.as<uint32_t>(),
                                e->d_keys0.as<uint64_t>(), gstat + 4 * t, s),
              "depth");
      size_t tb = e->d_cub.bytes;
      HIP_TRY(sort_keys(e->d_cub.p, &tb, e->d_keys0.as<uint64_t>(),
                        e->d_skeys.as<uint64_t>() + static_cast<size_t>(t) * n, n, s),
              "sort");
      HIP_TRY(launch_level_starts(e->d_skeys.as<uint64_t>() + static_cast<size_t>(t) * n, n,
                                  e->d_lvl.as<uint32_t>() + 512 * t, s),
              "level starts");
    }
    // (level starts of unreachable peers' keys land in slot 255: ignored)
    gs.assign(static_cast<size_t>(nt) * 4, 0);
    lh.assign(static_cast<size_t>(nt) * 512, 0);
    HIP_TRY(hipMemcpyAsync(gs.data(), gstat, gs.size() * 4, hipMemcpyDeviceToHost, s), "read build stats");
    HIP_TRY(hipMemcpyAsync(lh.data(), e->d_lvl.p, lh.size() * 4, hipMemcpyDeviceToHost, s), "read level starts");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    bool redo = false;
    for (uint32_t t = 0; t < nt; ++t)
      if (e->topics[t].exists && gs[4 * t + 3]) {
        jumps[t] = depth_jumps_full(n);
        redo = true;
      }
    if (!redo) break;
  }
  const auto tb2 = clk::now();
  for (uint32_t t = 0; t < nt; ++t)
    if (e->topics[t].exists && gs[4 * t + 1] >= kBuildMaxDepth) {
      *fallback = true;  // deeper than the key's depth field
      return PS_OK;
    }
  // 3. layout: topic t's nodes at [nbase_t, nbase_t + R_t)
  uint64_t n_total = 0;
  e->roots_host.clear();
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    T.nbase = static_cast<uint32_t>(n_total);
    T.n_nodes = T.exists ? gs[4 * t] : 0;
    if (T.n_nodes) e->roots_host.push_back(T.nbase);
    n_total += T.n_nodes;
  }
  if (n_total >= 0xFFFFFFF0ull) return e->fail(PS_E_NOMEM, "node space exceeds 2^32 nodes");
  const uint32_t nn = static_cast<uint32_t>(n_total);
  e->n_nodes = nn;
  e->n_pad = std::max<uint32_t>(16, ((nn + 15) / 16) * 16);
  HIP_TRY(e->d_row_ptr.ensure((static_cast<size_t>(nn) + 1) * 4), "alloc row_ptr");
  HIP_TRY(e->d_col.ensure(std::max<size_t>(nn, 1) * 4), "alloc col");
  HIP_TRY(e->d_node_topic.ensure(std::max<size_t>(nn, 1) * 2), "alloc node_topic");
  HIP_TRY(e->d_node_peer.ensure(std::max<size_t>(nn, 1) * 4), "alloc node_peer");
  HIP_TRY(e->d_node_parent.ensure(std::max<size_t>(nn, 1) * 4), "alloc node_parent");
  HIP_TRY(e->d_node_flags.ensure(e->n_pad + 16), "alloc node_flags");
  HIP_TRY(e->d_deg.ensure((static_cast<size_t>(nn) + 1) * 4), "alloc fan-out");
  HIP_TRY(e->d_first.ensure(std::max<size_t>(nn, 1) * 4), "alloc first child");
  HIP_TRY(e->d_local.ensure(static_cast<size_t>(n) * 4), "alloc local ids");
  HIP_TRY(hipMemsetAsync(e->d_deg.p, 0, (static_cast<size_t>(nn) + 1) * 4, s), "clear fan-out");
  HIP_TRY(hipMemsetAsync(e->d_first.p, 0xFF, std::max<size_t>(nn, 1) * 4, s), "clear first child");
  uint32_t* lvl = e->d_lvl.as<uint32_t>();  // [t][0..255] level start, [t][256..511] internal count
  // BFS placement, level by level and without sorting: the keys are already
  // grouped by level and, within a level, by parent peer with siblings in peer
  // order; the groups go in parent node order (an exclusive scan of the
  // parents' fan-out), each child at its sibling rank
  HIP_TRY(e->d_cnt.ensure(static_cast<size_t>(n) * 4), "alloc fan-out by peer");
  HIP_TRY(e->d_fidx.ensure(static_cast<size_t>(n) * 4), "alloc first child index");
  HIP_TRY(e->d_childoff.ensure(static_cast<size_t>(n) * 4 + 4), "alloc child offsets");
  {
    size_t sb = 0;
    HIP_TRY(scan_u32(nullptr, &sb, nullptr, nullptr, n, s), "scan size");
    HIP_TRY(e->d_cub.ensure(std::max<size_t>(sb, 16)), "alloc scan temp");
  }
  uint32_t* cnt = e->d_cnt.as<uint32_t>();
  uint32_t* fidx = e->d_fidx.as<uint32_t>();
  uint32_t* childoff = e->d_childoff.as<uint32_t>();
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    if (!T.n_nodes) continue;
    const uint32_t depth = gs[4 * t + 1];
    const uint64_t* keys = e->d_skeys.as<uint64_t>() + static_cast<size_t>(t) * n;
    const uint16_t tt = static_cast<uint16_t>(t);
    HIP_TRY(hipMemsetAsync(cnt, 0, static_cast<size_t>(n) * 4, s), "clear fan-out by peer");
    HIP_TRY(hipMemsetAsync(fidx, 0xFF, static_cast<size_t>(n) * 4, s), "clear first child index");
    HIP_TRY(launch_child_stats(keys, T.n_nodes, cnt, fidx, s), "child stats");
    // the small top levels (and their parents) go in one single-block launch
    auto lvl_end = [&](uint32_t d) { return d == depth ? T.n_nodes : lh[512 * t + d + 1]; };
    uint32_t d_small = 1;
    while (d_small <= depth && lvl_end(d_small) - lh[512 * t + d_small] <= e->small_place &&
           lh[512 * t + d_small] - lh[512 * t + d_small - 1] <= e->small_place)
      ++d_small;
    if (d_small > 1) {
      HIP_TRY(launch_place_small(keys, e->d_lvl.as<uint32_t>() + 512 * t, d_small, depth, T.n_nodes, T.nbase, tt,
                                 cnt, fidx, e->d_node_peer.as<uint32_t>(), e->d_node_topic.as<uint16_t>(),
                                 e->d_local.as<uint32_t>(), e->d_node_parent.as<uint32_t>(),
                                 e->d_deg.as<uint32_t>(), e->d_first.as<uint32_t>(), s),
              "place small levels");
    } else {
      HIP_TRY(launch_place_root(keys, T.nbase, tt, cnt, e->d_node_peer.as<uint32_t>(),
                                e->d_node_topic.as<uint16_t>(), e->d_local.as<uint32_t>(),
                                e->d_node_parent.as<uint32_t>(), e->d_deg.as<uint32_t>(), s),
              "place root");
    }
    for (uint32_t d = d_small; d <= depth; ++d) {
      const uint32_t plo = lh[512 * t + d - 1];
      const uint32_t lo = lh[512 * t + d];
      const uint32_t hi = d == depth ? T.n_nodes : lh[512 * t + d + 1];
      size_t tb = e->d_cub.bytes;
      HIP_TRY(scan_u32(e->d_cub.p, &tb, e->d_deg.as<uint32_t>() + T.nbase + plo, childoff, lo - plo, s),
              "scan fan-out");
      HIP_TRY(launch_place_level(keys, lo, hi, T.nbase, T.nbase + plo, childoff, cnt, fidx, tt,
                                 e->d_node_peer.as<uint32_t>(), e->d_node_topic.as<uint16_t>(),
                                 e->d_local.as<uint32_t>(), e->d_node_parent.as<uint32_t>(),
                                 e->d_deg.as<uint32_t>(), e->d_first.as<uint32_t>(), s),
              "place level");
    }
  }
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicHost& T = e->topics[t];
    if (!T.n_nodes) continue;
    HIP_TRY(launch_level_internal(e->d_deg.as<uint32_t>(), T.nbase, T.n_nodes, lvl + 512 * t, gs[4 * t + 1],
                                  lvl + 512 * t + 256, gstat + 4 * t + 2, s),
            "level stats");
  }
  // 4. CSR: row_ptr = exclusive scan of the fan-out; children consecutive
  HIP_TRY(scan_u32(nullptr, &scan_bytes, nullptr, nullptr, nn + 1, s), "scan size");
  HIP_TRY(e->d_cub.ensure(std::max<size_t>(scan_bytes, 16)), "alloc scan temp");
  size_t tb = e->d_cub.bytes;
  HIP_TRY(scan_u32(e->d_cub.p, &tb, e->d_deg.as<uint32_t>(), e->d_row_ptr.as<uint32_t>(), nn + 1, s), "scan");
  HIP_TRY(launch_fill_col(e->d_row_ptr.as<uint32_t>(), e->d_first.as<uint32_t>(), nn, e->d_col.as<uint32_t>(), s),
          "fill col");
  // 5. level tables back to the host (rounds, chunks, grid bounds)
  const auto tb3 = clk::now();
  HIP_TRY(hipMemcpyAsync(lh.data(), lvl, lh.size() * 4, hipMemcpyDeviceToHost, s), "read level tables");
  HIP_TRY(hipMemcpyAsync(gs.data(), gstat, gs.size() * 4, hipMemcpyDeviceToHost, s), "read build stats");
  HIP_TRY(hipStreamSynchronize(s), "sync");
  if (e->host_timing) {
    auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    std::fprintf(stderr, "[psengine] gpu build: deltas %.3f ms (%zu), depth+sort+readback %.3f ms, "
                 "placement enqueue %.3f ms, drain %.3f ms\n", ms(tb0, tb1), pairs.size() / 2,
                 ms(tb1, tb2), ms(tb2, tb3), ms(tb3, clk::now()));
  }
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    T.mesh = false;
    T.root_local = true;
    T.cross.clear();
    T.depth = T.n_nodes ? gs[4 * t + 1] : 0;
    T.max_deg = gs[4 * t + 2];
    T.level_off.assign(T.depth + 2, 0);
    T.level_internal.assign(T.depth + 1, 0);
    if (!T.n_nodes) continue;
    for (uint32_t d = 0; d <= T.depth; ++d) {
      T.level_off[d] = lh[512 * t + d];
      T.level_internal[d] = lh[512 * t + 256 + d];
    }
    T.level_off[T.depth + 1] = T.n_nodes;
  }
  e->remote_fed.clear();
  e->gpu_graph = true;
  e->mirrors_valid = false;
  return PS_OK;
}

int upload_graph(ps_engine* e) {
  // nothing changed: no uploads, and no stream sync (a pipelined run must not
  // wait here for the previous run's kernels)
  if (!e->graph_dirty && !e->flags_dirty) return PS_OK;
  if (e->graph_dirty) {
    bool built = false;
    if (can_gpu_build(e)) {
      bool fallback = false;
      int rc = gpu_build_graph(e, &fallback);
      if (rc) return rc;
      built = !fallback;
    }
    if (!built) {
      int rc = build_graph(e);
      if (rc) return rc;
      e->gpu_graph = false;
      e->mirrors_valid = true;
      const size_t nn = e->n_nodes;
      HIP_TRY(e->d_row_ptr.ensure((nn + 1) * 4), "alloc row_ptr");
      HIP_TRY(e->d_col.ensure(std::max<size_t>(e->col.size(), 1) * 4), "alloc col");
      HIP_TRY(e->d_node_topic.ensure(std::max<size_t>(nn, 1) * 2), "alloc node_topic");
      HIP_TRY(e->d_node_peer.ensure(std::max<size_t>(nn, 1) * 4), "alloc node_peer");
      HIP_TRY(e->d_node_parent.ensure(std::max<size_t>(nn, 1) * 4), "alloc node_parent");
      // padded to n_pad: the expand kernel stages flag bytes as whole dwords
      HIP_TRY(e->d_node_flags.ensure(e->n_pad + 16), "alloc node_flags");
      HIP_TRY(hipMemcpyAsync(e->d_row_ptr.p, e->row_ptr.data(), (nn + 1) * 4, hipMemcpyHostToDevice, e->stream),
              "upload row_ptr");
      if (!e->col.empty())
        HIP_TRY(hipMemcpyAsync(e->d_col.p, e->col.data(), e->col.size() * 4, hipMemcpyHostToDevice, e->stream),
                "upload col");
      if (nn) {
        HIP_TRY(hipMemcpyAsync(e->d_node_topic.p, e->node_topic.data(), nn * 2, hipMemcpyHostToDevice, e->stream),
                "upload node_topic");
        HIP_TRY(hipMemcpyAsync(e->d_node_peer.p, e->node_peer.data(), nn * 4, hipMemcpyHostToDevice, e->stream),
                "upload node_peer");
        HIP_TRY(hipMemcpyAsync(e->d_node_parent.p, e->node_parent.data(), nn * 4, hipMemcpyHostToDevice,
                               e->stream),
                "upload node_parent");
      }
    }
    const size_t nn = e->n_nodes;
    bool fresh = false;
    const size_t flag_bytes = static_cast<size_t>(ceil_div(e->n_pad, kFlagsPerBlock)) * kFlagsPerBlock;
    HIP_TRY(e->d_flags.ensure(flag_bytes, &fresh), "alloc flags");
    HIP_TRY(hipMemsetAsync(e->d_flags.p, 0, e->d_flags.bytes, e->stream), "clear flags");
    const size_t n_blk = ceil_div(e->n_pad, kFlagsPerBlock);
    HIP_TRY(e->d_blk.ensure(n_blk), "alloc block flags");
    HIP_TRY(hipMemsetAsync(e->d_blk.p, 0, e->d_blk.bytes, e->stream), "clear block flags");
    HIP_TRY(e->d_gen.ensure(e->n_pad + 16), "alloc generations");
    e->n_remote_fed = static_cast<uint32_t>(e->remote_fed.size());
    HIP_TRY(e->d_remote_fed.ensure(std::max<size_t>(e->remote_fed.size(), 1) * 4), "alloc remote list");
    if (!e->remote_fed.empty())
      HIP_TRY(hipMemcpyAsync(e->d_remote_fed.p, e->remote_fed.data(), e->remote_fed.size() * 4,
                             hipMemcpyHostToDevice, e->stream),
              "upload remote list");
    HIP_TRY(hipMemsetAsync(e->d_gen.p, 0, e->d_gen.bytes, e->stream), "clear generations");
    e->gen_cur = 0;  // node ids changed: every row is stale
    HIP_TRY(e->d_frontier.ensure(std::max<size_t>(nn, 1) * 4), "alloc frontier");
    HIP_TRY(e->d_wgcount.ensure(static_cast<size_t>(ceil_div(e->n_pad, kFlagsPerBlock)) * 4),
            "alloc wg_count");
    e->graph_dirty = false;
    e->flags_dirty = true;
    e->have_window = false;  // the node space of the last window is gone
    ++e->graph_epoch;
  }
  if (e->flags_dirty) {
    ++e->flags_epoch;
    if (e->gpu_graph) {
      const uint32_t n = e->cfg.n_peers;
      HIP_TRY(e->d_live.ensure(n), "alloc live mask");
      HIP_TRY(e->d_roots.ensure(std::max<size_t>(e->roots_host.size(), 1) * 4), "alloc roots");
      HIP_TRY(hipMemcpyAsync(e->d_live.p, e->live.data(), n, hipMemcpyHostToDevice, e->stream), "upload live");
      if (!e->roots_host.empty())
        HIP_TRY(hipMemcpyAsync(e->d_roots.p, e->roots_host.data(), e->roots_host.size() * 4,
                               hipMemcpyHostToDevice, e->stream),
                "upload roots");
      HIP_TRY(launch_node_flags(e->d_node_peer.as<uint32_t>(), e->d_row_ptr.as<uint32_t>(),
                                e->d_live.as<uint8_t>(), e->n_nodes, e->d_roots.as<uint32_t>(),
                                static_cast<uint32_t>(e->roots_host.size()), e->d_node_flags.as<uint8_t>(),
                                e->stream),
              "node flags");
      e->mirrors_valid = false;
    } else {
      build_flags(e);
      if (e->n_nodes)
        HIP_TRY(hipMemcpyAsync(e->d_node_flags.p, e->node_flags.data(), e->n_nodes, hipMemcpyHostToDevice,
                               e->stream),
                "upload node_flags");
    }
    e->flags_dirty = false;
  }
  // host mirrors may be rebuilt by the next call: finish the uploads now
  HIP_TRY(hipStreamSynchronize(e->stream), "sync uploads");
  return PS_OK;
}

// Level mode.  In a window whose topics are all trees with a
// single start round s_t each, a node at BFS level d receives the window's
// messages exactly in round s_t + d (if every ancestor is live) and forwards
// them in round s_t + d + 1, so each round writes one BFS level per topic.
//
// Per-level launches (k_pull): round q writes the rows of BFS level q - s_t
// of every active topic t (children pull from their parents), cut into
// chunks of at most kPullMaxKids nodes and about kPullWords words, one wave
// each.  Cached: rebuilt only when the node space, the flags or the start
// rounds change.
int build_pull_chunks(ps_engine* e, const std::vector<TopicDev>& tab,
                      const std::vector<std::vector<StartGroup>>& groups, uint32_t rounds) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  std::vector<uint64_t> key{e->graph_epoch, e->flags_epoch, rounds, e->pull_words};
  for (uint32_t t = 0; t < nt; ++t) {
    key.push_back(tab[t].W ? groups[t].size() : ~0ull);
    key.push_back(tab[t].W);
    key.push_back(tab[t].wbase << 1 | ((tab[t].flags & kTopicGroups) ? 1 : 0));
    if (tab[t].W)
      for (const StartGroup& g : groups[t]) key.push_back(static_cast<uint64_t>(g.start) << 32 | g.w0);
  }
  if (key == e->pull_key) return PS_OK;
  e->pull_key.clear();
  // parent-range staging reads the host mirror of node_parent; a GPU-built
  // node space (BFS order too) gets the ranges on the device
  const bool gpu = e->gpu_graph;
  auto& C = e->pull_host;
  auto& off = e->pull_off;
  C.clear();
  off.assign(rounds + 2, 0);
  e->pull_bytes.assign(rounds + 2, 0);
  for (uint32_t q = 1; q <= rounds; ++q) {
    off[q] = static_cast<uint32_t>(C.size());
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (const StartGroup& g : groups[t]) {
        if (q < g.start + 1) continue;
        const uint32_t d = q - g.start;  // level of the nodes whose block g is written this round
        if (d + 1 >= T.level_off.size()) continue;
        const uint32_t lo = T.level_off[d], hi = T.level_off[d + 1];
        const uint32_t per = std::max<uint32_t>(1, std::min<uint32_t>(kPullMaxKids, e->pull_words / g.wn));
        e->pull_bytes[q] += static_cast<uint64_t>(hi - lo) * g.wn * 8;
        for (uint32_t u = lo; u < hi; u += per) {
          PullChunk c{};
          c.node_begin = T.nbase + u;
          c.node_end = T.nbase + std::min(u + per, hi);
          c.topic = t;
          c.p_lo = gpu ? kNone : e->node_parent[c.node_begin];
          c.p_hi = gpu ? kNone : e->node_parent[c.node_end - 1];
          // the block rows: group-major blocks, or whole rows
          const bool gm = (tab[t].flags & kTopicGroups) != 0;
          const uint64_t row0 = tab[t].wbase + (gm ? static_cast<uint64_t>(tab[t].n_nodes) * g.w0 : 0);
          c.W = gm ? g.wn : tab[t].W;
          c.row0_lo = static_cast<uint32_t>(row0);
          c.row0_hi = static_cast<uint32_t>(row0 >> 32);
          C.push_back(c);
        }
      }
    }
  }
  off[rounds + 1] = static_cast<uint32_t>(C.size());
  HIP_TRY(e->d_pull.ensure(std::max<size_t>(C.size(), 1) * sizeof(PullChunk)), "alloc pull chunks");
  if (!C.empty())
    HIP_TRY(hipMemcpyAsync(e->d_pull.p, C.data(), C.size() * sizeof(PullChunk),
                           hipMemcpyHostToDevice, e->stream),
            "upload pull chunks");
  if (gpu && !C.empty())  // parent ranges for the generation staging
    HIP_TRY(launch_chunk_parents(e->d_pull.as<PullChunk>(), static_cast<uint32_t>(C.size()),
                                 e->d_node_parent.as<uint32_t>(), e->stream),
            "chunk parents");
  e->pull_key = key;
  e->ghost_key.clear();  // multi-GPU: the chunks' shipping ranges are assigned again
  return PS_OK;
}

// Pair launches (k_pull_pair): one launch writes rounds q
// and q + 1, each wave a run of level-d nodes and then every child of the run
// from the rows it holds in LDS, so round q + 1 reads no parent row from HBM.
// Which rounds pair up is a small dynamic program over the rounds after
// k_flood's: a pair saves round q + 1's parent-row reads (level d's internal
// nodes x row bytes) and one launch (priced as kLaunchBytes of traffic).  A
// round pairs only if each row it writes (and each level-1 row of a start
// group entering at round q) fits the LDS stage.  Fills e->pp_kind (PS_K_*
// per round); cached with the pull chunks.
int build_pair_chunks(ps_engine* e, const std::vector<TopicDev>& tab,
                      const std::vector<std::vector<StartGroup>>& groups, uint32_t rounds, uint32_t first) {
  std::vector<uint64_t> key = e->pull_key;  // (graph, flags, rounds, row widths, start groups)
  key.push_back(first);
  key.push_back(e->pair_on ? 1 : 0);
  if (key == e->pp_key) return PS_OK;
  constexpr uint32_t stage = kPairWords;
  constexpr double kLaunchBytes = 16e6;  // ~3 us of launch ramp and tail at ~5.5 TB/s (64, 200 MB: same plan on cfg3)
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  auto& kind = e->pp_kind;
  kind.assign(rounds + 2, PS_K_NONE);
  for (uint32_t q = 1; q <= first && q <= rounds; ++q) kind[q] = PS_K_FLOOD;
  auto width = [&](uint32_t t, const StartGroup& g) { return (tab[t].flags & kTopicGroups) ? g.wn : tab[t].W; };
  // per round: parent-row bytes read (estimate), and whether it can pair
  std::vector<double> rd(rounds + 2, 0.0);
  std::vector<uint8_t> can(rounds + 2, 0);
  for (uint32_t q = first + 1; q <= rounds; ++q) {
    bool ok = e->pair_on && q + 1 <= rounds;
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (const StartGroup& g : groups[t]) {
        const uint32_t W = width(t, g);
        if (q >= g.start + 1) {
          const uint32_t d = q - g.start;
          if (d + 1 >= T.level_off.size()) continue;
          const double parents = d == 1 ? 1.0 : (d - 1 < T.level_internal.size() ? T.level_internal[d - 1] : 0);
          rd[q] += parents * W * 8.0;
          ok = ok && W <= stage;
        } else if (g.start == q && T.level_off.size() > 2) {
          ok = ok && W <= stage;  // its level 1 runs in the pair launch as a plain run
        }
      }
    }
    can[q] = ok;
  }
  // best[q]: traffic of rounds q..rounds
  std::vector<double> best(rounds + 3, 0.0);
  std::vector<uint8_t> take(rounds + 2, 0);
  auto cost = [&](uint32_t q) {
    const double b = static_cast<double>(e->pull_bytes[q]);
    return b + rd[q] + (b > 0 ? kLaunchBytes : 0.0);
  };
  for (uint32_t q = rounds; q > first; --q) {
    best[q] = cost(q) + best[q + 1];
    if (can[q]) {
      const double wb = static_cast<double>(e->pull_bytes[q]) + static_cast<double>(e->pull_bytes[q + 1]);
      const double pc = wb + rd[q] + kLaunchBytes + best[q + 2];
      if (pc < best[q]) {
        best[q] = pc;
        take[q] = 1;
      }
    }
  }
  auto& C = e->pp_host;
  C.clear();
  e->pp_lo.assign(rounds + 2, 0);
  e->pp_hi.assign(rounds + 2, 0);
  const bool gpu = e->gpu_graph;
  for (uint32_t q = first + 1; q <= rounds; ++q) {
    if (!take[q]) {
      kind[q] = e->pull_bytes[q] ? PS_K_PULL : PS_K_NONE;
      continue;
    }
    kind[q] = PS_K_PAIR;
    kind[q + 1] = PS_K_PAIR2;
    e->pp_lo[q] = static_cast<uint32_t>(C.size());
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      const bool gm = (tab[t].flags & kTopicGroups) != 0;
      for (const StartGroup& g : groups[t]) {
        const uint32_t W = width(t, g);
        uint32_t d, per;
        bool late = false;
        if (q >= g.start + 1) {
          d = q - g.start;
          if (d + 1 >= T.level_off.size()) continue;
          const uint32_t n = T.level_off[d + 1] - T.level_off[d];
          const uint32_t kids = d + 2 < T.level_off.size() ? T.level_off[d + 2] - T.level_off[d + 1] : 0;
          // about 2 x pull_words row words per wave, parents and children together
          const double f = static_cast<double>(kids) / std::max<uint32_t>(1, n);
          per = static_cast<uint32_t>(std::max(1.0, 2.0 * e->pull_words / (W * (1.0 + f))));
        } else if (g.start == q && T.level_off.size() > 2) {
          d = 1;
          late = true;
          per = std::max<uint32_t>(1, e->pull_words / W);
        } else {
          continue;
        }
        per = std::min<uint32_t>({per, kPairPar, stage / W});
        const uint32_t lo = T.level_off[d], hi = T.level_off[d + 1];
        const uint64_t row0 = tab[t].wbase + (gm ? static_cast<uint64_t>(tab[t].n_nodes) * g.w0 : 0);
        for (uint32_t u = lo; u < hi; u += per) {
          PullChunk c{};
          c.node_begin = T.nbase + u;
          c.node_end = T.nbase + std::min(u + per, hi);
          c.topic = t;
          c.p_lo = gpu ? kNone : e->node_parent[c.node_begin];
          c.p_hi = gpu ? kNone : e->node_parent[c.node_end - 1];
          c.W = W;
          c.row0_lo = static_cast<uint32_t>(row0);
          c.row0_hi = static_cast<uint32_t>(row0 >> 32);
          c.c_lo = late ? kNoneNode : 0;  // children: filled in on the device
          C.push_back(c);
        }
      }
    }
    e->pp_hi[q] = static_cast<uint32_t>(C.size());
    ++q;  // round q + 1 is the pair's second round
  }
  HIP_TRY(e->d_pp.ensure(std::max<size_t>(C.size(), 1) * sizeof(PullChunk)), "alloc pair chunks");
  if (!C.empty()) {
    HIP_TRY(hipMemcpyAsync(e->d_pp.p, C.data(), C.size() * sizeof(PullChunk), hipMemcpyHostToDevice, e->stream),
            "upload pair chunks");
    if (gpu)
      HIP_TRY(launch_chunk_parents(e->d_pp.as<PullChunk>(), static_cast<uint32_t>(C.size()),
                                   e->d_node_parent.as<uint32_t>(), e->stream),
              "pair chunk parents");
    HIP_TRY(launch_pair_kids(e->d_pp.as<PullChunk>(), static_cast<uint32_t>(C.size()), e->d_row_ptr.as<uint32_t>(),
                             e->d_col.as<uint32_t>(), e->stream),
            "pair chunk children");
  }
  e->pp_key = key;
  return PS_OK;
}

// Multi-GPU level mode: the per-round exchange of ghost
// parents.  Region (a -> b, round q) holds, for the topics active in round q
// in topic order, one record per a -> b ghost parent of that round's level:
// [pad if W even][reach word][W row words] (ghost_record_words).  Every rank
// computes every region from the same topology (gcnt) and message counts, so
// sender and receiver agree on sizes and offsets without a handshake.  This
// rank's pack entries (its parents to ship, with their record offsets in the
// send buffer) and each ghost-fed node's row offset in the receive buffer
// follow.  Cached per node space, start rounds and row widths.
int build_ghost_plan(ps_engine* e, const std::vector<TopicDev>& tab, const std::vector<uint32_t>& wglob,
                     const std::vector<uint32_t>& tstart, uint32_t rounds) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const int32_t world = e->world, me = e->rank;
  // Every size here is computed from message-derived widths (wglob) and the
  // global cross counts, identically on every rank -- also on a rank that
  // owns none of a topic's nodes (its tab entry is idle): the ranks must agree
  // on which rounds exchange and on every region's size.
  std::vector<uint64_t> key{e->graph_epoch, rounds};
  for (uint32_t t = 0; t < nt; ++t) {
    key.push_back(wglob[t] ? tstart[t] : ~0ull);
    key.push_back(wglob[t]);
    key.push_back(tab[t].W);
  }
  if (key == e->ghost_key) return PS_OK;
  e->ghost_key.clear();
  auto level_of = [&](uint32_t q, uint32_t t) -> uint32_t {  // level written in round q, 0: none
    const TopicHost& T = e->topics[t];
    if (!wglob[t] || !T.exists || q <= tstart[t] || T.gcnt.empty()) return 0;
    const uint32_t d = q - tstart[t];
    return d <= T.depth ? d : 0;
  };
  auto gcnt = [&](uint32_t t, uint32_t d, int32_t a, int32_t b) -> uint64_t {
    return e->topics[t].gcnt[(static_cast<size_t>(d) * world + a) * world + b];
  };
  e->ghost_rounds.assign(rounds + 2, ps_engine::GhostRound{});
  struct ShipRange {
    uint32_t round, topic, e0, e1;
  };
  std::vector<ShipRange> ship;
  e->pack_host.clear();
  e->pack_seg_host.clear();
  e->ghost_off_host.assign(e->n_nodes, kGhostNone);
  e->ghost_send_max = e->ghost_recv_max = 0;
  std::vector<uint64_t> rec_off(static_cast<size_t>(world) * nt);  // per peer, per topic: first record (words)
  for (uint32_t q = 1; q <= rounds; ++q) {
    auto& R = e->ghost_rounds[q];
    R.s_off.assign(world, 0);
    R.s_len.assign(world, 0);
    R.r_off.assign(world, 0);
    R.r_len.assign(world, 0);
    // region a -> b: bytes, and (into rec_off[peer]) each topic's first record
    auto region = [&](int32_t a, int32_t b, int32_t peer) -> uint64_t {
      uint64_t words = 0;
      for (uint32_t t = 0; t < nt; ++t) {
        rec_off[static_cast<size_t>(peer) * nt + t] = words;
        const uint32_t d = level_of(q, t);
        if (d) words += gcnt(t, d, a, b) * ghost_record_words(wglob[t]);
      }
      return words * 8;
    };
    for (int32_t a = 0; a < world && !R.any; ++a)
      for (int32_t b = 0; b < world && !R.any; ++b)
        for (uint32_t t = 0; t < nt && a != b; ++t) {
          const uint32_t d = level_of(q, t);
          if (d && gcnt(t, d, a, b)) {
            R.any = true;
            break;
          }
        }
    // send regions (me -> b) and this rank's pack entries
    uint64_t so = 0;
    for (int32_t b = 0; b < world; ++b) {
      if (b == me) continue;
      R.s_off[b] = so;
      R.s_len[b] = region(me, b, b);
      so += R.s_len[b];
    }
    // Records of level-0 parents (roots, seeded) are packed by k_pack this
    // round; deeper parents' records are written by the k_pull launch of the
    // round before, which writes those parents' rows (PullChunk e_lo/e_hi)
    R.pack0 = static_cast<uint32_t>(e->pack_host.size());
    R.seg0 = static_cast<uint32_t>(e->pack_seg_host.size());
    uint64_t word0 = 0;
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t d = level_of(q, t);
      if (!d) continue;
      const TopicHost& T = e->topics[t];
      const uint32_t W = wglob[t], rw = ghost_record_words(W);
      const uint32_t e0 = static_cast<uint32_t>(e->pack_host.size());
      for (uint32_t i = T.send_lvl[d]; i < T.send_lvl[d + 1]; ++i) {
        const uint32_t b = T.send_dst[i] >> kRemoteRankShift, k = T.send_dst[i] & kRemoteIdMask;
        PackEntry pe{};
        pe.node = T.send_node[i];
        pe.row_off = R.s_off[b] / 8 + rec_off[static_cast<size_t>(b) * nt + t] + static_cast<uint64_t>(k) * rw +
                     (rw - W);
        e->pack_host.push_back(pe);
      }
      const uint32_t e1 = static_cast<uint32_t>(e->pack_host.size());
      if (e1 == e0) continue;
      if (d == 1) {
        e->pack_seg_host.push_back(PackSeg{e0, e1, t, W, word0});
        word0 += static_cast<uint64_t>(e1 - e0) * pack_units(W);
      } else {
        ship.push_back(ShipRange{q - 1, t, e0, e1});
      }
    }
    R.pack1 = static_cast<uint32_t>(e->pack_host.size());
    R.seg1 = static_cast<uint32_t>(e->pack_seg_host.size());
    // receive regions (a -> me) and the rows the ghost-fed nodes read
    uint64_t ro = 0;
    for (int32_t a = 0; a < world; ++a) {
      if (a == me) continue;
      R.r_off[a] = ro;
      R.r_len[a] = region(a, me, a);
      ro += R.r_len[a];
    }
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t d = level_of(q, t);
      if (!d) continue;
      const TopicHost& T = e->topics[t];
      const uint32_t W = wglob[t], rw = ghost_record_words(W);
      for (uint32_t u = T.nbase + T.level_off[d]; u < T.nbase + T.level_off[d + 1]; ++u) {
        const uint32_t g = e->ghost_ref[u];
        if (g == kNone) continue;
        const uint32_t a = g >> kRemoteRankShift, k = g & kRemoteIdMask;
        e->ghost_off_host[u] = R.r_off[a] / 8 + rec_off[static_cast<size_t>(a) * nt + t] +
                               static_cast<uint64_t>(k) * rw + (rw - W);
      }
    }
    e->ghost_send_max = std::max(e->ghost_send_max, so);
    e->ghost_recv_max = std::max(e->ghost_recv_max, ro);
  }
  // each shipping range to the chunks of round q - 1 that write its parents
  // (entries and chunks both in node order within a topic)
  for (PullChunk& c : e->pull_host) c.e_lo = c.e_hi = 0;
  for (const ShipRange& sr : ship) {
    uint32_t k = sr.e0;
    for (uint32_t ci = e->pull_off[sr.round]; ci < e->pull_off[sr.round + 1]; ++ci) {
      PullChunk& c = e->pull_host[ci];
      if (c.topic != sr.topic) continue;
      while (k < sr.e1 && e->pack_host[k].node < c.node_begin) ++k;  // (never: every parent is in a chunk)
      c.e_lo = k;
      while (k < sr.e1 && e->pack_host[k].node < c.node_end) ++k;
      c.e_hi = k;
    }
    if (k != sr.e1) return e->fail(PS_E_STATE, "ghost records outside the round's chunks");
  }
  if (!e->pull_host.empty()) {
    HIP_TRY(hipMemcpyAsync(e->d_pull.p, e->pull_host.data(), e->pull_host.size() * sizeof(PullChunk),
                           hipMemcpyHostToDevice, e->stream),
            "upload pull chunks");
    if (e->gpu_graph)  // parent ranges again (the host copy holds none)
      HIP_TRY(launch_chunk_parents(e->d_pull.as<PullChunk>(), static_cast<uint32_t>(e->pull_host.size()),
                                   e->d_node_parent.as<uint32_t>(), e->stream),
              "chunk parents");
  }
  HIP_TRY(e->d_pack.ensure(std::max<size_t>(e->pack_host.size(), 1) * sizeof(PackEntry)), "alloc pack entries");
  HIP_TRY(e->d_pack_seg.ensure(std::max<size_t>(e->pack_seg_host.size(), 1) * sizeof(PackSeg)), "alloc pack segments");
  HIP_TRY(e->d_ghost_off.ensure(std::max<size_t>(e->n_nodes, 1) * 8), "alloc ghost offsets");
  HIP_TRY(e->d_send.ensure(std::max<uint64_t>(e->ghost_send_max, 16)), "alloc send buffer");
  HIP_TRY(e->d_recv.ensure(std::max<uint64_t>(e->ghost_recv_max, 16)), "alloc recv buffer");
  if (!e->pack_host.empty())
    HIP_TRY(hipMemcpyAsync(e->d_pack.p, e->pack_host.data(), e->pack_host.size() * sizeof(PackEntry),
                           hipMemcpyHostToDevice, e->stream),
            "upload pack entries");
  if (!e->pack_seg_host.empty())
    HIP_TRY(hipMemcpyAsync(e->d_pack_seg.p, e->pack_seg_host.data(), e->pack_seg_host.size() * sizeof(PackSeg),
                           hipMemcpyHostToDevice, e->stream),
            "upload pack segments");
  if (e->n_nodes)
    HIP_TRY(hipMemcpyAsync(e->d_ghost_off.p, e->ghost_off_host.data(), static_cast<size_t>(e->n_nodes) * 8,
                           hipMemcpyHostToDevice, e->stream),
            "upload ghost offsets");
  e->ghost_key = key;
  return PS_OK;
}

// One persistent launch (k_flood, flood.hip): every level of every active
// topic cut into tasks of at most kFloodMaxNodes nodes and about flood_words
// row words, listed round by round -- a topological order of "reads the
// parent rows the previous round wrote".  A level's tasks publish granules of
// gsz nodes (32, or the task size when smaller: a granule never spans two
// tasks).  Each task records the parent level's segment; k_flood_deps turns it
// into the parent range and its granules.  Per round, the tasks share
// min(256, tasks) counter slots (slot 0 is the window's timeout word).
// Cached per node space, rounds, start rounds and row widths.
int build_flood_tasks(ps_engine* e, const std::vector<TopicDev>& tab,
                      const std::vector<std::vector<StartGroup>>& groups, uint32_t rounds) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  std::vector<uint64_t> key{e->graph_epoch, rounds, e->flood_words};
  for (uint32_t t = 0; t < nt; ++t) {
    key.push_back(tab[t].W ? groups[t].size() : ~0ull);
    key.push_back(tab[t].W);
    key.push_back(tab[t].wbase << 1 | ((tab[t].flags & kTopicGroups) ? 1 : 0));
    if (tab[t].W)
      for (const StartGroup& g : groups[t]) key.push_back(static_cast<uint64_t>(g.start) << 32 | g.w0);
  }
  if (key == e->flood_key) return PS_OK;
  e->flood_key.clear();
  auto& TK = e->flood_tasks;
  auto& SG = e->flood_segs;
  TK.clear();
  SG.clear();
  e->flood_slot0.assign(rounds + 2, 0);
  e->flood_nslot.assign(rounds + 2, 0);
  // each (topic, start group)'s segment of the previous round
  std::vector<std::vector<uint32_t>> seg_prev(nt);
  for (uint32_t t = 0; t < nt; ++t) seg_prev[t].assign(groups[t].size(), kNone);
  uint32_t slot = 1, gran = 0;
  for (uint32_t q = 1; q <= rounds; ++q) {
    const size_t first = TK.size();
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      const bool gm = (tab[t].flags & kTopicGroups) != 0;
      for (size_t gi = 0; gi < groups[t].size(); ++gi) {
        const StartGroup& g = groups[t][gi];
        const uint32_t W = gm ? g.wn : tab[t].W;
        if (q < g.start + 1) continue;
        const uint32_t d = q - g.start;
        if (d + 1 >= T.level_off.size()) continue;
        const uint32_t lo = T.level_off[d], hi = T.level_off[d + 1];
        if (lo == hi) continue;
        uint32_t per = std::max<uint32_t>(1, std::min<uint32_t>(kFloodMaxNodes, e->flood_words / W));
        const uint32_t gsz = std::min(per, kFloodGranule);
        per -= per % gsz;  // whole granules per task
        const uint32_t pseg = d == 1 ? kNone : seg_prev[t][gi];  // level 1: the seeded root
        const uint32_t seg = static_cast<uint32_t>(SG.size());
        seg_prev[t][gi] = seg;
        FloodSeg sg{};
        sg.task0 = static_cast<uint32_t>(TK.size());
        sg.node0 = T.nbase + lo;
        sg.per = per;
        sg.n_tasks = ceil_div(hi - lo, per);
        sg.gbase = gran;
        sg.gsz = gsz;
        sg.nodes = hi - lo;  // nodes of the level
        sg.W = W;
        sg.row0 = tab[t].wbase + (gm ? static_cast<uint64_t>(tab[t].n_nodes) * g.w0 : 0);
        SG.push_back(sg);
        gran += ceil_div(hi - lo, gsz);
        for (uint32_t u = lo; u < hi; u += per) {
          FloodTask k{};
          k.nb = T.nbase + u;
          k.ne = T.nbase + std::min(u + per, hi);
          k.topic = t;
          k.round = q;
          k.g_own = sg.gbase + (u - lo) / gsz;
          k.gsz = gsz;
          k.pseg = pseg;
          k.seg = seg;
          TK.push_back(k);
        }
      }
    }
    const uint32_t n_round = static_cast<uint32_t>(TK.size() - first);
    if (!n_round) continue;
    const uint32_t ns = std::min<uint32_t>(kPullSlots, n_round);
    e->flood_slot0[q] = slot;
    e->flood_nslot[q] = ns;
    for (size_t i = first; i < TK.size(); ++i) {
      TK[i].slot0 = slot;
      TK[i].nslot = ns;
    }
    slot += ns;
  }
  e->flood_slots = slot;
  const size_t n = TK.size();
  HIP_TRY(e->d_flood_tasks.ensure(std::max<size_t>(n, 1) * sizeof(FloodTask)), "alloc flood tasks");
  HIP_TRY(e->d_flood_segs.ensure(std::max<size_t>(SG.size(), 1) * sizeof(FloodSeg)), "alloc flood segments");
  bool fresh = false;  // granules of a fresh allocation carry no epoch yet
  HIP_TRY(e->d_flood_gran.ensure(std::max<size_t>(gran, 1) * 8, &fresh), "alloc flood granules");
  if (fresh) HIP_TRY(hipMemsetAsync(e->d_flood_gran.p, 0, e->d_flood_gran.bytes, e->stream), "clear granules");
  if (n) {
    HIP_TRY(hipMemcpyAsync(e->d_flood_tasks.p, TK.data(), n * sizeof(FloodTask), hipMemcpyHostToDevice, e->stream),
            "upload flood tasks");
    HIP_TRY(hipMemcpyAsync(e->d_flood_segs.p, SG.data(), SG.size() * sizeof(FloodSeg), hipMemcpyHostToDevice,
                           e->stream),
            "upload flood segments");
    HIP_TRY(launch_flood_deps(e->d_flood_tasks.as<FloodTask>(), static_cast<uint32_t>(n),
                              e->d_flood_segs.as<FloodSeg>(), e->d_node_parent.as<uint32_t>(), e->stream),
            "flood dependencies");
  }
  e->flood_key = key;
  return PS_OK;
}

// Counters of one window (rows r x kNumCtr, apply rows for multi-GPU) into
// the run's stats.
// Returns false when a k_flood dependency wait timed out (its timeout word
// is folded into row 0).
bool accumulate_window(ps_stats* st, const uint64_t* hs, const uint64_t* ha, uint32_t r, uint32_t planned0,
                       uint32_t mode, uint32_t flood_rounds, uint32_t launches, int32_t world,
                       const std::vector<uint8_t>& kinds) {
  const bool pull = mode == PS_MODE_LEVEL_PULL || mode == PS_MODE_FLOOD;
  std::memset(st->round_kernel, 0, sizeof(st->round_kernel));
  for (uint32_t q = 1; q <= r; ++q) {
    const uint8_t kind = q < kinds.size() ? kinds[q] : static_cast<uint8_t>(pull ? PS_K_PULL : PS_K_EXPAND);
    const uint64_t* c = &hs[static_cast<size_t>(q) * kNumCtr];
    const uint64_t app_d = (world > 1 && q <= planned0) ? ha[static_cast<size_t>(q) * kNumCtr + kCtrDeliveries] : 0;
    const uint64_t app_u = (world > 1 && q <= planned0) ? ha[static_cast<size_t>(q) * kNumCtr + kCtrDuplicates] : 0;
    st->deliveries += c[kCtrDeliveries] + app_d;
    st->duplicates += c[kCtrDuplicates] + app_u;
    st->frontier_entries += c[kCtrEntries];
    st->child_visits += c[kCtrChildren];
    st->edge_words += c[kCtrSeenWrites];
    // algorithmic bytes of the expand kernel (DESIGN.md §5.1 byte model):
    // per entry frontier id 4 + topic 2 + row_ptr pair 8 + first child 4;
    // per entry word the arrival read 8 (+ 8 when cleared); per child its
    // flag byte + generation read/write (tree) or col id 4 (mesh); per
    // seen read / seen write / arrival write 8.
    uint64_t b;
    if (pull)  // pull model: per node parent id 4 + flag 1 + parent generation 1 (k_flood:
               // + its own generation 1, the seen test; the second round of a k_pull_pair
               // launch: no parent generation, its parents' reach and rows are in LDS),
               // per reached node its generation write 1; parent rows read once (from
               // HBM: none in a pair's second round); rows written
      b = c[kCtrChildren] * (kind == PS_K_FLOOD ? 7 : kind == PS_K_PAIR2 ? 5 : 6) + c[kCtrMeshChildren] * 1 +
          c[kCtrEntryWords] * 8 + c[kCtrSeenWrites] * 8;
    else
      b = c[kCtrEntries] * 18 + c[kCtrEntryWords] * 8 + c[kCtrClearWords] * 8 + c[kCtrChildren] * 3 +
          c[kCtrMeshChildren] * 4 + c[kCtrSeenReads] * 8 + c[kCtrSeenWrites] * 8 + c[kCtrArrivalWrites] * 8;
    st->expand_bytes += b;
    if (q < PS_MAX_ROUNDS) {
      st->round_kernel[q] = kind;
      st->expand_bytes_per_round[q] += b;
      st->deliveries_per_round[q] += c[kCtrDeliveries] + app_d;
      st->frontier_per_round[q] += static_cast<uint32_t>(c[kCtrEntries]);
    }
  }
  st->rounds += r;
  st->expand_launches += launches;
  st->expand_mode = mode;
  st->flood_rounds = flood_rounds;
  st->windows += 1;
  return mode != PS_MODE_FLOOD || hs[kCtrDeliveries] == 0;
}

// Propagates one window: per topic t, win[t] lists the messages (indices into
// `msgs`) whose bits form t's block of W_t = ceil(|win[t]|/64) words.
// Host -> device copies of one window through a pinned staging slot
// (ps_engine::Staging): asynchronous for the host, stream-ordered.
struct Upload {
  void* dst;
  const void* src;
  size_t bytes;
};
// With `fold` set and the copy-kernel form, nothing is launched: *fold gets
// the copies for a kernel that folds them in, and staged[i] the device-mapped
// address of upload i's staged bytes (else its destination).
int stage_uploads(ps_engine* e, const Upload* ups, size_t n, hipStream_t s, StageCopy* fold = nullptr,
                  const void** staged = nullptr) {
  if (fold) *fold = StageCopy{};
  for (size_t i = 0; staged && i < n; ++i) staged[i] = ups[i].dst;
  size_t need = 0;
  for (size_t i = 0; i < n; ++i) need += (ups[i].bytes + 255) & ~size_t(255);
  if (need == 0) return PS_OK;
  // the slot of the asynchronous run being enqueued (its previous user was
  // waited for before the run slot was reused); synchronous runs start with
  // nothing in flight
  ps_engine::Staging& g = e->stg[e->defer_into ? e->defer_into - e->infl : 0];
  if (need > g.cap) {
    if (g.h) HIP_TRY(hipHostFree(g.h), "free staging");
    g.h = nullptr;
    g.cap = 0;
    const size_t cap = std::max<size_t>(need, 64 << 10);
    void* h = nullptr;
    HIP_TRY(hipHostMalloc(&h, cap, hipHostMallocMapped | hipHostMallocCoherent), "alloc staging");
    g.h = static_cast<uint8_t*>(h);
    g.cap = cap;
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, h, 0), "map staging");
    g.d = static_cast<uint8_t*>(d);
  }
  // one copy kernel for up to kStageMax arrays of whole u32 words; blits
  // otherwise
  bool kernel = n <= kStageMax;
  for (size_t i = 0; i < n; ++i) kernel = kernel && ups[i].bytes % 4 == 0;
  StageCopy c{};
  size_t off = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!ups[i].bytes) continue;
    std::memcpy(g.h + off, ups[i].src, ups[i].bytes);
    if (kernel) {
      if (staged && fold) staged[i] = g.d + off;
      c.src[c.n] = reinterpret_cast<const uint32_t*>(g.d + off);
      c.dst[c.n] = static_cast<uint32_t*>(ups[i].dst);
      c.words[c.n++] = static_cast<uint32_t>(ups[i].bytes / 4);
    } else {
      HIP_TRY(hipMemcpyAsync(ups[i].dst, g.h + off, ups[i].bytes, hipMemcpyHostToDevice, s), "upload");
    }
    off += (ups[i].bytes + 255) & ~size_t(255);
  }
  if (kernel && fold)
    *fold = c;
  else if (kernel)
    HIP_TRY(launch_stage_copy(c, s), "stage copy");
  return PS_OK;
}

// Debug (PSAMD_FLOOD_PROFILE=1): where k_flood's waves spent the last launch.
void flood_profile_report(ps_engine* e) {
  const uint32_t nw = e->flood_prof_waves;
  std::vector<uint64_t> p(static_cast<size_t>(nw) * kFloodProf);
  if (hipMemcpy(p.data(), e->d_flood_prof.p, p.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  uint64_t t0 = ~0ull, t1 = 0, smax = 0;
  double sum[kFloodProf] = {};
  std::vector<double> ends;
  for (uint32_t w = 0; w < nw; ++w) {
    const uint64_t* q = &p[static_cast<size_t>(w) * kFloodProf];
    t0 = std::min(t0, q[0]);
    t1 = std::max(t1, q[1]);
    smax = std::max(smax, q[0]);
    for (uint32_t k = 2; k < kFloodProf; ++k) sum[k] += static_cast<double>(q[k]);
    ends.push_back(static_cast<double>(q[1]));
  }
  std::sort(ends.begin(), ends.end());
  auto us = [](double ticks) { return ticks / 100.0; };  // s_memrealtime: 100 MHz
  const double busy = sum[2] + sum[3] + sum[4] + sum[5];
  std::fprintf(stderr,
               "[psengine] k_flood profile: %u waves, span %.1f us, start skew %.1f us, ends p50 %.1f p90 %.1f "
               "max %.1f us; per wave avg: wait %.1f resolve %.1f stream %.1f publish %.1f us (%.0f%%/%.0f%%/%.0f%%/"
               "%.0f%%), %.1f tasks; waits in the last third of the rounds %.1f us\n",
               nw, us(static_cast<double>(t1 - t0)), us(static_cast<double>(smax - t0)),
               us(ends[ends.size() / 2] - t0), us(ends[ends.size() * 9 / 10] - t0), us(ends.back() - t0),
               us(sum[2] / nw), us(sum[3] / nw), us(sum[4] / nw), us(sum[5] / nw), 100 * sum[2] / busy,
               100 * sum[3] / busy, 100 * sum[4] / busy, 100 * sum[5] / busy, sum[6] / nw, us(sum[7] / nw));
}

int run_window(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<WinSlice>& win,
               ps_stats* st) {
  const auto t_g0 = std::chrono::steady_clock::now();
  int rc = upload_graph(e);
  if (rc) return rc;
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const int32_t world = e->world, me = e->rank;
  const auto t_w0 = std::chrono::steady_clock::now();
  if (e->host_timing)
    std::fprintf(stderr, "[psengine] graph upload/build %.3f ms (%s)\n",
                 std::chrono::duration<double, std::milli>(t_w0 - t_g0).count(),
                 e->gpu_graph ? "gpu" : "host");
  std::vector<TopicDev> tab(std::max<uint32_t>(nt, 1));
  uint64_t wtot = 0;
  uint32_t max_depth = 0, max_start = 0;
  bool need_direct = world > 1;
  std::vector<uint32_t> tstart(std::max<uint32_t>(nt, 1), 0);  // single-start topics
  std::vector<std::vector<StartGroup>> groups(std::max<uint32_t>(nt, 1));
  std::vector<std::vector<uint32_t>> pos(std::max<uint32_t>(nt, 1));  // window slot -> row bit
  bool multi_any = false;  // some topic's window has several start rounds
  std::vector<uint32_t> wglob(std::max<uint32_t>(nt, 1), 0);  // row words of every active topic, on every rank
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicHost& T = e->topics[t];
    TopicDev& d = tab[t];
    d = TopicDev{};
    d.nbase = T.nbase;
    d.n_nodes = T.n_nodes;
    d.flags = (T.mesh ? kTopicMesh : 0u) | (T.root_local ? kTopicRootLocal : 0u);
    if (!T.exists || win[t].n == 0) continue;
    // every rank plans the same rounds: global depth, global start rounds
    max_depth = std::max(max_depth, T.depth);
    uint32_t s_lo = ~0u, s_hi = 0;
    if (!e->run_zero_start)  // else: every message of the run starts in round 0
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t s0 = msgs[win[t].idx[li]].start;
        s_lo = std::min(s_lo, s0);
        s_hi = std::max(s_hi, s0);
      }
    if (e->run_zero_start) s_lo = s_hi = 0;
    max_start = std::max(max_start, s_hi);
    const bool one_start = s_lo == s_hi;
    // (decided from the window's messages alone: the same on every rank,
    // also on one that owns none of the topic's nodes)
    multi_any |= !one_start && !T.mesh;
    // a tree topic whose window messages share one start round: every node
    // receives once, so arrival rows are its seen rows (kTopicSingleStart)
    if (one_start && !T.mesh) d.flags |= kTopicSingleStart;
    tstart[t] = msgs[win[t].idx[0]].start;
    // (the row layout depends on the window's messages only: every rank
    // computes the same W, also one that owns none of the topic's nodes --
    // its tab entry then stays idle, W = 0, but wglob keeps the width the
    // cross-rank sizes are computed with)
    if (one_start || T.mesh) {
      d.W = ceil_div(win[t].n, 64);
      d.w_msgs = d.W;
      // rows of >= 64 words are padded to an even length so that every row
      // starts 16-B aligned (the expand kernel stores them as dwordx4)
      if (d.W >= 64) d.W += d.W & 1u;
      groups[t].push_back(StartGroup{s_lo, 0, d.W});
    } else {
      // Start groups (a tree's messages entering at different rounds): the
      // (virtual) row holds one word block per start round, in start order,
      // each of an even number of words: a node at level d receives block s
      // -- and only block s -- in round s + d.  Slot li's bit is its rank
      // within its group from the block's first bit (counting sort by start,
      // window order kept inside a group).  Level mode stores the blocks
      // group-major (kTopicGroups, set below).
      std::vector<uint32_t> cnt(s_hi - s_lo + 2, 0);
      for (uint32_t li = 0; li < win[t].n; ++li) cnt[msgs[win[t].idx[li]].start - s_lo + 1]++;
      std::vector<uint32_t> wfirst(s_hi - s_lo + 1, 0);
      uint32_t w = 0;
      for (uint32_t k = 0; k <= s_hi - s_lo; ++k) {
        const uint32_t n_k = cnt[k + 1];
        if (!n_k) continue;
        const uint32_t wn = (ceil_div(n_k, 64) + 1) & ~1u;
        wfirst[k] = w;
        groups[t].push_back(StartGroup{s_lo + k, w, wn});
        w += wn;
      }
      d.W = w;
      d.w_msgs = w;  // every block's words (padding words stay zero)
      auto& P = pos[t];
      P.resize(win[t].n);
      std::vector<uint32_t> fill(s_hi - s_lo + 1, 0);
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t k = msgs[win[t].idx[li]].start - s_lo;
        P[li] = wfirst[k] * 64 + fill[k]++;
      }
    }
    wglob[t] = d.W;
    if (T.n_nodes == 0) {
      d.W = d.w_msgs = 0;
      continue;
    }
    wtot = (wtot + 15) & ~15ull;  // topic blocks start on a 128-B line
    d.wbase = wtot;
    wtot += static_cast<uint64_t>(T.n_nodes) * d.W;
    if (T.mesh || T.max_deg > 64) need_direct = true;
  }
  if (wtot == 0 && world == 1) return PS_OK;
  const auto t_w1 = std::chrono::steady_clock::now();
  const bool record = (e->cfg.flags & PS_F_RECORD_HOPS) != 0;
  HIP_TRY(e->d_seen.ensure(wtot * 8), "alloc seen");
  HIP_TRY(e->d_arr0.ensure(wtot * 8), "alloc arrivals");
  HIP_TRY(e->d_arr1.ensure(wtot * 8), "alloc arrivals");
  bool any_mesh = false;
  for (uint32_t t = 0; t < nt; ++t) any_mesh |= (tab[t].W && (tab[t].flags & kTopicMesh));
  if (record) HIP_TRY(e->d_hop.ensure(wtot * 64 * 2), "alloc hop record");
  const uint32_t n_waves = e->expand_grid * (kBlock / 64);
  // staged + direct kernel counters side by side
  HIP_TRY(e->d_partials.ensure(static_cast<size_t>(2) * n_waves * kNumCtr * 8), "alloc partials");
  // no simple path is longer than a topic's peers: a window ends within
  // n_peers + the latest start round (chains of any depth run to the end; the
  // bound is the same on every rank)
  const uint32_t round_cap = static_cast<uint32_t>(
      std::max<uint64_t>(kMaxRoundsCap, static_cast<uint64_t>(e->cfg.n_peers) + max_start + 2));
  // per-round counter rows: the planned rounds plus slack, grown (content kept)
  // if a mesh path outlives them
  uint32_t stats_rows = std::min<uint32_t>(round_cap, std::max<uint32_t>(kMaxRoundsCap, max_depth + max_start + 32));
  HIP_TRY(e->d_stats.ensure(static_cast<size_t>(stats_rows + 1) * kNumCtr * 8), "alloc stats");
  HIP_TRY(e->d_apply_stats.ensure(static_cast<size_t>(stats_rows + 1) * kNumCtr * 8),
          "alloc apply stats");
  HIP_TRY(e->d_topics.ensure(tab.size() * sizeof(TopicDev)), "alloc topics");
  HIP_TRY(e->d_nfront.ensure(4), "alloc n_front");
  const uint32_t planned0 = max_depth + max_start + 1;
  // level mode: every active topic a tree.  One rank: the leading rounds
  // whose rows are small (latency bound: a launch each would cost more than
  // their bytes) run as ONE persistent k_flood launch, the rest one k_pull
  // launch per round (bandwidth bound); several ranks: one k_pull launch per
  // round (the frontier exchange separates the rounds).  PSAMD_FLOOD=0
  // selects the per-round launches on one rank too.  A window with start
  // groups (a tree's messages entering at several rounds) runs level mode on
  // one rank, one k_pull launch per round over every group's level of that
  // round, its blocks stored group-major; PS_F_COMPACT sends every window
  // through the compaction path.
  const bool multi = multi_any;
  const bool level =
      !(e->cfg.flags & PS_F_COMPACT) && !any_mesh && planned0 + 1 < round_cap && !(multi && world > 1);
  std::vector<GroupDev> gtab;  // start groups of the group-major topics
  for (uint32_t t = 0; t < nt; ++t) {
    TopicDev& d = tab[t];
    d.root_words = d.W;
    if (!level || !d.W || groups[t].size() < 2) continue;
    d.flags |= kTopicGroups;
    d.group_lo = static_cast<uint32_t>(gtab.size());
    d.group_n = static_cast<uint32_t>(groups[t].size());
    d.root_words = groups[t][0].wn;
    for (const StartGroup& g : groups[t]) gtab.push_back(GroupDev{g.w0, g.wn});
  }
  HIP_TRY(e->d_groups.ensure(std::max<size_t>(gtab.size(), 1) * sizeof(GroupDev)), "alloc groups");
  // word offset of virtual word w of node u's row (u relative to the topic)
  auto phys = [&](uint32_t t, uint64_t u, uint32_t w) { return phys_word(tab[t], groups[t], u, w); };

  // root injections (owned roots only), grouped by round: mask[t][round][word]
  std::vector<std::vector<uint64_t>> inj(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicDev& d = tab[t];
    if (d.W == 0 || !(d.flags & kTopicRootLocal)) continue;
    inj[t].assign(static_cast<size_t>(max_start + 1) * d.W, 0);
    if (e->run_zero_start) {  // bits 0 .. n-1 of round 0
      for (uint32_t w = 0; w < win[t].n / 64; ++w) inj[t][w] = ~0ull;
      if (win[t].n % 64) inj[t][win[t].n / 64] = (1ull << (win[t].n % 64)) - 1;
    } else {
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t b = pos[t].empty() ? li : pos[t][li];
        inj[t][static_cast<size_t>(msgs[win[t].idx[li]].start) * d.W + (b >> 6)] |= 1ull << (b & 63);
      }
    }
  }
  std::vector<SeedDev> seeds;
  std::vector<uint32_t> seed_off(max_start + 2, 0);
  for (uint32_t r = 0; r <= max_start; ++r) {
    for (uint32_t t = 0; t < nt; ++t) {
      TopicDev& d = tab[t];
      if (r == 0) d.seed_lo = static_cast<uint32_t>(seeds.size());
      if (inj[t].empty()) continue;
      if (d.flags & kTopicGroups) {
        // group-major: the root's block of the group starting this round is
        // set whole (k_window_init zeroes block 0 only)
        for (const StartGroup& g : groups[t])
          if (g.start == r)
            for (uint32_t w = g.w0; w < g.w0 + g.wn; ++w)
              seeds.push_back(SeedDev{phys(t, 0, w), inj[t][static_cast<size_t>(r) * d.W + w], d.nbase, 1});
      } else {
        for (uint32_t w = 0; w < d.W; ++w) {
          const uint64_t m = inj[t][static_cast<size_t>(r) * d.W + w];
          if (m) seeds.push_back(SeedDev{d.wbase + w, m, d.nbase, 0});  // root = node 0
        }
      }
      if (r == 0) d.seed_n = static_cast<uint32_t>(seeds.size()) - d.seed_lo;
    }
    seed_off[r + 1] = static_cast<uint32_t>(seeds.size());
  }
  HIP_TRY(e->d_seeds.ensure(seeds.size() * sizeof(SeedDev)), "alloc seeds");
  const auto t_w2 = std::chrono::steady_clock::now();

  // Start rounds present per topic.  A node at BFS level d receives a
  // message started at round s in round s + d and is expanded in round
  // s + d + 1: that bounds each round's frontier (grid size) and, for the
  // multi-GPU exchange, each round's cross-rank traffic exactly.
  std::vector<std::vector<uint8_t>> starts_of(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    if (win[t].n == 0 || !e->topics[t].exists) continue;
    starts_of[t].assign(max_start + 1, 0);
    if (e->run_zero_start)
      starts_of[t][0] = 1;
    else
      for (uint32_t li = 0; li < win[t].n; ++li) starts_of[t][msgs[win[t].idx[li]].start] = 1;
  }
  auto round_grid = [&](uint32_t r) -> uint32_t {
    if (any_mesh) return e->expand_grid;
    uint64_t bound = 0;
    for (uint32_t t = 0; t < nt; ++t) {
      if (tab[t].W == 0) continue;
      const auto& li = e->topics[t].level_internal;
      for (uint32_t s0 = 0; s0 <= max_start; ++s0) {
        if (!starts_of[t][s0] || r < 1 + s0) continue;
        const uint32_t d = r - 1 - s0;
        if (d < li.size()) bound += li[d];
      }
    }
    const uint64_t blocks = (bound + 3) / 4;  // ~1 entry per wave at least
    return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(e->expand_grid, blocks)));
  };
  const bool flood_ok = level && world == 1 && e->flood_on && !e->flood_broken &&
                        e->flood_grid > 0 && e->n_nodes < 0x80000000u;  // k_flood marks node ids with bit 31
  uint32_t flood_rounds = 0;    // rounds 1..flood_rounds: k_flood
  std::vector<uint32_t> lgrid;  // per-round launches: grid of every round
  uint32_t n_slots = 0;         // level mode: partial counter slots of the window
  if (level) {
    int rc2 = build_pull_chunks(e, tab, groups, planned0);
    if (!rc2 && flood_ok) {
      while (flood_rounds < planned0 && e->pull_bytes[flood_rounds + 1] <= e->flood_top_bytes) ++flood_rounds;
      if (flood_rounds) rc2 = build_flood_tasks(e, tab, groups, flood_rounds);
    }
    if (!rc2 && world > 1) rc2 = build_ghost_plan(e, tab, wglob, tstart, planned0);
    // one rank: rounds q, q + 1 in one k_pull_pair launch where it pays
    // (round_kind; several ranks: the exchange separates every round)
    if (!rc2 && world == 1) {
      rc2 = build_pair_chunks(e, tab, groups, planned0, flood_rounds);
      e->round_kind = e->pp_kind;
    } else {
      e->round_kind.assign(planned0 + 2, PS_K_PULL);
      for (uint32_t q = 1; q <= flood_rounds; ++q) e->round_kind[q] = PS_K_FLOOD;
    }
    if (rc2) return rc2;
    // desc[3q..]: round q's partial slots (first, end, stride) for the reduce
    auto& desc = e->desc_host;
    desc.assign(3 * (planned0 + 2), 0);
    uint32_t slot = 0;
    if (flood_rounds) {
      desc[0] = 0;  // row 0: k_flood's timeout word (slot 0)
      desc[1] = 1;
      desc[2] = 1;
      for (uint32_t q = 1; q <= flood_rounds; ++q) {
        desc[3 * q] = e->flood_slot0[q];
        desc[3 * q + 1] = e->flood_slot0[q] + e->flood_nslot[q];
        desc[3 * q + 2] = e->flood_nslot[q] ? 1 : 0;
      }
      slot = e->flood_slots;
    }
    // k_pull launch of round q owns the slots [woff[q], woff[q+1]): one per block, at most kPullSlots
    lgrid.assign(planned0 + 1, 0);
    auto& woff = e->woff_host;
    woff.assign(planned0 + 2, 0);
    woff[flood_rounds + 1] = slot;
    for (uint32_t q = flood_rounds + 1; q <= planned0; ++q) {
      const bool pair = e->round_kind[q] == PS_K_PAIR;
      lgrid[q] = pair ? e->pp_hi[q] - e->pp_lo[q]  // (one one-wave workgroup per chunk)
                      : ceil_div(e->pull_off[q + 1] - e->pull_off[q], kBlock / 64);
      for (uint32_t k = q; k <= q + (pair ? 1u : 0u); ++k) {  // a pair launch: the same slots for both rounds
        woff[k + 1] = woff[k] + std::min<uint32_t>(lgrid[q], pair ? kPairSlots : kPullSlots);
        desc[3 * k] = woff[k];
        desc[3 * k + 1] = woff[k + 1];
        desc[3 * k + 2] = 1;
      }
      if (pair) lgrid[++q] = 0;
    }
    n_slots = woff[planned0 + 1];
    HIP_TRY(e->d_partials.ensure(static_cast<size_t>(std::max<uint32_t>(n_slots, 1)) * kNumCtr * 8),
            "alloc level partials");
    HIP_TRY(e->d_woff.ensure(desc.size() * 4), "alloc reduce descriptors");
  }
  // cross-rank capacities (items = node words) per round: cap[r][from*world+to]
  std::vector<std::vector<uint64_t>> cap;
  uint64_t max_send = 0, max_recv = 0;
  if (world > 1 && !level) {  // compaction mode: delivery items (level mode ships ghost rows)
    cap.assign(planned0 + 1, std::vector<uint64_t>(static_cast<size_t>(world) * world, 0));
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (starts_of[t].empty()) continue;
      const uint64_t Wt = wglob[t];
      for (const auto& c : T.cross)
        for (uint32_t s0 = 0; s0 <= max_start; ++s0) {
          const uint32_t r = c.level + 1 + s0;
          if (starts_of[t][s0] && r <= planned0) cap[r][c.from * world + c.to] += c.count * Wt;
        }
    }
    for (uint32_t r = 1; r <= planned0; ++r) {
      uint64_t sb = 0, rb = 0;
      for (int32_t q = 0; q < world; ++q) {
        if (cap[r][me * world + q]) sb += kRegionHeader + cap[r][me * world + q] * sizeof(XItem);
        if (cap[r][q * world + me]) rb += kRegionHeader + cap[r][q * world + me] * sizeof(XItem);
      }
      max_send = std::max(max_send, sb);
      max_recv = std::max(max_recv, rb);
    }
    HIP_TRY(e->d_send.ensure(max_send), "alloc send regions");
    HIP_TRY(e->d_recv.ensure(max_recv), "alloc recv regions");
  }

  const bool flood = flood_rounds > 0;
  const uint32_t mode = flood ? PS_MODE_FLOOD : level ? PS_MODE_LEVEL_PULL : PS_MODE_COMPACT;
  const auto t_w3 = std::chrono::steady_clock::now();
  hipStream_t s = e->stream;
  // the window's first kernel also copies the staged uploads, applies the
  // round-0 seeds of tree roots and clears the pull partial slots (level
  // mode without meshes; the eager seen clear below would erase the seeds)
  const bool fold = level && !any_mesh && !(e->cfg.flags & PS_F_NO_LAZY_SEEN);
  WindowStart ws{};
  const void* staged[4] = {nullptr, nullptr, nullptr, nullptr};
  {
    const Upload ups[4] = {
        {e->d_topics.p, tab.data(), tab.size() * sizeof(TopicDev)},
        {e->d_seeds.p, seeds.data(), seeds.size() * sizeof(SeedDev)},
        {e->d_woff.p, e->desc_host.data(), level ? e->desc_host.size() * 4 : 0},
        {e->d_groups.p, gtab.data(), gtab.size() * sizeof(GroupDev)}};
    const int rcu = stage_uploads(e, ups, 4, s, fold ? &ws.copy : nullptr, staged);
    if (rcu) return rcu;
  }
  if (fold) {
    if (seed_off[1] > 0) ws.seeds = static_cast<const SeedDev*>(staged[1]);
    ws.zero = e->d_partials.as<uint64_t>();
    ws.zero_words = static_cast<uint64_t>(n_slots) * kNumCtr;
  }
  const bool seeds0_done = ws.seeds != nullptr;
  const bool partials_done = ws.zero != nullptr;
  HIP_TRY(hipEventRecord(e->ev_run0, s), "event");
  const auto t_first = std::chrono::steady_clock::now();
  // new window generation: every tree row from older windows becomes stale
  if (++e->gen_cur > 255) {
    HIP_TRY(hipMemsetAsync(e->d_gen.p, 0, e->d_gen.bytes, s), "clear generations");
    e->gen_cur = 1;
  }
  HIP_TRY(launch_window_init(static_cast<const TopicDev*>(fold ? staged[0] : e->d_topics.p), nt,
                             e->d_seen.as<uint64_t>(), e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>(),
                             e->d_gen.as<uint8_t>(), e->gen_cur, any_mesh, ws, s),
          "window init");
  if (e->n_remote_fed && !level)
    HIP_TRY(launch_init_nodes(e->d_remote_fed.as<uint32_t>(), e->n_remote_fed,
                              e->d_node_topic.as<uint16_t>(), e->d_topics.as<TopicDev>(),
                              e->d_seen.as<uint64_t>(), e->d_arr0.as<uint64_t>(),
                              e->d_arr1.as<uint64_t>(), e->d_gen.as<uint8_t>(), e->gen_cur, !level, s),
            "init remote-fed rows");
  if (e->cfg.flags & PS_F_NO_LAZY_SEEN) {
    // eager variant: clear every row and mark every node current, so the
    // expand kernel reads each child's seen word before it tests and sets it
    HIP_TRY(hipMemsetAsync(e->d_seen.p, 0, wtot * 8, s), "clear seen");
    HIP_TRY(hipMemsetAsync(e->d_gen.p, static_cast<int>(e->gen_cur), e->d_gen.bytes, s),
            "stamp generations");
  }
  if (record) HIP_TRY(hipMemsetAsync(e->d_hop.p, 0xFF, wtot * 64 * 2, s), "clear hop record");
  if (world > 1)  // (level mode: stays zero; the pull kernels count every delivery)
    HIP_TRY(hipMemsetAsync(e->d_apply_stats.p, 0, static_cast<size_t>(planned0 + 1) * kNumCtr * 8, s),
            "clear apply stats");

  ExpandArgs a{};
  bool host_stats_written = false;  // the reduce wrote the deferred slot's pinned rows
  a.frontier = e->d_frontier.as<uint32_t>();
  a.n_front = e->d_nfront.as<uint32_t>();
  a.row_ptr = e->d_row_ptr.as<uint32_t>();
  a.col = e->d_col.as<uint32_t>();
  a.node_topic = e->d_node_topic.as<uint16_t>();
  a.node_flags = e->d_node_flags.as<uint8_t>();
  a.topics = e->d_topics.as<TopicDev>();
  a.seen = e->d_seen.as<uint64_t>();
  a.gen = e->d_gen.as<uint8_t>();
  a.gen_cur = e->gen_cur;
  a.next_flag = e->d_flags.as<uint8_t>();
  a.blk_flag = e->d_blk.as<uint8_t>();
  a.hop_rec = record ? e->d_hop.as<uint16_t>() : nullptr;
  a.send = e->d_send.as<uint8_t>();
  uint64_t* const partials = e->d_partials.as<uint64_t>();
  uint64_t* arr[2] = {e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>()};
  uint64_t* stats = e->d_stats.as<uint64_t>();
  const bool timed = (e->cfg.flags & PS_F_TIME_KERNELS) != 0;

  auto seed_round = [&](uint32_t r, uint64_t* into) -> hipError_t {
    if (r > max_start) return hipSuccess;
    return launch_seed(e->d_seeds.as<SeedDev>(), seed_off[r], seed_off[r + 1], into, a.seen,
                       level ? nullptr : a.next_flag, level ? nullptr : a.blk_flag, s);
  };
  auto compact = [&](uint32_t r, uint32_t waves_r) -> hipError_t {
    hipError_t x = launch_flag_count(a.next_flag, a.blk_flag, e->n_pad,
                                     e->d_wgcount.as<uint32_t>(), partials, waves_r,
                                     r ? stats + r * kNumCtr : nullptr, s);
    if (x != hipSuccess) return x;
    return launch_flag_compact(a.next_flag, a.blk_flag, e->n_pad, e->d_wgcount.as<uint32_t>(),
                               e->d_frontier.as<uint32_t>(), e->d_nfront.as<uint32_t>(), s);
  };
  // multi-GPU round r: region layout, header reset, exchange, apply
  std::vector<uint64_t> s_off(world, 0), s_len(world, 0), r_off(world, 0), r_len(world, 0);
  auto layout = [&](uint32_t r) -> bool {
    if (world <= 1 || r > planned0 || cap.empty()) return false;
    uint64_t so = 0, ro = 0;
    bool any = false;
    for (int32_t q = 0; q < world; ++q) {
      const uint64_t cs = cap[r][me * world + q], cr = cap[r][q * world + me];
      s_off[q] = so;
      s_len[q] = cs ? kRegionHeader + cs * sizeof(XItem) : 0;
      so += s_len[q];
      r_off[q] = ro;
      r_len[q] = cr ? kRegionHeader + cr * sizeof(XItem) : 0;
      ro += r_len[q];
      for (int32_t z = 0; z < world; ++z) any |= cap[r][q * world + z] != 0;
    }
    for (int32_t q = 0; q < world && q < kMaxRanks; ++q) a.send_off[q] = s_off[q];
    return any;  // the same verdict on every rank
  };

  uint32_t planned = planned0;
  uint32_t r = 0;
  size_t ev_used = 0;
  std::vector<uint32_t> ev_round;  // round of every timed launch pair
  uint32_t launches = 0;
  auto time_mark = [&](bool begin) -> hipError_t {
    if (!timed) return hipSuccess;
    if (begin) ev_round.push_back(r);
    if (begin && ev_used + 2 > e->ev_k.size()) {
      hipEvent_t x, y;
      hipError_t c = hipEventCreate(&x);
      if (c == hipSuccess) c = hipEventCreate(&y);
      if (c != hipSuccess) return c;
      e->ev_k.push_back(x);
      e->ev_k.push_back(y);
    }
    const hipError_t c = hipEventRecord(e->ev_k[ev_used + (begin ? 0 : 1)], s);
    if (!begin) ev_used += 2;
    return c;
  };
  // all-to-allv of this round's send regions, then the apply kernel
  auto xchg = [&](uint32_t rr) -> int {
    std::string xerr;
    hipError_t xe = e->transport->exchange(a.send, s_off, s_len, e->d_recv.as<uint8_t>(), r_off,
                                           r_len, s, &xerr);
    if (xe != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
    ApplyArgs ap{};
    ap.recv = e->d_recv.as<uint8_t>();
    ap.world = static_cast<uint32_t>(world);
    ap.cap_pre[0] = 0;
    for (int32_t q = 0; q < world; ++q) {
      ap.recv_off[q] = r_off[q];
      ap.cap_pre[q + 1] = ap.cap_pre[q] + cap[rr][q * world + me];
    }
    ap.node_topic = a.node_topic;
    ap.node_flags = a.node_flags;
    ap.topics = a.topics;
    ap.seen = a.seen;
    ap.a_next = a.a_next;
    ap.next_flag = level ? nullptr : a.next_flag;
    ap.blk_flag = level ? nullptr : a.blk_flag;
    ap.hop_rec = a.hop_rec;
    ap.stats = e->d_apply_stats.as<uint64_t>() + static_cast<size_t>(rr) * kNumCtr;
    ap.gen = level ? a.gen : nullptr;
    ap.gen_cur = a.gen_cur;
    HIP_TRY(launch_apply(ap, rr, record, s), "apply");
    return PS_OK;
  };
  if (level) {
    // static frontier, counters reduced once per window
    if (!partials_done)  // blocks / waves add into shared partial slots
      HIP_TRY(hipMemsetAsync(partials, 0, static_cast<size_t>(n_slots) * kNumCtr * 8, s), "clear partials");
    if (!seeds0_done) HIP_TRY(seed_round(0, arr[0]), "seed");
    // k_flood, or start groups: every root row is seeded up front into arr[0]
    // (and seen: k_flood reads parent rows from there), the blocks of later
    // start rounds included -- a block is read only in its own rounds
    bool pairs = false;
    for (uint32_t q = 1; q <= planned0; ++q) pairs |= e->round_kind[q] == PS_K_PAIR;
    const bool upfront = flood || multi || pairs;  // (a pair launch's plain level-1 runs read roots)
    if (upfront && max_start > 0)
      HIP_TRY(launch_seed(e->d_seeds.as<SeedDev>(), seed_off[1], seed_off[max_start + 1], arr[0], a.seen, nullptr,
                          nullptr, s),
              "seed");
    if (flood) {
      FloodArgs fa{};
      fa.tasks = e->d_flood_tasks.as<FloodTask>();
      fa.segs = e->d_flood_segs.as<FloodSeg>();
      fa.node_parent = e->d_node_parent.as<uint32_t>();
      fa.node_flags = a.node_flags;
      fa.topics = a.topics;
      fa.seen = a.seen;
      fa.gen = a.gen;
      fa.hop_rec = a.hop_rec;
      fa.granules = e->d_flood_gran.as<uint64_t>();
      fa.partials = partials;
      fa.err = reinterpret_cast<uint32_t*>(partials);  // slot 0, reduced into row 0
      fa.n_tasks = static_cast<uint32_t>(e->flood_tasks.size());
      if (++e->flood_epoch == 0) ++e->flood_epoch;  // granules of older launches carry older epochs
      fa.epoch = e->flood_epoch;
      fa.gen_cur = a.gen_cur;
      fa.spin_ticks = e->flood_spin_ticks;
      const uint32_t flood_blocks = std::min<uint32_t>(e->flood_grid, ceil_div(fa.n_tasks, kBlock / 64));
      if (e->flood_profile) {
        HIP_TRY(e->d_flood_prof.ensure(static_cast<size_t>(flood_blocks) * 4 * kFloodProf * 8), "alloc flood profile");
        fa.prof = e->d_flood_prof.as<uint64_t>();
        fa.prof_split = flood_rounds * 2 / 3;
        e->flood_prof_waves = flood_blocks * 4;
      }
      r = 1;  // the per-round kernel times of a timed run go to round 1
      HIP_TRY(time_mark(true), "event");
      ++launches;
      HIP_TRY(launch_flood(fa, flood_blocks, record, s), "flood");
      HIP_TRY(time_mark(false), "event");
    }
    {
      for (r = flood_rounds + 1; r <= planned0; ++r) {
        a.a_cur = upfront ? arr[0] : arr[(r - 1) & 1];
        a.a_next = arr[r & 1];
        // multi-GPU: this round's ghost parents (rows written last round, or
        // seeded roots) to the ranks owning their children, then the exchange
        if (world > 1 && e->ghost_rounds[r].any) {
          const auto& R = e->ghost_rounds[r];
          if (R.seg1 > R.seg0) {
            const PackSeg& last = e->pack_seg_host[R.seg1 - 1];
            HIP_TRY(launch_pack(e->d_pack.as<PackEntry>(), e->d_pack_seg.as<PackSeg>() + R.seg0, R.seg1 - R.seg0,
                                last.unit0 + static_cast<uint64_t>(last.e1 - last.e0) * pack_units(last.W), a.topics, a.seen,
                                a.gen, a.gen_cur, e->d_send.as<uint64_t>(), s),
                    "pack");
          }
          std::string xerr;
          const hipError_t xe = e->transport->exchange(e->d_send.as<uint8_t>(), R.s_off, R.s_len,
                                                       e->d_recv.as<uint8_t>(), R.r_off, R.r_len, s, &xerr);
          if (xe != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
        }
        if (lgrid[r]) {
          HIP_TRY(time_mark(true), "event");
          ++launches;
          PullArgs pa{};
          pa.node_parent = e->d_node_parent.as<uint32_t>();
          pa.node_flags = a.node_flags;
          pa.topics = a.topics;
          pa.a_cur = a.a_cur;
          pa.seen = a.seen;
          pa.gen = a.gen;
          pa.hop_rec = a.hop_rec;
          pa.partials = partials + static_cast<size_t>(e->woff_host[r]) * kNumCtr;
          pa.gen_cur = a.gen_cur;
          pa.slot_mod = kPullSlots;
          pa.ghost_off = world > 1 ? e->d_ghost_off.as<uint64_t>() : nullptr;
          pa.recv = e->d_recv.as<uint64_t>();
          pa.ship = world > 1 ? e->d_pack.as<PackEntry>() : nullptr;
          pa.send = e->d_send.as<uint64_t>();
          // rows nobody re-reads while they can still sit in the 256 MB MALL
          // (large rounds and the last round) store non-temporally
          const bool pair = e->round_kind[r] == PS_K_PAIR;
          const uint32_t rw = pair ? r + 1 : r;  // the round whose rows the next launch reads
          const bool nt = rw < e->pull_bytes.size() && (e->pull_bytes[rw] >= (64ull << 20) || rw == planned0);
          if (pair) {
            pa.partials2 = partials + static_cast<size_t>(e->woff_host[r + 1]) * kNumCtr;
            pa.slot_mod = kPairSlots;
            pa.all_current = (e->cfg.flags & PS_F_NO_LAZY_SEEN) ? 1u : 0u;
            HIP_TRY(launch_pull_pair(pa, e->d_pp.as<PullChunk>() + e->pp_lo[r], e->pp_hi[r] - e->pp_lo[r], lgrid[r],
                                     r, record, nt, s),
                    "pull pair");
          } else {
            // one rank: big rounds at 5 blocks per CU (+6 %); N ranks keep full
            // residency (4 loopback ranks on one GPU: 6.49 -> 7.13 ms capped)
            HIP_TRY(launch_pull(pa, e->d_pull.as<PullChunk>() + e->pull_off[r], e->pull_off[r + 1] - e->pull_off[r],
                                lgrid[r], r, record, nt, world == 1, s),
                    "pull");
          }
          HIP_TRY(time_mark(false), "event");
        }
        if (!upfront) HIP_TRY(seed_round(r, a.a_next), "seed");
      }
    }
    r = planned0;
    // a deferred window's counters go straight into its pinned rows
    const bool direct = e->defer_last && e->defer_into && !record && !timed && r <= PS_MAX_ROUNDS &&
                        (world == 1 || planned0 <= PS_MAX_ROUNDS);
    host_stats_written = direct;
    HIP_TRY(launch_reduce_rounds(partials, e->d_woff.as<uint32_t>(), planned0, stats,
                                 direct ? e->defer_into->hs_dev : nullptr, s),
            "reduce rounds");
  } else {
  e->round_kind.clear();  // (accumulate_window: every round k_expand)
  HIP_TRY(seed_round(0, arr[0]), "seed");
  HIP_TRY(compact(0, 0), "compact");
  while (true) {
    for (; r < planned && r < round_cap; ) {
      ++r;
      a.a_cur = arr[(r - 1) & 1];
      a.a_next = arr[r & 1];
      const bool xr = layout(r);
      if (xr)
        for (int32_t q = 0; q < world; ++q)
          if (s_len[q]) HIP_TRY(hipMemsetAsync(a.send + s_off[q], 0, kRegionHeader, s), "reset header");
      HIP_TRY(time_mark(true), "event");
      ++launches;
      const uint32_t grid_r = r <= planned0 ? round_grid(r) : e->expand_grid;
      a.partials = partials;
      HIP_TRY(launch_expand(a, r, record, grid_r, s), "expand");
      uint32_t waves_r = grid_r * (kBlock / 64);
      if (need_direct) {
        a.partials = partials + static_cast<size_t>(waves_r) * kNumCtr;
        HIP_TRY(launch_expand_direct(a, r, record, e->expand_grid, s), "expand direct");
        waves_r += n_waves;
      }
      HIP_TRY(time_mark(false), "event");
      if (xr) {
        const int rc3 = xchg(r);
        if (rc3) return rc3;
      }
      HIP_TRY(seed_round(r, a.a_next), "seed");
      HIP_TRY(compact(r, waves_r), "compact");
    }
    uint32_t left = 0;
    HIP_TRY(hipMemcpyAsync(&left, e->d_nfront.p, 4, hipMemcpyDeviceToHost, s), "read frontier");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    if (left == 0 || r >= round_cap) {
      if (left) return e->fail(PS_E_STATE, "propagation did not converge");
      break;
    }
    if (world > 1) return e->fail(PS_E_STATE, "multi-GPU frontier outlived the planned rounds");
    planned = r + 8;  // live mask lengthened a mesh path beyond the BFS depth
    if (planned + 1 > stats_rows) {  // grow the round rows, keeping the counted ones
      const uint32_t rows = std::min<uint32_t>(round_cap, std::max(planned + 1, 2 * stats_rows));
      DevBuf grown;
      HIP_TRY(grown.ensure(static_cast<size_t>(rows + 1) * kNumCtr * 8), "grow stats");
      HIP_TRY(hipMemcpyAsync(grown.p, e->d_stats.p, static_cast<size_t>(stats_rows + 1) * kNumCtr * 8,
                             hipMemcpyDeviceToDevice, s),
              "keep stats");
      HIP_TRY(hipStreamSynchronize(s), "sync");
      std::swap(grown.p, e->d_stats.p);
      std::swap(grown.bytes, e->d_stats.bytes);
      stats = e->d_stats.as<uint64_t>();
      stats_rows = rows;
    }
  }
  }
  const bool defer = e->defer_last && e->defer_into && !record && !timed && r <= PS_MAX_ROUNDS &&
                     (world == 1 || planned0 <= PS_MAX_ROUNDS);  // the pinned slots hold PS_MAX_ROUNDS + 1 rows
  if (!defer) HIP_TRY(hipEventRecord(e->ev_run1, s), "event");
  const auto t_enq = std::chrono::steady_clock::now();
  if (defer) {
    // asynchronous run: the counters follow the kernels on the stream into
    // pinned memory (level mode: written there by the reduce itself); the
    // window's end event marks their arrival; ps_wait accumulates them
    ps_engine::Inflight& f = *e->defer_into;
    if (!host_stats_written)
      HIP_TRY(hipMemcpyAsync(f.hs, stats, static_cast<size_t>(r + 1) * kNumCtr * 8, hipMemcpyDeviceToHost, s),
              "read stats");
    if (world > 1)
      HIP_TRY(hipMemcpyAsync(f.ha, e->d_apply_stats.p, static_cast<size_t>(planned0 + 1) * kNumCtr * 8,
                             hipMemcpyDeviceToHost, s),
              "read apply stats");
    HIP_TRY(hipEventRecord(e->ev_run1, s), "event");
    f.deferred = true;
    f.planned0 = planned0;
    f.world = world;
    f.r = r;
    f.launches = launches;
    f.mode = mode;
    f.flood_rounds = flood_rounds;
    f.kinds = e->round_kind;
    e->last_topics = tab;
    for (uint32_t t = 0; t < nt; ++t) {
      e->last_cnt[t] = tab[t].W ? win[t].n : 0;
      e->last_lo[t] = win[t].n ? e->run_rank[win[t].idx[0]] : 0;
    }
    e->last_pos.swap(pos);
    e->last_groups.swap(groups);
    e->have_window = true;
    if (e->host_timing) {
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      std::fprintf(stderr, "[psengine] async window: plan %.3f ms (run->window %.3f, topics %.3f, seeds %.3f, "
                   "schedule %.3f, uploads %.3f), enqueue %.3f ms\n",
                   ms(e->t_run0, t_first), ms(e->t_run0, t_w0), ms(t_w0, t_w1), ms(t_w1, t_w2),
                   ms(t_w2, t_w3), ms(t_w3, t_first), ms(t_first, t_enq));
    }
    return PS_OK;
  }
  HIP_TRY(hipEventSynchronize(e->ev_run1), "sync");
  const auto t_sync = std::chrono::steady_clock::now();
  const ps_stats keep = *st;  // a k_flood timeout re-runs the window from these stats
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e->ev_run0, e->ev_run1), "elapsed");
  st->run_ms += ms;
  for (size_t i = 0; i < ev_used; i += 2) {
    float k = 0.f;
    HIP_TRY(hipEventElapsedTime(&k, e->ev_k[i], e->ev_k[i + 1]), "elapsed");
    st->expand_ms += k;
    const size_t q = ev_round[i / 2];  // round of this launch
    if (q < PS_MAX_ROUNDS) st->expand_ms_per_round[q] += k;
  }
  std::vector<uint64_t> hs(static_cast<size_t>(r + 1) * kNumCtr), ha;
  HIP_TRY(hipMemcpyAsync(hs.data(), stats, hs.size() * 8, hipMemcpyDeviceToHost, s), "read stats");
  if (world > 1) {
    ha.resize(static_cast<size_t>(planned0 + 1) * kNumCtr);
    HIP_TRY(hipMemcpyAsync(ha.data(), e->d_apply_stats.p, ha.size() * 8, hipMemcpyDeviceToHost, s),
            "read apply stats");
  }
  HIP_TRY(hipStreamSynchronize(s), "sync");
  if (mode == PS_MODE_FLOOD && e->flood_profile && e->flood_prof_waves) flood_profile_report(e);
  if (!accumulate_window(st, hs.data(), ha.data(), r, planned0, mode, flood_rounds, launches, world,
                         e->round_kind)) {
    // a k_flood dependency wait timed out (its waves were not all resident:
    // another engine or process shares the GPU): this window's rows are
    // incomplete.  Run the same window again with per-round launches under a
    // fresh generation, and keep those from now on.
    e->flood_broken = true;
    *st = keep;
    if (e->host_timing) std::fprintf(stderr, "[psengine] k_flood timed out: window re-run per round\n");
    return run_window(e, msgs, win, st);
  }
  if (e->host_timing) {
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr, "[psengine] window: plan %.3f ms (run->window %.3f, topics %.3f, seeds %.3f, "
                 "schedule %.3f, uploads %.3f), enqueue %.3f ms, wait %.3f ms, tail %.3f ms\n",
                 ms(e->t_run0, t_first), ms(e->t_run0, t_w0), ms(t_w0, t_w1), ms(t_w1, t_w2),
                 ms(t_w2, t_w3), ms(t_w3, t_first), ms(t_first, t_enq), ms(t_enq, t_sync),
                 ms(t_sync, std::chrono::steady_clock::now()));
  }

  if (record) {
    {
      int rcm = ensure_mirrors(e);
      if (rcm) return rcm;
    }
    std::vector<uint16_t> hr(wtot * 64);
    if (!hr.empty()) {
      HIP_TRY(hipMemcpyAsync(hr.data(), e->d_hop.p, hr.size() * 2, hipMemcpyDeviceToHost, s), "read hops");
      HIP_TRY(hipStreamSynchronize(s), "sync");
    }
    const uint32_t np = e->cfg.n_peers;
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicDev& d = tab[t];
      if (d.W == 0) continue;
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t mi = win[t].idx[li];
        const uint32_t s0 = msgs[mi].start;
        const uint32_t b = pos[t].empty() ? li : pos[t][li];
        uint8_t* row = e->hops.data() + static_cast<size_t>(mi) * np;
        for (uint32_t u = 0; u < d.n_nodes; ++u) {
          const uint16_t v = hr[phys(t, u, b >> 6) * 64 + (b & 63)];
          // hop = round - start round, saturated at 254 (0xFF: not delivered)
          if (v != kHopRecNone) row[e->node_peer[d.nbase + u]] = static_cast<uint8_t>(std::min<uint32_t>(v - s0, 254u));
        }
      }
    }
  }
  // remember the last window for ps_read_delivered / ps_seen_digest
  e->last_topics = tab;
  for (uint32_t t = 0; t < nt; ++t) {
    e->last_cnt[t] = tab[t].W ? win[t].n : 0;
    e->last_lo[t] = win[t].n ? e->run_rank[win[t].idx[0]] : 0;
  }
  e->last_pos.swap(pos);
  e->last_groups.swap(groups);
  e->have_window = true;
  return PS_OK;
}

// Messages of one phase (per topic, a slice of the run's topic-sorted index
// array), split into windows of at most msg_window messages per topic.
int run_phase(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<WinSlice>& per,
              ps_stats* st) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const uint32_t cap = e->cfg.msg_window;
  uint32_t n_win = 0;
  for (const auto& v : per) n_win = std::max(n_win, (v.n + cap - 1) / cap);
  std::vector<WinSlice> win(nt);
  for (uint32_t k = 0; k < n_win; ++k) {
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t lo = k * cap;
      win[t].idx = per[t].idx + std::min(lo, per[t].n);
      win[t].n = lo < per[t].n ? std::min(cap, per[t].n - lo) : 0;
    }
    e->defer_last = e->defer_phase && k + 1 == n_win;
    int rc = run_window(e, msgs, win, st);
    e->defer_last = false;
    if (rc) return rc;
  }
  return PS_OK;
}

}  // namespace

extern "C" {

const char* ps_version(void) { return "psengine-mi355x 0.1 (gfx950)"; }

int ps_create(const ps_config* cfg, ps_engine** out) {
  if (!cfg || !out) return PS_E_INVAL;
  *out = nullptr;
  if (cfg->n_peers == 0 || cfg->n_topics == 0 || cfg->n_topics > 65535) return PS_E_INVAL;
  auto* e = new (std::nothrow) ps_engine();
  if (!e) return PS_E_NOMEM;
  e->cfg = *cfg;
  if (!e->cfg.tree_width) e->cfg.tree_width = 2;            // pubsub.go:16
  if (!e->cfg.tree_max_width) e->cfg.tree_max_width = 5;    // pubsub.go:17
  if (!e->cfg.msg_window) e->cfg.msg_window = kDefaultWindow;
  e->cfg.msg_window = ((e->cfg.msg_window + 63) / 64) * 64;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    delete e;
    return PS_E_DEVICE;
  }
  if (cfg->device < 0 || cfg->device >= ndev || hipSetDevice(cfg->device) != hipSuccess) {
    delete e;
    return PS_E_DEVICE;
  }
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess &&
      cus > 0)
    e->n_cus = static_cast<uint32_t>(cus);
  // resident 256-thread blocks per CU: k_expand needs 80 VGPRs / 106 SGPRs,
  // which admits 6 (MI355X_MICROARCH.md §Residency)
  e->expand_grid = e->n_cus * 6;
  // k_flood's waves must all be resident at once (its tasks wait on earlier
  // tasks): the grid stays within the occupancy the runtime reports, capped
  // at kFloodBlocksPerCu for margin (MI355X_MICROARCH.md §Residency)
  {
    int bpc = 0;
    if (flood_blocks_per_cu(&bpc) == hipSuccess && bpc > 0)
      e->flood_grid = e->n_cus * std::min<uint32_t>(static_cast<uint32_t>(bpc), kFloodBlocksPerCu);
  }
  // switches: debug timing, and the modes the parity tests cover
  if (const char* v = std::getenv("PSAMD_HOST_TIMING")) e->host_timing = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_GPU_BUILD")) e->gpu_build_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FLOOD")) e->flood_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_PULL_PAIR")) e->pair_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FLOOD_PROFILE")) e->flood_profile = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FLOOD_WORDS"))
    e->flood_words = static_cast<uint32_t>(std::min(1 << 16, std::max(64, std::atoi(v))));
  if (const char* v = std::getenv("PSAMD_FLOOD_SPIN_TICKS"))  // tests: 0 forces the timeout fallback
    e->flood_spin_ticks = static_cast<uint32_t>(std::strtoul(v, nullptr, 0));
  if (const char* v = std::getenv("PSAMD_FLOOD_TOP_BYTES"))  // the k_flood / k_pull split (tests: ~0 = all k_flood)
    e->flood_top_bytes = std::strtoull(v, nullptr, 0);
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e->ev_run0) != hipSuccess || hipEventCreate(&e->ev_run1) != hipSuccess) {
    delete e;
    return PS_E_DEVICE;
  }
  for (auto& f : e->infl) {
    void* h = nullptr;
    if (hipEventCreate(&f.ev0) != hipSuccess || hipEventCreate(&f.ev1) != hipSuccess ||
        hipHostMalloc(&h, 2 * (PS_MAX_ROUNDS + 1) * kNumCtr * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      ps_destroy(e);
      return PS_E_DEVICE;
    }
    f.hs = static_cast<uint64_t*>(h);
    void* hd = nullptr;
    if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) {
      ps_destroy(e);
      return PS_E_DEVICE;
    }
    f.hs_dev = static_cast<uint64_t*>(hd);
    f.ha = f.hs + (PS_MAX_ROUNDS + 1) * kNumCtr;
  }

  e->topics.resize(cfg->n_topics);
  e->live.assign(cfg->n_peers, 1);
  if (e->d_digest.ensure(8) != hipSuccess) {
    delete e;
    return PS_E_NOMEM;
  }
  *out = e;
  return PS_OK;
}

void ps_destroy(ps_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto ev : e->ev_k) (void)hipEventDestroy(ev);
  if (e->ev_run0) (void)hipEventDestroy(e->ev_run0);
  if (e->ev_run1) (void)hipEventDestroy(e->ev_run1);
  for (auto& f : e->infl) {
    if (f.ev0) (void)hipEventDestroy(f.ev0);
    if (f.ev1) (void)hipEventDestroy(f.ev1);
    if (f.hs) (void)hipHostFree(f.hs);
  }
  for (auto& g : e->stg)
    if (g.h) (void)hipHostFree(g.h);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

const char* ps_last_error(const ps_engine* e) { return e ? e->err.c_str() : "null engine"; }

int ps_topic_create(ps_engine* e, uint32_t topic, uint32_t root, uint32_t w, uint32_t mw) {
  if (!e) return PS_E_INVAL;
  if (topic >= e->topics.size()) return e->fail(PS_E_RANGE, "topic id out of range");
  if (root >= e->cfg.n_peers) return e->fail(PS_E_INVAL, "root out of range");
  if (e->topics[topic].exists) return e->fail(PS_E_STATE, "topic exists");
  TopicHost& T = e->topics[topic];
  T = TopicHost{};
  T.exists = true;
  T.kind = Kind::Join;
  T.root = root;
  T.width = w ? w : e->cfg.tree_width;          // TreeOpts (pubsub.go:66-72)
  T.max_width = mw ? mw : e->cfg.tree_max_width;
  T.tree = SubscriptionTree(e->cfg.n_peers, root, T.width, T.max_width,
                            e->cfg.seed ^ (0xA5A5A5A5ull * (topic + 1)));
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_close(ps_engine* e, uint32_t topic) {
  if (!e) return PS_E_INVAL;
  if (!topic_ok(e, topic)) return e->fail(PS_E_STATE, "no such topic");
  for (const auto& m : e->pending)
    if (m.topic == topic) return e->fail(PS_E_STATE, "topic has unsent messages");
  e->topics[topic] = TopicHost{};
  e->graph_dirty = true;
  return PS_OK;
}

static TopicHost* join_topic(ps_engine* e, uint32_t topic) {
  if (!topic_ok(e, topic)) {
    e->fail(PS_E_STATE, "no such topic");
    return nullptr;
  }
  TopicHost& T = e->topics[topic];
  if (T.kind != Kind::Join) {
    e->fail(PS_E_STATE, "topic topology was set explicitly");
    return nullptr;
  }
  return &T;
}

int ps_topic_join(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n,
                  int32_t* status_out) {
  if (!e || (n && !peers)) return PS_E_INVAL;
  TopicHost* T = join_topic(e, topic);
  if (!T) return PS_E_STATE;
  int first = PS_OK;
  for (size_t i = 0; i < n; ++i) {
    int rc = T->tree.subscribe(peers[i]);
    if (status_out) status_out[i] = rc;
    if (rc && !first) {
      first = rc;
      e->err = "join of peer " + std::to_string(peers[i]) + " failed";
    }
  }
  e->graph_dirty = true;
  return first;
}

int ps_topic_leave(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n) {
  if (!e || (n && !peers)) return PS_E_INVAL;
  TopicHost* T = join_topic(e, topic);
  if (!T) return PS_E_STATE;
  int first = PS_OK;
  // leaving peers are scattered over the tree: their entries are fetched a
  // few peers ahead (two stages: the peer, then the lists it points to)
  constexpr size_t kAhead0 = 16, kAhead1 = 8;
  for (size_t i = 0; i < std::min(n, kAhead0); ++i) T->tree.prefetch_leave(peers[i], 0);
  for (size_t i = 0; i < std::min(n, kAhead1); ++i) T->tree.prefetch_leave(peers[i], 1);
  for (size_t i = 0; i < n; ++i) {
    if (i + kAhead0 < n) T->tree.prefetch_leave(peers[i + kAhead0], 0);
    if (i + kAhead1 < n) T->tree.prefetch_leave(peers[i + kAhead1], 1);
    int rc = T->tree.close_client(peers[i]);
    if (rc && !first) first = rc;
  }
  e->graph_dirty = true;
  return first;
}

int ps_topic_drop(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n) {
  if (!e || (n && !peers)) return PS_E_INVAL;
  TopicHost* T = join_topic(e, topic);
  if (!T) return PS_E_STATE;
  int first = PS_OK;
  for (size_t i = 0; i < n; ++i) {
    int rc = T->tree.close_host(peers[i]);
    if (rc && !first) first = rc;
  }
  e->graph_dirty = true;
  return first;
}

int ps_topic_set_tree(ps_engine* e, uint32_t topic, uint32_t root, const uint32_t* parent) {
  if (!e || !parent) return PS_E_INVAL;
  if (topic >= e->topics.size()) return e->fail(PS_E_RANGE, "topic id out of range");
  if (root >= e->cfg.n_peers) return e->fail(PS_E_INVAL, "root out of range");
  for (uint32_t c = 0; c < e->cfg.n_peers; ++c)
    if (parent[c] != PS_NONE && parent[c] >= e->cfg.n_peers)
      return e->fail(PS_E_INVAL, "parent id out of range");
  TopicHost& T = e->topics[topic];
  T = TopicHost{};
  T.exists = true;
  T.kind = Kind::Parent;
  T.root = root;
  T.parent.assign(parent, parent + e->cfg.n_peers);
  T.par_full_dirty = true;
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_set_children(ps_engine* e, uint32_t topic, uint32_t root, const uint32_t* row_ptr,
                          const uint32_t* col) {
  if (!e || !row_ptr) return PS_E_INVAL;
  if (topic >= e->topics.size()) return e->fail(PS_E_RANGE, "topic id out of range");
  const uint32_t n = e->cfg.n_peers;
  if (root >= n) return e->fail(PS_E_INVAL, "root out of range");
  if (row_ptr[0] != 0) return e->fail(PS_E_INVAL, "row_ptr[0] != 0");
  for (uint32_t i = 0; i < n; ++i)
    if (row_ptr[i + 1] < row_ptr[i]) return e->fail(PS_E_INVAL, "row_ptr not monotone");
  if (row_ptr[n] && !col) return e->fail(PS_E_INVAL, "null col");
  for (uint32_t k = 0; k < row_ptr[n]; ++k)
    if (col[k] >= n) return e->fail(PS_E_INVAL, "child id out of range");
  TopicHost& T = e->topics[topic];
  T = TopicHost{};
  T.exists = true;
  T.kind = Kind::Children;
  T.root = root;
  T.rp.assign(row_ptr, row_ptr + n + 1);
  T.cl.assign(col, col + row_ptr[n]);
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_get_parents(ps_engine* e, uint32_t topic, uint32_t* parent_out) {
  if (!e || !parent_out) return PS_E_INVAL;
  if (!topic_ok(e, topic)) return e->fail(PS_E_STATE, "no such topic");
  const TopicHost& T = e->topics[topic];
  std::vector<uint32_t> par;
  if (T.kind == Kind::Join) {
    T.tree.attached_parents(par);
  } else {
    // BFS tree of the given topology (first parent in BFS order)
    std::vector<uint32_t> rp, cl;
    peer_children(e, T, rp, cl);
    par.assign(e->cfg.n_peers, kNone);
    std::vector<uint8_t> vis(e->cfg.n_peers, 0);
    std::vector<uint32_t> q{T.root};
    vis[T.root] = 1;
    for (size_t i = 0; i < q.size(); ++i)
      for (uint32_t k = rp[q[i]]; k < rp[q[i] + 1]; ++k)
        if (!vis[cl[k]]) {
          vis[cl[k]] = 1;
          par[cl[k]] = q[i];
          q.push_back(cl[k]);
        }
  }
  std::copy(par.begin(), par.end(), parent_out);
  return PS_OK;
}

int ps_topic_depth(ps_engine* e, uint32_t topic, uint32_t* depth_out, uint32_t* n_nodes_out) {
  if (!e) return PS_E_INVAL;
  if (!topic_ok(e, topic)) return e->fail(PS_E_STATE, "no such topic");
  int rc = upload_graph(e);
  if (rc) return rc;
  if (depth_out) *depth_out = e->topics[topic].depth;
  if (n_nodes_out) *n_nodes_out = e->topics[topic].n_nodes;
  return PS_OK;
}

int ps_set_flags(ps_engine* e, uint32_t flags) {
  if (!e) return PS_E_INVAL;
  if (flags & ~(PS_F_RECORD_HOPS | PS_F_TIME_KERNELS | PS_F_NO_LAZY_SEEN | PS_F_COMPACT))
    return e->fail(PS_E_INVAL, "unknown flag");
  e->cfg.flags = flags;
  return PS_OK;
}

int ps_set_live(ps_engine* e, const uint8_t* live) {
  if (!e || !live) return PS_E_INVAL;
  for (uint32_t p = 0; p < e->cfg.n_peers; ++p) e->live[p] = live[p] ? 1 : 0;
  e->flags_dirty = true;
  return PS_OK;
}

int ps_publish_at(ps_engine* e, const uint32_t* topic_of_msg, const uint32_t* start_round,
                  size_t n, uint32_t* first) {
  if (!e || (n && !topic_of_msg)) return PS_E_INVAL;
  for (size_t i = 0; i < n; ++i) {
    if (!topic_ok(e, topic_of_msg[i])) return e->fail(PS_E_STATE, "publish to a closed topic");
    if (start_round && start_round[i] > kMaxStartRound)
      return e->fail(PS_E_RANGE, "start round too large");
  }
  if (static_cast<uint64_t>(e->next_msg) + n >= 0xFFFFFFF0ull)
    return e->fail(PS_E_RANGE, "message id space exhausted");
  if (first) *first = e->next_msg;
  const size_t old = e->pending.size();
  e->pending.resize(old + n);
  RunMsg* out = e->pending.data() + old;
  for (size_t i = 0; i < n; ++i) {
    out[i] = RunMsg{topic_of_msg[i], start_round ? start_round[i] : 0u};
    e->pending_nonzero_start |= out[i].start != 0;
  }
  e->next_msg += static_cast<uint32_t>(n);
  return PS_OK;
}

int ps_publish(ps_engine* e, const uint32_t* topic_of_msg, size_t n, uint32_t* first) {
  return ps_publish_at(e, topic_of_msg, nullptr, n, first);
}

}  // extern "C"

namespace {

// ps_run's body.  may_defer: the last window of the final phase may leave its
// counters on the stream (ps_run_async); *stp is completed by ps_wait then.
int run_body(ps_engine* e, ps_stats* stp, bool may_defer) {
  const auto t_host0 = std::chrono::steady_clock::now();
  e->t_run0 = t_host0;
  ps_stats& st = *stp;
  if (hipSetDevice(e->cfg.device) != hipSuccess) return e->fail(PS_E_DEVICE, "hipSetDevice");
  e->last_msgs.clear();
  e->last_msgs.swap(e->pending);
  e->run_zero_start = !e->pending_nonzero_start;
  e->pending_nonzero_start = false;
  const std::vector<RunMsg>& msgs = e->last_msgs;
  const uint32_t nmsg = static_cast<uint32_t>(msgs.size());
  e->last_first = e->next_msg - nmsg;
  e->last_n = nmsg;
  e->have_hops = false;
  e->have_window = false;
  const bool record = (e->cfg.flags & PS_F_RECORD_HOPS) != 0;
  if (record) {
    const uint64_t bytes = static_cast<uint64_t>(nmsg) * e->cfg.n_peers;
    if (bytes > (8ull << 30)) return e->fail(PS_E_NOMEM, "hop record larger than 8 GiB");
    e->hops.assign(bytes, PS_HOP_NONE);
  }
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  // one counting sort: message indices grouped by topic, publish order kept
  auto& off = e->run_topic_off;
  off.assign(nt + 1, 0);
  for (uint32_t i = 0; i < nmsg; ++i) off[msgs[i].topic + 1]++;
  for (uint32_t t = 0; t < nt; ++t) off[t + 1] += off[t];
  e->run_sorted.resize(nmsg);
  e->run_rank.resize(nmsg);
  {
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint32_t i = 0; i < nmsg; ++i) {
      const uint32_t t = msgs[i].topic;
      e->run_rank[i] = fill[t] - off[t];
      e->run_sorted[fill[t]++] = i;
    }
  }
  e->last_lo.assign(nt, 0);
  e->last_cnt.assign(nt, 0);
  std::vector<uint32_t> head(nt, 0);
  auto slice = [&](uint32_t t, uint32_t from, uint32_t n) {
    WinSlice w;
    w.idx = e->run_sorted.data() + off[t] + from;
    w.n = n;
    return w;
  };
  // Abruptly dropped hosts: the first message through the failed edge is lost
  // below it, then the parent repairs (subtree.go:333-351): that message runs
  // on its own over the current tree, the rest over the repaired one.
  while (true) {
    std::vector<WinSlice> solo(nt);
    bool any = false;
    for (uint32_t t = 0; t < nt; ++t) {
      TopicHost& T = e->topics[t];
      const uint32_t cnt = off[t + 1] - off[t];
      if (T.exists && T.kind == Kind::Join && T.tree.has_pending_failures() && head[t] < cnt) {
        solo[t] = slice(t, head[t], 1);
        head[t]++;
        any = true;
      }
    }
    if (!any) break;
    int rc = run_phase(e, msgs, solo, &st);
    if (rc) return rc;
    for (uint32_t t = 0; t < nt; ++t)
      if (solo[t].n) {
        e->topics[t].tree.after_message();
        e->graph_dirty = true;
      }
  }
  {
    std::vector<WinSlice> rest(nt);
    bool any = false;
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t cnt = off[t + 1] - off[t];
      rest[t] = slice(t, head[t], cnt - head[t]);
      any |= rest[t].n > 0;
    }
    if (any) {
      e->defer_phase = may_defer && !record;
      int rc = run_phase(e, msgs, rest, &st);
      e->defer_phase = false;
      if (rc) return rc;
    }
  }
  // lazy prune of Part'ed children at every forwarding node (subtree.go:326-331)
  const auto t_am = std::chrono::steady_clock::now();
  const bool gpu_reach = e->gpu_graph && !e->graph_dirty;  // the node space the messages ran on
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    if (T.exists && T.kind == Kind::Join && head[t] < off[t + 1] - off[t] &&
        T.tree.needs_message_pass()) {
      // on a GPU-built node space the message's reach is a lookup there (a
      // host walk to the root per Part'ed parent costs ~0.2 us each)
      SubscriptionTree::ReachQuery q = [e, &T](const std::vector<uint32_t>& peers,
                                               std::vector<uint8_t>& outv) -> int {
        const uint32_t k = static_cast<uint32_t>(peers.size());
        if (!k) return PS_OK;
        HIP_TRY(e->d_pairs.ensure(static_cast<size_t>(k) * 4 + k + 16), "alloc reach query");
        uint32_t* dp = e->d_pairs.as<uint32_t>();
        uint8_t* dout = reinterpret_cast<uint8_t*>(dp + k);
        HIP_TRY(hipMemcpyAsync(dp, peers.data(), static_cast<size_t>(k) * 4, hipMemcpyHostToDevice, e->stream),
                "upload reach query");
        HIP_TRY(launch_reach_query(dp, k, e->cfg.n_peers, e->d_local.as<uint32_t>(),
                                   e->d_node_peer.as<uint32_t>(), T.nbase, T.n_nodes, dout, e->stream),
                "reach query");
        HIP_TRY(hipMemcpyAsync(outv.data(), dout, k, hipMemcpyDeviceToHost, e->stream), "read reach query");
        HIP_TRY(hipStreamSynchronize(e->stream), "sync");
        if (e->host_timing)
          std::fprintf(stderr, "[psengine] prune reach query: %u parents, done at %.3f ms\n", k,
                       std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - e->t_run0).count());
        return PS_OK;
      };
      int rc = T.tree.after_message(gpu_reach ? &q : nullptr);
      if (rc) return rc;
      e->graph_dirty = true;
    }
  }
  e->have_hops = record;
  if (e->host_timing)
    std::fprintf(stderr, "[psengine] after-message prune %.3f ms (started at %.3f ms)\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_am).count(),
                 std::chrono::duration<double, std::milli>(t_am - e->t_run0).count());
  st.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
  return PS_OK;
}

}  // namespace

extern "C" {

int ps_run(ps_engine* e, ps_stats* out) {
  if (!e) return PS_E_INVAL;
  if (e->infl_count) return e->fail(PS_E_STATE, "asynchronous runs pending: ps_wait first");
  ps_stats st{};
  const int rc = run_body(e, &st, false);
  if (rc) return rc;
  if (out) *out = st;
  return PS_OK;
}

int ps_run_async(ps_engine* e) {
  if (!e) return PS_E_INVAL;
  if (e->infl_count >= 2) return e->fail(PS_E_STATE, "two runs in flight: ps_wait first");
  ps_engine::Inflight& f = e->infl[(e->infl_head + e->infl_count) % 2];
  f.st = ps_stats{};
  f.deferred = false;
  hipEvent_t ev0 = e->ev_run0, ev1 = e->ev_run1;
  e->ev_run0 = f.ev0;  // this run's window events belong to its slot
  e->ev_run1 = f.ev1;
  e->defer_into = &f;
  const int rc = run_body(e, &f.st, true);
  e->ev_run0 = ev0;
  e->ev_run1 = ev1;
  e->defer_into = nullptr;
  if (rc) {
    (void)hipStreamSynchronize(e->stream);
    return rc;
  }
  ++e->infl_count;
  return PS_OK;
}

int ps_wait(ps_engine* e, ps_stats* out) {
  if (!e) return PS_E_INVAL;
  if (!e->infl_count) return e->fail(PS_E_NOTREADY, "no asynchronous run pending");
  ps_engine::Inflight& f = e->infl[e->infl_head];
  e->infl_head = (e->infl_head + 1) % 2;
  --e->infl_count;
  if (f.deferred) {
    HIP_TRY(hipEventSynchronize(f.ev1), "sync");
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, f.ev0, f.ev1), "elapsed");
    f.st.run_ms += ms;
    f.deferred = false;
    if (!accumulate_window(&f.st, f.hs, f.ha, f.r, f.planned0, f.mode, f.flood_rounds, f.launches, f.world,
                           f.kinds)) {
      e->flood_broken = true;
      return e->fail(PS_E_DEVICE, "k_flood: a dependency wait timed out (waves not co-resident?); "
                                  "per-round launches from now on");
    }
  }
  if (out) *out = f.st;
  return PS_OK;
}

int ps_read_hops(ps_engine* e, uint32_t msg, uint8_t* hop_per_peer) {
  if (!e || !hop_per_peer) return PS_E_INVAL;
  if (!e->have_hops) return e->fail(PS_E_NOTREADY, "no hop record (PS_F_RECORD_HOPS)");
  if (msg < e->last_first || msg >= e->last_first + e->last_n)
    return e->fail(PS_E_RANGE, "message not in the last run");
  const uint32_t np = e->cfg.n_peers;
  std::memcpy(hop_per_peer, e->hops.data() + static_cast<size_t>(msg - e->last_first) * np, np);
  return PS_OK;
}

int ps_read_delivered(ps_engine* e, uint32_t msg, uint8_t* out) {
  if (!e || !out) return PS_E_INVAL;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  if (msg < e->last_first || msg >= e->last_first + e->last_n)
    return e->fail(PS_E_RANGE, "message not in the last run");
  const uint32_t i = msg - e->last_first;
  const uint32_t t = e->last_msgs[i].topic;
  const uint32_t rank = e->run_rank[i];
  if (rank < e->last_lo[t] || rank >= e->last_lo[t] + e->last_cnt[t])
    return e->fail(PS_E_NOTREADY, "message not in the last window");
  const uint32_t li = rank - e->last_lo[t];
  const uint32_t b = t < e->last_pos.size() && !e->last_pos[t].empty() ? e->last_pos[t][li] : li;
  const TopicDev& d = e->last_topics[t];
  {
    int rcm = ensure_mirrors(e);
    if (rcm) return rcm;
  }
  std::memset(out, 0, e->cfg.n_peers);
  std::vector<uint64_t> col(d.n_nodes);
  // one word per node: strided copy of this message's word column (row
  // stride W, or its group's block width when group-major)
  static const std::vector<StartGroup> kNoGroups;
  const auto& G = t < e->last_groups.size() ? e->last_groups[t] : kNoGroups;
  uint64_t stride = d.W;
  if (d.flags & kTopicGroups)
    for (const StartGroup& g : G)
      if ((b >> 6) < g.w0 + g.wn) {
        stride = g.wn;
        break;
      }
  HIP_TRY(hipMemcpy2DAsync(col.data(), 8, e->d_seen.as<uint64_t>() + phys_word(d, G, 0, b >> 6), stride * 8ull, 8,
                           d.n_nodes, hipMemcpyDeviceToHost, e->stream),
          "read seen");
  std::vector<uint8_t> gen(d.n_nodes);
  HIP_TRY(hipMemcpyAsync(gen.data(), e->d_gen.as<uint8_t>() + d.nbase, d.n_nodes,
                         hipMemcpyDeviceToHost, e->stream),
          "read generations");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  const bool mesh = (d.flags & kTopicMesh) != 0;
  const uint64_t bit = 1ull << (b & 63);
  for (uint32_t u = 1; u < d.n_nodes; ++u)  // the root is not a recipient
    if ((mesh || gen[u] == e->gen_cur) && (col[u] & bit)) out[e->node_peer[d.nbase + u]] = 1;
  return PS_OK;
}

int ps_read_peer_messages(ps_engine* e, uint32_t topic, uint32_t peer, uint32_t* msg_out, size_t cap,
                          size_t* n_out) {
  if (!e || !n_out || (cap && !msg_out)) return PS_E_INVAL;
  *n_out = 0;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  if (topic >= e->topics.size() || peer >= e->cfg.n_peers) return e->fail(PS_E_RANGE, "topic or peer out of range");
  const TopicDev& d = e->last_topics[topic];
  if (!d.W || !e->last_cnt[topic]) return PS_OK;
  {
    int rcm = ensure_mirrors(e);
    if (rcm) return rcm;
  }
  // the peer's node in this topic (the root is the publisher, not a recipient):
  // a peer -> node map per topic, built once per node space
  auto& pm = e->peer_node[topic];
  if (e->peer_node_epoch.size() != e->topics.size()) e->peer_node_epoch.assign(e->topics.size(), ~0ull);
  if (e->peer_node_epoch[topic] != e->graph_epoch) {
    pm.assign(e->cfg.n_peers, kNone);
    for (uint32_t k = 1; k < d.n_nodes; ++k) pm[e->node_peer[d.nbase + k]] = k;
    e->peer_node_epoch[topic] = e->graph_epoch;
  }
  const uint32_t u = pm[peer];
  if (u == kNone) return PS_OK;  // not subscribed (or not owned by this rank)
  std::vector<uint64_t> row(d.W);
  uint8_t g = 0;
  if (d.flags & kTopicGroups) {  // the row's blocks, one per start group
    for (const StartGroup& sg : e->last_groups[topic])
      HIP_TRY(hipMemcpyAsync(row.data() + sg.w0, e->d_seen.as<uint64_t>() + phys_word(d, e->last_groups[topic], u, sg.w0),
                             sg.wn * 8ull, hipMemcpyDeviceToHost, e->stream),
              "read seen row");
  } else {
    HIP_TRY(hipMemcpyAsync(row.data(), e->d_seen.as<uint64_t>() + d.wbase + static_cast<uint64_t>(u) * d.W,
                           d.W * 8ull, hipMemcpyDeviceToHost, e->stream),
            "read seen row");
  }
  HIP_TRY(hipMemcpyAsync(&g, e->d_gen.as<uint8_t>() + d.nbase + u, 1, hipMemcpyDeviceToHost, e->stream),
          "read generation");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  if (!(d.flags & kTopicMesh) && g != e->gen_cur) return PS_OK;  // stale row: saw nothing
  // window slot li -> message: the window holds the topic's ranks
  // [last_lo, last_lo + last_cnt)
  const uint32_t lo = e->last_lo[topic], cnt = e->last_cnt[topic];
  std::vector<std::pair<uint64_t, uint32_t>> got;  // (start round << 32 | id, id)
  for (uint32_t i = 0; i < e->last_n; ++i) {
    if (e->last_msgs[i].topic != topic) continue;
    const uint32_t r = e->run_rank[i];
    if (r < lo || r >= lo + cnt) continue;
    const uint32_t li = r - lo;
    const uint32_t b = topic < e->last_pos.size() && !e->last_pos[topic].empty() ? e->last_pos[topic][li] : li;
    if (row[b >> 6] >> (b & 63) & 1ull)
      got.emplace_back((static_cast<uint64_t>(e->last_msgs[i].start) << 32) | i, e->last_first + i);
  }
  // arrival order: paced messages by entry round, then publish order
  std::sort(got.begin(), got.end());
  *n_out = got.size();
  if (got.size() > cap) return e->fail(PS_E_RANGE, "output buffer too small");
  for (size_t k = 0; k < got.size(); ++k) msg_out[k] = got[k].second;
  return PS_OK;
}

int ps_seen_digest(ps_engine* e, uint64_t* digest_out) {
  if (!e || !digest_out) return PS_E_INVAL;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  HIP_TRY(hipMemsetAsync(e->d_digest.p, 0, 8, e->stream), "clear digest");
  HIP_TRY(launch_digest(e->d_seen.as<uint64_t>(), e->d_gen.as<uint8_t>(), e->gen_cur,
                        e->d_node_peer.as<uint32_t>(),
                        e->d_node_topic.as<uint16_t>(), e->d_topics.as<TopicDev>(), e->d_groups.as<GroupDev>(),
                        e->n_nodes,
                        e->d_digest.as<uint64_t>(), e->stream),
          "digest");
  HIP_TRY(hipMemcpyAsync(digest_out, e->d_digest.p, 8, hipMemcpyDeviceToHost, e->stream),
          "read digest");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  return PS_OK;
}

int ps_dist_unique_id(uint8_t id_out[PS_UNIQUE_ID_BYTES]) {
  if (!id_out) return PS_E_INVAL;
  return rccl_unique_id(id_out) == 0 ? PS_OK : PS_E_DEVICE;
}

static int dist_common(ps_engine* e, const ps_dist_config* dc) {
  if (!e || !dc) return PS_E_INVAL;
  if (dc->world < 1 || dc->world > kMaxRanks || dc->rank < 0 || dc->rank >= dc->world)
    return e->fail(PS_E_INVAL, "rank/world out of range (world <= 16)");
  if (dc->partition != PS_PART_PEER && dc->partition != PS_PART_SUBTREE)
    return e->fail(PS_E_INVAL, "unknown partition");
  if (!e->pending.empty()) return e->fail(PS_E_STATE, "messages pending");
  e->rank = dc->rank;
  e->world = dc->world;
  e->partition = dc->partition;
  e->split_depth = dc->split_depth;
  e->graph_dirty = true;
  return PS_OK;
}

int ps_dist_init(ps_engine* e, const ps_dist_config* dc, const uint8_t id[PS_UNIQUE_ID_BYTES]) {
  if (!id) return PS_E_INVAL;
  int rc = dist_common(e, dc);
  if (rc) return rc;
  if (dc->world == 1) return PS_OK;
  if (hipSetDevice(e->cfg.device) != hipSuccess) return e->fail(PS_E_DEVICE, "hipSetDevice");
  std::string err;
  e->transport = make_rccl_transport(dc->rank, dc->world, id, &err);
  if (!e->transport) return e->fail(PS_E_DEVICE, err);
  return PS_OK;
}

struct ps_loopback {
  psamd::LoopbackGroup* g;
};

int ps_loopback_create(int32_t world, ps_loopback** out) {
  if (!out || world < 1 || world > kMaxRanks) return PS_E_INVAL;
  auto* lb = new (std::nothrow) ps_loopback{loopback_create(world)};
  if (!lb || !lb->g) {
    delete lb;
    return PS_E_NOMEM;
  }
  *out = lb;
  return PS_OK;
}

void ps_loopback_destroy(ps_loopback* lb) {
  if (!lb) return;
  loopback_destroy(lb->g);
  delete lb;
}

int ps_dist_init_loopback(ps_engine* e, const ps_dist_config* dc, ps_loopback* lb) {
  if (!lb) return PS_E_INVAL;
  int rc = dist_common(e, dc);
  if (rc) return rc;
  if (dc->world == 1) return PS_OK;
  e->transport = make_loopback_transport(lb->g, dc->rank, e->cfg.device);
  if (!e->transport) return e->fail(PS_E_INVAL, "loopback group size != world");
  return PS_OK;
}

int ps_partition_owner(uint32_t n_peers, uint32_t root, const uint32_t* parent, uint32_t topic,
                       const ps_dist_config* dc, int32_t* owner_out) {
  if (!parent || !dc || !owner_out || root >= n_peers) return PS_E_INVAL;
  if (dc->world < 1 || dc->world > kMaxRanks) return PS_E_INVAL;
  // children lists, then the same BFS the engine uses
  std::vector<uint32_t> rp(n_peers + 1, 0), cl;
  for (uint32_t c = 0; c < n_peers; ++c)
    if (parent[c] != PS_NONE && c != root) {
      if (parent[c] >= n_peers) return PS_E_INVAL;
      rp[parent[c] + 1]++;
    }
  for (uint32_t i = 0; i < n_peers; ++i) rp[i + 1] += rp[i];
  cl.assign(rp[n_peers], 0);
  {
    std::vector<uint32_t> fill(rp.begin(), rp.end() - 1);
    for (uint32_t c = 0; c < n_peers; ++c)
      if (parent[c] != PS_NONE && c != root) cl[fill[parent[c]]++] = c;
  }
  std::vector<uint32_t> order{root}, bfs_parent{kNone}, level{0}, local(n_peers, kNone);
  local[root] = 0;
  for (size_t qi = 0; qi < order.size(); ++qi)
    for (uint32_t k = rp[order[qi]]; k < rp[order[qi] + 1]; ++k)
      if (local[cl[k]] == kNone) {
        local[cl[k]] = static_cast<uint32_t>(order.size());
        order.push_back(cl[k]);
        bfs_parent.push_back(static_cast<uint32_t>(qi));
        level.push_back(level[qi] + 1);
      }
  std::vector<int32_t> owner;
  partition_topic(order, bfs_parent, level, topic, dc->world, dc->partition, dc->split_depth, owner);
  for (uint32_t p = 0; p < n_peers; ++p) owner_out[p] = -1;
  for (size_t u = 0; u < order.size(); ++u) owner_out[order[u]] = owner[u];
  return PS_OK;
}

}  // extern "C"
