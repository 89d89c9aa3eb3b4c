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
#include <string>
#include <vector>

#include "kernels.hpp"
#include "psengine.h"
#include "tree.hpp"

using namespace psamd;

namespace {

constexpr uint32_t kMaxRoundsCap = 4096;
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
  std::vector<uint32_t> level_internal;  // BFS level -> nodes with children
};

struct RunMsg {
  uint32_t topic;
  uint32_t start;
};

struct WindowMsg {
  uint32_t run_idx;  // index into the run's message list
  uint32_t local;    // bit index within the topic's window block
};

uint32_t ceil_div(uint64_t a, uint64_t b) { return static_cast<uint32_t>((a + b - 1) / b); }

}  // namespace

struct ps_engine {
  ps_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev_run0 = nullptr, ev_run1 = nullptr;
  std::vector<hipEvent_t> ev_k;  // pairs around expand launches
  uint32_t n_cus = 256, expand_grid = 2048;

  std::vector<TopicHost> topics;
  std::vector<uint8_t> live;
  bool graph_dirty = true, flags_dirty = true;

  // fused node space (host mirror)
  uint32_t n_nodes = 0, n_pad = 16;
  std::vector<uint32_t> node_peer, row_ptr, col;
  std::vector<uint16_t> node_topic;
  std::vector<uint8_t> node_flags;

  DevBuf d_row_ptr, d_col, d_node_topic, d_node_flags, d_node_peer;
  DevBuf d_seen, d_arr0, d_arr1, d_hop, d_flags, d_blk, d_gen, d_frontier, d_nfront, d_wgcount,
      d_partials, d_stats, d_topics, d_seeds, d_digest;
  uint32_t gen_cur = 0;  // window generation stamped into d_gen (1..255)

  // publishes not yet run
  std::vector<RunMsg> pending;
  uint32_t next_msg = 0;

  // results of the last run
  uint32_t last_first = 0, last_n = 0;
  bool have_hops = false;
  std::vector<uint8_t> hops;  // [msg][peer]
  std::vector<RunMsg> last_msgs;
  std::vector<int32_t> last_win_local;  // per run msg: bit index in the last window, -1 if not there
  std::vector<TopicDev> last_topics;
  bool have_window = false;

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

// Builds the fused node space: per topic, the nodes reachable from the root
// in BFS order (siblings contiguous, root = first node), CSR over node ids.
int build_graph(ps_engine* e) {
  const uint32_t n = e->cfg.n_peers;
  e->node_peer.clear();
  e->node_topic.clear();
  e->row_ptr.assign(1, 0);
  e->col.clear();
  std::vector<uint32_t> local(n, kNone);
  std::vector<uint32_t> rp, cl, order, indeg;
  uint64_t n_total = 0;
  for (uint32_t t = 0; t < e->topics.size(); ++t) {
    TopicHost& T = e->topics[t];
    T.nbase = static_cast<uint32_t>(n_total);
    T.n_nodes = 0;
    T.depth = 0;
    T.mesh = false;
    if (!T.exists) continue;
    peer_children(e, T, rp, cl);
    order.clear();
    order.push_back(T.root);
    local[T.root] = 0;
    size_t level_end = 1;
    uint32_t depth = 0;
    for (size_t qi = 0; qi < order.size(); ++qi) {
      if (qi == level_end) {
        level_end = order.size();
        ++depth;
      }
      const uint32_t p = order[qi];
      for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
        const uint32_t c = cl[k];
        if (c >= n) return e->fail(PS_E_INVAL, "child id out of range");
        if (local[c] == kNone) {
          local[c] = static_cast<uint32_t>(order.size());
          order.push_back(c);
        }
      }
    }
    if (order.size() > level_end) ++depth;
    T.depth = depth;
    // internal nodes per BFS level: bounds the frontier of every round
    T.level_internal.assign(depth + 1, 0);
    {
      std::vector<uint32_t> lvl(order.size(), 0);
      for (uint32_t u = 0; u < order.size(); ++u) {
        const uint32_t p = order[u];
        bool internal = false;
        for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
          const uint32_t lc = local[cl[k]];
          if (lc > u && lvl[lc] == 0) lvl[lc] = lvl[u] + 1;  // BFS discovery
          internal = true;
        }
        if (internal) T.level_internal[lvl[u]]++;
      }
    }
    T.n_nodes = static_cast<uint32_t>(order.size());
    if (n_total + order.size() >= 0xFFFFFFF0ull)
      return e->fail(PS_E_NOMEM, "node space exceeds 2^32 nodes");
    indeg.assign(order.size(), 0);
    for (uint32_t u = 0; u < order.size(); ++u) {
      const uint32_t p = order[u];
      e->node_peer.push_back(p);
      e->node_topic.push_back(static_cast<uint16_t>(t));
      for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
        const uint32_t lc = local[cl[k]];
        e->col.push_back(T.nbase + lc);
        indeg[lc]++;
      }
      e->row_ptr.push_back(static_cast<uint32_t>(e->col.size()));
      if (e->col.size() >= 0xFFFFFFF0ull) return e->fail(PS_E_NOMEM, "edge space exceeds 2^32");
    }
    for (uint32_t u = 0; u < order.size(); ++u)
      if (indeg[u] > (u == 0 ? 0u : 1u)) T.mesh = true;
    for (uint32_t p : order) local[p] = kNone;
    n_total += order.size();
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
    e->node_flags[u] = f;
  }
  for (const auto& T : e->topics)
    if (T.exists && T.n_nodes) e->node_flags[T.nbase] |= kNodeLive;  // roots always forward
}

int upload_graph(ps_engine* e) {
  if (e->graph_dirty) {
    int rc = build_graph(e);
    if (rc) return rc;
    const size_t nn = e->n_nodes;
    HIP_TRY(e->d_row_ptr.ensure((nn + 1) * 4), "alloc row_ptr");
    HIP_TRY(e->d_col.ensure(std::max<size_t>(e->col.size(), 1) * 4), "alloc col");
    HIP_TRY(e->d_node_topic.ensure(std::max<size_t>(nn, 1) * 2), "alloc node_topic");
    HIP_TRY(e->d_node_peer.ensure(std::max<size_t>(nn, 1) * 4), "alloc node_peer");
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
    }
    bool fresh = false;
    const size_t flag_bytes = static_cast<size_t>(ceil_div(e->n_pad, kFlagsPerBlock)) * kFlagsPerBlock;
    HIP_TRY(e->d_flags.ensure(flag_bytes, &fresh), "alloc flags");
    HIP_TRY(hipMemsetAsync(e->d_flags.p, 0, e->d_flags.bytes, e->stream), "clear flags");
    const size_t n_blk = ceil_div(e->n_pad, kFlagsPerBlock);
    HIP_TRY(e->d_blk.ensure(n_blk), "alloc block flags");
    HIP_TRY(hipMemsetAsync(e->d_blk.p, 0, e->d_blk.bytes, e->stream), "clear block flags");
    HIP_TRY(e->d_gen.ensure(e->n_pad + 16), "alloc generations");
    HIP_TRY(hipMemsetAsync(e->d_gen.p, 0, e->d_gen.bytes, e->stream), "clear generations");
    e->gen_cur = 0;  // node ids changed: every row is stale
    HIP_TRY(e->d_frontier.ensure(std::max<size_t>(nn, 1) * 4), "alloc frontier");
    HIP_TRY(e->d_wgcount.ensure(static_cast<size_t>(ceil_div(e->n_pad, kFlagsPerBlock)) * 4),
            "alloc wg_count");
    e->graph_dirty = false;
    e->flags_dirty = true;
    e->have_window = false;  // the node space of the last window is gone
  }
  if (e->flags_dirty) {
    build_flags(e);
    if (e->n_nodes)
      HIP_TRY(hipMemcpyAsync(e->d_node_flags.p, e->node_flags.data(), e->n_nodes, hipMemcpyHostToDevice, e->stream),
              "upload node_flags");
    e->flags_dirty = false;
  }
  // host mirrors may be rebuilt by the next call: finish the uploads now
  HIP_TRY(hipStreamSynchronize(e->stream), "sync uploads");
  return PS_OK;
}

// Propagates one window: per topic t, win[t] lists the messages (indices into
// `msgs`) whose bits form t's block of W_t = ceil(|win[t]|/64) words.
int run_window(ps_engine* e, const std::vector<RunMsg>& msgs,
               const std::vector<std::vector<uint32_t>>& win, ps_stats* st) {
  int rc = upload_graph(e);
  if (rc) return rc;
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  std::vector<TopicDev> tab(std::max<uint32_t>(nt, 1));
  uint64_t wtot = 0;
  uint32_t max_depth = 0, max_start = 0;
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicHost& T = e->topics[t];
    TopicDev& d = tab[t];
    d = TopicDev{};
    d.nbase = T.nbase;
    d.n_nodes = T.n_nodes;
    d.flags = T.mesh ? kTopicMesh : 0;
    if (!T.exists || win[t].empty() || T.n_nodes == 0) continue;
    d.W = ceil_div(win[t].size(), 64);
    d.w_msgs = d.W;
    // rows of >= 64 words are padded to an even length so that every row
    // starts 16-B aligned (the expand kernel stores them as dwordx4)
    if (d.W >= 64) d.W += d.W & 1u;
    wtot = (wtot + 15) & ~15ull;  // topic blocks start on a 128-B line
    d.wbase = wtot;
    wtot += static_cast<uint64_t>(T.n_nodes) * d.W;
    max_depth = std::max(max_depth, T.depth);
    for (uint32_t i : win[t]) max_start = std::max(max_start, msgs[i].start);
  }
  if (wtot == 0) return PS_OK;
  const bool record = (e->cfg.flags & PS_F_RECORD_HOPS) != 0;
  HIP_TRY(e->d_seen.ensure(wtot * 8), "alloc seen");
  HIP_TRY(e->d_arr0.ensure(wtot * 8), "alloc arrivals");
  HIP_TRY(e->d_arr1.ensure(wtot * 8), "alloc arrivals");
  bool any_mesh = false;
  for (uint32_t t = 0; t < nt; ++t) any_mesh |= (tab[t].W && (tab[t].flags & kTopicMesh));
  if (record) HIP_TRY(e->d_hop.ensure(wtot * 64), "alloc hop record");
  const uint32_t n_waves = e->expand_grid * (kBlock / 64);
  HIP_TRY(e->d_partials.ensure(static_cast<size_t>(n_waves) * kNumCtr * 8), "alloc partials");
  HIP_TRY(e->d_stats.ensure(static_cast<size_t>(kMaxRoundsCap + 1) * kNumCtr * 8), "alloc stats");
  HIP_TRY(e->d_topics.ensure(tab.size() * sizeof(TopicDev)), "alloc topics");
  HIP_TRY(e->d_nfront.ensure(4), "alloc n_front");

  // root injections, grouped by round: mask[t][round][word]
  std::vector<std::vector<uint64_t>> inj(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicDev& d = tab[t];
    if (d.W == 0) continue;
    inj[t].assign(static_cast<size_t>(max_start + 1) * d.W, 0);
    for (uint32_t li = 0; li < win[t].size(); ++li)
      inj[t][static_cast<size_t>(msgs[win[t][li]].start) * d.W + (li >> 6)] |= 1ull << (li & 63);
  }
  std::vector<SeedDev> seeds;
  std::vector<uint32_t> seed_off(max_start + 2, 0);
  for (uint32_t r = 0; r <= max_start; ++r) {
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicDev& d = tab[t];
      for (uint32_t w = 0; w < d.W; ++w) {
        const uint64_t m = inj[t][static_cast<size_t>(r) * d.W + w];
        if (m) seeds.push_back(SeedDev{d.wbase + w, m, d.nbase, 0});  // root = node 0
      }
    }
    seed_off[r + 1] = static_cast<uint32_t>(seeds.size());
  }
  HIP_TRY(e->d_seeds.ensure(seeds.size() * sizeof(SeedDev)), "alloc seeds");

  // Upper bound of the frontier expanded in round r (tree topics: a node at
  // BFS level d receives a message started at round s in round s + d), used
  // to size each round's grid; mesh topics (paths lengthen under the live
  // mask) use the full grid.
  bool any_mesh_active = false;
  std::vector<std::vector<uint8_t>> starts_of(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    if (tab[t].W == 0) continue;
    if (e->topics[t].mesh) any_mesh_active = true;
    starts_of[t].assign(max_start + 1, 0);
    for (uint32_t i : win[t]) starts_of[t][msgs[i].start] = 1;
  }
  auto round_grid = [&](uint32_t r) -> uint32_t {
    if (any_mesh_active) return e->expand_grid;
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

  hipStream_t s = e->stream;
  HIP_TRY(hipMemcpyAsync(e->d_topics.p, tab.data(), tab.size() * sizeof(TopicDev),
                         hipMemcpyHostToDevice, s),
          "upload topics");
  HIP_TRY(hipMemcpyAsync(e->d_seeds.p, seeds.data(), seeds.size() * sizeof(SeedDev),
                         hipMemcpyHostToDevice, s),
          "upload seeds");
  HIP_TRY(hipEventRecord(e->ev_run0, s), "event");
  // new window generation: every tree row from older windows becomes stale
  if (++e->gen_cur > 255) {
    HIP_TRY(hipMemsetAsync(e->d_gen.p, 0, e->d_gen.bytes, s), "clear generations");
    e->gen_cur = 1;
  }
  HIP_TRY(launch_window_init(e->d_topics.as<TopicDev>(), nt, e->d_seen.as<uint64_t>(),
                             e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>(),
                             e->d_gen.as<uint8_t>(), e->gen_cur, any_mesh, s),
          "window init");
  if (e->cfg.flags & PS_F_NO_LAZY_SEEN) {
    // eager variant: clear every row and mark every node current, so the
    // expand kernel reads each child's seen word before it tests and sets it
    HIP_TRY(hipMemsetAsync(e->d_seen.p, 0, wtot * 8, s), "clear seen");
    HIP_TRY(hipMemsetAsync(e->d_gen.p, static_cast<int>(e->gen_cur), e->d_gen.bytes, s),
            "stamp generations");
  }
  if (record) HIP_TRY(hipMemsetAsync(e->d_hop.p, 0xFF, wtot * 64, s), "clear hop record");

  ExpandArgs a{};
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
  a.dbg = 0;
  if (const char* v = std::getenv("PSAMD_DEBUG_EXPAND")) a.dbg = static_cast<uint32_t>(std::atoi(v));
  a.partials = e->d_partials.as<uint64_t>();
  a.hop_rec = record ? e->d_hop.as<uint8_t>() : nullptr;
  uint64_t* arr[2] = {e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>()};
  uint64_t* stats = e->d_stats.as<uint64_t>();
  const bool timed = (e->cfg.flags & PS_F_TIME_KERNELS) != 0;

  auto seed_round = [&](uint32_t r, uint64_t* into) -> hipError_t {
    if (r > max_start) return hipSuccess;
    return launch_seed(e->d_seeds.as<SeedDev>(), seed_off[r], seed_off[r + 1], into,
                       a.seen, a.next_flag, a.blk_flag, s);
  };
  auto compact = [&](uint32_t r, uint32_t waves_r) -> hipError_t {
    hipError_t x = launch_flag_count(a.next_flag, a.blk_flag, e->n_pad,
                                     e->d_wgcount.as<uint32_t>(), a.partials, waves_r,
                                     r ? stats + r * kNumCtr : nullptr, s);
    if (x != hipSuccess) return x;
    return launch_flag_compact(a.next_flag, a.blk_flag, e->n_pad, e->d_wgcount.as<uint32_t>(),
                               e->d_frontier.as<uint32_t>(), e->d_nfront.as<uint32_t>(), s);
  };

  HIP_TRY(seed_round(0, arr[0]), "seed");
  HIP_TRY(compact(0, 0), "compact");
  uint32_t planned = max_depth + max_start + 1;
  uint32_t r = 0;
  size_t ev_used = 0;
  while (true) {
    for (; r < planned && r < kMaxRoundsCap; ) {
      ++r;
      a.a_cur = arr[(r - 1) & 1];
      a.a_next = arr[r & 1];
      if (timed) {
        if (ev_used + 2 > e->ev_k.size()) {
          hipEvent_t x, y;
          HIP_TRY(hipEventCreate(&x), "event");
          HIP_TRY(hipEventCreate(&y), "event");
          e->ev_k.push_back(x);
          e->ev_k.push_back(y);
        }
        HIP_TRY(hipEventRecord(e->ev_k[ev_used], s), "event");
      }
      const uint32_t grid_r = r <= planned ? round_grid(r) : e->expand_grid;
      HIP_TRY(launch_expand(a, r, record, grid_r, s), "expand");
      if (timed) HIP_TRY(hipEventRecord(e->ev_k[ev_used + 1], s), "event");
      if (timed) ev_used += 2;
      HIP_TRY(seed_round(r, a.a_next), "seed");
      HIP_TRY(compact(r, grid_r * (kBlock / 64)), "compact");
    }
    uint32_t left = 0;
    HIP_TRY(hipMemcpyAsync(&left, e->d_nfront.p, 4, hipMemcpyDeviceToHost, s), "read frontier");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    if (left == 0 || r >= kMaxRoundsCap) {
      if (left) return e->fail(PS_E_STATE, "propagation did not converge");
      break;
    }
    planned = r + 8;  // live mask lengthened a mesh path beyond the BFS depth
  }
  HIP_TRY(hipEventRecord(e->ev_run1, s), "event");
  HIP_TRY(hipEventSynchronize(e->ev_run1), "sync");
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e->ev_run0, e->ev_run1), "elapsed");
  st->run_ms += ms;
  for (size_t i = 0; i < ev_used; i += 2) {
    float k = 0.f;
    HIP_TRY(hipEventElapsedTime(&k, e->ev_k[i], e->ev_k[i + 1]), "elapsed");
    st->expand_ms += k;
    const size_t q = i / 2 + 1;  // round of this launch
    if (q < PS_MAX_ROUNDS) st->expand_ms_per_round[q] += k;
  }
  std::vector<uint64_t> hs(static_cast<size_t>(r + 1) * kNumCtr);
  HIP_TRY(hipMemcpyAsync(hs.data(), stats, hs.size() * 8, hipMemcpyDeviceToHost, s), "read stats");
  HIP_TRY(hipStreamSynchronize(s), "sync");
  for (uint32_t q = 1; q <= r; ++q) {
    const uint64_t* c = &hs[static_cast<size_t>(q) * kNumCtr];
    st->deliveries += c[kCtrDeliveries];
    st->duplicates += c[kCtrDuplicates];
    st->frontier_entries += c[kCtrEntries];
    st->child_visits += c[kCtrChildren];
    st->edge_words += c[kCtrSeenWrites];
    // algorithmic bytes of the expand kernel (DESIGN.md §5.1 byte model):
    // per entry frontier id 4 + topic 2 + row_ptr pair 8 + first child 4;
    // per entry word the arrival read 8 (+ 8 when cleared); per child its
    // flag byte + generation read/write (tree) or col id 4 (mesh); per
    // seen read / seen write / arrival write 8.
    st->expand_bytes += c[kCtrEntries] * 18 + c[kCtrEntryWords] * 8 + c[kCtrClearWords] * 8 +
                        c[kCtrChildren] * 3 + c[kCtrMeshChildren] * 4 + c[kCtrSeenReads] * 8 +
                        c[kCtrSeenWrites] * 8 + c[kCtrArrivalWrites] * 8;
    if (q < PS_MAX_ROUNDS) {
      st->deliveries_per_round[q] += c[kCtrDeliveries];
      st->frontier_per_round[q] += static_cast<uint32_t>(c[kCtrEntries]);
    }
  }
  st->rounds += r;
  st->expand_launches += r;
  st->windows += 1;

  if (record) {
    std::vector<uint8_t> hr(wtot * 64);
    HIP_TRY(hipMemcpyAsync(hr.data(), e->d_hop.p, hr.size(), hipMemcpyDeviceToHost, s), "read hops");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    const uint32_t np = e->cfg.n_peers;
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicDev& d = tab[t];
      if (d.W == 0) continue;
      for (uint32_t li = 0; li < win[t].size(); ++li) {
        const uint32_t mi = win[t][li];
        const uint32_t s0 = msgs[mi].start;
        uint8_t* row = e->hops.data() + static_cast<size_t>(mi) * np;
        for (uint32_t u = 0; u < d.n_nodes; ++u) {
          const uint8_t v = hr[(d.wbase + static_cast<uint64_t>(u) * d.W + (li >> 6)) * 64 + (li & 63)];
          if (v != 0xFF) row[e->node_peer[d.nbase + u]] = static_cast<uint8_t>(v - s0);
        }
      }
    }
  }
  // remember the last window for ps_read_delivered / ps_seen_digest
  e->last_topics = tab;
  std::fill(e->last_win_local.begin(), e->last_win_local.end(), -1);
  for (uint32_t t = 0; t < nt; ++t)
    for (uint32_t li = 0; li < win[t].size(); ++li) e->last_win_local[win[t][li]] = static_cast<int32_t>(li);
  e->have_window = true;
  return PS_OK;
}

// Messages of one phase, split into windows of at most msg_window per topic.
int run_phase(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<uint32_t>& idx,
              ps_stats* st) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  std::vector<std::vector<uint32_t>> per(nt);
  for (uint32_t i : idx) per[msgs[i].topic].push_back(i);
  const uint32_t cap = e->cfg.msg_window;
  size_t n_win = 0;
  for (const auto& v : per) n_win = std::max(n_win, (v.size() + cap - 1) / cap);
  std::vector<std::vector<uint32_t>> win(nt);
  for (size_t k = 0; k < n_win; ++k) {
    for (uint32_t t = 0; t < nt; ++t) {
      win[t].clear();
      const size_t lo = k * cap, hi = std::min(per[t].size(), lo + cap);
      for (size_t q = lo; q < hi; ++q) win[t].push_back(per[t][q]);
    }
    int rc = run_window(e, msgs, win, st);
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
  // which admits 6 (MI355X_MICROARCH.md §Residency); PSAMD_EXPAND_BPC overrides
  uint32_t bpc = 6;
  if (const char* v = std::getenv("PSAMD_EXPAND_BPC")) bpc = std::max(1, std::atoi(v));
  e->expand_grid = e->n_cus * bpc;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e->ev_run0) != hipSuccess || hipEventCreate(&e->ev_run1) != hipSuccess) {
    delete e;
    return PS_E_DEVICE;
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
  for (size_t i = 0; i < n; ++i) {
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
  for (size_t i = 0; i < n; ++i)
    e->pending.push_back(RunMsg{topic_of_msg[i], start_round ? start_round[i] : 0u});
  e->next_msg += static_cast<uint32_t>(n);
  return PS_OK;
}

int ps_publish(ps_engine* e, const uint32_t* topic_of_msg, size_t n, uint32_t* first) {
  return ps_publish_at(e, topic_of_msg, nullptr, n, first);
}

int ps_run(ps_engine* e, ps_stats* out) {
  if (!e) return PS_E_INVAL;
  const auto t_host0 = std::chrono::steady_clock::now();
  ps_stats st{};
  if (hipSetDevice(e->cfg.device) != hipSuccess) return e->fail(PS_E_DEVICE, "hipSetDevice");
  std::vector<RunMsg> msgs;
  msgs.swap(e->pending);
  const uint32_t nmsg = static_cast<uint32_t>(msgs.size());
  e->last_first = e->next_msg - nmsg;
  e->last_n = nmsg;
  e->last_msgs = msgs;
  e->last_win_local.assign(nmsg, -1);
  e->have_hops = false;
  e->have_window = false;
  const bool record = (e->cfg.flags & PS_F_RECORD_HOPS) != 0;
  if (record) {
    const uint64_t bytes = static_cast<uint64_t>(nmsg) * e->cfg.n_peers;
    if (bytes > (8ull << 30)) return e->fail(PS_E_NOMEM, "hop record larger than 8 GiB");
    e->hops.assign(bytes, PS_HOP_NONE);
  }
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  std::vector<std::vector<uint32_t>> queue(nt);
  for (uint32_t i = 0; i < nmsg; ++i) queue[msgs[i].topic].push_back(i);
  std::vector<size_t> head(nt, 0);
  // Abruptly dropped hosts: the first message through the failed edge is lost
  // below it, then the parent repairs (subtree.go:333-351): that message runs
  // on its own over the current tree, the rest over the repaired one.
  while (true) {
    std::vector<uint32_t> solo;
    for (uint32_t t = 0; t < nt; ++t) {
      TopicHost& T = e->topics[t];
      if (T.exists && T.kind == Kind::Join && T.tree.has_pending_failures() &&
          head[t] < queue[t].size())
        solo.push_back(queue[t][head[t]++]);
    }
    if (solo.empty()) break;
    int rc = run_phase(e, msgs, solo, &st);
    if (rc) return rc;
    for (uint32_t i : solo) {
      e->topics[msgs[i].topic].tree.after_message();
      e->graph_dirty = true;
    }
  }
  std::vector<uint32_t> rest;
  rest.reserve(nmsg);
  {
    std::vector<size_t> seen_in_topic(nt, 0);  // publish order, minus the solo'd heads
    for (uint32_t i = 0; i < nmsg; ++i)
      if (seen_in_topic[msgs[i].topic]++ >= head[msgs[i].topic]) rest.push_back(i);
  }
  if (!rest.empty()) {
    int rc = run_phase(e, msgs, rest, &st);
    if (rc) return rc;
  }
  // lazy prune of Part'ed children at every forwarding node (subtree.go:326-331)
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    if (T.exists && T.kind == Kind::Join && head[t] < queue[t].size() &&
        T.tree.needs_message_pass()) {
      T.tree.after_message();
      e->graph_dirty = true;
    }
  }
  e->have_hops = record;
  st.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
  if (out) *out = st;
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
  const int32_t li = e->last_win_local[i];
  if (li < 0) return e->fail(PS_E_NOTREADY, "message not in the last window");
  const uint32_t t = e->last_msgs[i].topic;
  const TopicDev& d = e->last_topics[t];
  std::memset(out, 0, e->cfg.n_peers);
  std::vector<uint64_t> col(d.n_nodes);
  // one word per node: strided copy of this message's word column
  HIP_TRY(hipMemcpy2DAsync(col.data(), 8, e->d_seen.as<uint64_t>() + d.wbase + (li >> 6),
                           d.W * 8ull, 8, d.n_nodes, hipMemcpyDeviceToHost, e->stream),
          "read seen");
  std::vector<uint8_t> gen(d.n_nodes);
  HIP_TRY(hipMemcpyAsync(gen.data(), e->d_gen.as<uint8_t>() + d.nbase, d.n_nodes,
                         hipMemcpyDeviceToHost, e->stream),
          "read generations");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  const bool mesh = (d.flags & kTopicMesh) != 0;
  const uint64_t bit = 1ull << (li & 63);
  for (uint32_t u = 1; u < d.n_nodes; ++u)  // the root is not a recipient
    if ((mesh || gen[u] == e->gen_cur) && (col[u] & bit)) out[e->node_peer[d.nbase + u]] = 1;
  return PS_OK;
}

int ps_seen_digest(ps_engine* e, uint64_t* digest_out) {
  if (!e || !digest_out) return PS_E_INVAL;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  HIP_TRY(hipMemsetAsync(e->d_digest.p, 0, 8, e->stream), "clear digest");
  HIP_TRY(launch_digest(e->d_seen.as<uint64_t>(), e->d_gen.as<uint8_t>(), e->gen_cur,
                        e->d_node_peer.as<uint32_t>(),
                        e->d_node_topic.as<uint16_t>(), e->d_topics.as<TopicDev>(), e->n_nodes,
                        e->d_digest.as<uint64_t>(), e->stream),
          "digest");
  HIP_TRY(hipMemcpyAsync(digest_out, e->d_digest.p, 8, hipMemcpyDeviceToHost, e->stream),
          "read digest");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  return PS_OK;
}

}  // extern "C"
