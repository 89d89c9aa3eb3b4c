// plan.cpp -- one window's layout and launch plans.  Pure
// host code: nothing here touches the device, so the plans are unit-tested on
// the CPU through the planner probe (include/psengine_plan.h); run.cpp uploads
// them and drives the rounds.
#include <algorithm>
#include <cstring>

#include "engine.hpp"

namespace psamd {

uint64_t phys_word(const TopicDev& d, const std::vector<StartGroup>& G, uint64_t u, uint32_t w) {
  if (!(d.flags & kTopicGroups)) return d.wbase + u * d.W + w;
  for (const StartGroup& g : G)
    if (w < g.w0 + g.wn) return d.wbase + static_cast<uint64_t>(d.n_nodes) * g.w0 + u * g.wn + (w - g.w0);
  return d.wbase;  // (w < W always)
}

namespace {

// the row block a topic's start group g is written in: (width, word offset
// of the topic's first node's block)
uint32_t block_w(const TopicDev& d, const StartGroup& g) { return (d.flags & kTopicGroups) ? g.wn : d.W; }
uint64_t block_row0(const TopicDev& d, const StartGroup& g) {
  return d.wbase + ((d.flags & kTopicGroups) ? static_cast<uint64_t>(d.n_nodes) * g.w0 : 0);
}

}  // namespace

// Per topic t the window's messages win[t] (indices into msgs) form the
// topic's block of W_t = ceil(|win[t]| / 64) words per node -- or, when they
// start in several rounds, one even-length block per start round (start
// groups).  Every rank computes the same widths, rounds and start groups from
// the messages alone (also a rank that owns none of a topic's nodes: its tab
// entry stays idle, W = 0, while wglob keeps the width cross-rank sizes use).
int plan_window_layout(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<WinSlice>& win,
                       WindowLayout& L) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  L = WindowLayout{};
  L.tab.assign(std::max<uint32_t>(nt, 1), TopicDev{});
  L.groups.assign(std::max<uint32_t>(nt, 1), {});
  L.pos.assign(std::max<uint32_t>(nt, 1), {});
  L.tstart.assign(std::max<uint32_t>(nt, 1), 0);
  L.wglob.assign(std::max<uint32_t>(nt, 1), 0);
  L.need_direct = e->world > 1;
  // Level-aligned start groups (one rank, ps_plan_opts.align_groups).  In a
  // tree window, messages published in different rounds are independent:
  // the tree and the live mask do not change inside a window, so a message
  // published in round s reaches the same peers at the same hops as one
  // published in round 0, s rounds later (hop = depth, client.go:100-132).
  // Its topic's row is then the burst's row -- node-major, one bit per
  // message, the bits sorted by start round -- and the window runs the
  // burst's schedule over the BFS levels (every start taken as round 0).
  // Only the observable rounds differ: round s + d delivers level d of the
  // messages starting in s.  The per-round counters are split after the
  // window from each (topic, level)'s reached and frontier nodes
  // (k_level_reach, checked against the kernels' per-level counters).  The
  // reach rows ride in the window's counter reduce and must fit a run
  // slot's pinned rows.
  bool align = false;
  if (e->world == 1 && e->align_groups && !e->run_zero_start && !(e->cfg.flags & PS_F_COMPACT)) {
    bool multi = false, mesh = false;
    uint64_t segs = 0;
    uint32_t depth = 0;
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (!T.exists || win[t].n == 0) continue;
      mesh |= T.mesh;
      const uint32_t s0 = msgs[win[t].idx[0]].start;
      for (uint32_t li = 1; li < win[t].n && !multi; ++li) multi |= msgs[win[t].idx[li]].start != s0;
      segs += T.depth + 1;
      depth = std::max(depth, T.depth);
    }
    align = multi && !mesh && depth + 2 + ceil_div(2 * segs, static_cast<uint64_t>(kNumCtr)) <= kAlignedRowsMax;
  }
  uint32_t true_max_start = 0;
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicHost& T = e->topics[t];
    TopicDev& d = L.tab[t];
    d.nbase = T.nbase;
    d.n_nodes = T.n_nodes;
    d.flags = (T.mesh ? kTopicMesh : 0u) | (T.root_local ? kTopicRootLocal : 0u);
    if (!T.exists || win[t].n == 0) continue;
    L.max_depth = std::max(L.max_depth, T.depth);  // global depth: every rank plans the same rounds
    uint32_t s_lo = ~0u, s_hi = 0;
    if (!e->run_zero_start)  // else: every message of the run starts in round 0
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t s0 = msgs[win[t].idx[li]].start;
        s_lo = std::min(s_lo, s0);
        s_hi = std::max(s_hi, s0);
      }
    if (e->run_zero_start) s_lo = s_hi = 0;
    true_max_start = std::max(true_max_start, s_hi);
    if (align) {
      // the topic's start groups over its packed row: bits by (start, window order)
      auto& G = L.split.groups;
      G.resize(nt);
      std::vector<uint32_t> cnt(s_hi - s_lo + 2, 0);
      for (uint32_t li = 0; li < win[t].n; ++li) cnt[msgs[win[t].idx[li]].start - s_lo + 1]++;
      for (uint32_t k = 0; k <= s_hi - s_lo; ++k) {
        if (cnt[k + 1]) G[t].push_back(AlignedGroup{s_lo + k, cnt[k], cnt[k + 1]});
        cnt[k + 1] += cnt[k];
      }
      if (s_lo != s_hi) {
        auto& P = L.pos[t];
        P.resize(win[t].n);
        for (uint32_t li = 0; li < win[t].n; ++li) P[li] = cnt[msgs[win[t].idx[li]].start - s_lo]++;
      }
      s_lo = s_hi = 0;  // (planned as one start, round 0)
    }
    L.max_start = std::max(L.max_start, s_hi);
    const bool one_start = s_lo == s_hi;
    L.multi |= !one_start && !T.mesh;
    // a tree topic whose window messages share one start round: every node
    // receives once, so arrival rows are its seen rows (kTopicSingleStart)
    if (one_start && !T.mesh) d.flags |= kTopicSingleStart;
    L.tstart[t] = s_lo;
    if (one_start || T.mesh) {
      d.W = ceil_div(win[t].n, 64);
      d.w_msgs = d.W;
      // rows of >= pad_words (16) words are padded to an even length so that
      // every row starts 16-B aligned (the kernels store them as dwordx4):
      // <= 1/16 more bytes against half the store instructions (cfg3 1.015
      // -> 1.003 ms/step, the 4-rank cfg4 loopback's 63-word rows 2.49x ->
      // 2.32x; profiles/r03/ab_pad.txt)
      // (16-word alignment measured no faster: profiles/r04/ab/NOTES.md)
      if (d.W >= e->pad_words) d.W = (d.W + 1) & ~1u;
      L.groups[t].push_back(StartGroup{s_lo, 0, d.W});
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
        L.groups[t].push_back(StartGroup{s_lo + k, w, wn});
        w += wn;
      }
      d.W = w;
      d.w_msgs = w;  // every block's words (padding words stay zero)
      auto& P = L.pos[t];
      P.resize(win[t].n);
      std::vector<uint32_t> fill(s_hi - s_lo + 1, 0);
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t k = msgs[win[t].idx[li]].start - s_lo;
        P[li] = wfirst[k] * 64 + fill[k]++;
      }
    }
    L.wglob[t] = d.W;
    if (T.n_nodes == 0) {
      d.W = d.w_msgs = 0;
      continue;
    }
    L.wtot = (L.wtot + 15) & ~15ull;  // topic blocks start on a 128-B line
    d.wbase = L.wtot;
    L.wtot += static_cast<uint64_t>(T.n_nodes) * d.W;
    if (T.mesh || T.max_deg > 64) L.need_direct = true;
  }
  for (uint32_t t = 0; t < nt; ++t) L.any_mesh |= (L.tab[t].W && (L.tab[t].flags & kTopicMesh));
  // no simple path is longer than a topic's peers: a window ends within
  // n_peers + the latest start round (the bound is the same on every rank)
  L.round_cap = static_cast<uint32_t>(
      std::max<uint64_t>(kMaxRoundsCap, static_cast<uint64_t>(e->cfg.n_peers) + L.max_start + 2));
  L.planned0 = L.max_depth + L.max_start + 1;
  // level mode: every active topic a tree (any rank count, start groups
  // included); PS_F_COMPACT sends every window through the compaction path
  L.level = !(e->cfg.flags & PS_F_COMPACT) && !L.any_mesh && L.planned0 + 1 < L.round_cap;
  for (uint32_t t = 0; t < nt; ++t) {
    TopicDev& d = L.tab[t];
    d.root_words = d.W;
    if (!L.level || !L.wglob[t] || L.groups[t].size() < 2) continue;
    d.flags |= kTopicGroups;  // (also an idle entry on a rank owning none of the nodes)
    d.group_lo = static_cast<uint32_t>(L.gtab.size());
    d.group_n = static_cast<uint32_t>(L.groups[t].size());
    d.root_words = L.groups[t][0].wn;
    for (const StartGroup& g : L.groups[t]) L.gtab.push_back(GroupDev{g.w0, g.wn, 0, 0});
  }
  L.true_rounds = L.planned0;
  if (align && !L.level) return e->fail(PS_E_STATE, "aligned window outside level mode");  // (unreachable)
  if (align) {
    AlignedSplit& sp = L.split;
    L.aligned = true;
    L.true_rounds = L.planned0 + true_max_start;
    sp.seg_lo.assign(nt, kNone);
    sp.seg_n.assign(nt, 0);
    for (uint32_t t = 0; t < nt; ++t) {
      if (!L.tab[t].W) continue;
      TopicDev& d = L.tab[t];
      if (sp.groups[t].size() > 1) {  // the digest's virtual group-major words
        d.flags |= kTopicPacked;
        d.group_lo = static_cast<uint32_t>(L.gtab.size());
        d.group_n = static_cast<uint32_t>(sp.groups[t].size());
        uint32_t w0 = 0;
        for (const AlignedGroup& g : sp.groups[t]) {
          const uint32_t wn = (ceil_div(g.n, 64) + 1) & ~1u;
          L.gtab.push_back(GroupDev{w0, wn, g.b0, g.n});
          w0 += wn;
        }
      }
      sp.seg_lo[t] = sp.n_segs;
      sp.seg_n[t] = e->topics[t].depth + 1;  // levels 0 .. depth
      sp.n_segs += sp.seg_n[t];
    }
    sp.row0 = L.planned0 + 1;
    sp.eager = (e->cfg.flags & PS_F_NO_LAZY_SEEN) != 0;
  } else {
    L.split = AlignedSplit{};
  }
  return PS_OK;
}

// Level mode.  In a tree window, a node at BFS level d
// receives start group g's block exactly in round s_g + d (if every ancestor
// is live), so each round writes one BFS level per (topic, group).  Per-level
// launches (k_pull): round q writes level q - s_g of every active (topic,
// group), cut into chunks of at most kPullMaxKids nodes and about pull_words
// words, one wave each.  On N ranks a level's nodes fed by a local parent
// come first (graph.cpp): their chunks are listed first in the round and run
// while the round's records are exchanged; the ghost-fed chunks follow from
// gsplit[q].  Cached: rebuilt only when the node space, the flags, the
// widths or the start rounds change.  Returns true when the plan changed.
bool plan_pull_chunks(ps_engine* e, const WindowLayout& L) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const uint32_t rounds = L.planned0;
  const auto& tab = L.tab;
  std::vector<uint64_t> key{e->graph_epoch, e->flags_epoch, rounds, e->pull_words};
  for (uint32_t t = 0; t < nt; ++t) {
    key.push_back(tab[t].W ? L.groups[t].size() : ~0ull);
    key.push_back(tab[t].W);
    key.push_back(tab[t].wbase << 1 | ((tab[t].flags & kTopicGroups) ? 1 : 0));
    if (tab[t].W)
      for (const StartGroup& g : L.groups[t]) key.push_back(static_cast<uint64_t>(g.start) << 32 | g.w0);
  }
  PullPlan& P = e->pull;
  if (key == P.key) return false;
  // parent-range staging reads the host mirror of node_parent; a GPU-built
  // node space gets the ranges on the device (run.cpp)
  const bool gpu = e->gpu_graph;
  P.key = key;
  P.chunks.clear();
  P.off.assign(rounds + 2, 0);
  P.gsplit.assign(rounds + 2, 0);
  P.bytes.assign(rounds + 2, 0);
  std::vector<PullChunk> ghost;
  auto cut = [&](std::vector<PullChunk>& out, uint32_t t, uint32_t gi, uint32_t u0, uint32_t u1, uint32_t per,
                 uint32_t W, uint64_t row0) {
    const TopicHost& T = e->topics[t];
    for (uint32_t u = u0; u < u1; u += per) {
      PullChunk c{};
      c.node_begin = T.nbase + u;
      c.node_end = T.nbase + std::min(u + per, u1);
      c.topic = t;
      c.p_lo = gpu ? kNone : e->node_parent[c.node_begin];
      c.p_hi = gpu ? kNone : e->node_parent[c.node_end - 1];
      c.W = W;
      c.row0_lo = static_cast<uint32_t>(row0);
      c.row0_hi = static_cast<uint32_t>(row0 >> 32);
      c.gin = c.gout = kNoneNode;
      c.group = gi;
      out.push_back(c);
    }
  };
  for (uint32_t q = 1; q <= rounds; ++q) {
    P.off[q] = static_cast<uint32_t>(P.chunks.size());
    ghost.clear();
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (uint32_t gi = 0; gi < L.groups[t].size(); ++gi) {
        const StartGroup& g = L.groups[t][gi];
        if (q < g.start + 1) continue;
        const uint32_t d = q - g.start;  // level of the nodes whose block g is written this round
        if (d + 1 >= T.level_off.size()) continue;
        const uint32_t lo = T.level_off[d], hi = T.level_off[d + 1];
        const uint32_t nl = d < T.level_local.size() ? std::min(T.level_local[d], hi - lo) : hi - lo;
        const uint32_t W = block_w(tab[t], g);
        const uint32_t per = std::max<uint32_t>(1, std::min<uint32_t>(kPullMaxKids, e->pull_words / W));
        P.bytes[q] += static_cast<uint64_t>(hi - lo) * W * 8;
        cut(P.chunks, t, gi, lo, lo + nl, per, W, block_row0(tab[t], g));
        cut(ghost, t, gi, lo + nl, hi, per, W, block_row0(tab[t], g));
      }
    }
    P.gsplit[q] = static_cast<uint32_t>(P.chunks.size());
    P.chunks.insert(P.chunks.end(), ghost.begin(), ghost.end());
  }
  P.off[rounds + 1] = static_cast<uint32_t>(P.chunks.size());
  ++P.version;
  return true;
}

// Multi-round launches: k_pull_pair writes rounds
// q and q + 1, k_pull_chain rounds q .. q + L - 1 (L = 3 .. kChainLevels) --
// each wave a run of level-d nodes and then every descendant of the run from
// the rows it holds in LDS, so only round q reads parent rows from HBM.  Which rounds go
// together is a small dynamic program over the rounds after k_flood's: a
// launch costs its rows, round q's parent-row reads (level d - 1's internal
// nodes x row bytes) and kLaunchBytes of launch ramp and tail.  A pair needs
// each row of round q (and each level-1 row of a start group entering at q)
// to fit the kPairWords stage; a chain slices wide rows into columns instead
// and sizes its runs by the levels' growth (chain_size).
// On N ranks a launch spans only rounds whose successors exchange nothing
// (every child is local and nothing written inside ships), and a chain also
// needs round q itself exchange-free.  Fills pair.kind (PS_K_* per round);
// cached with the pull chunks and the ghost plan's exchange rounds.
bool plan_pair_chunks(ps_engine* e, const WindowLayout& L, uint32_t first) {
  const uint32_t rounds = L.planned0;
  const auto& tab = L.tab;
  const auto& xchg = e->ghost.rounds;
  std::vector<uint64_t> key = e->pull.key;  // (graph, flags, rounds, row widths, start groups)
  key.push_back(first);
  key.push_back(e->chain_max);
  key.push_back(e->chain_max_groups);
  key.push_back(e->chain_words);
  key.push_back(e->chain_words_lead);
  key.push_back(static_cast<uint64_t>(e->launch_bytes));
  key.push_back(e->chain_tail ? 1 : 0);
  for (size_t q = 0; q < xchg.size(); ++q) key.push_back(xchg[q].any);
  PairPlan& PP = e->pair;
  if (key == PP.key) return false;
  PP.key = key;
  constexpr uint32_t stage = kPairWords;
  const double kLaunchBytes = e->launch_bytes;  // ~3 us of launch ramp and tail at ~5.5 TB/s
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const uint32_t chain_max = L.multi ? e->chain_max_groups : e->chain_max;
  const uint32_t max_len = std::max<uint32_t>(1, std::min<uint32_t>(chain_max, kChainLevels));
  auto& kind = PP.kind;
  kind.assign(rounds + 2, PS_K_NONE);
  for (uint32_t q = 1; q <= first && q <= rounds; ++q) kind[q] = PS_K_FLOOD;
  auto exch = [&](uint32_t q) { return q < xchg.size() && xchg[q].any; };
  // per round: parent-row bytes read (estimate), and whether a pair fits
  std::vector<double> rd(rounds + 2, 0.0);
  std::vector<uint8_t> can2(rounds + 2, 0);
  for (uint32_t q = first + 1; q <= rounds; ++q) {
    bool ok = max_len >= 2 && q + 1 <= rounds && !exch(q + 1) && !exch(q + 2);
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (const StartGroup& g : L.groups[t]) {
        const uint32_t W = block_w(tab[t], g);
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
    can2[q] = ok;
  }
  // A chain of `levels` levels from level d of (topic t, block of W words):
  // its runs, column slice and per-level growth.  Runs are sized so that the
  // stage holds their rows (slices of the stage width for wider rows), the
  // expected widest level range is half of the level tables (k_chain_ranges checks
  // the real ranges), and a wave writes about chain_words row words.
  struct ChainSize {
    uint32_t R = 0, S = 0;  // R = 0: no chain of this length
  };
  constexpr uint32_t stage_w = kChainWords, cap = kChainCap;
  auto chain_size = [&](const TopicHost& T, uint32_t d, uint32_t levels, uint32_t W, uint32_t words) {
    ChainSize z;
    const double n0 = static_cast<double>(T.level_off[d + 1] - T.level_off[d]);
    if (n0 == 0) {  // no node of the level on this rank: nothing to cut
      z.R = 1;
      z.S = std::max<uint32_t>(1, std::min(W, stage_w));
      return z;
    }
    double gmax = 1.0, gsum = 1.0;
    for (uint32_t k = 1; k < levels && d + k + 1 < T.level_off.size(); ++k) {
      const double g = static_cast<double>(T.level_off[d + k + 1] - T.level_off[d + k]) / n0;
      gmax = std::max(gmax, g);
      gsum += g;
    }
    if (gmax > cap / 2) return z;  // even one node's subtree is expected too wide
    z.S = W <= stage_w ? W : stage_w;
    const double r = std::min({static_cast<double>(kChainPar), static_cast<double>(stage_w / z.S),
                               std::floor(cap / 2 / gmax),
                               std::floor(static_cast<double>(words) / (z.S * gsum))});
    z.R = static_cast<uint32_t>(std::max(1.0, r));
    // (Rejected in round 4, profiles/r04/ab/NOTES.md: one-node runs of huge
    // subtrees cut into column slices for parallelism -- cfg2 0.0536 either
    // way, cfg3 0.908 vs 0.898 -- and two-round launches as two-level chains
    // instead of pairs.)
    return z;
  };
  // the (topic, group)s a launch of rounds q .. q + len - 1 writes: level d
  // from round q + r0 for `levels` levels
  auto chain_parts = [&](uint32_t q, uint32_t len, auto&& fn) {
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (uint32_t gi = 0; gi < L.groups[t].size(); ++gi) {
        const StartGroup& g = L.groups[t][gi];
        uint32_t d, r0;
        if (q >= g.start + 1) {
          d = q - g.start;
          r0 = 0;
        } else if (g.start + 1 < q + len) {
          d = 1;
          r0 = g.start + 1 - q;
        } else {
          continue;
        }
        if (d > T.depth || d + 1 >= T.level_off.size()) continue;
        fn(t, gi, d, r0, std::min(len - r0, T.depth - d + 1));
      }
    }
  };
  const bool chains_ok = key != e->chain_fail_key;  // (ranges overflowed under this plan once)
  // the window's last round with rows: a chain ending there may take one
  // round more than chain_max (the last level is the leaves' partial level;
  // it saves the tail round's own launch)
  uint32_t last_r = 0;
  for (uint32_t q = 1; q <= rounds && q < e->pull.bytes.size(); ++q)
    if (e->pull.bytes[q]) last_r = q;
  // (A/B: the launches before the window's last one sized by chain_words_lead)
  auto words_of = [&](uint32_t q, uint32_t len) {
    return e->chain_words_lead && q + len - 1 < last_r ? e->chain_words_lead : e->chain_words;
  };
  auto can_chain = [&](uint32_t q, uint32_t len) {
    const bool tail = e->chain_tail && len == max_len + 1 && q + len - 1 == last_r && max_len >= 3;
    if (!chains_ok || (len > max_len && !tail) || len > kChainLevels || q + len - 1 > rounds || exch(q)) return false;
    for (uint32_t k = 1; k <= len; ++k)
      if (exch(q + k)) return false;
    bool ok = true;
    chain_parts(q, len, [&](uint32_t t, uint32_t gi, uint32_t d, uint32_t, uint32_t levels) {
      ok = ok && chain_size(e->topics[t], d, levels, block_w(tab[t], L.groups[t][gi]), words_of(q, len)).R > 0;
    });
    return ok;
  };
  auto can = [&](uint32_t q, uint32_t len) {
    if (len == 1) return true;
    if (len == 2) return static_cast<bool>(can2[q]);
    return can_chain(q, len);
  };
  // best[q]: traffic of rounds q..rounds; take[q]: rounds of the launch starting at q
  std::vector<double> best(rounds + 6, 0.0);
  std::vector<uint8_t> take(rounds + 2, 1);
  for (uint32_t q = rounds; q > first; --q) {
    best[q] = 1e300;
    double wb = 0;
    for (uint32_t len = 1; len <= std::min<uint32_t>(kChainLevels, rounds - q + 1); ++len) {
      if (len > max_len + 1) break;
      wb += static_cast<double>(e->pull.bytes[q + len - 1]);
      if (!can(q, len)) continue;
      const double c = wb + rd[q] + (wb > 0 ? kLaunchBytes : 0.0) + best[q + len];
      if (c < best[q]) {
        best[q] = c;
        take[q] = static_cast<uint8_t>(len);
      }
    }
  }
  auto& C = PP.chunks;
  C.clear();
  PP.chain.clear();
  PP.lo.assign(rounds + 2, 0);
  PP.hi.assign(rounds + 2, 0);
  PP.gsplit.assign(rounds + 2, 0);
  PP.len.assign(rounds + 2, 0);
  const bool gpu = e->gpu_graph;
  std::vector<PullChunk> ghost;
  for (uint32_t q = first + 1; q <= rounds; ++q) {
    const uint32_t len = take[q];
    if (len == 1) {
      kind[q] = e->pull.bytes[q] ? PS_K_PULL : PS_K_NONE;
      continue;
    }
    PP.len[q] = len;
    if (len >= 3) {
      kind[q] = PS_K_CHAIN;
      for (uint32_t k = 1; k < len; ++k) kind[q + k] = PS_K_CHAIN2;
      PP.lo[q] = static_cast<uint32_t>(PP.chain.size());
      std::vector<ChainChunk> sliced;  // rows wider than the stage: after the whole-row chunks
      chain_parts(q, len, [&](uint32_t t, uint32_t gi, uint32_t d, uint32_t r0, uint32_t levels) {
        const TopicHost& T = e->topics[t];
        const StartGroup& g = L.groups[t][gi];
        const uint32_t W = block_w(tab[t], g);
        const ChainSize z = chain_size(T, d, levels, W, words_of(q, len));
        const uint64_t row0 = block_row0(tab[t], g);
        const uint32_t lo = T.level_off[d], hi = T.level_off[d + 1];
        for (uint32_t u = lo; u < hi; u += z.R)
          for (uint32_t w0 = 0; w0 < W; w0 += z.S) {
            ChainChunk c{};
            c.node_begin = T.nbase + u;
            c.node_end = T.nbase + std::min(u + z.R, hi);
            c.topic = t;
            c.p_lo = gpu ? kNone : e->node_parent[c.node_begin];
            c.p_hi = gpu ? kNone : e->node_parent[c.node_end - 1];
            c.W = W;
            c.row0_lo = static_cast<uint32_t>(row0);
            c.row0_hi = static_cast<uint32_t>(row0 >> 32);
            c.w0 = w0;
            c.S = std::min(z.S, W - w0);
            c.levels = static_cast<uint8_t>(levels);
            c.r0 = static_cast<uint8_t>(r0);
            c.group = static_cast<uint16_t>(gi);
            c.nbase = T.nbase;
            c.root = T.root_local ? T.nbase : kNoneNode;
            for (uint32_t k = 0; k <= levels && k <= kChainLevels; ++k)
              c.first[k] = T.nbase + (d + k < T.level_off.size() ? T.level_off[d + k] : T.n_nodes);
            (z.S < W ? sliced : PP.chain).push_back(c);
          }
      });
      // (heaviest chunks first measured no difference: profiles/r04/ab/chain_lpt.log)
      PP.gsplit[q] = static_cast<uint32_t>(PP.chain.size());
      PP.chain.insert(PP.chain.end(), sliced.begin(), sliced.end());
      PP.hi[q] = static_cast<uint32_t>(PP.chain.size());
      q += len - 1;
      continue;
    }
    kind[q] = PS_K_PAIR;
    kind[q + 1] = PS_K_PAIR2;
    PP.lo[q] = static_cast<uint32_t>(C.size());
    ghost.clear();
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (uint32_t gi = 0; gi < L.groups[t].size(); ++gi) {
        const StartGroup& g = L.groups[t][gi];
        const uint32_t W = block_w(tab[t], g);
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
        const uint32_t nl = d < T.level_local.size() ? std::min(T.level_local[d], hi - lo) : hi - lo;
        const uint64_t row0 = block_row0(tab[t], g);
        for (int part = 0; part < 2; ++part) {
          const uint32_t u0 = part ? lo + nl : lo, u1 = part ? hi : lo + nl;
          for (uint32_t u = u0; u < u1; u += per) {
            PullChunk c{};
            c.node_begin = T.nbase + u;
            c.node_end = T.nbase + std::min(u + per, u1);
            c.topic = t;
            c.p_lo = gpu ? kNone : e->node_parent[c.node_begin];
            c.p_hi = gpu ? kNone : e->node_parent[c.node_end - 1];
            c.W = W;
            c.row0_lo = static_cast<uint32_t>(row0);
            c.row0_hi = static_cast<uint32_t>(row0 >> 32);
            c.c_lo = late ? kNoneNode : 0;  // children: filled in on the device
            c.gin = c.gout = kNoneNode;
            c.group = gi;
            (part ? ghost : C).push_back(c);
          }
        }
      }
    }
    PP.gsplit[q] = static_cast<uint32_t>(C.size());
    C.insert(C.end(), ghost.begin(), ghost.end());
    PP.hi[q] = static_cast<uint32_t>(C.size());
    ++q;  // round q + 1 is the pair's second round
  }
  ++PP.version;
  return true;
}

// k_flood (one rank) runs the leading rounds that each write at most
// flood_top_bytes of rows: latency bound, one launch each would cost more
// than their bytes.
// (Windows under overlap_min_bytes never overlap -- run.cpp's byte floor --
// so they keep k_flood: a small deep tree has nothing to gain from chains.)
bool deep_window(const ps_engine* e, const WindowLayout& L) {
  if (!(e->overlap_on && L.level && e->world == 1 && !L.any_mesh && !(e->cfg.flags & PS_F_RECORD_HOPS) &&
        !L.multi && L.planned0 >= e->overlap_min_rounds))
    return false;
  uint64_t rows = 0;  // the window's row bytes, as run.cpp's floor counts them
  for (uint32_t t = 0; t < L.tab.size(); ++t)
    rows += static_cast<uint64_t>(L.tab[t].n_nodes) * L.tab[t].W * 8;
  return rows >= e->overlap_min_bytes;
}

// (Fewer than flood_min_rounds leading rounds cost less as a chain launch:
// k_flood's dependency hand-offs are a few us per round -- cfg2, 3 rounds:
// 0.066 ms/step with k_flood, 0.058 without; cfg4, 5 rounds: 0.447 with,
// 0.457 without; profiles/r04/ab/NOTES.md.)
uint32_t plan_flood_rounds(const ps_engine* e, const WindowLayout& L) {
  uint32_t r = 0;
  while (r < L.planned0 && e->pull.bytes[r + 1] <= e->flood_top_bytes) ++r;
  return r >= e->flood_min_rounds ? r : 0;
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
bool plan_flood_tasks(ps_engine* e, const WindowLayout& L, uint32_t rounds) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const auto& tab = L.tab;
  std::vector<uint64_t> key{e->graph_epoch, rounds, e->flood_words};
  for (uint32_t t = 0; t < nt; ++t) {
    key.push_back(tab[t].W ? L.groups[t].size() : ~0ull);
    key.push_back(tab[t].W);
    key.push_back(tab[t].wbase << 1 | ((tab[t].flags & kTopicGroups) ? 1 : 0));
    if (tab[t].W)
      for (const StartGroup& g : L.groups[t]) key.push_back(static_cast<uint64_t>(g.start) << 32 | g.w0);
  }
  FloodPlan& F = e->flood;
  if (key == F.key) return false;
  F.key = key;
  auto& TK = F.tasks;
  auto& SG = F.segs;
  TK.clear();
  SG.clear();
  F.slot0.assign(rounds + 2, 0);
  F.nslot.assign(rounds + 2, 0);
  // each (topic, start group)'s segment of the previous round
  std::vector<std::vector<uint32_t>> seg_prev(nt);
  for (uint32_t t = 0; t < nt; ++t) seg_prev[t].assign(L.groups[t].size(), kNone);
  uint32_t slot = 1, gran = 0;
  for (uint32_t q = 1; q <= rounds; ++q) {
    const size_t first = TK.size();
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (tab[t].W == 0) continue;
      for (size_t gi = 0; gi < L.groups[t].size(); ++gi) {
        const StartGroup& g = L.groups[t][gi];
        const uint32_t W = block_w(tab[t], g);
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
        sg.row0 = block_row0(tab[t], g);
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
    F.slot0[q] = slot;
    F.nslot[q] = ns;
    for (size_t i = first; i < TK.size(); ++i) {
      TK[i].slot0 = slot;
      TK[i].nslot = ns;
    }
    slot += ns;
  }
  F.slots = slot;
  F.granules = gran;
  ++F.version;
  return true;
}

// Multi-GPU level mode: the per-round exchange of ghost
// parents.  Round q writes, for every active (topic, start group), level d =
// q - s_g; its ghost-fed nodes read their parents' records, which every rank
// a ships to every rank b once per parent with a child there.  Region (a ->
// b, round q) = for each active (topic, group) in order, gcnt(t, d, a, b)
// records of the block's W words, each (topic, group) block padded to 16
// words (128 B), so regions and blocks stay line-aligned.  Every size comes
// from the global cross counts and message-derived widths (wglob), identical
// on every rank -- also one that owns none of a topic's nodes -- so senders
// and receivers agree without a handshake.  One GhostSeg per (round, topic,
// group) holds this rank's record bases (receive side per source rank, send
// side per destination rank, in the round's half of the double-buffered send
// buffer); the pull / pair chunks are annotated with the segment they read
// (gin) and ship into (gout) and their ship entries.  *changed: the plan (and
// the chunks' annotations) were rebuilt.
int plan_ghost(ps_engine* e, const WindowLayout& L, bool* changed) {
  *changed = false;
  GhostPlan& G = e->ghost;
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const int32_t world = e->world, me = e->rank;
  const uint32_t rounds = L.planned0;
  if (world <= 1) {
    if (!G.key.empty()) *changed = true;
    G = GhostPlan{};
    return PS_OK;
  }
  std::vector<uint64_t> key{e->graph_epoch, rounds};
  for (uint32_t t = 0; t < nt; ++t) {
    key.push_back(L.wglob[t]);
    if (L.wglob[t])
      for (const StartGroup& g : L.groups[t]) key.push_back(static_cast<uint64_t>(g.start) << 32 | g.wn);
  }
  if (key == G.key) return PS_OK;
  *changed = true;
  G = GhostPlan{};
  G.key = key;
  auto gcnt = [&](uint32_t t, uint32_t d, int32_t a, int32_t b) -> uint64_t {
    const auto& g = e->topics[t].gcnt;
    const size_t i = (static_cast<size_t>(d) * world + a) * world + b;
    return i < g.size() ? g[i] : 0;
  };
  auto pad16 = [](uint64_t w) { return (w + 15) & ~15ull; };
  // the (topic, group)s active in round q: level d = q - s_g, 1 <= d <= depth
  struct Act {
    uint32_t t, gi, d, rw;
  };
  std::vector<Act> act;
  G.rounds.assign(rounds + 2, GhostRound{});
  G.seg_of.assign(rounds + 2, {});
  std::vector<uint32_t> seg_round;  // round of every segment
  struct SegAt {
    uint32_t t, gi, d;
  };
  std::vector<SegAt> seg_at;  // (topic, group, level) of every segment
  for (uint32_t q = 1; q <= rounds; ++q) {
    GhostRound& R = G.rounds[q];
    R.s_off.assign(world, 0);
    R.s_len.assign(world, 0);
    R.r_off.assign(world, 0);
    R.r_len.assign(world, 0);
    act.clear();
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (!L.wglob[t] || !T.exists || T.gcnt.empty()) continue;
      for (uint32_t gi = 0; gi < L.groups[t].size(); ++gi) {
        const StartGroup& g = L.groups[t][gi];
        if (q <= g.start || q - g.start > T.depth) continue;
        act.push_back(Act{t, gi, q - g.start, g.wn});  // (one group: wn = the row width)
      }
    }
    for (int32_t a = 0; a < world && !R.any; ++a)
      for (int32_t b = 0; b < world && !R.any; ++b)
        for (const Act& x : act)
          if (a != b && gcnt(x.t, x.d, a, b)) {
            R.any = true;
            break;
          }
    if (!R.any) continue;
    // region a -> b: each active (topic, group) block in order
    auto region = [&](int32_t a, int32_t b) {
      uint64_t w = 0;
      for (const Act& x : act) w += pad16(gcnt(x.t, x.d, a, b) * x.rw);
      return w;
    };
    uint64_t so = 0, ro = 0;
    for (int32_t b = 0; b < world; ++b) {
      if (b == me) continue;
      R.s_off[b] = so * 8;
      R.s_len[b] = region(me, b) * 8;
      so += R.s_len[b] / 8;
    }
    for (int32_t a = 0; a < world; ++a) {
      if (a == me) continue;
      R.r_off[a] = ro * 8;
      R.r_len[a] = region(a, me) * 8;
      ro += R.r_len[a] / 8;
    }
    G.send_half = std::max(G.send_half, so);
    G.recv_words = std::max(G.recv_words, ro);
    // each block's base in every region of this rank
    std::vector<uint64_t> s_run(world, 0), r_run(world, 0);
    for (int32_t b = 0; b < world; ++b) {
      s_run[b] = R.s_off[b] / 8;
      r_run[b] = R.r_off[b] / 8;
    }
    R.pack0 = static_cast<uint32_t>(G.pack.size());
    uint64_t units = 0;
    for (const Act& x : act) {
      GhostSeg S{};
      S.rw = x.rw;
      S.topic = x.t;
      for (int32_t b = 0; b < world; ++b) {
        if (b == me) continue;
        S.sbase[b] = s_run[b];  // (+ the round's half, below)
        s_run[b] += pad16(gcnt(x.t, x.d, me, b) * x.rw);
        S.rbase[b] = r_run[b];
        r_run[b] += pad16(gcnt(x.t, x.d, b, me) * x.rw);
      }
      const uint32_t si = static_cast<uint32_t>(G.segs.size());
      auto& so_q = G.seg_of[q];
      if (so_q.size() <= x.t) so_q.resize(nt);
      if (so_q[x.t].size() <= x.gi) so_q[x.t].resize(L.groups[x.t].size(), kNone);
      so_q[x.t][x.gi] = si;
      G.segs.push_back(S);
      seg_round.push_back(q);
      seg_at.push_back(SegAt{x.t, x.gi, x.d});
      const bool in_place = e->inplace && x.d >= 2;  // (level-1 nodes: the root's records)
      if (!in_place)
        for (int32_t a = 0; a < world; ++a)
          if (a != me) R.rec_bytes += gcnt(x.t, x.d, a, me) * x.rw * 8;
      // level-1 records come from the seeded root: packed by k_pack
      const TopicHost& T = e->topics[x.t];
      if (x.d == 1 && T.root_local && T.send_lvl.size() > 2 && T.send_lvl[2] > T.send_lvl[1]) {
        PackSeg ps{};
        ps.e0 = T.ship0 + T.send_lvl[1];
        ps.e1 = T.ship0 + T.send_lvl[2];
        ps.gseg = si;
        ps.W = x.rw;
        ps.row = block_row0(L.tab[x.t], L.groups[x.t][x.gi]);  // the root: the topic's first node
        ps.unit0 = units;
        units += static_cast<uint64_t>(ps.e1 - ps.e0) * pack_units(ps.W);
        G.pack.push_back(ps);
      }
    }
    R.pack1 = static_cast<uint32_t>(G.pack.size());
    R.pack_units = units;
  }
  G.send_half = std::max<uint64_t>(16, pad16(G.send_half));
  // PS_DIST_F_INPLACE: the owners' row sets and layouts (every rank plans
  // the same ghost key, so all of them reach this exchange together)
  if (e->inplace && e->transport && !G.segs.empty()) {
    Transport::Share mine;
    mine.seen = e->d_seen.p;
    mine.gen = e->d_gen.p;
    mine.gen_cur = e->gen_cur;
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicDev& d = L.tab[t];
      mine.topics.insert(mine.topics.end(), {d.wbase, d.n_nodes, d.nbase, d.flags});
    }
    std::vector<Transport::Share> all;
    std::string xerr;
    if (e->transport->share(mine, all, &xerr) != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
    e->rrows_host.assign(kMaxRanks, RankRows{nullptr, nullptr});
    for (int32_t a = 0; a < world; ++a) {
      if (all[a].gen_cur != e->gen_cur || all[a].topics.size() != mine.topics.size())
        return e->fail(PS_E_STATE, "in-place rows: the ranks' windows differ");
      e->rrows_host[a] = RankRows{static_cast<const uint64_t*>(all[a].seen), static_cast<const uint8_t*>(all[a].gen)};
    }
    e->rrows_dirty = true;
    for (size_t si = 0; si < G.segs.size(); ++si) {
      const SegAt& x = seg_at[si];
      if (x.d < 2) continue;
      GhostSeg& S = G.segs[si];
      S.flags |= kSegInPlace;
      const StartGroup& g = L.groups[x.t][x.gi];
      for (int32_t a = 0; a < world; ++a) {
        if (a == me) continue;
        const uint64_t* o = &all[a].topics[4 * static_cast<size_t>(x.t)];  // the owner's topic block
        TopicDev od{};
        od.wbase = o[0];
        od.n_nodes = static_cast<uint32_t>(o[1]);
        od.flags = static_cast<uint32_t>(o[3]);
        S.rbase[a] = block_row0(od, g);
        S.gbase[a] = static_cast<uint32_t>(o[2]);
      }
    }
  }
  // each round's records go to its half of the send buffer (round q + 1's are
  // written while round q's are in flight)
  for (size_t si = 0; si < G.segs.size(); ++si)
    for (int32_t b = 0; b < world; ++b)
      if (b != me) G.segs[si].sbase[b] += (seg_round[si] % kSendBufs) * G.send_half;
  return PS_OK;
}

// The ghost plan's segments and ship entries on the level-mode chunks: a
// chunk's ghost-fed nodes read records of its own round's segment (gin); its
// nodes with children on other ranks ship records into the next round's
// segment (gout), entries [e_lo, e_hi) of the engine's ship array.  Pair
// launches never ship (they pair only rounds whose successors exchange
// nothing); a pair launch's level-1 run belongs to its second round.
void annotate_chunks(ps_engine* e, const WindowLayout& L) {
  const GhostPlan& G = e->ghost;
  const uint32_t rounds = L.planned0;
  auto seg = [&](uint32_t q, uint32_t t, uint32_t gi) -> uint32_t {
    if (q > rounds || q >= G.seg_of.size() || t >= G.seg_of[q].size() || gi >= G.seg_of[q][t].size())
      return kNoneNode;
    return G.seg_of[q][t][gi];
  };
  auto annotate = [&](std::vector<PullChunk>& C, uint32_t c0, uint32_t c1, uint32_t q, bool ship) {
    for (uint32_t ci = c0; ci < c1; ++ci) {
      PullChunk& c = C[ci];
      c.gin = c.gout = kNoneNode;
      c.e_lo = c.e_hi = 0;
      if (e->world <= 1) continue;
      const uint32_t t = c.topic, gi = c.group;
      const TopicHost& T = e->topics[t];
      const bool late = !ship && c.c_lo == kNoneNode;  // a pair launch's level-1 run (round q + 1)
      const uint32_t qq = late ? q + 1 : q;
      c.gin = seg(qq, t, gi);
      if (!ship) continue;
      const uint32_t d = qq - L.groups[t][gi].start;
      c.gout = seg(qq + 1, t, gi);
      if (c.gout == kNoneNode || d + 2 >= T.send_lvl.size()) {
        c.gout = kNoneNode;
        continue;
      }
      // this chunk's nodes among the level's parents with children elsewhere
      const auto b0 = T.send_node.begin() + T.send_lvl[d + 1], b1 = T.send_node.begin() + T.send_lvl[d + 2];
      const auto lo = std::lower_bound(b0, b1, c.node_begin), hi = std::lower_bound(b0, b1, c.node_end);
      c.e_lo = T.ship0 + static_cast<uint32_t>(lo - T.send_node.begin());
      c.e_hi = T.ship0 + static_cast<uint32_t>(hi - T.send_node.begin());
      if (c.e_lo == c.e_hi) c.gout = kNoneNode;
    }
  };
  PullPlan& P = e->pull;
  for (uint32_t q = 1; q <= rounds && q + 1 < P.off.size(); ++q) annotate(P.chunks, P.off[q], P.off[q + 1], q, true);
  PairPlan& PP = e->pair;
  for (uint32_t q = 1; q < PP.lo.size(); ++q)
    if (PP.len[q] == 2 && PP.hi[q] > PP.lo[q]) annotate(PP.chunks, PP.lo[q], PP.hi[q], q, false);
  ++P.version;
  ++PP.version;
}

}  // namespace psamd
