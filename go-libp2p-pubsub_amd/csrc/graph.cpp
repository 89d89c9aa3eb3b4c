// graph.cpp -- the node space of the engine: per topic the
// owned tree nodes reachable from the root, numbered level by level, CSR child
// lists, node flags; built on the host (any rank count) or rebuilt on the GPU
// after churn (gbuild.hip, one rank).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <tuple>

#include "engine.hpp"
#include "gbuild.hpp"

namespace psamd {

bool topic_ok(const ps_engine* e, uint32_t topic) { return topic < e->topics.size() && e->topics[topic].exists; }

// Child lists of one topic in peer space, insertion order.
void peer_children(const ps_engine* e, const TopicHost& T, std::vector<uint32_t>& rp, std::vector<uint32_t>& cl) {
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
// least-loaded rank; the levels above L stay with the root's owner.  L =
// split_depth, or (0) the first level holding >= 64*world nodes, so only
// edges out of level L - 1 cross ranks.
void partition_topic(const std::vector<uint32_t>& order, const std::vector<uint32_t>& bfs_parent,
                     const std::vector<uint32_t>& level, int32_t world, uint32_t part, uint32_t split_depth,
                     std::vector<int32_t>& owner) {
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
  for (size_t u = 0; u < n; ++u)
    if (level[u] > L) owner[u] = owner[anc[u]];
}

namespace {

// One topic's BFS over its child lists: global positions in BFS order, each
// position's BFS parent and level; local[peer] = position (reset by caller).
struct TopicBfs {
  std::vector<uint32_t> rp, cl, order, bfs_parent, level;
  std::vector<int32_t> owner;
};

int topic_bfs(ps_engine* e, const TopicHost& T, std::vector<uint32_t>& local, TopicBfs& B) {
  const uint32_t n = e->cfg.n_peers;
  peer_children(e, T, B.rp, B.cl);
  B.order.assign(1, T.root);
  B.bfs_parent.assign(1, kNone);
  B.level.assign(1, 0);
  local[T.root] = 0;
  for (size_t qi = 0; qi < B.order.size(); ++qi) {
    const uint32_t p = B.order[qi];
    for (uint32_t k = B.rp[p]; k < B.rp[p + 1]; ++k) {
      const uint32_t c = B.cl[k];
      if (c >= n) return e->fail(PS_E_INVAL, "child id out of range");
      if (local[c] == kNone) {
        local[c] = static_cast<uint32_t>(B.order.size());
        B.order.push_back(c);
        B.bfs_parent.push_back(static_cast<uint32_t>(qi));
        B.level.push_back(B.level[qi] + 1);
      }
    }
  }
  partition_topic(B.order, B.bfs_parent, B.level, e->world, e->partition, e->split_depth, B.owner);
  return PS_OK;
}

}  // namespace

// Builds this rank's node space.  Per topic, every rank's owned nodes are
// numbered level by level (each rank computes every rank's numbering, so
// remote ids and ghost record indices agree without a handshake).  Level d + 1
// of rank r: first the nodes whose parent r owns, in (parent id, sibling)
// order -- so the children of consecutive parents are consecutive ids, as in
// BFS order, which is what one rank gets -- then the ghost-fed nodes, grouped
// by the parent's owner a and ordered by record index k (a numbers its
// parents with children on r in its own node order).  A round's nodes that
// need no exchange are therefore one contiguous range ahead of those that
// read records.  CSR over node ids; a child owned by another rank is
// kRemoteBit | rank << 27 | its id at that rank.
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
  e->ship_host.clear();
  std::vector<uint32_t> local(n, kNone);  // peer -> BFS position
  TopicBfs B;
  const uint32_t ntop = static_cast<uint32_t>(e->topics.size());
  // node-space base of every topic at every rank (a remote child is addressed
  // by its fused node id at its owner)
  std::vector<uint64_t> base_at(static_cast<size_t>(ntop) * std::max(world, 1), 0);
  if (world > 1) {
    std::vector<uint64_t> run(world, 0);
    for (uint32_t t = 0; t < ntop; ++t) {
      for (int32_t q = 0; q < world; ++q) base_at[static_cast<size_t>(t) * world + q] = run[q];
      TopicHost& T = e->topics[t];
      if (!T.exists) continue;
      int rc = topic_bfs(e, T, local, B);
      if (rc) return rc;
      for (size_t u = 0; u < B.order.size(); ++u) run[B.owner[u]]++;
      for (uint32_t p : B.order) local[p] = kNone;
    }
  }
  std::vector<uint32_t> loc, ghost_of, mine;
  std::vector<std::vector<uint32_t>> cur(std::max(world, 1)), nxt_local(std::max(world, 1));
  std::vector<std::vector<uint32_t>> nxt_ghost(static_cast<size_t>(std::max(world, 1)) * std::max(world, 1));
  uint64_t n_total = 0;
  for (uint32_t t = 0; t < ntop; ++t) {
    TopicHost& T = e->topics[t];
    T.nbase = static_cast<uint32_t>(n_total);
    T.n_nodes = 0;
    T.depth = 0;
    T.mesh = false;
    T.root_local = true;
    T.max_deg = 0;
    T.cross.clear();
    T.level_internal.clear();
    T.level_off.clear();
    T.level_local.clear();
    T.gcnt.clear();
    T.send_node.clear();
    T.send_dst.clear();
    T.send_lvl.clear();
    T.ship0 = static_cast<uint32_t>(e->ship_host.size());
    if (!T.exists) continue;
    {
      int rc = topic_bfs(e, T, local, B);
      if (rc) return rc;
    }
    const auto& rp = B.rp;
    const auto& cl = B.cl;
    const auto& order = B.order;
    const auto& owner = B.owner;
    const uint32_t N = static_cast<uint32_t>(order.size());
    for (uint32_t p : order) T.max_deg = std::max(T.max_deg, rp[p + 1] - rp[p]);
    T.depth = B.level.back();
    {
      std::vector<uint32_t> indeg(N, 0);
      for (uint32_t u = 0; u < N; ++u)
        for (uint32_t k = rp[order[u]]; k < rp[order[u] + 1]; ++k) indeg[local[cl[k]]]++;
      for (uint32_t u = 0; u < N; ++u)
        if (indeg[u] > (u == 0 ? 0u : 1u)) T.mesh = true;
    }
    if (T.mesh && world > 1) return e->fail(PS_E_STATE, "multi-GPU engines support tree topics only");
    T.root_local = owner[0] == me;
    // per-rank numbering, level by level (see above)
    const int32_t W = std::max(world, 1);
    loc.assign(N, 0);
    if (world > 1) ghost_of.assign(N, kNone);
    mine.clear();
    std::vector<uint32_t> next_id(W, 0);
    for (auto& v : cur) v.clear();
    cur[owner[0]].push_back(0);
    loc[0] = next_id[owner[0]]++;
    T.level_off.assign(T.depth + 2, 0);
    T.level_local.assign(T.depth + 1, 0);
    T.gcnt.assign(world > 1 ? static_cast<size_t>(T.depth + 2) * world * world : 0, 0);
    T.send_lvl.assign(T.depth + 3, 0);
    if (owner[0] == me) {
      mine.push_back(0);
      T.level_local[0] = 1;
    }
    T.level_off[1] = static_cast<uint32_t>(mine.size());
    std::vector<uint32_t> kk(W);
    for (uint32_t d = 0; d < T.depth; ++d) {
      for (auto& v : nxt_local) v.clear();
      for (auto& v : nxt_ghost) v.clear();
      uint32_t* gc = world > 1 ? &T.gcnt[static_cast<size_t>(d + 1) * world * world] : nullptr;
      for (int32_t a = 0; a < W; ++a)
        for (uint32_t u : cur[a]) {
          const uint32_t p = order[u];
          uint32_t mask = 0;
          for (uint32_t k = rp[p]; k < rp[p + 1]; ++k) {
            const uint32_t v = local[cl[k]];
            if (B.bfs_parent[v] != u) continue;  // (a mesh edge into an earlier-numbered node)
            const int32_t b = owner[v];
            if (b == a) {
              nxt_local[a].push_back(v);
              continue;
            }
            // PS_DIST_F_INPLACE: below the root a ghost parent is addressed by
            // its topic-relative id at its owner (its row is read there); the
            // roots' rows still ship as records (their seeded row)
            const bool in_place = e->inplace && d >= 1;
            if (!(mask >> b & 1u)) {
              mask |= 1u << b;
              kk[b] = gc[a * world + b]++;
              if (kk[b] > kRemoteIdMask) return e->fail(PS_E_NOMEM, "ghost rows of one level exceed 2^27");
              if (a == me && !in_place) {
                e->ship_host.push_back(ShipEntry{T.nbase + loc[u], static_cast<uint32_t>(b) << kRemoteRankShift | kk[b]});
                T.send_node.push_back(T.nbase + loc[u]);
                T.send_dst.push_back(static_cast<uint32_t>(b) << kRemoteRankShift | kk[b]);
              }
            }
            if (in_place && loc[u] > kRemoteIdMask) return e->fail(PS_E_NOMEM, "a rank's topic exceeds 2^27 nodes");
            ghost_of[v] = static_cast<uint32_t>(a) << kRemoteRankShift | (in_place ? loc[u] : kk[b]);
            nxt_ghost[static_cast<size_t>(b) * W + a].push_back(v);
          }
        }
      T.send_lvl[d + 2] = static_cast<uint32_t>(T.send_node.size());
      for (int32_t r = 0; r < W; ++r) {
        auto& c = cur[r];
        c.swap(nxt_local[r]);
        if (r == me) T.level_local[d + 1] = static_cast<uint32_t>(c.size());
        for (int32_t a = 0; a < W; ++a) {
          const auto& g = nxt_ghost[static_cast<size_t>(r) * W + a];
          c.insert(c.end(), g.begin(), g.end());
        }
        for (uint32_t v : c) loc[v] = next_id[r]++;
        if (r == me) {
          mine.insert(mine.end(), c.begin(), c.end());
          T.level_off[d + 2] = static_cast<uint32_t>(mine.size());
        }
      }
    }
    for (uint32_t d = 1; d < T.send_lvl.size(); ++d) T.send_lvl[d] = std::max(T.send_lvl[d], T.send_lvl[d - 1]);
    // emit the owned nodes in local-id order
    T.level_internal.assign(T.depth + 1, 0);
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> cross;
    if (world > 1)
      for (uint32_t u = 0; u < N; ++u)
        for (uint32_t k = rp[order[u]]; k < rp[order[u] + 1]; ++k) {
          const uint32_t v = local[cl[k]];
          if (owner[v] != owner[u])
            cross[{B.level[u], static_cast<uint32_t>(owner[u]), static_cast<uint32_t>(owner[v])}]++;
        }
    for (uint32_t u : mine) {
      const uint32_t p = order[u];
      const uint32_t deg = rp[p + 1] - rp[p];
      const uint32_t bp = B.bfs_parent[u];
      e->node_peer.push_back(p);
      if (world > 1) e->ghost_ref.push_back(u ? ghost_of[u] : kNone);
      e->node_parent.push_back(u && owner[bp] == me ? T.nbase + loc[bp] : kNone);
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
      if (deg) T.level_internal[B.level[u]]++;
      if (u && owner[bp] != me) e->remote_fed.push_back(T.nbase + loc[u]);
      if (e->col.size() >= 0xFFFFFFF0ull) return e->fail(PS_E_NOMEM, "edge space exceeds 2^32");
    }
    for (const auto& kv : cross)
      T.cross.push_back({std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), kv.second});
    T.n_nodes = static_cast<uint32_t>(mine.size());
    for (uint32_t p : order) local[p] = kNone;
    n_total += T.n_nodes;
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

namespace {

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
  HIP_TRY(e->d_orph.ensure(static_cast<size_t>(nt) * n), "alloc orphan bytes");
  static_assert(SubscriptionTree::kOrphanUp == kOrphanCode, "one orphan code");
  // 1. parent deltas of every topic, one upload
  auto& pairs = e->pairs_host;
  pairs.clear();
  e->pair_off.assign(nt + 1, 0);
  std::vector<uint32_t> cand, codes;
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    e->pair_off[t] = pairs.size() / 2;
    if (!T.exists) continue;
    uint32_t* par_t = e->d_tpar.as<uint32_t>() + static_cast<size_t>(t) * n;
    bool full = false;
    uint8_t* orph_t = e->d_orph.as<uint8_t>() + static_cast<size_t>(t) * n;
    if (!T.par_dev_valid) {
      HIP_TRY(hipMemsetAsync(par_t, 0xFF, static_cast<size_t>(n) * 4, s), "clear parents");
      HIP_TRY(hipMemsetAsync(orph_t, 0, n, s), "clear orphan bytes");
      if (T.kind != Kind::Join) T.par_mirror.assign(n, kNone);  // (joined trees ship their touched codes)
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
      // the tree recorded each touched peer's upstream code when it changed:
      // ship them as they are (a peer touched without a net change costs one
      // idempotent pair, not a visit of its scattered line here)
      T.tree.take_touched(cand, codes);
      if (full) {
        for (uint32_t p = 0; p < n; ++p) {
          const uint32_t v = T.tree.upstream_code(p);
          if (v != kNone) {
            pairs.push_back(p);
            pairs.push_back(v);
          }
        }
      } else {
        for (size_t i = 0; i < cand.size(); ++i) {
          pairs.push_back(cand[i]);
          pairs.push_back(codes[i]);
        }
      }
    } else if (T.par_full_dirty || full) {
      for (uint32_t p = 0; p < n; ++p) diff(p, p == T.root ? kNone : T.parent[p]);
      T.par_full_dirty = false;
    }
  }
  e->pair_off[nt] = pairs.size() / 2;
  if (!pairs.empty()) {
    HIP_TRY(e->d_pairs.ensure(pairs.size() * 4), "alloc deltas");
    // through pinned memory: an asynchronous DMA (a pageable source is staged
    // by the runtime, synchronously); the build syncs before the next reuse
    if (e->pairs_pinned_cap < pairs.size()) {
      if (e->pairs_pinned) HIP_TRY(hipHostFree(e->pairs_pinned), "free pinned deltas");
      e->pairs_pinned = nullptr;
      e->pairs_pinned_cap = 0;
      const size_t cap = std::max<size_t>(pairs.size() + pairs.size() / 2, 1 << 16);
      void* h = nullptr;
      HIP_TRY(hipHostMalloc(&h, cap * 4, hipHostMallocDefault), "alloc pinned deltas");
      e->pairs_pinned = static_cast<uint32_t*>(h);
      e->pairs_pinned_cap = cap;
    }
    std::memcpy(e->pairs_pinned, pairs.data(), pairs.size() * 4);
    HIP_TRY(hipMemcpyAsync(e->d_pairs.p, e->pairs_pinned, pairs.size() * 4, hipMemcpyHostToDevice, s),
            "upload deltas");
    for (uint32_t t = 0; t < nt; ++t)
      HIP_TRY(launch_scatter_pairs(e->d_pairs.as<uint32_t>() + 2 * e->pair_off[t],
                                   static_cast<uint32_t>(e->pair_off[t + 1] - e->pair_off[t]),
                                   e->d_tpar.as<uint32_t>() + static_cast<size_t>(t) * n,
                                   e->d_orph.as<uint8_t>() + static_cast<size_t>(t) * n, s),
              "scatter deltas");
  }
  using clk = std::chrono::steady_clock;
  const auto tb1 = clk::now();
  // 2. node capacity: every peer of every existing topic (the reachable
  //    counts are known only once placed); the node arrays are written in place
  std::vector<uint32_t> act;  // existing topics in node-space order
  for (uint32_t t = 0; t < nt; ++t)
    if (e->topics[t].exists) act.push_back(t);
  const uint32_t na = static_cast<uint32_t>(act.size());
  const uint64_t cap = static_cast<uint64_t>(na) * n + 16;
  if (cap >= 0xFFFFFFF0ull) {  // (every peer of every topic as a node: the host build sizes exactly)
    *fallback = true;
    return PS_OK;
  }
  HIP_TRY(e->d_row_ptr.ensure((cap + 1) * 4), "alloc row_ptr");
  HIP_TRY(e->d_col.ensure(cap * 4), "alloc col");
  HIP_TRY(e->d_node_topic.ensure(cap * 2), "alloc node_topic");
  HIP_TRY(e->d_node_peer.ensure(cap * 4), "alloc node_peer");
  HIP_TRY(e->d_node_parent.ensure(cap * 4), "alloc node_parent");
  HIP_TRY(e->d_node_flags.ensure(((cap + 15) / 16) * 16 + 16), "alloc node_flags");
  HIP_TRY(e->d_first.ensure(cap * 4), "alloc first child");
  HIP_TRY(e->d_ndeg.ensure(cap * 4), "alloc node fan-out");
  HIP_TRY(e->d_nkat.ensure(cap * 4), "alloc node child index");
  HIP_TRY(e->d_local.ensure(static_cast<size_t>(n) * 4), "alloc local ids");
  {
    bool fresh = false;
    HIP_TRY(e->d_live.ensure(n, &fresh), "alloc live mask");
    if (fresh) e->live_dev_valid = false;
  }
  // the peer-space CSR scratch (one topic at a time)
  HIP_TRY(e->d_cnt.ensure((static_cast<size_t>(n) + 1) * 4), "alloc fan-out by peer");
  HIP_TRY(e->d_childoff.ensure((static_cast<size_t>(n) + 1) * 4), "alloc child offsets");
  HIP_TRY(e->d_fidx.ensure(static_cast<size_t>(n) * 4), "alloc scatter fill");
  HIP_TRY(e->d_kids.ensure(static_cast<size_t>(n) * 4 + 4), "alloc children");
  HIP_TRY(e->d_big.ensure(static_cast<size_t>(n) * 4 + 4), "alloc long child lists");
  size_t scan_bytes = 0;
  HIP_TRY(scan_u32(nullptr, &scan_bytes, nullptr, nullptr, n + 1, s), "scan size");
  HIP_TRY(e->d_cub.ensure(std::max<size_t>(scan_bytes, 16)), "alloc scan temp");
  // one block, one clear and one readback: per-topic stat words, the error
  // word, per-topic level tables, the active topics' bases
  const size_t o_err = static_cast<size_t>(nt) * kGstWords, o_lvl = (o_err + 4 + 3) & ~size_t(3),
               o_tb = o_lvl + static_cast<size_t>(nt) * 512, blk_words = o_tb + 2 * static_cast<size_t>(na) + 2;
  HIP_TRY(e->d_gstat.ensure(blk_words * 4), "alloc build stats");
  uint32_t* gstat = e->d_gstat.as<uint32_t>();
  uint32_t* err = gstat + o_err;
  auto& blk = e->gstat_host;
  blk.assign(blk_words, 0);
  const uint32_t* gs = blk.data();
  const uint32_t* lh = blk.data() + o_lvl;
  const uint32_t* tb = blk.data() + o_tb;
  if (!e->live_dev_valid) {
    HIP_TRY(hipMemcpyAsync(e->d_live.p, e->live.data(), n, hipMemcpyHostToDevice, s), "upload live");
    e->live_dev_valid = true;
  }
  // per topic: the levels the look-back launches take (from the top kernel's
  // last reach to 2 past the last depth: the pass past the deepest level
  // closes its leaves' CSR rows) and each launch's grid, from the last build's
  // level sizes (a level that outgrew its grid is redone with full grids)
  const uint32_t full = lb_tiles(n);
  std::vector<uint32_t> d_from(nt, 1), d_to(nt, 0);
  for (uint32_t t : act) {
    const TopicHost& T = e->topics[t];
    if (T.level_off.size() >= 2 && T.depth) {
      d_from[t] = std::max<uint32_t>(1, T.top_levels);
      d_to[t] = std::min<uint32_t>(kBuildMaxDepth - 1, T.depth + 2);
    } else {
      d_to[t] = 24;
    }
  }
  bool full_grids = false;
  const auto tb2 = clk::now();
  for (int attempt = 0;; ++attempt) {
    if (attempt >= 8) {
      *fallback = true;
      return PS_OK;
    }
    // look-back status words: one region per level launch
    size_t st_words = 0;
    std::vector<std::vector<uint32_t>> grids(nt);
    for (uint32_t t : act) {
      const TopicHost& T = e->topics[t];
      for (uint32_t d = d_from[t]; d <= d_to[t]; ++d) {
        uint32_t g = full;
        if (!full_grids && d < T.level_off.size() && d >= 1 && T.level_off.size() >= 2) {
          const uint64_t np = T.level_off[d] - T.level_off[d - 1];
          g = std::min<uint32_t>(full, lb_tiles(static_cast<uint32_t>(std::min<uint64_t>(np + np / 4 + 2048, n))));
        }
        grids[t].push_back(g);
        st_words += g + 1;  // (+ the launch's tile ticket, first)
      }
    }
    HIP_TRY(e->d_lbstat.ensure(std::max<size_t>(st_words, 1) * 8), "alloc look-back status");
    {
      ClearRegions cr{};
      cr.p[0] = gstat;
      cr.words[0] = blk_words;
      cr.p[1] = e->d_lbstat.as<uint32_t>();
      cr.words[1] = 2 * std::max<size_t>(st_words, 1);
      cr.n = 2;
      HIP_TRY(launch_clear(cr, s), "clear build block");
    }
    uint64_t* lbst = e->d_lbstat.as<uint64_t>();
    for (uint32_t ai = 0; ai < na; ++ai) {
      const uint32_t t = act[ai];
      const TopicHost& T = e->topics[t];
      {
        ClearRegions cr{};
        cr.p[0] = e->d_cnt.as<uint32_t>();
        cr.words[0] = static_cast<uint64_t>(n) + 1;
        cr.p[1] = e->d_fidx.as<uint32_t>();
        cr.words[1] = n;
        cr.p[2] = e->d_big.as<uint32_t>() + n;
        cr.words[2] = 1;
        cr.n = 3;
        HIP_TRY(launch_clear(cr, s), "clear child-list scratch");
      }
      HIP_TRY(build_kids(e->d_tpar.as<uint32_t>() + static_cast<size_t>(t) * n, n, e->d_cnt.as<uint32_t>(),
                         e->d_childoff.as<uint32_t>(), e->d_fidx.as<uint32_t>(), e->d_kids.as<uint32_t>(),
                         e->d_big.as<uint32_t>(), e->d_big.as<uint32_t>() + n, e->d_cub.p, e->d_cub.bytes, s),
              "child lists");
      PlaceArgs P{};
      P.kids = e->d_kids.as<uint32_t>();
      P.koff = e->d_childoff.as<uint32_t>();
      P.cnt = e->d_cnt.as<uint32_t>();
      P.live = e->d_live.as<uint8_t>();
      P.node_peer = e->d_node_peer.as<uint32_t>();
      P.node_topic = e->d_node_topic.as<uint16_t>();
      P.local = e->d_local.as<uint32_t>();
      P.node_parent = e->d_node_parent.as<uint32_t>();
      P.row_ptr = e->d_row_ptr.as<uint32_t>();
      P.col = e->d_col.as<uint32_t>();
      P.first = e->d_first.as<uint32_t>();
      P.flags = e->d_node_flags.as<uint8_t>();
      P.ndeg = e->d_ndeg.as<uint32_t>();
      P.nkat = e->d_nkat.as<uint32_t>();
      P.lvl = gstat + o_lvl + 512 * static_cast<size_t>(t);
      P.gst = gstat + static_cast<size_t>(t) * kGstWords;
      P.tb = gstat + o_tb;
      P.err = err;
      P.a = ai;
      P.root = T.root;
      P.topic = static_cast<uint16_t>(t);
      HIP_TRY(launch_place_top(P, d_from[t] > 1 ? d_from[t] : kBuildMaxDepth, s), "place top levels");
      for (uint32_t i = 0, d = d_from[t]; d <= d_to[t]; ++d, ++i) {
        HIP_TRY(launch_place_lb(P, d, grids[t][i], lbst + 1, s), "place level");
        lbst += grids[t][i] + 1;
      }
    }
    // the lazy prune's reach queries over this node space (run.cpp): their
    // answers come back with the build block, one sync for both
    {
      size_t qw = 0;
      for (const auto& q : e->early_q) qw += q.peers.size() + (q.peers.size() + 3) / 4 + 4;
      if (qw) HIP_TRY(e->d_query.ensure(qw * 4), "alloc reach query");
      uint32_t* qp = e->d_query.as<uint32_t>();
      for (auto& q : e->early_q) {
        q.launched = q.ready = false;
        const uint32_t k = static_cast<uint32_t>(q.peers.size());
        if (!k || std::find(act.begin(), act.end(), q.topic) == act.end()) continue;
        uint8_t* dout = reinterpret_cast<uint8_t*>(qp + k);
        HIP_TRY(hipMemcpyAsync(qp, q.peers.data(), static_cast<size_t>(k) * 4, hipMemcpyHostToDevice, s),
                "upload reach query");
        const TopicHost& T = e->topics[q.topic];
        HIP_TRY(launch_reach_query(qp, k, n, e->d_tpar.as<uint32_t>() + static_cast<size_t>(q.topic) * n,
                                   e->d_orph.as<uint8_t>() + static_cast<size_t>(q.topic) * n, T.root, dout, s),
                "reach query");
        q.out.resize(k);
        HIP_TRY(hipMemcpyAsync(q.out.data(), dout, k, hipMemcpyDeviceToHost, s), "read reach query");
        q.launched = true;
        qp += k + (k + 3) / 4 + 4;
      }
    }
    HIP_TRY(hipMemcpyAsync(blk.data(), gstat, blk_words * 4, hipMemcpyDeviceToHost, s), "read build block");
    HIP_TRY(hipStreamSynchronize(s), "sync");
    const uint32_t ev = gs[o_err];
    if (ev & kBuildErrStall) {
      *fallback = true;  // a stalled look-back: build on the host
      return PS_OK;
    }
    bool redo = false;
    if (ev & kBuildErrGrid) {
      full_grids = true;
      redo = true;
    }
    if (ev & kBuildErrOrder) {  // a top level outgrew the top kernel: every level by look-back launches
      for (uint32_t t : act) d_from[t] = 1;
      redo = true;
    }
    for (uint32_t t : act) {  // a tree deeper than the launches: more levels
      const uint32_t done = gs[static_cast<size_t>(t) * kGstWords + kGstDone];
      if (lh[512 * t + done + 1] != lh[512 * t + done] || done < d_to[t]) {
        if (d_to[t] >= kBuildMaxDepth - 1 && lh[512 * t + done + 1] != lh[512 * t + done]) {
          *fallback = true;  // deeper than the level tables
          return PS_OK;
        }
        if (!(ev & (kBuildErrGrid | kBuildErrOrder)) && done >= d_to[t]) {
          d_to[t] = std::min<uint32_t>(kBuildMaxDepth - 1, 2 * d_to[t] + 8);
          redo = true;
        }
      }
    }
    if (!redo) break;
  }
  for (auto& q : e->early_q) q.ready = q.launched;
  const auto tb3 = clk::now();
  // 3. layout: topic t's nodes at [nbase_t, nbase_t + R_t) (the device's bases)
  e->roots_host.clear();
  for (uint32_t t = 0; t < nt; ++t) e->topics[t].n_nodes = 0;
  for (uint32_t ai = 0; ai < na; ++ai) {
    TopicHost& T = e->topics[act[ai]];
    T.nbase = tb[2 * ai];
    T.n_nodes = tb[2 * ai + 2] - tb[2 * ai];
    e->roots_host.push_back(T.nbase);
  }
  const uint32_t nn = na ? tb[2 * na] : 0u;
  e->n_nodes = nn;
  e->n_pad = std::max<uint32_t>(16, ((nn + 15) / 16) * 16);
  if (e->host_timing) {
    auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    std::fprintf(stderr, "[psengine] gpu build: deltas %.3f ms (%zu), scratch %.3f ms, child lists + placement "
                 "+ readback %.3f ms\n", ms(tb0, tb1), pairs.size() / 2, ms(tb1, tb2), ms(tb2, tb3));
  }
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    T.mesh = false;
    T.root_local = true;
    T.cross.clear();
    const uint32_t* g = gs + static_cast<size_t>(t) * kGstWords;
    T.depth = T.n_nodes ? g[kGstDepth] : 0;
    T.max_deg = g[kGstMaxDeg];
    T.level_off.assign(T.depth + 2, 0);
    T.level_internal.assign(T.depth + 1, 0);
    T.level_local.clear();
    T.gcnt.clear();
    T.send_node.clear();
    T.send_dst.clear();
    T.send_lvl.clear();
    T.top_levels = 1;
    if (!T.n_nodes) continue;
    for (uint32_t d = 0; d <= T.depth; ++d) {
      T.level_off[d] = lh[512 * t + d];
      T.level_internal[d] = lh[512 * t + 256 + d];
    }
    T.level_off[T.depth + 1] = T.n_nodes;
    // the levels the top kernel places (parents of at most kBuildTopLevel)
    while (T.top_levels <= T.depth && T.level_off[T.top_levels] - T.level_off[T.top_levels - 1] <= kBuildTopLevel)
      ++T.top_levels;
    T.level_local.assign(T.depth + 1, 0);
    for (uint32_t d = 0; d <= T.depth; ++d) T.level_local[d] = T.level_off[d + 1] - T.level_off[d];
  }
  e->remote_fed.clear();
  e->ghost_ref.clear();
  e->ship_host.clear();
  e->gpu_graph = true;
  e->mirrors_valid = false;
  e->flags_built = true;  // (node flags from the current live mask: the flags pass can skip them)
  return PS_OK;
}

}  // namespace

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
      if (e->world > 1) {  // ghost parents: the record each ghost-fed node reads, the records each parent ships
        HIP_TRY(e->d_ghost_ref.ensure(std::max<size_t>(nn, 1) * 4), "alloc ghost refs");
        HIP_TRY(e->d_ship.ensure(std::max<size_t>(e->ship_host.size(), 1) * sizeof(ShipEntry)), "alloc ship entries");
        if (nn)
          HIP_TRY(hipMemcpyAsync(e->d_ghost_ref.p, e->ghost_ref.data(), nn * 4, hipMemcpyHostToDevice, e->stream),
                  "upload ghost refs");
        if (!e->ship_host.empty())
          HIP_TRY(hipMemcpyAsync(e->d_ship.p, e->ship_host.data(), e->ship_host.size() * sizeof(ShipEntry),
                                 hipMemcpyHostToDevice, e->stream),
                  "upload ship entries");
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
      bool fresh = false;
      HIP_TRY(e->d_live.ensure(n, &fresh), "alloc live mask");
      HIP_TRY(e->d_roots.ensure(std::max<size_t>(e->roots_host.size(), 1) * 4), "alloc roots");
      if (fresh || !e->live_dev_valid) {
        HIP_TRY(hipMemcpyAsync(e->d_live.p, e->live.data(), n, hipMemcpyHostToDevice, e->stream), "upload live");
        e->live_dev_valid = true;
      }
      // (the GPU build wrote every node's flags from this live mask itself)
      if (!e->flags_built) {
        if (!e->roots_host.empty())
          HIP_TRY(hipMemcpyAsync(e->d_roots.p, e->roots_host.data(), e->roots_host.size() * 4,
                                 hipMemcpyHostToDevice, e->stream),
                  "upload roots");
        HIP_TRY(launch_node_flags(e->d_node_peer.as<uint32_t>(), e->d_row_ptr.as<uint32_t>(),
                                  e->d_live.as<uint8_t>(), e->n_nodes, e->d_roots.as<uint32_t>(),
                                  static_cast<uint32_t>(e->roots_host.size()), e->d_node_flags.as<uint8_t>(),
                                  e->stream),
                "node flags");
      }
      e->flags_built = false;
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

}  // namespace psamd
