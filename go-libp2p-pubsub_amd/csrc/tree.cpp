// tree.cpp -- host-side subscription tree maintenance (see tree.hpp).
#include "tree.hpp"

#include <algorithm>
#include <deque>

#include "psengine.h"

namespace psamd {

SubscriptionTree::SubscriptionTree(uint32_t n_peers, uint32_t root, uint32_t width,
                                   uint32_t max_width, uint64_t seed)
    : n_(n_peers), root_(root), width_(width), max_width_(max_width), rng_(seed),
      touched_at_(n_peers, 0), rec_(n_peers) {
  rec_[root].state = PeerState::In;
}

void SubscriptionTree::kid_push(uint32_t p, const ChildRec& r) {
  PeerRec& R = rec_[p];
  if (R.spill == kNone && R.n < kInline) {
    R.kin[R.n++] = r;
    return;
  }
  if (R.spill == kNone) {  // the list outgrows the line: move it to a spill vector
    uint32_t s;
    if (!spill_free_.empty()) {
      s = spill_free_.back();
      spill_free_.pop_back();
    } else {
      s = static_cast<uint32_t>(spill_.size());
      spill_.emplace_back();
    }
    spill_[s].assign(R.kin, R.kin + R.n);
    R.spill = s;
  }
  auto& v = spill_[R.spill];
  v.resize(R.n);
  v.push_back(r);
  R.n = static_cast<uint32_t>(v.size());
}

void SubscriptionTree::kid_clear(uint32_t p) {
  PeerRec& R = rec_[p];
  if (R.spill != kNone) {
    spill_[R.spill].clear();
    spill_free_.push_back(R.spill);
    R.spill = kNone;
  }
  R.n = 0;
}

// Called after every change of p's state or upstream: records p's upstream
// code while its line is hot (take_touched hands the codes out without
// visiting the peers again).
void SubscriptionTree::touch(uint32_t p) {
  const uint32_t code = upstream_code(p);
  if (touched_at_[p]) {
    touched_code_[touched_at_[p] - 1] = code;
    return;
  }
  touched_.push_back(p);
  touched_code_.push_back(code);
  touched_at_[p] = static_cast<uint32_t>(touched_.size());
}

void SubscriptionTree::take_touched(std::vector<uint32_t>& out) {
  std::vector<uint32_t> codes;
  take_touched(out, codes);
}

void SubscriptionTree::take_touched(std::vector<uint32_t>& peers, std::vector<uint32_t>& codes) {
  peers.swap(touched_);
  codes.swap(touched_code_);
  touched_.clear();
  touched_code_.clear();
  for (uint32_t p : peers) touched_at_[p] = 0;
}

bool SubscriptionTree::reachable_memo(uint32_t p) {
  const uint32_t yes = 2 * reach_pass_, no = yes + 1;
  walk_.clear();
  bool ok = false;
  for (uint32_t hops = 0; hops <= n_; ++hops) {
    if (p == root_ || reach_stamp_[p] == yes) {
      ok = true;
      break;
    }
    if (reach_stamp_[p] == no || rec_[p].state != PeerState::In || rec_[p].up == kNone) break;
    walk_.push_back(p);
    p = rec_[p].up;
  }
  for (uint32_t q : walk_) reach_stamp_[q] = ok ? yes : no;
  return ok;
}

// Memoised over one pass like reachable_memo (unreached Part'ed parents of a
// decayed tree share their upstream paths): orphan_stamp_ = 2*pass + 1 for
// "an Orphan cuts the path", 2*pass for "it does not".
bool SubscriptionTree::below_orphan(uint32_t p) {
  const uint32_t no = 2 * reach_pass_, yes = no + 1;
  if (orphan_stamp_.size() != n_) orphan_stamp_.assign(n_, 0xFFFFFFFFu);
  walk_.clear();
  bool cut = false;
  for (uint32_t hops = 0; hops <= n_ && p != root_ && p != kNone; ++hops) {
    if (orphan_stamp_[p] == yes || orphan_stamp_[p] == no) {
      cut = orphan_stamp_[p] == yes;
      break;
    }
    if (rec_[p].state == PeerState::Orphan) {
      cut = true;
      break;
    }
    if (rec_[p].state != PeerState::In) break;
    walk_.push_back(p);
    p = rec_[p].up;
  }
  for (uint32_t q : walk_) orphan_stamp_[q] = cut ? yes : no;
  return cut;
}

void SubscriptionTree::below_orphan_many(const std::vector<uint32_t>& ps, std::vector<uint8_t>& cut) {
  constexpr size_t kWalks = 16;
  const uint32_t no = 2 * reach_pass_, yes = no + 1;
  if (orphan_stamp_.size() != n_) orphan_stamp_.assign(n_, 0xFFFFFFFFu);
  cut.assign(ps.size(), 0);
  std::vector<uint32_t> path[kWalks];
  for (size_t b = 0; b < ps.size(); b += kWalks) {
    const size_t m = std::min(kWalks, ps.size() - b);
    uint32_t cur[kWalks], hops[kWalks];
    bool done[kWalks];
    for (size_t j = 0; j < m; ++j) {
      cur[j] = ps[b + j];
      hops[j] = 0;
      done[j] = false;
      path[j].clear();
      if (cur[j] < n_) {
        __builtin_prefetch(&rec_[cur[j]]);
        __builtin_prefetch(&orphan_stamp_[cur[j]]);
      }
    }
    size_t active = m;
    while (active) {
      for (size_t j = 0; j < m; ++j) {
        if (done[j]) continue;
        const uint32_t p = cur[j];
        int res = -1;  // -1: continue upward, 0: not cut, 1: cut
        if (p == root_ || p == kNone || p >= n_ || hops[j] > n_) {
          res = 0;
        } else if (orphan_stamp_[p] == yes || orphan_stamp_[p] == no) {
          res = orphan_stamp_[p] == yes;
        } else if (rec_[p].state == PeerState::Orphan) {
          res = 1;
        } else if (rec_[p].state != PeerState::In) {
          res = 0;
        }
        if (res < 0) {
          path[j].push_back(p);
          cur[j] = rec_[p].up;
          ++hops[j];
          if (cur[j] < n_) {
            __builtin_prefetch(&rec_[cur[j]]);
            __builtin_prefetch(&orphan_stamp_[cur[j]]);
          }
          continue;
        }
        for (uint32_t q : path[j]) orphan_stamp_[q] = res ? yes : no;
        cut[b + j] = static_cast<uint8_t>(res);
        done[j] = true;
        --active;
      }
    }
  }
}

// SplitMix64: stands in for Go's randomised map iteration (rule Q2).
uint64_t SubscriptionTree::next_random() {
  uint64_t z = (rng_ += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Walk of one join request: handleJoin at `at` (subtree.go:110-154), each
// redirectJoin hop (156-194) followed by the joiner's next Join in
// joinParents (241-307) at prio=false.
int SubscriptionTree::attach(uint32_t at, uint32_t joiner, bool prio) {
  while (true) {
    const uint32_t cnt = rec_[at].n;
    const size_t cap = prio ? max_width_ : width_;
    if (cnt < cap) {
      kid_push(at, ChildRec{joiner, kNone, 0, 0});
      rec_[joiner].up = at;
      rec_[joiner].state = PeerState::In;
      touch(joiner);
      // State{Peers:[joiner], NumPeers: sub.size(=0)} upstream (137-147);
      // only a node holding a live `in` stream sends it (client.go:106).
      const uint32_t gp = rec_[at].up;
      if (at != root_ && gp != kNone && rec_[at].state == PeerState::In) {
        ChildRec* k = kids(gp);
        for (uint32_t i = 0, m = rec_[gp].n; i < m; ++i)
          if (k[i].id == at) {
            k[i].redirects = 1;
            k[i].last_state = joiner;
            break;
          }
      }
      return PS_OK;
    }
    if (cnt == 0) return PS_E_NOPARENT;
    ChildRec* list = kids(at);
    // the walk continues at one of these children: start fetching their
    // lines (state, upstream, child list) while the redirect choice is made
    for (uint32_t i = 0; i < cnt; ++i) __builtin_prefetch(&rec_[list[i].id]);
    int64_t best = 10000000000ll;
    uint32_t ties = 0;
    for (uint32_t i = 0; i < cnt; ++i) {
      const ChildRec& r = list[i];
      if (r.parted) continue;
      if (r.redirects < best) {
        best = r.redirects;
        ties = 1;
      } else if (r.redirects == best) {
        ++ties;
      }
    }
    if (ties == 0) return PS_E_NOPARENT;
    uint32_t k = ties > 1 ? static_cast<uint32_t>(next_random() % ties) : 0;
    ChildRec* pick = nullptr;
    for (uint32_t i = 0; i < cnt; ++i) {
      ChildRec& r = list[i];
      if (r.parted || r.redirects != best) continue;
      if (k-- == 0) {
        pick = &r;
        break;
      }
    }
    pick->redirects += 1;
    const uint32_t target = pick->id;
    if (rec_[target].state == PeerState::Failed) return PS_E_UNREACHABLE;
    at = target;
    prio = false;
  }
}

int SubscriptionTree::subscribe(uint32_t peer) {
  if (peer >= n_) return PS_E_INVAL;
  if (peer == root_ || rec_[peer].state != PeerState::Out) return PS_E_STATE;
  return attach(root_, peer, false);
}

// `gone` left the tree under `at`: every child of `gone` loses its upstream;
// the last one `gone` reported (`rescue`) is re-joined at `at` with prio
// (redistributeChildren, subtree.go:356-375); the rest are orphaned (Q5).
void SubscriptionTree::depart(uint32_t at, uint32_t gone, uint32_t rescue) {
  {
    const ChildRec* k = kids(gone);
    for (uint32_t i = 0, m = rec_[gone].n; i < m; ++i)
      if (k[i].id != rescue && rec_[k[i].id].state == PeerState::In) {
        rec_[k[i].id].state = PeerState::Orphan;
        touch(k[i].id);
      }
  }
  kid_clear(gone);
  if (rescue == kNone) return;
  if (rec_[rescue].state != PeerState::In || rec_[rescue].up != gone) return;
  rec_[rescue].state = PeerState::Out;
  touch(rescue);
  if (attach(at, rescue, true) != PS_OK) {
    rec_[rescue].state = PeerState::Orphan;
    rec_[rescue].up = gone;
    touch(rescue);
  }
}

int SubscriptionTree::close_client(uint32_t peer) {
  if (peer >= n_) return PS_E_INVAL;
  if (peer == root_ || rec_[peer].state != PeerState::In) return PS_E_STATE;
  const uint32_t at = rec_[peer].up;
  rec_[peer].state = PeerState::Dead;
  touch(peer);
  ChildRec* rec = nullptr;
  if (at != kNone && rec_[at].state != PeerState::Failed) {  // a Part to a closed host is lost
    ChildRec* k = kids(at);
    for (uint32_t i = 0, m = rec_[at].n; i < m; ++i)
      if (k[i].id == peer) {
        rec = &k[i];
        break;
      }
  }
  if (rec == nullptr) {
    depart(at, peer, kNone);
    return PS_OK;
  }
  rec->parted = 1;  // handleChildMessages Part (subtree.go:62-70)
  needs_pass_ = true;
  parted_at_.push_back(at);
  depart(at, peer, rec->last_state);
  return PS_OK;
}

void SubscriptionTree::prefetch_leave(uint32_t peer, int stage) const {
  if (peer >= n_) return;
  if (stage == 0) {
    __builtin_prefetch(&rec_[peer]);
    return;
  }
  const PeerRec& R = rec_[peer];
  if (R.spill != kNone) __builtin_prefetch(spill_[R.spill].data());
  const uint32_t at = R.up;
  if (at < n_) {
    __builtin_prefetch(&rec_[at]);
    if (rec_[at].spill != kNone) __builtin_prefetch(spill_[rec_[at].spill].data());
  }
  // the rescued child re-joins at `at`; the orphans' lines are written
  const ChildRec* k = kids(peer);
  for (uint32_t i = 0, m = R.n; i < m; ++i) __builtin_prefetch(&rec_[k[i].id]);
}

int SubscriptionTree::close_host(uint32_t peer) {
  if (peer >= n_) return PS_E_INVAL;
  if (peer == root_) return PS_E_STATE;
  if (rec_[peer].state != PeerState::In && rec_[peer].state != PeerState::Orphan) return PS_E_STATE;
  rec_[peer].state = PeerState::Failed;
  touch(peer);
  pending_failures_ = true;
  needs_pass_ = true;
  return PS_OK;
}

const std::vector<uint32_t>& SubscriptionTree::part_parents() {
  // distinct parents (the pass is order free): marked once, marks reset
  if (dedup_mark_.size() != n_) dedup_mark_.assign(n_, 0);
  size_t w = 0;
  for (uint32_t p : parted_at_)
    if (p < n_ && !dedup_mark_[p]) {
      dedup_mark_[p] = 1;
      parted_at_[w++] = p;
    }
  parted_at_.resize(w);
  for (uint32_t p : parted_at_) dedup_mark_[p] = 0;
  return parted_at_;
}

int SubscriptionTree::after_message(const ReachQuery* reach) {
  if (!needs_pass_) return PS_OK;
  if (!pending_failures_) {
    // Parts only: the lazy prune at each forwarding node deletes Part'ed
    // entries (subtree.go:329-331), draws nothing from the tie-break stream,
    // so the order does not matter -- visit just the parents holding one,
    // if the message reached them (an In-state path from the root).
    part_parents();
    // reachability of the message's tree, before this pass mutates anything
    // (the prune below only edits child lists of reached parents and puts Dead
    // children Out: no reached peer's path changes)
    if (reach_stamp_.size() != n_) reach_stamp_.assign(n_, 0xFFFFFFFFu);
    if (++reach_pass_ >= 0x7FFFFFF0u) {
      std::fill(reach_stamp_.begin(), reach_stamp_.end(), 0xFFFFFFFFu);
      std::fill(orphan_stamp_.begin(), orphan_stamp_.end(), 0xFFFFFFFFu);
      reach_pass_ = 1;
    }
    std::vector<uint8_t> reached(parted_at_.size());
    std::vector<uint8_t> cut;  // per unreached entry, in order
    if (reach) {
      int rc = (*reach)(parted_at_, reached);
      if (rc) return rc;
      for (size_t i = 0; i < parted_at_.size(); ++i)
        if (reached[i] != 1 && parted_at_[i] < n_) cut.push_back(reached[i] == 2);
      for (auto& x : reached) x = x == 1;
    } else {
      for (size_t i = 0; i < parted_at_.size(); ++i)
        reached[i] = parted_at_[i] < n_ && reachable_memo(parted_at_[i]);
      // the unreached ones: cut for good (below an Orphan) or kept for a
      // later message, decided by walks run in lockstep
      std::vector<uint32_t> unreached;
      for (size_t i = 0; i < parted_at_.size(); ++i)
        if (!reached[i] && parted_at_[i] < n_) unreached.push_back(parted_at_[i]);
      below_orphan_many(unreached, cut);
    }
    size_t ui = 0;
    std::vector<uint32_t> keep;
    // scattered parents: their lines are fetched 16 ahead, their children's 8 ahead
    constexpr size_t kAhead0 = 16, kAhead1 = 8;
    const size_t np = parted_at_.size();
    auto fetch_kids = [&](uint32_t q) {
      if (q >= n_) return;
      const ChildRec* k = kids(q);
      for (uint32_t j = 0, m = rec_[q].n; j < m; ++j)
        if (k[j].parted) __builtin_prefetch(&rec_[k[j].id]);
    };
    for (size_t i = 0; i < std::min(np, kAhead0); ++i)
      if (parted_at_[i] < n_) __builtin_prefetch(&rec_[parted_at_[i]]);
    for (size_t i = 0; i < std::min(np, kAhead1); ++i) fetch_kids(parted_at_[i]);
    for (size_t i = 0; i < np; ++i) {
      if (i + kAhead0 < np && parted_at_[i + kAhead0] < n_) __builtin_prefetch(&rec_[parted_at_[i + kAhead0]]);
      if (i + kAhead1 < np) fetch_kids(parted_at_[i + kAhead1]);
      const uint32_t p = parted_at_[i];
      if (!reached[i]) {
        // pruned by a later message that reaches it -- unless an orphan cuts
        // it off for good (an Orphan never becomes In again, Q5)
        if (p < n_ && !cut[ui++]) keep.push_back(p);
        continue;
      }
      ChildRec* list = kids(p);
      uint32_t w = 0;
      for (uint32_t k = 0, m = rec_[p].n; k < m; ++k) {
        const ChildRec r = list[k];
        if (r.parted) {
          if (rec_[r.id].state == PeerState::Dead) {
            rec_[r.id].state = PeerState::Out;
            rec_[r.id].up = kNone;
            touch(r.id);
          }
          continue;
        }
        list[w++] = r;
      }
      kid_shrink(p, w);
    }
    parted_at_.swap(keep);
    needs_pass_ = !parted_at_.empty();
    return PS_OK;
  }
  // forwarding nodes in BFS order over subscribed peers
  std::vector<uint32_t> order;
  order.reserve(64);
  std::deque<uint32_t> q{root_};
  while (!q.empty()) {
    uint32_t p = q.front();
    q.pop_front();
    order.push_back(p);
    for (const ChildRec& r : children(p))
      if (rec_[r.id].state == PeerState::In) q.push_back(r.id);
  }
  for (uint32_t p : order) {
    ChildRec* list = kids(p);
    std::vector<ChildRec> failed;
    uint32_t w = 0;
    for (uint32_t i = 0, m = rec_[p].n; i < m; ++i) {
      ChildRec r = list[i];
      if (r.parted) {  // delete(sub.children, c.id), subtree.go:329-331
        if (rec_[r.id].state == PeerState::Dead) {
          rec_[r.id].state = PeerState::Out;
          rec_[r.id].up = kNone;
          touch(r.id);
        }
        continue;
      }
      if (rec_[r.id].state == PeerState::Failed) {  // write error, subtree.go:333-336
        failed.push_back(r);
        continue;
      }
      list[w++] = r;
    }
    kid_shrink(p, w);
    for (const auto& r : failed) depart(p, r.id, r.last_state);  // 342-349
  }
  pending_failures_ = false;
  needs_pass_ = false;
  // Part'ed entries under parents this message did not reach stay listed
  std::vector<uint32_t> keep;
  for (uint32_t p : parted_at_)
    for (const ChildRec& r : children(p))
      if (r.parted) {
        keep.push_back(p);
        needs_pass_ = true;
        break;
      }
  parted_at_.swap(keep);
  for (uint32_t p = 0; p < n_ && !pending_failures_; ++p)
    if (rec_[p].state == PeerState::Failed && rec_[p].up != kNone) {
      for (const ChildRec& r : children(rec_[p].up))
        if (r.id == p) {
          pending_failures_ = true;
          needs_pass_ = true;
          break;
        }
    }
  return PS_OK;
}

void SubscriptionTree::attached_parents(std::vector<uint32_t>& parent) const {
  parent.assign(n_, kNone);
  std::vector<uint32_t> stack{root_};
  while (!stack.empty()) {
    uint32_t p = stack.back();
    stack.pop_back();
    for (const ChildRec& r : children(p))
      if (rec_[r.id].state == PeerState::In) {
        parent[r.id] = p;
        stack.push_back(r.id);
      }
  }
}

}  // namespace psamd
