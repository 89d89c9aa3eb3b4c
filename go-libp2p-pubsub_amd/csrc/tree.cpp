// tree.cpp -- host-side subscription tree maintenance (see tree.hpp).
#include "tree.hpp"

#include <algorithm>
#include <deque>

#include "psengine.h"

namespace psamd {

SubscriptionTree::SubscriptionTree(uint32_t n_peers, uint32_t root, uint32_t width,
                                   uint32_t max_width, uint64_t seed)
    : n_(n_peers), root_(root), width_(width), max_width_(max_width), rng_(seed),
      touched_mark_(n_peers, 0), state_(n_peers, PeerState::Out), up_(n_peers, kNone),
      kids_(n_peers) {
  state_[root] = PeerState::In;
}

void SubscriptionTree::touch(uint32_t p) {
  if (!touched_mark_[p]) {
    touched_mark_[p] = 1;
    touched_.push_back(p);
  }
}

void SubscriptionTree::take_touched(std::vector<uint32_t>& out) {
  out.swap(touched_);
  touched_.clear();
  for (uint32_t p : out) touched_mark_[p] = 0;
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
    if (reach_stamp_[p] == no || state_[p] != PeerState::In || up_[p] == kNone) break;
    walk_.push_back(p);
    p = up_[p];
  }
  for (uint32_t q : walk_) reach_stamp_[q] = ok ? yes : no;
  return ok;
}

bool SubscriptionTree::below_orphan(uint32_t p) const {
  for (uint32_t hops = 0; hops <= n_ && p != root_ && p != kNone; ++hops) {
    if (state_[p] == PeerState::Orphan) return true;
    if (state_[p] != PeerState::In) return false;
    p = up_[p];
  }
  return false;
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
    auto& list = kids_[at];
    const size_t cap = prio ? max_width_ : width_;
    if (list.size() < cap) {
      list.push_back(ChildRec{joiner, kNone, 0, false});
      up_[joiner] = at;
      state_[joiner] = PeerState::In;
      touch(joiner);
      // State{Peers:[joiner], NumPeers: sub.size(=0)} upstream (137-147);
      // only a node holding a live `in` stream sends it (client.go:106).
      const uint32_t gp = up_[at];
      if (at != root_ && gp != kNone && state_[at] == PeerState::In) {
        for (auto& r : kids_[gp])
          if (r.id == at) {
            r.redirects = 1;
            r.last_state = joiner;
            break;
          }
      }
      return PS_OK;
    }
    if (list.empty()) return PS_E_NOPARENT;
    // the walk continues at one of these children: start fetching their
    // entries while the redirect choice is made
    for (const auto& r : list) {
      __builtin_prefetch(&kids_[r.id]);
      __builtin_prefetch(&state_[r.id]);
    }
    int64_t best = 10000000000ll;
    uint32_t ties = 0;
    for (const auto& r : list) {
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
    for (auto& r : list) {
      if (r.parted || r.redirects != best) continue;
      if (k-- == 0) {
        pick = &r;
        break;
      }
    }
    pick->redirects += 1;
    const uint32_t target = pick->id;
    if (state_[target] == PeerState::Failed) return PS_E_UNREACHABLE;
    at = target;
    prio = false;
  }
}

int SubscriptionTree::subscribe(uint32_t peer) {
  if (peer >= n_) return PS_E_INVAL;
  if (peer == root_ || state_[peer] != PeerState::Out) return PS_E_STATE;
  return attach(root_, peer, false);
}

// `gone` left the tree under `at`: every child of `gone` loses its upstream;
// the last one `gone` reported (`rescue`) is re-joined at `at` with prio
// (redistributeChildren, subtree.go:356-375); the rest are orphaned (Q5).
void SubscriptionTree::depart(uint32_t at, uint32_t gone, uint32_t rescue) {
  for (const auto& r : kids_[gone])
    if (r.id != rescue && state_[r.id] == PeerState::In) {
      state_[r.id] = PeerState::Orphan;
      touch(r.id);
    }
  kids_[gone].clear();
  if (rescue == kNone) return;
  if (state_[rescue] != PeerState::In || up_[rescue] != gone) return;
  state_[rescue] = PeerState::Out;
  touch(rescue);
  if (attach(at, rescue, true) != PS_OK) {
    state_[rescue] = PeerState::Orphan;
    up_[rescue] = gone;
  }
}

int SubscriptionTree::close_client(uint32_t peer) {
  if (peer >= n_) return PS_E_INVAL;
  if (peer == root_ || state_[peer] != PeerState::In) return PS_E_STATE;
  const uint32_t at = up_[peer];
  state_[peer] = PeerState::Dead;
  touch(peer);
  ChildRec* rec = nullptr;
  if (at != kNone && state_[at] != PeerState::Failed)  // a Part to a closed host is lost
    for (auto& r : kids_[at])
      if (r.id == peer) {
        rec = &r;
        break;
      }
  if (rec == nullptr) {
    depart(at, peer, kNone);
    return PS_OK;
  }
  rec->parted = true;  // handleChildMessages Part (subtree.go:62-70)
  needs_pass_ = true;
  parted_at_.push_back(at);
  depart(at, peer, rec->last_state);
  return PS_OK;
}

void SubscriptionTree::prefetch_leave(uint32_t peer, int stage) const {
  if (peer >= n_) return;
  if (stage == 0) {
    __builtin_prefetch(&state_[peer]);
    __builtin_prefetch(&up_[peer]);
    __builtin_prefetch(&kids_[peer]);
    return;
  }
  if (!kids_[peer].empty()) __builtin_prefetch(kids_[peer].data());
  const uint32_t at = up_[peer];
  if (at < n_) {
    __builtin_prefetch(&kids_[at]);
    __builtin_prefetch(&state_[at]);
    if (!kids_[at].empty()) __builtin_prefetch(kids_[at].data());
  }
}

int SubscriptionTree::close_host(uint32_t peer) {
  if (peer >= n_) return PS_E_INVAL;
  if (peer == root_) return PS_E_STATE;
  if (state_[peer] != PeerState::In && state_[peer] != PeerState::Orphan) return PS_E_STATE;
  state_[peer] = PeerState::Failed;
  touch(peer);
  pending_failures_ = true;
  needs_pass_ = true;
  return PS_OK;
}

int SubscriptionTree::after_message(const ReachQuery* reach) {
  if (!needs_pass_) return PS_OK;
  if (!pending_failures_) {
    // Parts only: the lazy prune at each forwarding node deletes Part'ed
    // entries (subtree.go:329-331), draws nothing from the tie-break stream,
    // so the order does not matter -- visit just the parents holding one,
    // if the message reached them (an In-state path from the root).
    std::sort(parted_at_.begin(), parted_at_.end());
    parted_at_.erase(std::unique(parted_at_.begin(), parted_at_.end()), parted_at_.end());
    // reachability of the message's tree, before this pass mutates anything
    // (the prune below only edits child lists of reached parents and puts Dead
    // children Out: no reached peer's path changes)
    if (reach_stamp_.size() != n_) reach_stamp_.assign(n_, 0xFFFFFFFFu);
    if (++reach_pass_ >= 0x7FFFFFF0u) {
      std::fill(reach_stamp_.begin(), reach_stamp_.end(), 0xFFFFFFFFu);
      reach_pass_ = 1;
    }
    std::vector<uint8_t> reached(parted_at_.size());
    if (reach) {
      int rc = (*reach)(parted_at_, reached);
      if (rc) return rc;
    } else {
      for (size_t i = 0; i < parted_at_.size(); ++i)
        reached[i] = parted_at_[i] < n_ && reachable_memo(parted_at_[i]);
    }
    std::vector<uint32_t> keep;
    for (size_t i = 0; i < parted_at_.size(); ++i) {
      const uint32_t p = parted_at_[i];
      if (!reached[i]) {
        // pruned by a later message that reaches it -- unless an orphan cuts
        // it off for good (an Orphan never becomes In again, Q5)
        if (p < n_ && !below_orphan(p)) keep.push_back(p);
        continue;
      }
      auto& list = kids_[p];
      size_t w = 0;
      for (size_t k = 0; k < list.size(); ++k) {
        const ChildRec r = list[k];
        if (r.parted) {
          if (state_[r.id] == PeerState::Dead) {
            state_[r.id] = PeerState::Out;
            up_[r.id] = kNone;
            touch(r.id);
          }
          continue;
        }
        list[w++] = r;
      }
      list.resize(w);
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
    for (const auto& r : kids_[p])
      if (state_[r.id] == PeerState::In) q.push_back(r.id);
  }
  for (uint32_t p : order) {
    auto& list = kids_[p];
    std::vector<ChildRec> failed;
    size_t w = 0;
    for (size_t i = 0; i < list.size(); ++i) {
      ChildRec r = list[i];
      if (r.parted) {  // delete(sub.children, c.id), subtree.go:329-331
        if (state_[r.id] == PeerState::Dead) {
          state_[r.id] = PeerState::Out;
          up_[r.id] = kNone;
          touch(r.id);
        }
        continue;
      }
      if (state_[r.id] == PeerState::Failed) {  // write error, subtree.go:333-336
        failed.push_back(r);
        continue;
      }
      list[w++] = r;
    }
    list.resize(w);
    for (const auto& r : failed) depart(p, r.id, r.last_state);  // 342-349
  }
  pending_failures_ = false;
  needs_pass_ = false;
  // Part'ed entries under parents this message did not reach stay listed
  std::vector<uint32_t> keep;
  for (uint32_t p : parted_at_)
    for (const auto& r : kids_[p])
      if (r.parted) {
        keep.push_back(p);
        needs_pass_ = true;
        break;
      }
  parted_at_.swap(keep);
  for (uint32_t p = 0; p < n_ && !pending_failures_; ++p)
    if (state_[p] == PeerState::Failed && up_[p] != kNone) {
      for (const auto& r : kids_[up_[p]])
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
    for (const auto& r : kids_[p])
      if (state_[r.id] == PeerState::In) {
        parent[r.id] = p;
        stack.push_back(r.id);
      }
  }
}

}  // namespace psamd
