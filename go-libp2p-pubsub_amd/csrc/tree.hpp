// tree.hpp -- host-side subscription tree of one topic (product code).
//
// Restates the reference's tree maintenance (subtree.go:16-307,356-375,
// client.go:36-98) under the quiescent rules Q1-Q5 documented in DESIGN.md
// §3.  This is the *input generator* for the GPU hot path: it decides which
// peer hangs below which; the dissemination itself never runs here.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace psamd {

constexpr uint32_t kNone = 0xFFFFFFFFu;

enum class PeerState : uint8_t { Out = 0, In = 1, Dead = 2, Failed = 3, Orphan = 4 };

// The parent's record of one child (subtree.go:36-44).
struct ChildRec {
  uint32_t id;
  uint32_t last_state;  // `children` of the last State message (one peer)
  int32_t redirects;    // `size`: reset to NumPeers+1 = 1 by State, ++ per redirect
  uint32_t parted;      // `dead`: set by a Part message
};

// A peer's child records, in insertion order (iteration only).
struct ChildSpan {
  const ChildRec* b;
  const ChildRec* e;
  const ChildRec* begin() const { return b; }
  const ChildRec* end() const { return e; }
  size_t size() const { return static_cast<size_t>(e - b); }
};

class SubscriptionTree {
 public:
  SubscriptionTree() = default;
  SubscriptionTree(uint32_t n_peers, uint32_t root, uint32_t width, uint32_t max_width,
                   uint64_t seed);

  // 0 or a negative PS_E_* code.
  int subscribe(uint32_t peer);
  int close_client(uint32_t peer);  // graceful: Part
  // Cache hint for a batch of leaves (no state change): stage 0 touches the
  // peer's own entries, stage 1 (a few peers later) its child lists and its
  // parent's list, so close_client() finds them resident.
  void prefetch_leave(uint32_t peer, int stage) const;
  void prefetch_peer(uint32_t peer) const { __builtin_prefetch(&rec_[peer]); }  // state, upstream, children
  // a joiner's own line and touched-list slot (written when it attaches)
  void prefetch_join(uint32_t peer) const {
    if (peer >= n_) return;
    __builtin_prefetch(&rec_[peer], 1);
    __builtin_prefetch(&touched_at_[peer], 1);
  }
  int close_host(uint32_t peer);    // abrupt
  // Called once per message that floods this topic: lazy prune and repair of
  // failed writes at every node the message reached (rule Q3).  `reach`, if
  // given, answers for a batch of peers: 1 = the message reached the peer,
  // 2 = it did not and an Orphan cuts the peer's upstream path for good, 0 =
  // neither (the engine asks the node space the message ran on); otherwise
  // the tree walks up from each peer.
  using ReachQuery = std::function<int(const std::vector<uint32_t>& peers, std::vector<uint8_t>& out)>;
  int after_message(const ReachQuery* reach = nullptr);
  // a Parts-only message pass is pending: its distinct Part'ed parents (the
  // peers after_message will ask `reach` about, deduplicated in place), so
  // that the engine can ask the GPU before the message runs
  bool parts_only_pass() const { return needs_pass_ && !pending_failures_; }
  const std::vector<uint32_t>& part_parents();
  bool has_pending_failures() const { return pending_failures_; }
  // a Part or a host failure happened since the last after_message()
  bool needs_message_pass() const { return needs_pass_; }
  size_t parted_parents() const { return parted_at_.size(); }  // pending lazy prunes (diagnostics)

  // Attached structure: parent of every peer reachable from the root through
  // subscribed peers, kNone elsewhere.
  void attached_parents(std::vector<uint32_t>& parent) const;
  // Upstream of every subscribed (In) peer, kNone elsewhere; reachability from
  // the root is left to the consumer (the GPU rebuild).  take_touched() hands
  // out the peers whose entry may have changed since the last call (and their
  // upstream codes, recorded when they changed).
  uint32_t in_parent(uint32_t p) const {
    return rec_[p].state == PeerState::In && p != root_ ? rec_[p].up : kNone;
  }
  // in_parent, or kOrphanUp for an Orphan (its subtree is cut for good): what
  // the GPU rebuild ships, so the lazy prune's orphan walks run there too
  static constexpr uint32_t kOrphanUp = 0xFFFFFFFEu;
  uint32_t upstream_code(uint32_t p) const {
    return rec_[p].state == PeerState::Orphan ? kOrphanUp : in_parent(p);
  }
  void take_touched(std::vector<uint32_t>& out);
  void take_touched(std::vector<uint32_t>& peers, std::vector<uint32_t>& codes);
  // Peers reachable for the NEXT message (failed hosts cut their subtree).
  // Children lists in insertion order.
  ChildSpan children(uint32_t p) const {
    const ChildRec* k = kids(p);
    return ChildSpan{k, k + rec_[p].n};
  }
  PeerState state(uint32_t p) const { return rec_[p].state; }
  uint32_t root() const { return root_; }
  uint32_t n_peers() const { return n_; }

 private:
  int attach(uint32_t at, uint32_t joiner, bool prio);
  void depart(uint32_t at, uint32_t gone, uint32_t rescue);
  uint64_t next_random();

  // In-state path from the root?  Memoised over one pass: every peer on a
  // walked path is stamped reachable / unreachable (top levels are shared).
  bool reachable_memo(uint32_t p);
  bool below_orphan(uint32_t p);  // an Orphan on the upstream path (cut for good); memoised per pass
  // below_orphan of many peers, kWalks walks in lockstep (their cache misses overlap)
  void below_orphan_many(const std::vector<uint32_t>& ps, std::vector<uint8_t>& cut);
  void touch(uint32_t p);             // (state, upstream) of p may have changed

  // One cache line per peer: upstream, state and (up to kInline) child
  // records, so a join walk touches one line per level (and prefetches the
  // candidate children's lines while it picks among them).  Longer lists
  // (prio re-joins up to MaxWidth, wide trees) live in spill_.
  static constexpr uint32_t kInline = 3;
  struct alignas(64) PeerRec {
    uint32_t up = kNone;  // upstream peer (the other end of `in`)
    PeerState state = PeerState::Out;
    uint8_t pad[3] = {0, 0, 0};
    uint32_t n = 0;          // children (TreeWidth / MaxWidth are unbounded: no 16-bit count)
    uint32_t spill = kNone;  // index into spill_, or kNone: the records are inline
    ChildRec kin[kInline];
  };
  static_assert(sizeof(PeerRec) == 64, "one cache line per peer");
  ChildRec* kids(uint32_t p) { return rec_[p].spill == kNone ? rec_[p].kin : spill_[rec_[p].spill].data(); }
  const ChildRec* kids(uint32_t p) const {
    return rec_[p].spill == kNone ? rec_[p].kin : spill_[rec_[p].spill].data();
  }
  void kid_push(uint32_t p, const ChildRec& r);
  void kid_clear(uint32_t p);
  void kid_shrink(uint32_t p, uint32_t n) { rec_[p].n = n; }

  uint32_t n_ = 0, root_ = 0, width_ = 2, max_width_ = 5;
  uint64_t rng_ = 0;
  bool pending_failures_ = false;
  bool needs_pass_ = false;
  std::vector<uint32_t> parted_at_;  // parents holding a Part'ed child entry
  std::vector<uint32_t> touched_;       // peers whose attachment may have changed
  std::vector<uint32_t> touched_code_;  // ... and their upstream_code() after the last change
  std::vector<uint32_t> touched_at_;    // per peer: its index in touched_ + 1 (0: not listed)
  std::vector<uint8_t> dedup_mark_;  // after_message: distinct Part'ed parents
  std::vector<uint32_t> reach_stamp_;  // 2*pass: reachable, 2*pass+1: not (reachable_memo)
  std::vector<uint32_t> orphan_stamp_;  // 2*pass: not cut, 2*pass+1: cut (below_orphan)
  uint32_t reach_pass_ = 0;
  std::vector<uint32_t> walk_;
  std::vector<PeerRec> rec_;
  std::vector<std::vector<ChildRec>> spill_;
  std::vector<uint32_t> spill_free_;
};

}  // namespace psamd
