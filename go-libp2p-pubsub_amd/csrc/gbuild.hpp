// gbuild.hpp -- GPU rebuild of the node space from per-topic parent arrays
// (DESIGN.md §4.1).  Single rank, tree topics.
//
// For each topic: the upstream of every subscribed peer (kNone otherwise,
// maintained on the host by the restated join / leave protocol and shipped as
// deltas) -> depth of every peer reachable from the root (pointer jumping) ->
// one radix sort of (depth, parent, peer) keys: each BFS level is a
// contiguous range, siblings consecutive -> node ids level by level (the
// sibling groups in parent node order: a scan of the parents' fan-out, no
// further sort) -> node_parent, CSR, flags.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace psamd {

constexpr uint32_t kBuildMaxDepth = 255;  // depth bits of the sort key
constexpr uint32_t kBuildPeerBits = 28;   // peer / parent bits of the sort key at most
// The sort key of a reachable peer p: depth << 2b | parent << b | p, with b =
// the bits of the largest peer id -- the radix sort covers 2b + 8 bits only
// (1M peers: 48 bits, 6 passes of 8 instead of 8).  Unreachable peers: ~0.
struct BuildKey {
  uint32_t b;
  __host__ __device__ uint64_t make(uint32_t depth, uint32_t parent, uint32_t peer) const {
    return static_cast<uint64_t>(depth) << (2 * b) | static_cast<uint64_t>(parent) << b | peer;
  }
  __host__ __device__ uint32_t peer(uint64_t k) const { return static_cast<uint32_t>(k & ((1ull << b) - 1)); }
  __host__ __device__ uint32_t parent(uint64_t k) const {
    return static_cast<uint32_t>((k >> b) & ((1ull << b) - 1));
  }
  __host__ __device__ uint32_t depth(uint64_t k) const { return static_cast<uint32_t>((k >> (2 * b)) & 0xFFu); }
  uint32_t sort_bits() const { return 2 * b + 8; }
};
inline BuildKey build_key(uint32_t n_peers) {
  uint32_t b = 1;
  while (b < kBuildPeerBits && (1ull << b) < n_peers) ++b;
  return BuildKey{b};
}
constexpr uint32_t kBuildSmallLevel = 8192;  // levels placed by the one-block kernel

// Pair value of an Orphan peer (not subscribed: no upstream; its subtree is
// cut for good, rule Q5): par[p] = kNone, orph[p] = 1.
constexpr uint32_t kOrphanCode = 0xFFFFFFFEu;
// (peer, value) pairs scattered into a parent array and its orphan bytes
hipError_t launch_scatter_pairs(const uint32_t* pairs, uint32_t n, uint32_t* par, uint8_t* orph, hipStream_t s);

// Depth of every peer (pointer jumping, `jumps` steps: depths up to 2^jumps
// resolve): keys[p] = kf.make(depth, parent, p) for peers reachable from
// root, ~0 otherwise; gstat[0] += reachable count, gstat[1] = max(depth),
// gstat[3] += unresolved peers (more jumps needed).  Scratch: anc[2][n],
// dep[2][n].
hipError_t launch_depth_keys(const uint32_t* par, uint32_t n, uint32_t root, uint32_t jumps,
                             uint32_t* anc0, uint32_t* anc1, uint32_t* dep0, uint32_t* dep1,
                             uint64_t* keys, uint32_t* gstat, BuildKey kf, hipStream_t s);
// jumps that resolve any depth below n
inline uint32_t depth_jumps_full(uint32_t n) {
  uint32_t j = 1;
  while ((1ull << j) < n) ++j;
  return j + 1;
}

// hipcub radix sort of n keys (in -> out); temp queried when temp == nullptr.
// peer_bits = false: only the (depth, parent) bits are sorted -- the radix
// sort is stable and the keys come in peer order (keys[p] is peer p's), so
// siblings still end up in peer order, with b fewer key bits to pass over
// (cfg5: 28 of 48 bits); true: every bit (A/B: PSAMD_SORT_PEER_BITS=1)
hipError_t sort_keys(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, uint32_t n,
                     BuildKey kf, bool peer_bits, hipStream_t s);
// exclusive scan of n u32 (in -> out)
hipError_t scan_u32(void* temp, size_t* temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                    hipStream_t s);

// level starts of a topic's sorted keys (lvl_start[d], topic-relative)
hipError_t launch_level_starts(const uint64_t* keys, uint32_t R, uint32_t* lvl_start, BuildKey kf, hipStream_t s);
hipError_t launch_level_internal(const uint32_t* deg, uint32_t nbase, uint32_t R,
                                 const uint32_t* lvl_start, uint32_t depth, uint32_t* lvl_internal,
                                 uint32_t* max_deg, hipStream_t s);
// Sort-free BFS placement: fan-out / first child index of every parent peer
// from the (depth, parent, peer)-sorted keys; the root; then level by level,
// each child at nbase + lo + childoff[parent node - prev0] + sibling rank,
// where childoff is the exclusive scan of the parents' fan-out (deg).
hipError_t launch_child_stats(const uint64_t* keys, uint32_t R, uint32_t* cnt, uint32_t* firstidx,
                              BuildKey kf, hipStream_t s);
hipError_t launch_place_root(const uint64_t* keys, uint32_t nbase, uint16_t topic, const uint32_t* cnt,
                             uint32_t* node_peer, uint16_t* node_topic, uint32_t* local,
                             uint32_t* node_parent, uint32_t* deg, BuildKey kf, hipStream_t s);
// root and levels 1 .. d_end - 1 in one block; every one of those levels and
// its parent level has at most kBuildSmallLevel nodes.  lvl: the topic's level
// starts on the device (level d ends at lvl[d + 1], the last one at n_nodes).
hipError_t launch_place_small(const uint64_t* keys, const uint32_t* lvl, uint32_t d_end, uint32_t depth, uint32_t n_nodes,
                              uint32_t nbase, uint16_t topic, const uint32_t* cnt, const uint32_t* firstidx,
                              uint32_t* node_peer, uint16_t* node_topic, uint32_t* local,
                              uint32_t* node_parent, uint32_t* deg, uint32_t* first, BuildKey kf, hipStream_t s);
hipError_t launch_place_level(const uint64_t* keys, uint32_t lo, uint32_t hi, uint32_t nbase, uint32_t prev0,
                              const uint32_t* childoff, const uint32_t* cnt, const uint32_t* firstidx,
                              uint16_t topic, uint32_t* node_peer, uint16_t* node_topic, uint32_t* local,
                              uint32_t* node_parent, uint32_t* deg, uint32_t* first, BuildKey kf, hipStream_t s);
// Level d placed in one launch from its parents (nodes pbase + [0, np) of
// level d - 1, already placed): children at cbase + the exclusive scan of the
// parents' fan-out + sibling rank, the scan by decoupled look-back over
// lb_tiles(np) tiles (status: that many zeroed words; *err set on a stalled
// look-back).
inline uint32_t lb_tiles(uint32_t np) { return (np + 255) / 256; }
hipError_t launch_place_level_lb(const uint64_t* keys, uint32_t np, uint32_t pbase, uint32_t cbase,
                                 const uint32_t* cnt, const uint32_t* firstidx, uint16_t topic, uint32_t* node_peer,
                                 uint16_t* node_topic, uint32_t* local, uint32_t* node_parent, uint32_t* deg,
                                 uint32_t* first, uint64_t* status, uint32_t* err, BuildKey kf, hipStream_t s);
// The lazy prune's questions about peers[i] (tree.hpp ReachQuery), from the
// last GPU build: out[i] = 1 if the peer holds a node of the topic at [nbase,
// nbase + n_nodes) (the message reached it), else 2 if its upstream path
// (par, from the peer itself) ends at an Orphan (cut for good), else 0.
hipError_t launch_reach_query(const uint32_t* peers, uint32_t n, uint32_t n_peers, const uint32_t* local,
                              const uint32_t* node_peer, uint32_t nbase, uint32_t n_nodes, const uint32_t* par,
                              const uint8_t* orph, uint32_t root, uint8_t* out, hipStream_t s);
// col[row_ptr[u] + j] = first[u] + j
hipError_t launch_fill_col(const uint32_t* row_ptr, const uint32_t* first, uint32_t n_nodes,
                           uint32_t* col, hipStream_t s);
// node flags from the live mask (per peer) and the fan-out; roots[] forced live
hipError_t launch_node_flags(const uint32_t* node_peer, const uint32_t* row_ptr,
                             const uint8_t* live, uint32_t n_nodes, const uint32_t* roots,
                             uint32_t n_roots, uint8_t* flags, hipStream_t s);

}  // namespace psamd
