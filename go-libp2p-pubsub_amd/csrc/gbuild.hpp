// gbuild.hpp -- GPU rebuild of the node space from per-topic parent arrays
// (DESIGN.md §4.1).  Single rank, tree topics.
//
// For each topic: the upstream of every subscribed peer (kNone otherwise,
// maintained on the host by the restated join / leave protocol and shipped as
// deltas) -> the children of every peer as a peer-space CSR (histogram of the
// parent array + exclusive scan + scatter, siblings in peer order) -> BFS
// numbering from the root, level by level, each level's node range from the
// exclusive scan of the fan-out of the level above -> node_parent, CSR,
// flags.  No depth pass and no sort.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace psamd {

constexpr uint32_t kBuildMaxDepth = 255;  // levels of the level tables
constexpr uint32_t kBuildPeerBits = 28;   // peer ids below 2^28 (the GPU build's bound)
constexpr uint32_t kBuildSmallLevel = 8192;  // the one-block kernel's LDS scan capacity
// levels whose parents number at most this many are placed by the one-block
// kernel (its levels are latency chains: 512 was the best cut of 0 / 512 /
// 2048 / 8192 in round 4, and 8192 cost 0.24 ms per cfg5 rebuild here)
constexpr uint32_t kBuildTopLevel = 512;

// Pair value of an Orphan peer (not subscribed: no upstream; its subtree is
// cut for good, rule Q5): par[p] = kNone, orph[p] = 1.
constexpr uint32_t kOrphanCode = 0xFFFFFFFEu;
// (peer, value) pairs scattered into a parent array and its orphan bytes
hipError_t launch_scatter_pairs(const uint32_t* pairs, uint32_t n, uint32_t* par, uint8_t* orph, hipStream_t s);

// exclusive scan of n u32 (in -> out)
hipError_t scan_u32(void* temp, size_t* temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                    hipStream_t s);

// ---- by-parent CSR BFS rebuild ------------------------------
// Per topic: the parent array's children as a peer-space CSR (histogram of
// the parent array, exclusive scan, scatter; siblings sorted by peer), then
// BFS numbering from the root, one level per launch, each level from the
// fan-out of the one above (no depth pass, no sort).  Node ids, topic bases
// and level tables stay on the device until one readback after the last
// topic.
// look-back tiles of a level of np parents (one 256-thread block each)
__host__ __device__ inline uint32_t lb_tiles(uint32_t np) { return (np + 255) / 256; }
// per-topic stat words (gst = d_gstat + kGstWords * t)
constexpr uint32_t kGstWords = 8;
constexpr uint32_t kGstDepth = 1, kGstMaxDeg = 2, kGstDone = 4;
// build error bits (one word): a level wider than its launch's grid, a level
// launched before its parent level was placed, a stalled look-back
constexpr uint32_t kBuildErrGrid = 1, kBuildErrOrder = 2, kBuildErrStall = 4;
struct PlaceArgs {
  const uint32_t* kids;  // the peer-space CSR: children of peer v at kids[koff[v] .. + cnt[v])
  const uint32_t* koff;
  const uint32_t* cnt;
  const uint8_t* live;
  uint32_t* node_peer;
  uint16_t* node_topic;
  uint32_t* local;  // peer -> node
  uint32_t* node_parent;
  uint32_t* row_ptr;
  uint32_t* col;
  uint32_t* first;
  uint8_t* flags;
  // node space, written with each placed node for the next level's pass
  // (coalesced there, instead of a dependent random read of the peer's):
  // its fan-out and the index of its first child in kids
  uint32_t* ndeg;
  uint32_t* nkat;
  uint32_t* lvl;  // this topic's table: [d] level start (topic-relative), [256 + d] internal nodes
  uint32_t* gst;  // this topic's stat words
  uint32_t* tb;   // [2 a] node base, [2 a + 1] edge base of active topic a (a + 1's written at the end)
  uint32_t* err;
  uint32_t a, root;
  uint16_t topic;
};
// Zeroes up to 8 regions of u32 words in one launch (the build's scratch and
// stat block: one launch instead of a fill per buffer)
struct ClearRegions {
  uint32_t* p[8];
  uint64_t words[8];
  uint32_t n;
};
hipError_t launch_clear(const ClearRegions& r, hipStream_t s);

// peer-space CSR of one topic's parent array (temp: the scan's, queried with
// scan_u32 over n + 1 entries; cnt has n + 1 entries)
// (cnt, fill and *n_big zeroed by the caller)
hipError_t build_kids(const uint32_t* par, uint32_t n, uint32_t* cnt, uint32_t* koff, uint32_t* fill, uint32_t* kids,
                      uint32_t* big, uint32_t* n_big, void* temp, size_t temp_bytes, hipStream_t s);
// the root and the top levels of at most kBuildSmallLevel parents each, levels < d_limit
hipError_t launch_place_top(const PlaceArgs& P, uint32_t d_limit, hipStream_t s);
// level d (grid: the host's estimate of the parent level's tiles; status: grid zeroed words)
hipError_t launch_place_lb(const PlaceArgs& P, uint32_t d, uint32_t grid, uint64_t* status, hipStream_t s);

// The lazy prune's questions about peers[i] (tree.hpp ReachQuery), over the
// topic's upstream array as the GPU build took it (par, orph: peer space):
// out[i] = 1 if the peer's upstream path reaches the root (it holds a node of
// the node space: the message reached it), else 2 if the path ends at an
// Orphan (cut for good), else 0.  (Not the peer -> node map: a peer of several
// topics maps to its node of the last topic placed.)
hipError_t launch_reach_query(const uint32_t* peers, uint32_t n, uint32_t n_peers, const uint32_t* par,
                              const uint8_t* orph, uint32_t root, uint8_t* out, hipStream_t s);
// node flags from the live mask (per peer) and the fan-out; roots[] forced live
hipError_t launch_node_flags(const uint32_t* node_peer, const uint32_t* row_ptr,
                             const uint8_t* live, uint32_t n_nodes, const uint32_t* roots,
                             uint32_t n_roots, uint8_t* flags, hipStream_t s);

}  // namespace psamd
