// kernels.hpp -- device data layout shared by the HIP kernels and the host
// runtime.  See DESIGN.md §4 (HBM layout) and §5 (kernels).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace psamd {

// node_flags bits (one byte per tree node)
enum : uint8_t {
  kNodeLive = 1,      // subscribed and live: receives and forwards
  kNodeInternal = 2,  // has at least one child: enters the next frontier
  kNodeSplit = 4,     // some child is owned by another rank (direct path)
};

// col[] entry of a child owned by another rank: rank and its local node id
constexpr uint32_t kRemoteBit = 0x80000000u;
constexpr uint32_t kRemoteRankShift = 27;
constexpr uint32_t kRemoteIdMask = (1u << kRemoteRankShift) - 1u;
constexpr int kMaxRanks = 16;

// One delivery addressed to a node of another rank: node id at the owner,
// word of its row, the arriving bits.  Regions: 16-B header (u32 count) +
// capacity items.
struct XItem {
  uint32_t node;
  uint32_t word;
  uint64_t mask;
};
constexpr uint32_t kRegionHeader = 16;

// TopicDev.flags
enum : uint32_t {
  // A node may have several parents (general child lists): the seen
  // test-and-set and the arrival OR are 64-bit atomics, rows are cleared
  // eagerly per window and consumed-and-cleared per round.
  kTopicMesh = 1,
  kTopicRootLocal = 2,  // this rank owns the topic root (node nbase)
  // Tree topic whose messages of this window all start in one round: every
  // node receives exactly once, so a node's arrival row equals its freshly
  // written seen row.  Arrival rows are then neither stored nor read: a
  // (non-root) parent's row is read from `seen`.
  kTopicSingleStart = 4,
};
constexpr uint32_t kEntrySplit = 0x100;  // per-entry flag bit next to TopicDev.flags

// One topic of the fused node space.  Node u of topic t (nbase <= u <
// nbase + n_nodes) owns the 64-message words [wbase + (u-nbase)*W, +W) of the
// seen bitset and of the two arrival buffers.  Tree topics are numbered in
// BFS order, so the children of a node are consecutive node ids.
// Hop record (parity mode): the delivery round of every (node, message) as
// u16, so paths deeper than 254 hops stay exact up to the host's saturation.
constexpr uint16_t kHopRecNone = 0xFFFF;
__host__ __device__ inline uint16_t hop_round(uint32_t round) {
  return static_cast<uint16_t>(round < 0xFFFEu ? round : 0xFFFEu);
}

struct TopicDev {
  uint64_t wbase;    // first word of the topic's mask block
  uint32_t w_msgs;   // message words in use (W may carry one pad word)
  uint32_t pad;
  uint32_t nbase;    // first node of the topic (its root)
  uint32_t n_nodes;  // nodes in the topic
  uint32_t W;        // 64-message words per node in this window (0 = idle)
  uint32_t flags;    // kTopic*
  uint32_t seed_lo, seed_n;  // the topic's round-0 seeds (k_window_init applies them when asked)
};

// One root injection: words of a topic root that start flooding in a round.
struct SeedDev {
  uint64_t woff;  // word offset (root row + word)
  uint64_t mask;  // messages entering at this round
  uint32_t node;  // root node index
  uint32_t pad;
};

// Per-wave counters written by the expand kernel, reduced per round; they
// also feed the algorithmic byte model.
enum : int {
  kCtrDeliveries = 0,
  kCtrDuplicates,
  kCtrEntries,
  kCtrEntryWords,
  kCtrChildren,
  kCtrMeshChildren,
  kCtrSeenReads,
  kCtrSeenWrites,
  kCtrArrivalWrites,
  kCtrClearWords,
  kNumCtr
};

struct ExpandArgs {
  const uint32_t* frontier;
  const uint32_t* n_front;
  const uint32_t* row_ptr;
  const uint32_t* col;
  const uint16_t* node_topic;
  const uint8_t* node_flags;
  const TopicDev* topics;
  uint64_t* a_cur;   // arrivals of the current frontier
  uint64_t* a_next;  // arrivals for the next frontier
  uint64_t* seen;    // per-node delivered bitset (the dedup record)
  uint8_t* gen;      // per-node window generation of its seen row (tree topics)
  uint8_t* next_flag;
  uint8_t* blk_flag;  // one byte per kFlagsPerBlock nodes: some flag set
  uint64_t* partials;  // [n_waves][kNumCtr]
  uint16_t* hop_rec;   // [word*64 + bit] = round (kHopRecNone: none), record mode only
  uint32_t gen_cur;
  uint32_t dbg;  // experiment knobs (kDbg*), 0 in production
  uint8_t* send;                  // send regions of this round (multi-GPU)
  uint64_t send_off[kMaxRanks];   // byte offset of the region for each rank
};

// Level mode, pull direction: one wave copies the parents' rows into the
// rows of a contiguous run of next-level nodes [node_begin, node_end) of one
// topic (at most kPullMaxKids nodes, about kPullWords words).
struct PullChunk {
  uint32_t node_begin, node_end;  // nodes written in round r (level d)
  uint32_t g_begin, g_end;        // fused launches: their children, written as round r + 1
  uint32_t topic;
  uint32_t p_lo, p_hi;  // parents of [node_begin, node_end) (consecutive ids), kNone: unknown
  uint32_t pad;
};
constexpr uint32_t kPullMaxKids = 512;
constexpr uint32_t kPullTopLevels = 32;  // levels of one top launch at most (ancestor walks)
constexpr uint32_t kNoneNode = 0xFFFFFFFFu;
constexpr uint32_t kPullWords = 1024;  // default; PSAMD_PULL_WORDS overrides

struct PullArgs {
  const uint32_t* node_parent;  // node-space parent (kNone for roots)
  const uint8_t* node_flags;
  const TopicDev* topics;
  const uint64_t* a_cur;  // arrivals of round-1 (topic roots' seeded rows)
  uint64_t* seen;
  uint8_t* gen;
  uint16_t* hop_rec;
  uint64_t* partials;  // [n_blocks][kNumCtr]
  uint32_t gen_cur;
  uint32_t dbg;
  uint32_t slot_mod;   // block b adds its counters into partial slot b % slot_mod (zeroed per window)
  uint32_t slot_base;  // top launch: round q's slots start at (q - slot_base) * kPullSlots
  uint32_t wave_flush;  // counters added per wave (no block barrier) instead of per block
  uint32_t* path_live;  // k_pull_top: per node, epoch << 2 | parent path live << 1 | node path live
  uint32_t pl_epoch;    // current flags epoch (< 2^30, never 0)
  uint32_t top_nt;      // k_pull_top: bit q - slot_base set = round q stores its rows non-temporally
  uint32_t xcd_remap;  // k_pull_top: XCD x runs one contiguous range of the blocks
  uint32_t top_odd_wide;  // k_pull_top odd W: 2 = 16-B pair stores, 1 = 8-B words 16 in flight, 0 = 8 in flight
};
constexpr uint32_t kPullSlots = 256;  // partial slots per round of a pull launch

struct ApplyArgs {
  const uint8_t* recv;
  uint64_t recv_off[kMaxRanks];  // region from each rank
  uint64_t cap_pre[kMaxRanks + 1];  // prefix of region capacities (items)
  uint32_t world;
  const uint16_t* node_topic;
  const uint8_t* node_flags;
  const TopicDev* topics;
  uint64_t* seen;
  uint64_t* a_next;
  uint8_t* next_flag;
  uint8_t* blk_flag;
  uint16_t* hop_rec;
  uint64_t* stats;  // [kNumCtr] of this round (deliveries, duplicates)
  uint8_t* gen;     // level mode: stamp a node reached (null: compaction mode)
  uint32_t gen_cur;
};

// k_expand experiment knobs (PSAMD_DEBUG_EXPAND); results are wrong when set
enum : uint32_t {
  kDbgNoArrivalLoad = 1,   // arrival words read as all-ones
  kDbgNoArrivalStore = 2,  // skip arrival-row stores
  kDbgNoByteStores = 4,    // skip frontier-flag and generation byte stores
  kDbgNoSeenStore = 8,     // skip seen-row stores
};

constexpr int kBlock = 256;
constexpr int kFlagsPerThread = 16;
constexpr int kFlagsPerBlock = kBlock * kFlagsPerThread;  // 4096 nodes
constexpr int kFlagBlockShift = 12;

// host-side launchers (kernels.hip)
// Per-window parameters (topic table, seeds, reduce descriptors) copied by
// one small kernel straight from the pinned staging slot (device-mapped host
// memory): one launch instead of a blit per array and its barrier packets.
constexpr uint32_t kStageMax = 4;
struct StageCopy {
  const uint32_t* src[kStageMax];
  uint32_t* dst[kStageMax];
  uint32_t words[kStageMax];
  uint32_t n;
};
hipError_t launch_stage_copy(const StageCopy& c, hipStream_t s);
// Window start: zero and stamp the roots' rows (every row of a mesh topic);
// optionally in the same launch (WindowStart): the staged per-window copies
// (topics_src / seeds_src then point at the staged sources), the round-0
// seeds of tree roots (each topic's block, after its zeroing), and zeroing
// of the pull partial slots.
struct WindowStart {
  StageCopy copy{};
  const SeedDev* seeds = nullptr;  // apply round-0 seeds (tree topics only)
  uint64_t* zero = nullptr;        // words to clear
  uint64_t zero_words = 0;
};
hipError_t launch_window_init(const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur,
                              bool any_mesh, const WindowStart& ws, hipStream_t s);
// stamp: mark the nodes' generation current (compaction mode)
hipError_t launch_init_nodes(const uint32_t* nodes, uint32_t n, const uint16_t* node_topic,
                             const TopicDev* topics, uint64_t* seen, uint64_t* a0, uint64_t* a1,
                             uint8_t* gen, uint32_t gen_cur, bool stamp, hipStream_t s);
// level mode, multi-GPU: rows of the reached split parents `list` to the
// send regions of their remote children's owners
hipError_t launch_send(const ExpandArgs& a, const uint32_t* list, uint32_t n, hipStream_t s);
hipError_t launch_apply(const ApplyArgs& a, uint32_t round, bool record, hipStream_t s);
// next_flag / blk_flag may be null (level mode: the root is in the schedule)
hipError_t launch_seed(const SeedDev* seeds, uint32_t lo, uint32_t hi, uint64_t* arrivals,
                       uint64_t* seen, uint8_t* next_flag, uint8_t* blk_flag, hipStream_t s);
// level = true: the frontier is a static level schedule (every entry a live
// internal node of the round's BFS level): entries not reached this window
// (stale generation) are skipped and no frontier flags are raised.
hipError_t launch_expand(const ExpandArgs& a, uint32_t round, bool record, bool level,
                         uint32_t grid, hipStream_t s);
// Level mode, pull direction: one wave per chunk (grid = ceil(n_chunks / 4));
// fuse: each chunk also writes its nodes' children (two levels per launch).
// unroll: 16-B loads in flight per lane (4: 8 waves/SIMD, 8: 6 waves/SIMD)
// grid: blocks, one chunk per wave (ceil(n_chunks / 4))
hipError_t launch_pull(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks,
                       uint32_t grid, uint32_t round, bool record, bool fuse, uint32_t unroll, uint32_t nt,
                       hipStream_t s);

// Fills PullChunk::p_lo / p_hi from the device node_parent (GPU-built graphs).
hipError_t launch_chunk_parents(PullChunk* chunks, uint32_t n, const uint32_t* node_parent, hipStream_t s);
// Level mode, top levels in one launch (one rank, every active topic
// starting together): chunks of several rounds (PullChunk::pad = round),
// each round's list padded to whole blocks of kBlock / 64 chunks.
hipError_t launch_pull_top(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks,
                           bool record, hipStream_t s, uint32_t lds_bytes = 0);
// Level mode: round q's counters = sum of the partial slots desc[3q],
// desc[3q] + desc[3q+2], ... < desc[3q+1], for q = 1..n_rounds.
// host_stats (nullable): device-mapped pinned rows that receive the same
// counters, so an asynchronous run needs no readback copy
hipError_t launch_reduce_rounds(const uint64_t* partials, const uint32_t* desc, uint32_t n_rounds,
                                uint64_t* round_stats, uint64_t* host_stats, hipStream_t s);
// second instance: entries the staged kernel leaves (mesh, split, wide rows,
// fan-out > 64); writes the same counters to partials + n_waves*kNumCtr
hipError_t launch_expand_direct(const ExpandArgs& a, uint32_t round, bool record, uint32_t grid,
                                hipStream_t s);
constexpr uint32_t kStageMaxWords = 704;  // widest row of the staged path
hipError_t launch_flag_count(const uint8_t* flags, const uint8_t* blk_flag, uint32_t n_pad,
                             uint32_t* wg_count, const uint64_t* partials, uint32_t n_waves,
                             uint64_t* round_stats, hipStream_t s);
hipError_t launch_flag_compact(uint8_t* flags, uint8_t* blk_flag, uint32_t n_pad,
                               const uint32_t* wg_count, uint32_t* frontier, uint32_t* n_front,
                               hipStream_t s);
hipError_t launch_digest(const uint64_t* seen, const uint8_t* gen, uint32_t gen_cur,
                         const uint32_t* node_peer, const uint16_t* node_topic,
                         const TopicDev* topics, uint32_t n_nodes, uint64_t* out, hipStream_t s);

}  // namespace psamd
