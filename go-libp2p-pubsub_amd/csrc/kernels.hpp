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
  // Tree topic whose window messages start in several rounds, laid out for
  // level mode (one rank): start group g (GroupDev [group_lo, + group_n))
  // owns the words [w0, w0 + wn) of every row -- "virtual" word w of node u
  // -- stored group-major: block g of node u at wbase + n_nodes * w0 +
  // (u - nbase) * wn, so a round's rows are contiguous per group.
  kTopicGroups = 8,
  // A level-aligned window's topic with several start rounds (one rank): one
  // node-major row, message bits sorted by start round; GroupDev [group_lo,
  // + group_n) hold each start group's bits [b0, b0 + n) of the row and the
  // virtual words [w0, w0 + wn) the group-major layout would give it, so the
  // digest reads both layouts alike.  Kernels other than the digest see a
  // single-start topic.
  kTopicPacked = 16,
};
struct GroupDev {
  uint32_t w0, wn;
  uint32_t b0, n;  // kTopicPacked: the group's bits of the packed row
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
  uint32_t group_lo;  // kTopicGroups: the topic's start groups in the GroupDev table
  uint32_t nbase;    // first node of the topic (its root)
  uint32_t n_nodes;  // nodes in the topic
  uint32_t W;        // 64-message words per node in this window (0 = idle)
  uint32_t flags;    // kTopic*
  uint32_t seed_lo, seed_n;  // the topic's round-0 seeds (k_window_init applies them when asked)
  uint32_t group_n;     // kTopicGroups: number of start groups
  uint32_t root_words;  // words at wbase k_window_init zeroes for the root (W; group-major: block 0)
};

// One root injection: words of a topic root that start flooding in a round.
struct SeedDev {
  uint64_t woff;    // word offset (root row + word)
  uint64_t mask;    // messages entering at this round
  uint32_t node;    // root node index
  uint32_t assign;  // 1: the word is set to mask (group-major root blocks, not zeroed by
                    // k_window_init), 0: or-ed in
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
  // arrival extents (one rank; nullptr: whole rows): per node the word range
  // [lo, hi) of its arrival row written this round (lo | hi << 16), kept for
  // multi-start tree topics of 64..kStageWords words; the row outside it is
  // stale and never read
  uint32_t* ext_cur;
  uint32_t* ext_next;
  uint8_t* gen;      // per-node window generation of its seen row (tree topics)
  uint8_t* next_flag;
  uint8_t* blk_flag;  // one byte per kFlagsPerBlock nodes: some flag set
  uint64_t* partials;  // [n_waves][kNumCtr]
  uint16_t* hop_rec;   // [word*64 + bit] = round (kHopRecNone: none), record mode only
  uint32_t gen_cur;
  uint8_t* send;                  // send regions of this round (multi-GPU compaction mode)
  uint64_t send_off[kMaxRanks];   // byte offset of the region for each rank
  uint32_t opts;                  // kExpand* switches (A/B)
};
constexpr uint32_t kExpandNoNarrow = 1;  // narrow entries one at a time (the entry loop), not flattened

// Level mode, pull direction: one wave copies the parents' rows into the
// rows of a contiguous run of next-level nodes [node_begin, node_end) of one
// topic (at most kPullMaxKids nodes, about kPullWords words).
struct PullChunk {
  uint32_t node_begin, node_end;  // nodes written in round r (level d)
  uint32_t topic;
  uint32_t p_lo, p_hi;  // parents of [node_begin, node_end) (consecutive ids), kNone: unknown
  uint32_t W;           // row words (a start group's block width for kTopicGroups)
  uint32_t row0_lo, row0_hi;  // word offset of the row of the topic's first node (nbase)
  // multi-GPU: PullArgs::ship entries [e_lo, e_hi) -- ghost records of the
  // next round for nodes of this chunk, written by the wave that writes them
  uint32_t e_lo, e_hi;
  // k_pull_pair: the children of [node_begin, node_end) (consecutive ids,
  // filled in on the device), written in round q + 1 by the same wave; c_lo =
  // kNoneNode: a run written in round q + 1 itself (level 1 under a root)
  uint32_t c_lo, c_hi;
  // multi-GPU: GhostSeg of this round (a ghost-fed node reads its parent's
  // record there) and of the next round (the records [e_lo, e_hi) ship
  // into); kNoneNode: none
  uint32_t gin, gout;
  uint32_t group;  // host: the start group (index in the topic's groups) whose block the chunk writes
  uint32_t pad;
};
constexpr uint32_t kPullMaxKids = 512;
constexpr uint32_t kNoneNode = 0xFFFFFFFFu;
constexpr uint32_t kPullWords = 1024;

// Multi-GPU level mode.  Before round q each rank ships the
// rows of its parents of the level written in round q - 1 that have children
// on other ranks -- once per destination rank -- as records of W words (the
// start group's block): record k of the (round, topic, group)'s a -> b block
// is a's k-th such parent in a's node order.  No header: a reached parent's
// block holds every message of its start group (a tree, one start round per
// block), so its first word is non-zero; an unreached parent's record starts
// with a zero word and its children stay unreached.
struct ShipEntry {
  uint32_t node;  // the parent (local node id)
  uint32_t dst;   // destination rank << 27 | record index k
};
struct GhostSeg {              // one (round, topic, start group)
  uint64_t rbase[kMaxRanks];   // recv buffer: first word of the records from rank a
                               // (kSegInPlace: the block's first row in rank a's seen rows)
  uint64_t sbase[kMaxRanks];   // send buffer: first word of the records to rank b (the round's half)
  uint32_t rw;                 // record words (the block width)
  uint32_t topic;
  uint32_t flags;              // kSegInPlace
  uint32_t gbase[kMaxRanks];   // kSegInPlace: the topic's first node at rank a (its generation bytes)
};
// PS_DIST_F_INPLACE: a ghost-fed node of this segment reads its parent's row
// where the owner wrote it (RankRows of the owner, the parent's topic-relative
// id there in ghost_ref), reached iff the owner stamped its generation byte
// this window -- no record is written or shipped
constexpr uint32_t kSegInPlace = 1u;
struct RankRows {
  const uint64_t* seen;
  const uint8_t* gen;
};
// k_pack: a topic root's records (round s_g + 1 of each start group g), from
// its seeded row; one segment per (round, topic, group).
struct PackSeg {
  uint32_t e0, e1;  // the root's ship entries
  uint32_t gseg;    // GhostSeg of the round
  uint32_t W;
  uint64_t row;     // word offset of the root's row (block)
  uint64_t unit0;   // the segment's first unit in the launch's flattened stream (pack_units)
};
__host__ __device__ inline uint32_t pack_units(uint32_t W) { return (W & 1u) ? W : W >> 1; }
struct PullArgs {
  const uint32_t* node_parent;  // node-space parent (kNone for roots and remote parents)
  // k_pull_chain: every chain chunk's node entries (16 bits: parent index
  // relative to the level above, live bit), levels in order, from
  // ChainChunk::first[kChainLevels] (k_chain_meta, once per plan)
  const uint32_t* chain_meta;
  const uint8_t* node_flags;
  const TopicDev* topics;
  const uint64_t* a_cur;  // arrivals of round-1 (topic roots' seeded rows)
  uint64_t* seen;
  uint8_t* gen;
  uint16_t* hop_rec;
  uint64_t* partials;  // [n_blocks][kNumCtr]
  // multi-GPU: a node whose parent lives on another rank (ghost_ref[node] =
  // rank << 27 | k, kNoneNode otherwise) reads record k of that rank in this
  // round's receive buffer (GhostSeg gin)
  const uint32_t* ghost_ref;  // null: one rank
  const GhostSeg* gsegs;
  const uint64_t* recv;
  // multi-GPU: the next round's records of the nodes written now
  // (PullChunk e_lo/e_hi, GhostSeg gout), stored into the send buffer
  const ShipEntry* ship;
  uint64_t* send;
  // per source rank a: the base its records are addressed from (record k of
  // (round, topic, group) block at rsrc[a] + GhostSeg::rbase[a] + k * rw):
  // the receive buffer for every rank, or -- the zero-copy loopback -- rank
  // a's own send region, offset so that the same rbase applies
  const uint64_t* rsrc[kMaxRanks];
  const RankRows* rrows;  // PS_DIST_F_INPLACE: every rank's row set (kSegInPlace segments)
  uint32_t gen_cur;
  uint32_t slot_mod;   // block b adds its counters into partial slot b % slot_mod (zeroed per window)
  // k_pull_pair: round q + 1's partial slots; all_current: every generation
  // byte was stamped up front (PS_F_NO_LAZY_SEEN), so every parent counts as
  // reached, as the generation test of a separate launch would find
  uint64_t* partials2;
  uint32_t all_current;
  // k_pull_chain: the CSR offsets (a run's children are consecutive ids) and
  // the partial slots of each round of the launch
  const uint32_t* row_ptr;
  uint64_t* partials_r[6];  // (kChainLevels)
  // debug (PSAMD_CHAIN_PROFILE): per chunk kChainProf words -- s_memrealtime
  // at the chunk's start and end, row words written, HW_ID and XCC_ID; null: off
  uint64_t* prof;
};
constexpr uint32_t kChainProf = 4;
// k_pull_pair: per wave, a run of at most kPairPar nodes
// whose rows (at most kPairWords words in all) stay in LDS for its children,
// streamed kPairKids children at a time
constexpr uint32_t kPairWords = 768;  // (1024: 17 resident waves/CU, cfg3 +3 % slower; 512: 1 parent of 330 words)
constexpr uint32_t kPairPar = 128;
constexpr uint32_t kPairKids = 256;
// k_pull_chain: up to kChainLevels rounds in one launch.  A
// wave owns a run of level-d nodes and a column slice [w0, w0 + S) of their
// rows (S = W: whole rows, the usual case; slices only for rows wider than
// the stage).  It writes the run (round q, the parents' rows from HBM) and
// keeps those rows in its LDS stage; then, level by level, every descendant
// of the run (round q + k: the level-(d + k) nodes of the subtree, one
// contiguous id range per level).  In a single-start window a reached node's
// row is its parent's row as round q + k - 1 wrote it, and that row is a
// stage row: a node's entry in the level table is the stage slot of the row
// its parent holds (kChainNone: unreached), so no level below the run reads
// a row from HBM.  Level ranges are at most kChainCap nodes (the host sizes
// the runs; k_chain_ranges fills and checks the ranges on the device).
constexpr uint32_t kChainLevels = 6;
static_assert(sizeof(PullArgs::partials_r) / sizeof(uint64_t*) == kChainLevels, "a slot row per chain level");
constexpr uint32_t kChainKids = 256;   // nodes resolved per sub-run of a level
constexpr uint32_t kChainPar = 128;    // nodes of a run at most (stage slots < kChainZero)
constexpr uint32_t kChainWords = 768;  // LDS stage words per wave: the run's rows (slices)
constexpr uint32_t kChainCap = 1024;   // nodes of one level of a chunk at most (the LDS level tables)
constexpr uint8_t kChainNone = 0xFF;   // level table: unreached
constexpr uint8_t kChainZero = 0xFE;   // level table: reached with a zero row (PS_F_NO_LAZY_SEEN only)
struct ChainChunk {
  uint32_t node_begin, node_end;  // the run (level d)
  uint32_t topic;
  uint32_t p_lo, p_hi;            // parents of the run (consecutive ids), kNone: unknown
  uint32_t W;                     // row stride, words
  uint32_t row0_lo, row0_hi;      // row of the topic's first node (its start group's block)
  uint32_t w0, S;                 // the column slice of every row (rows reach 2^24 words)
  uint8_t levels;                 // levels written: d .. d + levels - 1 (rounds r0 + k of the launch)
  uint8_t r0;                     // the run's round within the launch (a start group entering late: > 0)
  uint16_t group;                 // host: the start group
  // first node of levels d .. d + levels: a run [x0, x1) of level d + k has
  // the children [row_ptr[x0] - row_ptr[first[k]] + first[k + 1], ...x1...)
  uint32_t first[kChainLevels + 1];
  // level k >= 1 of the chunk: the descendants [lo[k], hi[k]) (k_chain_ranges)
  uint32_t lo[kChainLevels], hi[kChainLevels];
  // the topic's first node, and its root node if this rank owns it (the
  // root's row is the seeded arrival row), else kNoneNode: node-space
  // properties, so the kernel needs no topic-table read before its loads
  uint32_t nbase, root;
};
static_assert(sizeof(ChainChunk) == 128, "two chunk descriptors per 256-B line");
// ChainChunk::lo / hi from the device CSR; *overflow is set non-zero when a
// level range exceeds cap (the plan is then not used)
hipError_t launch_chain_ranges(ChainChunk* chunks, uint32_t n, const uint32_t* row_ptr, uint32_t cap,
                               uint32_t* overflow, hipStream_t s);
// The chunks' node entries (PullArgs::chain_meta) after their ranges: per
// chunk its node count (counts[i]), an exclusive scan into
// ChainChunk::first[kChainLevels] (the device copy's; first[] past the
// chain's levels is unused there), the entries from node_parent and the live
// flags.  *entries: the buffer's size in entries, read back by the caller
// with the ranges' overflow word (`tail`: counts[n] after the scan).
hipError_t launch_chain_meta(ChainChunk* chunks, uint32_t n, const uint32_t* node_parent, const uint8_t* node_flags,
                             uint32_t* counts, void* scan_temp, size_t scan_bytes, uint32_t* meta, bool fill,
                             hipStream_t s);
size_t chain_meta_scan_bytes(uint32_t n);
// slices: chunks of rows wider than the stage (column slices; their own launch)
// inner_nt: level 0 and the inner levels store non-temporally (false: plain, A/B)
// waves_per_cu: resident chain waves per CU at most (an LDS pad; 0: no cap)
hipError_t launch_pull_chain(const PullArgs& a, const ChainChunk* chunks, uint32_t n_chunks, uint32_t round,
                             bool record, bool nt, bool slices, bool inner_nt, uint32_t waves_per_cu,
                             hipStream_t s);
// ChainChunk::p_lo / p_hi from the device node_parent (GPU-built graphs)
hipError_t launch_chain_parents(ChainChunk* chunks, uint32_t n, const uint32_t* node_parent, hipStream_t s);
constexpr uint32_t kPullSlots = 256;  // partial slots per round of a pull launch
// k_pull_pair: every wave adds its counters with atomics (no block
// reduction) into slot wave % kPairSlots.  (4096 slots: no faster than 256,
// and k_reduce_rounds folds each round's slots in one block -- 26 us per
// step -- and k_window_init zeroes them.)
constexpr uint32_t kPairSlots = kPullSlots;

// k_flood (flood.hip): every round of a single-start tree
// window in one persistent launch.  A task = the nodes [nb, ne) of one BFS
// level of one topic (at most kFloodMaxNodes = one per lane, about
// kFloodWords row words), written in round `round`; tasks are listed level by
// level.  A task publishes which of its nodes were reached as granules: one
// 8-B word {epoch << 32 | reach bits} per `gsz` consecutive nodes of its level
// (data and flag in one store); its children's tasks poll those granules.
struct FloodTask {
  uint32_t nb, ne;          // nodes written (consecutive ids of one level)
  uint32_t topic, round;
  uint32_t slot0, nslot;    // the round's partial counter slots
  uint32_t g_own, gsz;      // granules written: g_own, g_own + 1, ... (gsz nodes each)
  uint32_t p_lo, p_hi;      // parents of the run (consecutive ids)              [k_flood_deps]
  uint32_t pg_lo, pg_hi;    // parent granules to poll; kNoneNode: parent = root [k_flood_deps]
  uint32_t pnode0, pgsz;    // parent level: first node and nodes per granule    [k_flood_deps]
  uint32_t pseg;            // host: the parent level's segment (kNoneNode: root)
  uint32_t seg;             // the task's own segment (row stride and base)
};
// One level of one topic (of one start group): tasks task0 .. task0 +
// n_tasks - 1 of `per` nodes each from node0, granules gbase .. of gsz nodes
// each; rows of W words, node u's at row0 + (u - nbase) * W.
struct FloodSeg {
  uint32_t task0, node0, per, n_tasks;
  uint32_t gbase, gsz, nodes, W;
  uint64_t row0;  // word offset of the topic's first node's row (its start group's block region)
};
struct FloodArgs {
  const FloodTask* tasks;
  const FloodSeg* segs;
  const uint32_t* node_parent;
  const uint8_t* node_flags;
  const TopicDev* topics;
  uint64_t* seen;
  uint8_t* gen;
  uint16_t* hop_rec;
  uint64_t* granules;   // per granule: epoch << 32 | reach bits, once its task's rows are stored
  uint64_t* partials;   // counter slots (FloodTask::slot0 ...), zeroed per window
  uint32_t* err;        // set when a dependency wait times out
  uint32_t n_tasks;
  uint32_t epoch;       // this launch's granule tag (never 0)
  uint32_t gen_cur;
  uint32_t spin_ticks;  // wait bound, s_memrealtime ticks (100 MHz)
  uint64_t* prof;       // debug (PSAMD_FLOOD_PROFILE): per wave kFloodProf s_memrealtime stamps / sums
  uint32_t prof_split;  // debug: pf[7] sums the waits of tasks of later rounds
};
// per-wave profile words: first task start, last task end, then summed ticks
// waiting, resolving, streaming, publishing; tasks run; waiting in rounds > prof_split
constexpr uint32_t kFloodProf = 8;
constexpr uint32_t kFloodMaxNodes = 64;       // one node per lane
constexpr uint32_t kFloodGranule = 32;        // reach bits per granule at most
constexpr uint32_t kFloodWords = 2048;        // row words per task (16 KB)
constexpr uint32_t kFloodBlocksPerCu = 4;     // resident 256-thread blocks per CU the grid uses

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

// Loopback exchange (one GPU): up to kMaxCopyRegions device regions of
// whole 16-B units copied by one launch.
constexpr uint32_t kMaxCopyRegions = 16;
struct CopyRegions {
  const uint4* src[kMaxCopyRegions];
  uint4* dst[kMaxCopyRegions];
  uint64_t units[kMaxCopyRegions];
  uint32_t n;
};
hipError_t launch_copy_regions(const CopyRegions& c, hipStream_t s);
// Process-shared exchange (dist.cpp IpcTransport): stream-ordered device
// flags in IPC-mapped memory.  launch_flag_set stores `value` into `flag`
// (system-scope release, after every launch before it on the stream);
// launch_flag_wait holds the stream until every non-null flag[q] >= value[q]
// (system-scope acquire polls) or `timeout_ticks` of the 100 MHz clock pass,
// then ORs 1 into *err (pinned host memory) and lets the stream go on.
struct FlagWait {
  const uint64_t* flag[kMaxRanks];
  uint64_t value[kMaxRanks];
};
hipError_t launch_flag_set(uint64_t* flag, uint64_t value, hipStream_t s);
hipError_t launch_flag_wait(const FlagWait& w, uint32_t* err, uint64_t timeout_ticks, hipStream_t s);
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
  uint64_t* t0 = nullptr;          // (signalled windows) the start stamp, s_memrealtime into pinned memory
};
// A signalled window's end, after its reduce on the same stream: the end
// stamp into sig[2], then seq into sig[0] (pinned; system-scope release) --
// ps_wait polls it instead of waiting on an event, whose record costs the
// queue ~10 us between windows (profiles/r04/cfg2)
hipError_t launch_window_done(uint64_t* sig, uint64_t seq, hipStream_t s);
// ... or raised by the reduce's last block (no launch of its own): ctr a
// zeroed device word (left zero again)
struct WindowSignal {
  uint64_t* flag = nullptr;
  uint32_t* ctr = nullptr;
  uint64_t seq = 0;
};
hipError_t launch_window_init(const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur,
                              bool any_mesh, const WindowStart& ws, hipStream_t s);
// A signalled window's reduce held back until the next window starts: the
// two run as one launch (the reduce's blocks first, then the init's), one
// kernel boundary less per pipelined window.  The two touch
// disjoint memory: the reduce reads its own slot's partials and descriptors,
// the init writes the other slot's.
// A level-aligned window's per-(topic, level) reach counts:
// the nodes [lo, hi) of segment seg (one BFS level of one topic; a level is
// cut into pieces of at most kReachPiece nodes).  out[2 * seg] += reached
// nodes, out[2 * seg + 1] += frontier nodes (reached and internal).  Reached:
// the generation byte is this window's (eager seen: the row's first word is
// non-zero -- its first message's bit); a topic root always.
struct ReachPiece {
  uint32_t seg, lo, hi, topic;
};
constexpr uint32_t kReachPiece = 16384;
hipError_t launch_level_reach(const ReachPiece* pieces, uint32_t n, const uint8_t* gen, uint32_t gen_cur,
                              const uint8_t* node_flags, const TopicDev* topics, const uint64_t* seen, bool eager,
                              uint64_t* out, hipStream_t s);

struct ReduceArgs {
  const uint64_t* partials = nullptr;
  const uint32_t* desc = nullptr;
  uint32_t n_rounds = 0;  // > 0
  uint64_t* round_stats = nullptr;
  uint64_t* host_stats = nullptr;
  WindowSignal sig{};
};
hipError_t launch_window_turn(const ReduceArgs& rd, const TopicDev* topics, uint32_t n_topics, uint64_t* seen,
                              uint64_t* a0, uint64_t* a1, uint8_t* gen, uint32_t gen_cur, bool any_mesh,
                              const WindowStart& ws, hipStream_t s);
// stamp: mark the nodes' generation current (compaction mode)
hipError_t launch_init_nodes(const uint32_t* nodes, uint32_t n, const uint16_t* node_topic,
                             const TopicDev* topics, uint64_t* seen, uint64_t* a0, uint64_t* a1,
                             uint8_t* gen, uint32_t gen_cur, bool stamp, hipStream_t s);
hipError_t launch_apply(const ApplyArgs& a, uint32_t round, bool record, hipStream_t s);
// next_flag / blk_flag may be null (level mode: the root is in the schedule)
hipError_t launch_seed(const SeedDev* seeds, uint32_t lo, uint32_t hi, uint64_t* arrivals,
                       uint64_t* seen, uint8_t* next_flag, uint8_t* blk_flag, hipStream_t s);
hipError_t launch_expand(const ExpandArgs& a, uint32_t round, bool record, uint32_t grid, hipStream_t s);
// Level mode, pull direction: one wave per chunk, grid = ceil(n_chunks / 4)
// blocks; nt: the row stores are non-temporal (rounds nobody re-reads soon);
// cap: an nt round runs at most 5 blocks per CU (one rank; N ranks keep full
// residency)
hipError_t launch_pull(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks,
                       uint32_t grid, uint32_t round, bool record, bool nt, bool cap, hipStream_t s);

// Level mode, rounds q and q + 1 in one launch (one rank): a wave writes its
// run's rows (round q, always non-temporal: the run's children are written
// from LDS, nothing re-reads them), then the children's rows (round q + 1;
// nt2: non-temporal too)
// One-wave workgroups, one chunk each (grid = n_chunks); a chunk's rows fit
// the kPairWords LDS stage
hipError_t launch_pull_pair(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks, uint32_t grid,
                            uint32_t round, bool record, bool nt2, hipStream_t s);
// Fills PullChunk::c_lo / c_hi of pair chunks from the device CSR (children
// of a BFS-numbered run are consecutive ids)
hipError_t launch_pair_kids(PullChunk* chunks, uint32_t n, const uint32_t* row_ptr, const uint32_t* col,
                            hipStream_t s);

// multi-GPU level mode: the roots' records of the round into the send buffer
hipError_t launch_pack(const ShipEntry* ship, const PackSeg* segs, uint32_t n_segs, uint64_t total_units,
                       const GhostSeg* gsegs, const uint64_t* seen, uint64_t* send, hipStream_t s);
// Fills PullChunk::p_lo / p_hi from the device node_parent (GPU-built graphs).
hipError_t launch_chunk_parents(PullChunk* chunks, uint32_t n, const uint32_t* node_parent, hipStream_t s);
// k_flood (flood.hip): grid = resident blocks (<= flood_blocks_per_cu x CUs)
hipError_t launch_flood(const FloodArgs& a, uint32_t grid, bool record, hipStream_t s);
// FloodTask::p_lo / p_hi / pg_lo / pg_hi / pnode0 / pgsz from node_parent and the segments
hipError_t launch_flood_deps(FloodTask* tasks, uint32_t n, const FloodSeg* segs, const uint32_t* node_parent,
                             hipStream_t s);
hipError_t flood_blocks_per_cu(int* out);
// Level mode: round q's counters = sum of the partial slots desc[3q],
// desc[3q] + desc[3q+2], ... < desc[3q+1], for q = 1..n_rounds.
// host_stats (nullable): device-mapped pinned rows that receive the same
// counters, so an asynchronous run needs no readback copy
hipError_t launch_reduce_rounds(const uint64_t* partials, const uint32_t* desc, uint32_t n_rounds,
                                uint64_t* round_stats, uint64_t* host_stats, const WindowSignal& sig, hipStream_t s);
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
                         const TopicDev* topics, const GroupDev* groups, uint32_t n_nodes, uint64_t* out,
                         hipStream_t s);

}  // namespace psamd
