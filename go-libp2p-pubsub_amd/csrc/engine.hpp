// engine.hpp -- internal state of the engine (include/psengine.h) shared by
// its translation units:
//   graph.cpp  the node space: per-topic BFS numbering (host, or rebuilt on
//              the GPU by gbuild.hip), multi-GPU partition and ghost tables
//   plan.cpp   one window's layout and its launch plans (pull chunks, round
//              pairs, k_flood tasks, the ghost exchange) -- pure host code,
//              tested on the CPU through include/psengine_plan.h
//   run.cpp    plan uploads and the round loop on the GPU (ps_run*)
//   api.cpp    the remaining C ABI (topics, membership, reads, multi-GPU)
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "dist.hpp"
#include "kernels.hpp"
#include "psengine.h"
#include "tree.hpp"

namespace psamd {

constexpr uint32_t kMaxRoundsCap = 4096;  // round buffers' minimum size (deeper windows grow them)
// counter rows of a level-aligned window at most (its rounds and its reach
// rows): a run slot's pinned block holds 2 x (PS_MAX_ROUNDS + 1) rows (the
// second half, the multi-rank apply rows, is free on one rank)
constexpr uint32_t kAlignedRowsMax = 2 * (PS_MAX_ROUNDS + 1);
constexpr uint32_t kMaxStartRound = 200;
constexpr uint32_t kDefaultWindow = 65536;
constexpr uint32_t kMaxWindow = 1u << 30;  // messages per topic per window at most (ps_config.msg_window)

inline uint32_t ceil_div(uint64_t a, uint64_t b) { return static_cast<uint32_t>((a + b - 1) / b); }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  uint64_t gen = 0;  // allocations made (a shadow of the contents is valid for one)
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) {
      (void)hipFree(p);
      psamd::note_device_free();  // (IPC exports of a freed range are stale)
    }
    p = nullptr;
    bytes = 0;
  }
  // Grow-only allocation; *fresh = a new allocation was made.
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
    ++gen;
    if (fresh) *fresh = true;
    return hipSuccess;
  }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(bytes, o.bytes);
    std::swap(gen, o.gen);
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
  // node space (set by build_graph / gpu_build_graph)
  uint32_t nbase = 0, n_nodes = 0, depth = 0;
  bool mesh = false;
  bool root_local = true;                // this rank owns the root
  uint32_t max_deg = 0;
  uint32_t top_levels = 1;  // GPU build: levels 1 .. top_levels - 1 fit the one-block top kernel
  std::vector<uint32_t> level_internal;  // BFS level -> owned nodes with children
  std::vector<uint32_t> level_off;       // BFS level -> first owned node (topic-relative)
  // multi-GPU: the owned nodes of level d are [level_off[d], level_off[d] +
  // level_local[d]) fed by a parent on this rank, then the ghost-fed ones
  // (parent on another rank), grouped by source rank (graph.cpp numbering)
  std::vector<uint32_t> level_local;
  // GPU rebuild: the upstream of every peer as last shipped to the device
  std::vector<uint32_t> par_mirror;
  bool par_dev_valid = false;  // the device parent array holds par_mirror
  bool par_full_dirty = true;  // Kind::Parent: re-diff the whole array
  // cross-rank edges by the parent's BFS level: (level, from rank, to rank, count)
  struct Cross {
    uint32_t level, from, to, count;
  };
  std::vector<Cross> cross;
  // Multi-GPU level mode: ghost parents.  gcnt[(d * world + a)
  // * world + b] = parents at level d - 1 owned by rank a with a child at
  // level d owned by rank b (a != b): each crosses once per round that writes
  // level d, as record k = its index among them (in a's node order).
  // This rank's parents to ship: send_node[i] (local node), send_dst[i]
  // (dest rank << 27 | k), grouped by the level of the children:
  // send_lvl[d] .. send_lvl[d + 1], node order within a level.
  std::vector<uint32_t> gcnt, send_node, send_dst, send_lvl;
  uint32_t ship0 = 0;  // this topic's first entry in the engine's ship array
};

struct RunMsg {
  uint32_t topic;
  uint32_t start;
  RunMsg() {}  // (left unset: ps_publish writes every element it appends)
  RunMsg(uint32_t t, uint32_t s) : topic(t), start(s) {}
};

// Messages of one topic in one window: a slice of the run's topic-sorted
// message index array (bit li of the topic block = message idx[li]).
struct WinSlice {
  const uint32_t* idx = nullptr;
  uint32_t n = 0;
};

// One start round of a topic's window and its word block [w0, w0 + wn) of
// every row: a tree node at level d receives the block in round start + d.
// A topic whose window messages share one start round has one group, the
// whole row.
struct StartGroup {
  uint32_t start, w0, wn;
};

// A level-aligned window (WindowLayout::aligned): the messages of one topic
// that start in one round, and their row bits [b0, b0 + n) (rows are packed
// node-major, bits sorted by start round).
struct AlignedGroup {
  uint32_t start, b0, n;
};
// The per-round split of a level-aligned window: reached and frontier
// counts per (topic, BFS level), from k_level_reach.  seg_lo[t]: topic t's
// first segment (levels 0 .. depth_t), kNone: inactive.
struct AlignedSplit {
  std::vector<uint32_t> seg_lo, seg_n;
  std::vector<std::vector<AlignedGroup>> groups;
  uint32_t n_segs = 0;
  uint32_t row0 = 0;  // the counter row of segment pair 0 (after the window's rounds)
  bool eager = false;
};

// Word offset of virtual word w of row u (relative to the topic's first
// node): node-major rows, or a kTopicGroups topic's group-major blocks.
uint64_t phys_word(const TopicDev& d, const std::vector<StartGroup>& G, uint64_t u, uint32_t w);

// One window's rows (plan_window_layout): the topic table, start groups,
// message bit positions, and how its rounds run.
struct WindowLayout {
  std::vector<TopicDev> tab;
  std::vector<std::vector<StartGroup>> groups;
  std::vector<std::vector<uint32_t>> pos;  // window slot -> row bit (start groups)
  std::vector<uint32_t> tstart;            // first start round per topic
  std::vector<uint32_t> wglob;             // row words of every active topic, on every rank
  std::vector<GroupDev> gtab;              // start groups of the group-major topics
  uint64_t wtot = 0;                       // row words of the window (this rank)
  uint32_t max_depth = 0, max_start = 0;
  uint32_t planned0 = 0;                   // rounds of the window: max depth + latest start + 1
  uint32_t round_cap = 0;
  bool multi = false;                      // some tree window has several start rounds
  // level-aligned start groups (one rank, ps_plan_opts.align_groups): every
  // topic's row is one node-major block with its messages' bits sorted by
  // start round (AlignedSplit::groups); the planners see one start (round
  // 0: planned0 = max depth + 1 launch rounds); true_rounds = planned0 +
  // the latest start round
  bool aligned = false;
  uint32_t true_rounds = 0;
  AlignedSplit split;
  bool any_mesh = false, need_direct = false;
  bool level = false;                      // level mode (else the compaction path)
};

// Level mode, one launch kind per round; the round's chunks are
// [off[q], off[q+1]); on N ranks the chunks of nodes fed by a ghost parent
// come last, from gsplit[q] (they wait for the round's exchange).
struct PullPlan {
  std::vector<uint64_t> key;
  uint64_t version = 0;  // bumped by every change (run.cpp uploads on a new version)
  std::vector<PullChunk> chunks;
  std::vector<uint32_t> off, gsplit;
  std::vector<uint64_t> bytes;  // row bytes written per round
};
struct PairPlan {
  std::vector<uint64_t> key;
  uint64_t version = 0;
  std::vector<PullChunk> chunks;         // pair launches
  std::vector<ChainChunk> chain;         // chain launches
  std::vector<uint32_t> lo, hi, gsplit;  // round q: chunks (pair) or chain chunks of the launch starting at q
                                         // (chains: whole rows [lo, gsplit), column slices [gsplit, hi))
  std::vector<uint32_t> len;             // round q: rounds of the launch starting at q (0: none)
  std::vector<uint8_t> kind;             // per round: PS_K_*
};
struct FloodPlan {
  std::vector<uint64_t> key;
  uint64_t version = 0;
  std::vector<FloodTask> tasks;
  std::vector<FloodSeg> segs;
  std::vector<uint32_t> slot0, nslot;  // per round: partial counter slots
  uint32_t slots = 1;                  // slots of a window (slot 0: the timeout word)
  uint32_t granules = 0;
};
// Multi-GPU: the ghost exchange of a window.
struct GhostRound {
  std::vector<uint64_t> s_off, s_len, r_off, r_len;  // transport regions, bytes (send: in the round's half)
  uint32_t pack0 = 0, pack1 = 0;                     // the round's root segments (k_pack)
  uint64_t pack_units = 0;                           // their units (k_pack's stream)
  bool any = false;                                  // some rank ships rows this round (same on every rank)
  uint64_t rec_bytes = 0;                            // record bytes this rank receives (in place: roots' only)
};
struct GhostPlan {
  std::vector<uint64_t> key;
  std::vector<GhostRound> rounds;
  std::vector<GhostSeg> segs;     // per (round, topic, start group): record bases
  std::vector<std::vector<std::vector<uint32_t>>> seg_of;  // [round][topic][group] -> segs index (kNoneNode: none)
  std::vector<PackSeg> pack;      // roots' records (level-1 rounds)
  uint64_t send_half = 0;         // words per part of the send buffer (kSendBufs parts, by round)
  uint64_t recv_words = 0;
};

}  // namespace psamd

struct ps_engine {
  ps_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  hipStream_t xstream = nullptr;  // multi-GPU: the exchange, beside the round's local chunks
  hipEvent_t ev_run0 = nullptr, ev_run1 = nullptr;
  hipEvent_t ev_round = nullptr, ev_xchg = nullptr;  // multi-GPU: round boundary, exchange done
  // the exchange on its own stream beside the round's locally fed chunks
  // (ps_plan_opts.xchg_overlap, -1 = auto): a transport that copies the
  // records (RCCL; the loopback with PS_DIST_F_COPY) yes; the zero-copy
  // loopback no -- there it only contends for the same GPU (4 loopback
  // ranks, cfg4: 7.06 vs 6.32 ms/step, profiles/r03/loopback)
  int xchg_overlap_env = -1;
  bool xchg_overlap = true;
  std::vector<hipEvent_t> ev_k;  // pairs around expand launches
  uint32_t n_cus = 256, expand_grid = 2048;
  bool host_only = false;        // a planner probe (psengine_plan.h): no device
  psamd::WindowLayout probe;     // the probe's last planned window
  bool host_timing = false;      // PSAMD_HOST_TIMING=1: host phase times to stderr
  bool sig_windows = true;        // pipelined one-rank windows end with a pinned flag, not an event (A/B: PSAMD_SIG_WINDOWS=0)
  // per-window uploads (topic table, seeds, descriptors) kept on the device:
  // the bytes last staged into each buffer, skipped when a window repeats them
  struct UploadShadow {
    uint64_t gen = 0;
    std::vector<uint8_t> data;
  };
  std::map<const psamd::DevBuf*, UploadShadow> upload_shadow;
  bool upload_reuse = true;  // (A/B: PSAMD_UPLOAD_REUSE=0)
  bool defer_into_signalled = false;  // the window being enqueued raises its flag in its reduce
  uint64_t sig_seq = 0;
  // a signalled window's reduce, held back to run in the next window's first
  // launch (k_window_turn) -- or alone, from ps_wait, if none comes first
  // (A/B: PSAMD_FUSE_REDUCE=0)
  bool fuse_reduce = true;
  struct PendingReduce {
    bool valid = false;
    const void* owner = nullptr;  // the Inflight slot whose flag it raises
    psamd::ReduceArgs args{};
  } pend_reduce;
  // GPU rebuild of the node space: on by default for one
  // rank and tree topics (PSAMD_GPU_BUILD=0: host build)
  bool gpu_build_on = true;
  bool gpu_graph = false;     // the current node space was built on the GPU
  bool mirrors_valid = true;  // host copies of node_peer / flags / CSR are current
  std::vector<uint32_t> pairs_host, gstat_host, roots_host;
  bool live_dev_valid = false;  // d_live holds `live` (uploaded again only after ps_set_live)
  bool flags_built = false;     // the last GPU build wrote the node flags (no flags pass needed)
  uint32_t* pairs_pinned = nullptr;  // pinned staging of the parent deltas
  size_t pairs_pinned_cap = 0;       // (u32 words)
  std::vector<size_t> pair_off;
  psamd::DevBuf d_tpar, d_orph, d_local, d_first,
      d_gstat, d_cub, d_pairs, d_live, d_roots, d_cnt, d_fidx, d_childoff, d_lbstat, d_sigctr, d_kids, d_big, d_ndeg, d_nkat, d_query;
  std::chrono::steady_clock::time_point t_run0;
  // the lazy prune's reach queries, enqueued with the GPU rebuild that
  // precedes the run's last phase (its result comes back with the build's
  // readback, no round trip of its own); the prune uses a result whose peers
  // match its question, else asks the GPU itself
  struct EarlyQuery {
    uint32_t topic = 0;
    std::vector<uint32_t> peers;
    std::vector<uint8_t> out;
    bool launched = false, ready = false;
  };
  std::vector<EarlyQuery> early_q;
  // k_flood: a single-rank level window's leading rounds in
  // one persistent launch; PSAMD_FLOOD=0 runs per-round launches instead
  bool flood_on = true;
  bool flood_broken = false;  // a dependency wait timed out once: per-level launches from then on
  uint32_t flood_grid = 0;    // resident blocks (0: k_flood unavailable)
  uint32_t flood_words = psamd::kFloodWords;  // row words per task (PSAMD_FLOOD_WORDS)
  uint32_t pull_words = psamd::kPullWords;    // row words per k_pull chunk (512..4096 measured: 1024 best)
  // k_flood runs the leading rounds writing at most this many row bytes (with
  // chains after it: 4 MB; 16 MB was best before them, profiles/r03/ab_flood_top.txt)
  uint64_t flood_top_bytes = 4ull << 20;
  uint32_t flood_min_rounds = 4;  // k_flood only for at least this many leading rounds (ps_plan_opts)
  bool align_groups = true;       // one-rank start-group windows run level-aligned (ps_plan_opts)
  uint32_t flood_epoch = 0;   // granule tag of the last launch (granules are never reset)
  uint32_t flood_spin_ticks = 200000000u;  // dependency-wait bound: 2 s of s_memrealtime (100 MHz); PSAMD_FLOOD_SPIN_TICKS
  psamd::FloodPlan flood;
  uint64_t flood_up = ~0ull;  // plan version of the tasks on the device
  psamd::DevBuf d_flood_tasks, d_flood_segs, d_flood_gran;
  bool flood_profile = false;  // PSAMD_FLOOD_PROFILE=1: per-wave phase times of k_flood to stderr (sync runs)
  psamd::DevBuf d_flood_prof;
  uint32_t flood_prof_waves = 0;
  // PSAMD_CHAIN_PROFILE=<file>: per-wave start / end / words of every
  // k_pull_chain launch of blocking windows, appended to <file> (debug)
  std::string chain_prof_path;
  psamd::DevBuf d_chain_prof;

  std::vector<psamd::TopicHost> topics;
  std::vector<uint8_t> live;
  bool graph_dirty = true, flags_dirty = true;
  uint64_t graph_epoch = 0, flags_epoch = 0;  // bumped by every upload

  // level mode, per-round counter slots and their reduce descriptors
  std::vector<uint32_t> woff_host, desc_host;
  psamd::DevBuf d_woff;
  // level-aligned windows: the (topic, level) pieces of k_level_reach, cached
  // per node space and active topic set
  psamd::DevBuf d_reach;
  std::vector<psamd::ReachPiece> reach_host;
  std::vector<uint64_t> reach_key;
  uint32_t n_reach = 0, reach_a = 0;  // pieces; those of levels <= the prefix P (first)
  // level mode, pull direction: per-round chunks of next-level nodes
  psamd::PullPlan pull;
  psamd::DevBuf d_pull;
  uint64_t pull_up = ~0ull;  // plan version of the chunks on the device
  // rounds per launch at most (ps_plan_opts.chain_max, 1..kChainLevels): 1 =
  // one k_pull per round, 2 = pairs (k_pull_pair), 3..6 chains.
  // Defaults by measurement (profiles/r03/ab_chain_v2.txt):
  // 4 for single-start windows (cfg3 burst 1.016 vs 1.033 ms at 6), 6 for
  // windows with start groups (paced cfg3 1.363 vs 1.443 ms at 4)
  uint32_t chain_max = 4, chain_max_groups = 6;
  psamd::DevBuf d_chain;
  uint32_t pad_words = 16;        // rows of at least this many words padded to even (PSAMD_PAD_WORDS)
  bool chain_tail = true;         // a chain ending at the last round may be one round longer (PSAMD_CHAIN_TAIL)
  double launch_bytes = 16e6;     // planner: a launch's ramp and tail as row bytes (PSAMD_LAUNCH_BYTES)
  uint32_t chain_words = 4096;    // row words per chain wave, the planner's target (8192 until r05: cfg4 0.444 -> 0.404, cfg3 -0.5..1 %, profiles/r05/ab/)
  uint32_t chain_words_lead = 0;  // A/B only (PSAMD_CHAIN_WORDS_LEAD): the same for all but the last launch
  uint32_t expand_opts = 0;       // ExpandArgs::opts (A/B only: PSAMD_NARROW=0 -> kExpandNoNarrow)
  uint32_t chain_waves = 12;      // chain launches: resident waves per CU at most (ps_plan_opts)
  bool chain_nt = true;           // chain launches: level 0 and the inner levels stored non-temporally
  std::vector<uint64_t> chain_fail_key;  // a pair plan whose chain ranges overflowed the level tables: no chains
  psamd::DevBuf d_chain_ovf;
  psamd::DevBuf d_chain_meta, d_chain_cnt, d_chain_scan;  // the chunks' node entries (k_chain_meta)
  // rows of rounds writing at least this much store non-temporally (the MALL
  // cannot hold them for the next launch: reversing launch order and cached
  // stores measured 0-50 % slower, profiles/r03/ab_mall_reverse.txt)
  static constexpr uint64_t kNtBytes = 64ull << 20;
  psamd::PairPlan pair;
  psamd::DevBuf d_pp;
  uint64_t pair_up = ~0ull;
  std::vector<uint8_t> round_kind;  // per round of the current window: PS_K_* (empty: k_expand)

  // fused node space (host mirror)
  uint32_t n_nodes = 0, n_pad = 16;
  std::vector<uint32_t> node_peer, row_ptr, col;
  std::vector<uint32_t> node_parent;  // node-space parent on this rank (kNone: root / remote)
  std::vector<uint16_t> node_topic;
  std::vector<uint8_t> node_flags;

  psamd::DevBuf d_row_ptr, d_col, d_node_topic, d_node_flags, d_node_peer, d_node_parent;
  psamd::DevBuf d_ext0, d_ext1;  // compaction mode, one rank: arrival extents (ExpandArgs::ext_cur)
  psamd::DevBuf d_seen, d_arr0, d_arr1, d_hop, d_flags, d_blk, d_gen, d_frontier, d_nfront, d_wgcount,
      d_partials, d_stats, d_topics, d_seeds, d_digest, d_groups;
  uint32_t gen_cur = 0;  // window generation stamped into d_gen (1..255)
  psamd::DevBuf d_remote_fed, d_send, d_recv, d_apply_stats;
  // multi-GPU level mode: ghost parents
  std::vector<uint32_t> ghost_ref;  // per node: remote parent's rank << 27 | record index, or kNone
  std::vector<psamd::ShipEntry> ship_host;  // every topic's send entries (TopicHost::ship0)
  psamd::GhostPlan ghost;
  psamd::DevBuf d_ghost_ref, d_ship, d_gsegs, d_pack;
  bool ghost_up = false;  // the ghost plan's segments and root segments are on the device
  uint32_t n_remote_fed = 0;
  std::vector<uint32_t> remote_fed;  // owned nodes whose parent is on another rank

  // multi-GPU: this engine owns a hash-partitioned share of every topic
  int32_t rank = 0, world = 1;
  bool inplace = false;  // PS_DIST_F_INPLACE: kSegInPlace segments, RankRows of every rank
  psamd::DevBuf d_rrows;
  std::vector<psamd::RankRows> rrows_host;
  bool rrows_dirty = false;
  uint32_t partition = PS_PART_PEER, split_depth = 0;
  std::unique_ptr<psamd::Transport> transport;

  // publishes not yet run
  std::vector<psamd::RunMsg> pending;
  bool pending_nonzero_start = false;  // some pending message starts after round 0
  bool pending_mixed = false;          // pending messages name more than one topic
  uint32_t pending_topic0 = 0;         // ... the topic of the first one
  uint32_t run_iota_n = 0;             // run_sorted / run_rank hold 0 .. n-1 (one-topic runs)
  bool run_zero_start = true;          // every message of the current run starts in round 0
  uint32_t next_msg = 0;

  // results of the last run
  uint32_t last_first = 0, last_n = 0;
  bool have_hops = false;
  std::vector<uint8_t> hops;  // [msg][peer]
  std::vector<psamd::RunMsg> last_msgs;  // messages of the last run, publish order
  std::vector<uint32_t> run_sorted;      // run message indices grouped by topic
  std::vector<uint32_t> run_topic_off;   // topic -> first position in run_sorted
  std::vector<uint32_t> run_rank;        // message -> position within its topic
  std::vector<uint32_t> last_lo, last_cnt;  // topic -> last window's rank range
  // topic -> the last window's row bit of each window message (empty: bit li
  // = the message's window slot; else the start-group layout, StartGroup)
  std::vector<std::vector<uint32_t>> last_pos;
  std::vector<std::vector<psamd::StartGroup>> last_groups;  // topic -> the last window's start groups
  std::vector<psamd::TopicDev> last_topics;
  bool have_window = false;
  std::map<uint32_t, std::vector<uint32_t>> peer_node;  // topic -> peer -> node (ps_read_peer_messages)
  std::vector<uint64_t> peer_node_epoch;                 // graph_epoch each map was built for

  // asynchronous runs (ps_run_async / ps_wait): the last window of a run may
  // leave its stats on the stream (pinned readback) so that the host plans
  // the next run while this one's kernels execute
  struct Inflight {
    ps_stats st{};
    bool deferred = false;
    uint32_t r = 0, launches = 0;
    uint32_t mode = PS_MODE_COMPACT, flood_rounds = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the window's kernels
    uint64_t* hs = nullptr;      // pinned: (PS_MAX_ROUNDS + 1) x kNumCtr counters
    uint64_t* hs_dev = nullptr;  // hs, device-mapped (k_reduce_rounds writes it)
    uint64_t* ha = nullptr;      // pinned: apply counters of a multi-GPU window
    // signalled windows (no end event): sig[0] = the window's sequence number
    // once done, sig[1] / sig[2] = its start / end s_memrealtime stamps
    uint64_t* sig = nullptr;
    uint64_t* sig_dev = nullptr;
    uint64_t seq = 0;
    bool signalled = false;
    uint32_t planned0 = 0;
    uint32_t true_rounds = 0;   // level-aligned windows: rounds by start round (else planned0)
    psamd::AlignedSplit split;  // level-aligned windows: the per-round split
    int32_t world = 1;
    std::vector<uint8_t> kinds;  // round_kind of the window
    hipStream_t stream = nullptr;  // the stream the window's kernels ran on
  };
  Inflight infl[2];
  uint32_t infl_head = 0, infl_count = 0;

  // per-window uploads (topic table, seeds, reduce descriptors) go through
  // pinned staging: a copy from pageable memory blocks the host until the
  // stream has drained, so the next batch's launches would only be issued
  // once the previous batch had finished (a ~35 us bubble per pipelined
  // step).  Two slots alternate; a slot is rewritten only after the copies
  // of its previous use have completed: slot i belongs to asynchronous run
  // slot i (synchronous runs use slot 0 with nothing in flight).
  struct Staging {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;  // the slot's device-mapped address
    size_t cap = 0;
  };
  Staging stg[2];
  bool defer_phase = false;  // the current phase may defer its last window's stats
  bool defer_last = false;   // ... and this window is that last window
  Inflight* defer_into = nullptr;

  // Cross-window overlap.  A deep single-rank window (at
  // least overlap_min_rounds rounds, one start round) plans no k_flood; its
  // leading launches -- a few % of its bytes, rounds 1..P, latency bound --
  // form the prefix.  Its gate is the launch that starts at round P + 1 (the
  // last one reading a level <= P).  A pipelined window whose predecessor
  // (other slot) is in flight with the same plan runs its window init and
  // prefix on pstream once that predecessor's gate is done, beside the
  // predecessor's remaining launches: they touch only levels > P + 1, and the
  // per-window tables (topics, seeds, reduce descriptors, partial slots) are
  // per slot.  PSAMD_OVERLAP=0: off.
  bool overlap_on = true;
  uint32_t overlap_min_rounds = 12;
  uint64_t overlap_min_bytes = 512ull << 20;  // row bytes of the window at least (PSAMD_OVERLAP_BYTES)
  hipStream_t pstream = nullptr;
  hipStream_t rstream = nullptr;  // a pipelined window's counter reduce, beside the next window
  // the lazy prune's reach queries: they read the node space of the window
  // just enqueued (its build is complete), not its rows, so they run beside
  // the window's kernels instead of behind them
  hipStream_t qstream = nullptr;
  hipEvent_t ev_gate[2] = {nullptr, nullptr}, ev_pre = nullptr, ev_end = nullptr;
  bool gate_valid = false;
  uint32_t gate_slot = 0;
  std::vector<uint64_t> gate_key;  // plan versions, node-space epochs and P of the gate's window
  uint64_t overlapped = 0;         // windows whose prefix ran beside their predecessor (stats)
  uint32_t last_slot = 0;          // the slot of the last enqueued window's tables
  psamd::DevBuf d_topics1, d_woff1, d_groups1, d_partials1, d_seeds1;  // slot 1's tables

  // Twin windows.  A pipelined one-rank level window whose
  // plan is already on the device runs ENTIRELY beside its predecessor: on
  // the other of two streams (stream / tstream), into the other of two row
  // sets (seen + arrivals + generation bytes, swapped so that d_seen & co.
  // always name the last window's), with its own slot's tables and signal
  // counter.  Nothing the two share is written by either (node space, plan
  // tables, reach pieces are read-only; uploads make a window a non-twin).
  // Work on `stream` that changes shared state first waits for tstream's
  // last window (twin_join); a twin window on tstream first waits for work
  // `stream` did since tstream last followed it (e_seq).  PSAMD_TWIN=0: off.
  bool twin_on = true;
  hipStream_t tstream = nullptr;
  hipEvent_t ev_tend = nullptr, ev_e2t = nullptr;
  bool t_pending = false;            // tstream ran a window `stream` has not waited for
  uint64_t e_seq = 1, t_seq = 0;     // shared-state work on `stream` / the last that tstream followed
  hipStream_t last_win_stream = nullptr;
  psamd::DevBuf d_seen_b, d_arr0_b, d_arr1_b, d_gen_b;  // the other row set
  uint32_t gen_cur_b = 0;
  void swap_row_sets() {
    d_seen.swap(d_seen_b);
    d_arr0.swap(d_arr0_b);
    d_arr1.swap(d_arr1_b);
    d_gen.swap(d_gen_b);
    std::swap(gen_cur, gen_cur_b);
  }

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
  int hip_fail(hipError_t e, const char* what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return PS_E_DEVICE;
  }
};

#define HIP_TRY(expr, what)                              \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return e->hip_fail(_e, what); \
  } while (0)

namespace psamd {

// graph.cpp
bool topic_ok(const ps_engine* e, uint32_t topic);
void peer_children(const ps_engine* e, const TopicHost& T, std::vector<uint32_t>& rp, std::vector<uint32_t>& cl);
void partition_topic(const std::vector<uint32_t>& order, const std::vector<uint32_t>& bfs_parent,
                     const std::vector<uint32_t>& level, int32_t world, uint32_t part, uint32_t split_depth,
                     std::vector<int32_t>& owner);
int build_graph(ps_engine* e);  // host node space (any rank count); no device calls
void build_flags(ps_engine* e);
int ensure_mirrors(ps_engine* e);
int upload_graph(ps_engine* e);
// run.cpp: the engine stream waits for tstream's last twin window (a no-op
// when none is pending); every change of shared device state goes after it
int twin_join(ps_engine* e);

// plan.cpp (host only: no device calls)
int plan_window_layout(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<WinSlice>& win,
                       WindowLayout& L);
bool plan_pull_chunks(ps_engine* e, const WindowLayout& L);  // true: the plan changed
bool plan_pair_chunks(ps_engine* e, const WindowLayout& L, uint32_t first);
bool plan_flood_tasks(ps_engine* e, const WindowLayout& L, uint32_t rounds);
int plan_ghost(ps_engine* e, const WindowLayout& L, bool* changed);
void annotate_chunks(ps_engine* e, const WindowLayout& L);
uint32_t plan_flood_rounds(const ps_engine* e, const WindowLayout& L);
// A deep single-start window: chains from round 1, no k_flood.
bool deep_window(const ps_engine* e, const WindowLayout& L);

// run.cpp
int run_body(ps_engine* e, ps_stats* st, bool may_defer);
bool accumulate_window(ps_stats* st, const uint64_t* hs, const uint64_t* ha, uint32_t r, uint32_t planned0,
                       uint32_t mode, uint32_t flood_rounds, uint32_t launches, int32_t world,
                       const std::vector<uint8_t>& kinds, bool by_round = true);
// A level-aligned window's per-round deliveries and frontier entries from
// its reach rows (hs rows split.row0 ..): false when they disagree with the
// kernels' per-level counters (rows 1 .. r)
bool split_aligned_window(ps_stats* st, const uint64_t* hs, uint32_t r, uint32_t true_rounds,
                          const AlignedSplit& sp, std::string* why = nullptr);

}  // namespace psamd
