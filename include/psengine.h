/*
 * psengine.h -- C ABI of the MI355X subtree-dissemination engine.
 *
 * Drop-in boundary for the one hot path of go-libp2p-pubsub v0: flooding
 * published messages down each topic's subscription tree (subtree.go).
 * Plain C types only (no torch, no HIP types): a cgo shim, ctypes or C++ binds
 * it directly.  Every entry point names the reference interface it replaces.
 *
 * Conventions:
 *  - return codes: 0 = PS_OK, negative = PS_E_*; the cgo shim turns a negative
 *    code plus ps_last_error() into a Go `error`.
 *  - caller arrays are borrowed for the duration of the call and copied;
 *    the engine owns all device memory.
 *  - an engine is NOT thread-safe; the caller serialises calls, as
 *    subtree.chlock does in the reference (subtree.go:18,320).
 *  - peers are dense u32 ids [0, n_peers) standing in for peer.ID
 *    (go-libp2p-peer); messages are u32 publish indices returned by
 *    ps_publish (the reference's Message has no ID, pubsub.go:146-153).
 */
#ifndef PSENGINE_H
#define PSENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PS_NONE 0xFFFFFFFFu
#define PS_HOP_NONE 0xFFu
#define PS_MAX_ROUNDS 256

enum ps_status {
  PS_OK = 0,
  PS_E_INVAL = -1,       /* bad argument                                        */
  PS_E_NOMEM = -2,       /* host or device allocation failed                    */
  PS_E_STATE = -3,       /* peer/topic in the wrong state for the request       */
  PS_E_NOPARENT = -4,    /* redirectJoin found no live child (subtree.go:172)   */
  PS_E_UNREACHABLE = -5, /* join redirected into a closed host (subtree.go:302) */
  PS_E_DEVICE = -6,      /* HIP runtime error                                   */
  PS_E_RANGE = -7,       /* message id / topic id out of range                  */
  PS_E_NOTREADY = -8     /* no completed run holds the requested record         */
};

/* ps_config.flags */
#define PS_F_RECORD_HOPS 0x1u  /* keep (peer,msg)->hop for ps_read_hops (parity) */
#define PS_F_TIME_KERNELS 0x2u /* HIP-event time every expand launch            */
#define PS_F_NO_LAZY_SEEN 0x4u /* clear the seen bitset eagerly per window      */
#define PS_F_COMPACT 0x8u      /* every window through the compaction path (the
                                  general-graph k_expand rounds), trees too     */

typedef struct ps_config {
  uint32_t n_peers;        /* peer id space [0, n_peers)                       */
  uint32_t n_topics;       /* topic slots [0, n_topics)                        */
  uint32_t tree_width;     /* DefaultTreeWidth  (pubsub.go:16), 0 -> 2         */
  uint32_t tree_max_width; /* DefaultTreeMaxWidth (pubsub.go:17), 0 -> 5       */
  uint32_t msg_window;     /* max messages per topic per window, 0 -> 65536,
                              at most 2^30 (PS_E_INVAL above)                  */
  int32_t device;          /* HIP device ordinal                               */
  uint32_t flags;          /* PS_F_*                                           */
  uint32_t reserved;
  uint64_t seed;           /* redirect tie-break stream (Go map order, Q2)     */
} ps_config;

/* ps_stats.expand_mode: how the last window's rounds ran */
#define PS_MODE_COMPACT 0u     /* k_expand over a compacted frontier (flags + scan) */
#define PS_MODE_LEVEL_PULL 2u  /* k_pull: one launch per round, each level pulls its
                                  parents' rows (start groups, multi-GPU windows) */
#define PS_MODE_FLOOD 3u       /* k_flood for the leading rounds (one persistent
                                  launch, each level pulls its parents' rows once
                                  the tasks writing them have published), then
                                  k_pull per round; see ps_stats.flood_rounds     */

typedef struct ps_stats {
  uint64_t deliveries;         /* (peer,msg) pairs delivered by this run        */
  uint64_t duplicates;         /* bits suppressed by the seen test (0 on trees)  */
  uint64_t frontier_entries;   /* frontier nodes expanded                        */
  uint64_t child_visits;       /* (frontier node, child) pairs                   */
  uint64_t edge_words;         /* (child, 64-message word) pairs tested          */
  uint64_t expand_bytes;       /* algorithmic HBM bytes of the expand kernel     */
  uint64_t windows;            /* propagation windows                            */
  uint64_t rounds;             /* synchronous rounds launched                    */
  uint64_t expand_launches;    /* expand kernel launches                         */
  double run_ms;               /* device time of the whole run (HIP events; a
                                  pipelined one-rank window: its start and
                                  reduce-end device stamps -- a reduce held back
                                  into the next window's first launch, or to
                                  ps_wait, ends there)                          */
  double expand_ms;            /* summed expand-kernel device time (TIME flag)   */
  double host_ms;              /* wall time of the ps_run call                   */
  uint32_t expand_mode;        /* hot kernel of the last window: PS_MODE_*       */
  uint32_t flood_rounds;       /* PS_MODE_FLOOD: leading rounds of the last
                                  window run by k_flood (the rest: k_pull)      */
  uint64_t deliveries_per_round[PS_MAX_ROUNDS];
  float expand_ms_per_round[PS_MAX_ROUNDS];   /* TIME flag, summed over windows  */
  uint32_t frontier_per_round[PS_MAX_ROUNDS]; /* expanded entries per round      */
  uint64_t expand_bytes_per_round[PS_MAX_ROUNDS]; /* algorithmic bytes per round */
  uint8_t round_kernel[PS_MAX_ROUNDS]; /* PS_K_*: the launch kind that wrote each
                                          round of the last window              */
  /* the effective plan of the last window (scheduling diagnostics) */
  uint32_t plan_max_rounds;    /* rounds of its longest launch (1: k_pull, 2: pair,
                                  3..7: chain; k_flood counts as 1)            */
  uint32_t prefix_rounds;      /* leading rounds that may run beside the previous
                                  window (0: none)             */
  uint32_t overlapped;         /* windows of this run whose prefix ran beside
                                  their predecessor                             */
  uint32_t xchg_path;          /* N ranks: PS_XCHG_* of the last window         */
  uint64_t xchg_rounds;        /* N ranks: rounds of this run that exchanged     */
  uint64_t xchg_bytes;         /* N ranks: ghost-record bytes this rank received */
  uint32_t level_aligned;      /* the last window ran level-aligned start groups
                                  (ps_plan_opts.align_groups): round_kernel,
                                  expand_bytes_per_round and expand_ms_per_round
                                  are indexed by launch round = BFS level;
                                  deliveries_per_round / frontier_per_round stay
                                  by round (start + level)                      */
  uint32_t reserved2;
} ps_stats;

/* ps_stats.xchg_path: how a multi-rank level window's ghost records moved */
#define PS_XCHG_NONE 0u       /* one rank, or nothing exchanged                */
#define PS_XCHG_ZERO_COPY 1u  /* read in place from the sender's send region
                                 (loopback ranks sharing one process and GPU)  */
#define PS_XCHG_COPY 2u       /* copied into this rank's receive buffer (RCCL
                                 send/recv; the loopback with PS_DIST_F_COPY)  */
#define PS_XCHG_IN_PLACE 3u   /* ghost parents' rows read where their owner
                                 wrote them (PS_DIST_F_INPLACE); only the topic
                                 roots' rows still move as records            */

/* ps_stats.round_kernel */
#define PS_K_NONE 0u
#define PS_K_FLOOD 1u   /* k_flood (its one launch is timed into round 1)      */
#define PS_K_PULL 2u    /* k_pull, one launch for this round                   */
#define PS_K_PAIR 3u    /* k_pull_pair: this round and the next in one launch   */
#define PS_K_PAIR2 4u   /* k_pull_pair: the second round of the launch above    */
#define PS_K_EXPAND 5u  /* k_expand (compaction mode)                          */
#define PS_K_CHAIN 6u   /* k_pull_chain: this round and the next 2-3 in one launch */
#define PS_K_CHAIN2 7u  /* k_pull_chain: a later round of the launch above      */

typedef struct ps_engine ps_engine;

/* ---- lifecycle: NewTopicManager (pubsub.go:26-31) ------------------------ */
int ps_create(const ps_config* cfg, ps_engine** out);
void ps_destroy(ps_engine* e);
const char* ps_last_error(const ps_engine* e);
const char* ps_version(void);

/* ABI guard.  The public structs' layouts are versioned by PS_ABI_VERSION
 * (5: ps_stats gained the plan diagnostics and xchg fields, ps_dist_config
 * its flags word -- a caller built against an older header would read or
 * write past its own structs).  A binding calls ps_abi_check once, with the
 * sizes it was compiled with (PS_ABI_CHECK() in C/C++); PS_E_INVAL on any
 * mismatch, with ps_last_error(NULL) naming it. */
#define PS_ABI_VERSION 5u
uint32_t ps_abi_version(void);
int ps_abi_check(uint32_t abi_version, size_t config_size, size_t stats_size,
                 size_t plan_opts_size, size_t dist_config_size);
#define PS_ABI_CHECK()                                                        \
  ps_abi_check(PS_ABI_VERSION, sizeof(ps_config), sizeof(ps_stats),           \
               sizeof(struct ps_plan_opts), sizeof(struct ps_dist_config))

/* ---- topics: TopicManager.NewTopic + TreeOpts (pubsub.go:49-97),
 *      Topic.Close (pubsub.go:99-103).  width 0 -> engine default.            */
int ps_topic_create(ps_engine* e, uint32_t topic, uint32_t root,
                    uint32_t tree_width, uint32_t tree_max_width);
int ps_topic_close(ps_engine* e, uint32_t topic);

/* ---- membership, restated on the host (sequential by nature):
 * ps_topic_join:  TopicManager.Subscribe -> joinToPeer -> handleJoin /
 *                 redirectJoin / joinParents (client.go:65-94,
 *                 subtree.go:100-307).  status_out[i] (nullable) gets the
 *                 per-peer PS_* code; the call returns the first failure.
 * ps_topic_leave: client.Close -> Part -> redistributeChildren
 *                 (client.go:30-34, subtree.go:46-98,356-375).
 * ps_topic_drop:  host.Close(): abrupt; the parent notices on its next write
 *                 (subtree.go:333-351); that message is lost below the peer. */
int ps_topic_join(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n,
                  int32_t* status_out);
int ps_topic_leave(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n);
int ps_topic_drop(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n);

/* ---- explicit topology (harness / parity inputs) ---------------------------
 * set_tree:     parent[p] for every peer (PS_NONE = not in the tree); the tree
 *               printTree walks (pubsub_test.go:204-229).
 * set_children: general child lists in peer space (row_ptr[n_peers+1],
 *               col[row_ptr[n_peers]]); a peer may have several parents
 *               (mesh), in which case the seen bitset deduplicates.
 * get_parents:  current attached tree (PS_NONE = not attached / orphaned).   */
int ps_topic_set_tree(ps_engine* e, uint32_t topic, uint32_t root, const uint32_t* parent);
int ps_topic_set_children(ps_engine* e, uint32_t topic, uint32_t root,
                          const uint32_t* row_ptr, const uint32_t* col);
int ps_topic_get_parents(ps_engine* e, uint32_t topic, uint32_t* parent_out);
int ps_topic_depth(ps_engine* e, uint32_t topic, uint32_t* depth_out, uint32_t* n_nodes_out);

/* Replace the engine's PS_F_* flags (e.g. PS_F_TIME_KERNELS for an
 * instrumented run between untimed ones); applies to the next ps_run. */
int ps_set_flags(ps_engine* e, uint32_t flags);

/* ---- launch-plan options ----------------------------------
 * The schedule knobs whose defaults were chosen by measurement (the A/B
 * records under profiles/).  ps_create starts from the defaults; a caller
 * pins or changes them only through ps_set_plan_opts -- the environment does
 * not touch them, except for A/B tools that set PSAMD_AB=1 (then the PSAMD_*
 * variables are read at ps_create).  Plans are rebuilt on the next run. */
typedef struct ps_plan_opts {
  uint64_t flood_top_bytes;    /* k_flood runs the leading rounds that each write at
                                  most this many row bytes (4 MiB)              */
  uint64_t overlap_min_bytes;  /* windows of fewer row bytes never overlap (512 MiB) */
  uint64_t launch_bytes;       /* planner: a launch's ramp and tail, as row bytes (16e6) */
  uint32_t flood;              /* 1: k_flood for a one-rank window's leading rounds (1) */
  uint32_t chain_max;          /* rounds per launch at most, single-start windows:
                                  1 = one k_pull per round, 2 = pairs, 3..6 chains (4) */
  uint32_t chain_max_groups;   /* the same for windows with start groups (6)     */
  uint32_t chain_tail;         /* 1: a chain ending at the last round may take one
                                  round more (1)                                */
  uint32_t chain_words;        /* row words a chain wave writes, planner target (4096) */
  uint32_t flood_words;        /* row words per k_flood task (2048)              */
  uint32_t pad_words;          /* rows of at least this many words padded to even (16) */
  uint32_t overlap;            /* 1: pipelined deep windows overlap their leading
                                  launches with the previous window (1)          */
  uint32_t overlap_min_rounds; /* ... windows of at least this many rounds (12) */
  int32_t xchg_overlap;        /* N ranks: exchange on its own stream beside the
                                  locally fed chunks: -1 auto (RCCL yes, loopback
                                  no), 0, 1 (-1)                                */
  uint32_t gpu_build;          /* 1: rebuild a one-rank node space on the GPU (1) */
  uint32_t flood_spin_ticks;   /* k_flood dependency-wait bound, 100-MHz ticks (2e8) */
  uint32_t chain_nt;           /* 1: chain launches store level 0 and their inner
                                  levels non-temporally, 0: plain stores (1)    */
  uint32_t chain_waves;        /* chain launches: resident waves per CU at most,
                                  1..16 (an LDS pad), 0: as many as fit (12)    */
  uint32_t flood_min_rounds;   /* k_flood only when it would run at least this many
                                  leading rounds; fewer go to chain launches (4) */
  uint32_t align_groups;       /* 1: a one-rank window with start groups (paced
                                  publishing) runs level-aligned -- launch round q
                                  writes BFS level q of every start group, each
                                  group's deliveries counted and recorded in its
                                  own round (start + level) -- instead of one
                                  launch schedule over start + depth rounds (1) */
} ps_plan_opts;

int ps_plan_opts_default(ps_plan_opts* out);
/* effective options of an engine (the defaults, or what ps_set_plan_opts set) */
int ps_get_plan_opts(const ps_engine* e, ps_plan_opts* out);
/* PS_E_INVAL on an out-of-range value; PS_E_STATE with runs in flight */
int ps_set_plan_opts(ps_engine* e, const ps_plan_opts* opts);

/* Subscribed-and-live mask over peers (1 = receives and forwards).  A peer
 * whose client stopped reading (client.go:103-131) is 0. Default: all 1. */
int ps_set_live(ps_engine* e, const uint8_t* live);

/* ---- the hot path ----------------------------------------------------------
 * ps_publish:    Topic.PublishMessage (pubsub.go:111-120) for a batch; message
 *                i of the batch gets id *first_msg_id_out + i.
 * ps_publish_at: same, message i enters its topic root at round start_round[i]
 *                (paced / pipelined publishing; hop = round - start_round).
 * ps_run:        forwardMessage (subtree.go:319-354) + processMessages
 *                (client.go:100-132) for every enqueued message, as
 *                synchronous rounds on the GPU, to quiescence.               */
int ps_publish(ps_engine* e, const uint32_t* topic_of_msg, size_t n_msgs,
               uint32_t* first_msg_id_out);
int ps_publish_at(ps_engine* e, const uint32_t* topic_of_msg, const uint32_t* start_round,
                  size_t n_msgs, uint32_t* first_msg_id_out);
int ps_run(ps_engine* e, ps_stats* out);
/* ps_run in two halves, for pipelined batches: ps_run_async plans and enqueues
 * the run and returns while its last window's kernels execute (at most two runs
 * in flight), so the caller can publish and enqueue the next batch; ps_wait
 * completes the oldest run in flight and returns its stats.  Reads
 * (ps_read_*, ps_seen_digest) and membership changes stay stream-ordered
 * behind the runs in flight; ps_run refuses while any is pending.  (A one-rank
 * run's counter reduce may be held back to ride in the next ps_run_async's
 * first launch; ps_wait launches it itself when no run came first.) */
int ps_run_async(ps_engine* e);
int ps_wait(ps_engine* e, ps_stats* out);

/* ---- results of the last ps_run (client.Messages, client.go:26-28) --------
 * ps_read_hops: hop of message `msg` at every peer (PS_HOP_NONE = not
 *               delivered; hops beyond 254 read as 254); needs PS_F_RECORD_HOPS.
 * ps_read_delivered: 1 where `msg` was delivered (seen bit set), any mode,
 *               for messages of the last window of the last run.            */
int ps_read_hops(ps_engine* e, uint32_t msg, uint8_t* hop_per_peer);
int ps_read_delivered(ps_engine* e, uint32_t msg, uint8_t* delivered_per_peer);
/* ps_read_peer_messages: what one subscriber's client.Messages() channel
 *               (client.go:26-28, fed by processMessages client.go:124-128)
 *               yields for `topic` from the last window of the last run: the
 *               delivered message ids in publish order (a tree path is FIFO,
 *               so publish order is arrival order).  *n_out = count; returns
 *               PS_E_RANGE (with *n_out set) when cap is too small. */
int ps_read_peer_messages(ps_engine* e, uint32_t topic, uint32_t peer, uint32_t* msg_out,
                          size_t cap, size_t* n_out);
/* Order-independent digest of the final seen state of the last window:
 * sum over (peer, topic, word < message words) of
 * mix64(mix64(peer << 32 | topic << 16 | word) ^ mix64(seen word)); a
 * multi-GPU engine sums its owned nodes (the ranks' digests add up). */
int ps_seen_digest(ps_engine* e, uint64_t* digest_out);

/* Pipelined windows (ps_run_async) whose leading launches ran beside the
 * previous window's last launches (no reference
 * counterpart: a scheduling diagnostic). */
int ps_overlapped_windows(ps_engine* e, uint64_t* count_out);

/* ---- multi-GPU: one engine (process) per GPU --------------------------------
 * Every rank creates the same topics and memberships and publishes the same
 * messages; each owns a hash partition of every topic's tree nodes and ps_run
 * exchanges, each round, the deliveries addressed to other ranks' nodes
 * (stream-ordered all-to-allv over RCCL / xGMI).  Stats and ps_read_* cover
 * the owned nodes; sums over ranks give the job totals.
 *   PS_PART_PEER     owner(p) = splitmix64(p) mod world (the
 *                    default): every round ships each parent row whose
 *                    children live on other ranks once per such rank
 *   PS_PART_SUBTREE  a node below the split level belongs to the owner of its
 *                    ancestor at that level (the subtrees dealt largest first
 *                    to the least-loaded rank), so only edges out of the top
 *                    levels cross GPUs. */
#define PS_PART_PEER 0u
#define PS_PART_SUBTREE 1u
#define PS_UNIQUE_ID_BYTES 128

typedef struct ps_dist_config {
  int32_t rank;
  int32_t world;        /* <= 16 */
  uint32_t partition;   /* PS_PART_*                                    */
  uint32_t split_depth; /* PS_PART_SUBTREE: split level, 0 = automatic */
  uint32_t flags;       /* PS_DIST_F_*                                  */
  uint32_t reserved;
} ps_dist_config;
/* ps_dist_config.flags: the loopback transport copies every round's ghost
 * records into the receiver's buffer, the data path of the RCCL transport
 * (send parts, receive buffer, exchange stream), instead of reading them in
 * place (tests run the RCCL-shaped path on one GPU with it; RCCL: ignored) */
#define PS_DIST_F_COPY 0x1u
/* ps_dist_config.flags: ghost-fed nodes read their remote parents' rows in
 * the owner's own row set (no packed records, no shipping): the loopback's
 * ranks share one process; ps_dist_init_ipc's map each other's row sets
 * (across the GPUs of a node, xGMI peer reads).  Not with PS_DIST_F_COPY;
 * RCCL: refused. */
#define PS_DIST_F_INPLACE 0x2u

/* GPUs visible to this process (0 without one); a launcher decides from it
 * whether every rank gets a GPU of its own (RCCL) or ranks share (IPC) */
int ps_device_count(int32_t* out);
/* rank 0 creates the RCCL id; the caller ships it to every rank */
int ps_dist_unique_id(uint8_t id_out[PS_UNIQUE_ID_BYTES]);
int ps_dist_init(ps_engine* e, const ps_dist_config* dc, const uint8_t id[PS_UNIQUE_ID_BYTES]);
/* process-shared transport: one process per rank on one node -- their GPUs
 * map each other's memory (hipIpcGetMemHandle / hipIpcOpenMemHandle; several
 * ranks may share one GPU, which RCCL refuses).  Rank 0 calls ps_dist_ipc_id
 * (host only: a fresh POSIX shared-memory name) and the caller ships the id
 * to every rank, as with the RCCL id; ps_dist_init_ipc then meets the other
 * ranks there (host barriers in shared memory, 120 s timeout) and maps their
 * device flag blocks.  Each round is ordered by monotonic device flags in
 * IPC-mapped memory (a one-wave set kernel and a one-wave poll kernel with a
 * 30 s timeout, after which the next call fails with PS_E_DEVICE): no host
 * synchronisation with the GPU.  flags: PS_DIST_F_COPY copies the records
 * into the receive buffer (the RCCL data path), PS_DIST_F_INPLACE reads the
 * ghost parents' rows in their owner's row set, neither reads each sender's
 * records in place.  Replaces the cross-host child write subtree.go:333 and
 * the per-hop read client.go:104 for ranks that share a node. */
int ps_dist_ipc_id(uint8_t id_out[PS_UNIQUE_ID_BYTES]);
int ps_dist_init_ipc(ps_engine* e, const ps_dist_config* dc, const uint8_t id[PS_UNIQUE_ID_BYTES]);
/* in-process transport: `world` engines of one process (one thread each)
 * exchange through device copies -- runs the multi-GPU path on one GPU */
typedef struct ps_loopback ps_loopback;
int ps_loopback_create(int32_t world, ps_loopback** out);
void ps_loopback_destroy(ps_loopback* lb);
int ps_dist_init_loopback(ps_engine* e, const ps_dist_config* dc, ps_loopback* lb);
/* host-only: owner rank of every peer of a tree (parent array, PS_NONE =
 * absent) under a partition; -1 for peers outside the tree */
int ps_partition_owner(uint32_t n_peers, uint32_t root, const uint32_t* parent, uint32_t topic,
                       const ps_dist_config* dc, int32_t* owner_out);

/* ---- wire codec (host only, no engine needed) --------------------------------
 * The reference's stream framing, pubsub.go:122-153: writeMessage is
 * json.NewEncoder(s).Encode(m) and readMessage json.NewDecoder(r).Decode(m)
 * over
 *   type Message struct { Type MessageType; Data []byte `json:"data,omitempty"`;
 *     Peers []string `json:"parents,omitempty"`; TreeWidth, TreeMaxWidth,
 *     NumPeers int `json:"...,omitempty"` }
 * so a Go peer and this engine exchange byte-identical lines. */
#define PS_MSG_DATA 0   /* MessageType, pubsub.go:138-144 */
#define PS_MSG_JOIN 1
#define PS_MSG_PART 2
#define PS_MSG_UPDATE 3
#define PS_MSG_STATE 4

typedef struct ps_message {
  int32_t type;
  const uint8_t* data;      /* Data (base64 on the wire) */
  size_t data_len;
  const char* const* peers; /* Peers: NUL-terminated peer id strings */
  size_t n_peers;
  int64_t tree_width;
  int64_t tree_max_width;
  int64_t num_peers;
} ps_message;

/* decode target: caller-owned buffers; *_len / n_peers are always set, and
 * PS_E_RANGE is returned when data_cap / peers_cap is too small */
typedef struct ps_message_buf {
  int32_t type;
  int32_t reserved;
  uint8_t* data;
  size_t data_cap;
  size_t data_len;
  char* peers;              /* n_peers NUL-terminated strings, back to back */
  size_t peers_cap;
  size_t peers_len;
  size_t n_peers;
  int64_t tree_width;
  int64_t tree_max_width;
  int64_t num_peers;
} ps_message_buf;

/* one JSON line, '\n'-terminated; *len_out = bytes needed (PS_E_RANGE if cap
 * is short, nothing written) */
int ps_msg_encode(const ps_message* m, char* out, size_t cap, size_t* len_out);
/* one JSON value from in[0..len); *consumed = bytes up to the next value
 * (trailing whitespace included); PS_E_INVAL on malformed input */
int ps_msg_decode(const char* in, size_t len, ps_message_buf* out, size_t* consumed);

#ifdef __cplusplus
}
#endif
#endif /* PSENGINE_H */
