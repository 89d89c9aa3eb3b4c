/*
 * psoracle.h -- CPU restatement of go-libp2p-pubsub v0 (the "subtree" pubsub).
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X engine
 * in go-libp2p-pubsub_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path never links or calls it.
 *
 * Pinning: the reference ships no golden vectors or hop-level fixtures
 * (SURVEY.md §8c).  This restatement is pinned against (1) the reference's own
 * test assertions (pubsub_test.go:101-325, restated as deterministic scenarios
 * in tests/golden/scenarios.json) and (2) an independent pure-Python
 * event-driven restatement (oracle/event_sim.py) whose outputs are committed as
 * fixtures under tests/golden/.  Tree SHAPE parity with a live Go run is only
 * distributional (Go map order is random); hop/delivery parity is
 * exact given a tree.
 *
 * Go toolchain and the gx dependencies are absent, so the
 * reference itself cannot be built here; there is no oracle/_ref.
 */
#ifndef PSORACLE_H
#define PSORACLE_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define OR_NONE 0xFFFFFFFFu

/* peer states inside one topic tree */
enum { OR_OUT = 0, OR_IN = 1, OR_DEAD = 2, OR_FAILED = 3, OR_ORPHAN = 4 };

/* error codes (mirror include/psengine.h PS_E_*) */
enum {
  OR_OK = 0,
  OR_E_INVAL = -1,
  OR_E_NOMEM = -2,
  OR_E_STATE = -3,      /* peer in the wrong state for the request          */
  OR_E_NOPARENT = -4,   /* redirectJoin found no live child (subtree.go:172) */
  OR_E_UNREACHABLE = -5 /* join redirected into a failed host               */
};

typedef struct or_tree or_tree;

/* NewTopic (pubsub.go:54-97): tree rooted at `root`, widths from TreeOpts.  */
or_tree* or_tree_new(uint32_t n_peers, uint32_t root, uint32_t tree_width,
                     uint32_t tree_max_width, uint64_t seed);
void or_tree_free(or_tree* t);
/* Subscribe -> joinToPeer -> handleJoin/redirectJoin/joinParents, quiescent
 * (client.go:65-94, subtree.go:100-307). */
int or_tree_join(or_tree* t, uint32_t peer);
/* client.Close -> Part -> redistributeChildren (subtree.go:46-98,356-375). */
int or_tree_leave(or_tree* t, uint32_t peer);
/* host.Close(): abrupt; detected by the parent's next failed write
 * (subtree.go:333-351). */
int or_tree_drop(or_tree* t, uint32_t peer);
/* One message flows through the tree (forwardMessage at every reached node):
 * writes the per-peer hop of THIS message into hop_out (0xFF = not delivered)
 * and then applies the lazy prune of Part'ed children and the repair of
 * children whose write failed (subtree.go:319-354), in BFS order. */
int or_tree_message(or_tree* t, uint8_t* hop_out);
/* Current attached structure: parent[p] for every peer reachable from the
 * root through IN peers, OR_NONE otherwise (printTree, pubsub_test.go:204). */
void or_tree_parents(const or_tree* t, uint32_t* parent_out);
/* Raw parent pointer / state, for debugging and scenario checks. */
uint32_t or_tree_state(const or_tree* t, uint32_t peer);
uint32_t or_tree_n_children(const or_tree* t, uint32_t peer);

/* ---- the hot path: round-synchronous dissemination (SURVEY.md §8 formal
 * semantics), restating subtree.forwardMessage (subtree.go:319-354),
 * client.processMessages (client.go:100-132) and Topic.PublishMessage
 * (pubsub.go:111-120).
 *
 * Graph given as child lists in node space (row_ptr[n+1], col[E]).
 * live[c] != 0 <=> c is subscribed and live.  Message m is injected at the
 * root in round start_round[m] (NULL = all 0).  A delivery of m to c in global
 * round r has hop r - start_round[m].  hop_out[m * n + c] (may be NULL) gets the
 * hop or 0xFF.  hist_out[h] (may be NULL, length hist_len) accumulates
 * deliveries per hop.  Returns total deliveries, or <0 on error.
 * n_threads > 1 splits the messages over OpenMP threads. */
int64_t or_disseminate(uint32_t n, const uint32_t* row_ptr, const uint32_t* col,
                       uint32_t root, const uint8_t* live, uint32_t n_msgs,
                       const uint32_t* start_round, uint8_t* hop_out,
                       uint64_t* hist_out, uint32_t hist_len, int n_threads);

/* The hot path as the GPU engine computes it (bench CPU baseline): messages
 * as bits (64 per u64), rounds level-synchronous, OpenMP over each level's
 * nodes.  Returns total deliveries, or <0 on error. */
int64_t or_levels_bits(uint32_t n, const uint32_t* row_ptr, const uint32_t* col, uint32_t root,
                       const uint8_t* live, uint32_t n_msgs, int n_threads);
/* The same, split like the engine: or_levels_new does the per-topology work
 * (BFS numbering, rows allocated and touched) once; or_levels_run is one pass
 * of a batch of n_msgs messages (what bench.py's cpu_baseline times). */
typedef struct or_levels or_levels;
or_levels* or_levels_new(uint32_t n, const uint32_t* row_ptr, const uint32_t* col, uint32_t root,
                         uint32_t n_msgs);
int64_t or_levels_run(or_levels* plan, const uint8_t* live, int n_threads);
void or_levels_free(or_levels* plan);

/* SplitMix64 (shared definition with the engine and the synthetic workload
 * generator). */
uint64_t or_splitmix64(uint64_t* state);
uint64_t or_mix64(uint64_t x);

#ifdef __cplusplus
}
#endif
#endif
