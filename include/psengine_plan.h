/*
 * psengine_plan.h -- host-only planner probe of libpsengine.so (tests).
 *
 * Not part of the drop-in boundary (include/psengine.h): these entry points
 * build one rank's node space and one window's launch plans on the host --
 * no device is touched -- so the planners (chunk cuts, round pairs, the
 * multi-GPU ghost exchange layout) are unit-tested on a machine without a GPU
 * (tests/test_plan_cpu.py replays the exchange from these tables with gloo
 * and checks the deliveries against the CPU restatement).
 */
#ifndef PSENGINE_PLAN_H
#define PSENGINE_PLAN_H

#include "psengine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A host-only engine of n_topics trees: parents[t * n_peers + p] (PS_NONE =
 * absent), roots[t]; dc (nullable) = this rank and the partition. */
int ps_plan_create(uint32_t n_peers, uint32_t n_topics, const uint32_t* roots, const uint32_t* parents,
                   const ps_dist_config* dc, ps_engine** out);
void ps_plan_destroy(ps_engine* e);
/* ps_config.msg_window of the probe (default 65536; PS_E_INVAL above 2^30) */
int ps_plan_set_msg_window(ps_engine* e, uint32_t msg_window);
/* Plans the first window of a batch (topic and start round per message; a
 * null start_round = all round 0), as ps_run would; flags: PS_F_* */
int ps_plan_window(ps_engine* e, const uint32_t* topic_of_msg, const uint32_t* start_round, size_t n_msgs,
                   uint32_t flags);

/* ps_plan_get(what, index): u64 values into out[0..cap), *n_out = how many
 * there are (PS_E_RANGE if cap is short). */
#define PS_PLAN_INFO 0        /* planned rounds, nodes, pull chunks, pair chunks, world, rank,
                                 send half words, recv words, ghost segments, level mode, ship entries */
#define PS_PLAN_NODES 1       /* per node: peer */
#define PS_PLAN_PARENT 2      /* per node: local parent node (PS_NONE: root or remote) */
#define PS_PLAN_GHOST_REF 3   /* per node: source rank << 27 | record index (PS_NONE: local parent) */
#define PS_PLAN_TOPIC 4       /* index = topic: nbase, n_nodes, depth, root_local, then level_off[0..depth+1],
                                 level_local[0..depth] */
#define PS_PLAN_LAYOUT 5      /* index = topic: W, wbase, flags, group count, then (start, w0, wn) per group */
#define PS_PLAN_ROUND_KIND 6  /* per round 0..planned+1: PS_K_* */
#define PS_PLAN_PULL 7        /* index = round: off, gsplit, end, then per chunk 13 values: node_begin,
                                 node_end, topic, W, row0, e_lo, e_hi, gin, gout, group, p_lo, p_hi,
                                 c_lo (pair launches: PS_NONE = a level-1 run of the second round) */
#define PS_PLAN_PAIR 8        /* index = round: lo, gsplit, hi, then the chunks as PS_PLAN_PULL */
#define PS_PLAN_XCHG 9        /* index = round: any, then per rank s_off, s_len, r_off, r_len (bytes) */
#define PS_PLAN_SEGS 10       /* per segment: topic, rw, rbase[world], sbase[world] */
#define PS_PLAN_SHIP 11       /* per ship entry: node, dst (rank << 27 | record index) */
#define PS_PLAN_PACK 12       /* index = round: per root segment e0, e1, gseg, W, row, unit0 */
#define PS_PLAN_CHAIN 13      /* index = round: rounds of the launch, then per chunk 17 values: node_begin,
                                 node_end, topic, W, row0, w0, S, levels, r0, group, first[0..6] */
int ps_plan_get(ps_engine* e, uint32_t what, uint32_t index, uint64_t* out, size_t cap, size_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* PSENGINE_PLAN_H */
