// api.cpp -- the C ABI of the engine (include/psengine.h) around the node
// space (graph.cpp), the planners (plan.cpp) and the round loop (run.cpp):
// lifecycle, topics and membership, publishes, result readbacks, multi-GPU
// set-up; and the host-only planner probe (include/psengine_plan.h).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "engine.hpp"
#include "psengine_plan.h"

using namespace psamd;

namespace {

TopicHost* join_topic(ps_engine* e, uint32_t topic) {
  if (!topic_ok(e, topic)) {
    e->fail(PS_E_STATE, "no such topic");
    return nullptr;
  }
  TopicHost& T = e->topics[topic];
  if (T.kind != Kind::Join) {
    e->fail(PS_E_STATE, "topic topology was set explicitly");
    return nullptr;
  }
  return &T;
}

int dist_common(ps_engine* e, const ps_dist_config* dc) {
  if (!e || !dc) return PS_E_INVAL;
  if (dc->world < 1 || dc->world > kMaxRanks || dc->rank < 0 || dc->rank >= dc->world)
    return e->fail(PS_E_INVAL, "rank/world out of range (world <= 16)");
  if (dc->partition != PS_PART_PEER && dc->partition != PS_PART_SUBTREE) return e->fail(PS_E_INVAL, "unknown partition");
  if (dc->flags & ~(PS_DIST_F_COPY | PS_DIST_F_INPLACE)) return e->fail(PS_E_INVAL, "unknown dist flag");
  if ((dc->flags & PS_DIST_F_COPY) && (dc->flags & PS_DIST_F_INPLACE))
    return e->fail(PS_E_INVAL, "PS_DIST_F_INPLACE reads rows in place: not with PS_DIST_F_COPY");
  if (!e->pending.empty()) return e->fail(PS_E_STATE, "messages pending");
  // (every check above passed: the mode changes together with rank and world)
  e->inplace = dc->world > 1 && (dc->flags & PS_DIST_F_INPLACE) != 0;
  e->rank = dc->rank;
  e->world = dc->world;
  e->partition = dc->partition;
  e->split_depth = dc->split_depth;
  e->graph_dirty = true;
  return PS_OK;
}

// a transport that failed to come up leaves the engine on one rank
int dist_undo(ps_engine* e, int code, const std::string& why) {
  e->transport.reset();
  e->rank = 0;
  e->world = 1;
  e->inplace = false;
  e->graph_dirty = true;
  return e->fail(code, why);
}

// N ranks: the exchange stream and the round events (the exchange of round q
// runs beside round q's locally fed chunks)
int dist_streams(ps_engine* e) {
  if (e->xstream) return PS_OK;
  HIP_TRY(hipSetDevice(e->cfg.device), "hipSetDevice");
  HIP_TRY(hipStreamCreateWithFlags(&e->xstream, hipStreamNonBlocking), "exchange stream");
  HIP_TRY(hipEventCreateWithFlags(&e->ev_round, kStreamEvent), "round event");
  HIP_TRY(hipEventCreateWithFlags(&e->ev_xchg, kStreamEvent), "exchange event");
  return PS_OK;
}

}  // namespace

namespace {

ps_plan_opts current_opts(const ps_engine* e) {
  ps_plan_opts o{};
  o.flood_top_bytes = e->flood_top_bytes;
  o.overlap_min_bytes = e->overlap_min_bytes;
  o.launch_bytes = static_cast<uint64_t>(e->launch_bytes);
  o.flood = e->flood_on ? 1 : 0;
  o.chain_max = e->chain_max;
  o.chain_max_groups = e->chain_max_groups;
  o.chain_tail = e->chain_tail ? 1 : 0;
  o.chain_words = e->chain_words;
  o.flood_words = e->flood_words;
  o.pad_words = e->pad_words;
  o.overlap = e->overlap_on ? 1 : 0;
  o.overlap_min_rounds = e->overlap_min_rounds;
  o.xchg_overlap = e->xchg_overlap_env;
  o.gpu_build = e->gpu_build_on ? 1 : 0;
  o.flood_spin_ticks = e->flood_spin_ticks;
  o.chain_nt = e->chain_nt ? 1 : 0;
  o.chain_waves = e->chain_waves;
  o.flood_min_rounds = e->flood_min_rounds;
  o.align_groups = e->align_groups ? 1 : 0;
  return o;
}

const char* check_opts(const ps_plan_opts& o) {
  if (o.chain_max < 1 || o.chain_max > kChainLevels || o.chain_max_groups < 1 || o.chain_max_groups > kChainLevels)
    return "chain_max / chain_max_groups out of 1..6";
  if (o.chain_words < 256 || o.chain_words > (1u << 20)) return "chain_words out of 256..2^20";
  if (o.flood_words < 64 || o.flood_words > (1u << 16)) return "flood_words out of 64..65536";
  if (o.pad_words < 2) return "pad_words < 2";
  if (o.overlap_min_rounds < 2) return "overlap_min_rounds < 2";
  if (o.xchg_overlap < -1 || o.xchg_overlap > 1) return "xchg_overlap not -1, 0 or 1";
  if (o.flood > 1 || o.chain_tail > 1 || o.overlap > 1 || o.gpu_build > 1 || o.chain_nt > 1 || o.chain_waves > 16 ||
      o.flood_min_rounds < 1 || o.align_groups > 1)
    return "switch not 0 or 1";
  return nullptr;
}

// the exchange stream of a multi-rank engine: forced by the options, or
// (auto) on whenever the transport copies the records
void refresh_xchg_overlap(ps_engine* e) {
  if (e->transport) e->xchg_overlap = e->xchg_overlap_env < 0 ? !e->transport->zero_copy() : e->xchg_overlap_env != 0;
}

void apply_opts(ps_engine* e, const ps_plan_opts& o) {
  e->flood_top_bytes = o.flood_top_bytes;
  e->overlap_min_bytes = o.overlap_min_bytes;
  e->launch_bytes = static_cast<double>(o.launch_bytes);
  e->flood_on = o.flood != 0;
  e->chain_max = o.chain_max;
  e->chain_max_groups = o.chain_max_groups;
  e->chain_tail = o.chain_tail != 0;
  e->chain_words = o.chain_words;
  e->flood_words = o.flood_words;
  e->pad_words = o.pad_words;
  e->overlap_on = o.overlap != 0;
  e->overlap_min_rounds = o.overlap_min_rounds;
  e->xchg_overlap_env = o.xchg_overlap;
  e->gpu_build_on = o.gpu_build != 0;
  e->flood_spin_ticks = o.flood_spin_ticks;
  e->chain_nt = o.chain_nt != 0;
  e->chain_waves = o.chain_waves;
  e->flood_min_rounds = o.flood_min_rounds;
  e->align_groups = o.align_groups != 0;
  refresh_xchg_overlap(e);
}

}  // namespace

struct ps_loopback {
  psamd::LoopbackGroup* g;
};

namespace {
thread_local std::string g_abi_error;  // ps_abi_check's last mismatch (ps_last_error(NULL))
}  // namespace

extern "C" {

const char* ps_version(void) { return "psengine-mi355x 0.5 (gfx950, abi 5)"; }

uint32_t ps_abi_version(void) { return PS_ABI_VERSION; }

int ps_abi_check(uint32_t abi_version, size_t config_size, size_t stats_size, size_t plan_opts_size,
                 size_t dist_config_size) {
  char buf[256];
  if (abi_version != PS_ABI_VERSION)
    std::snprintf(buf, sizeof buf, "ABI version %u, the library is %u", abi_version, PS_ABI_VERSION);
  else if (config_size != sizeof(ps_config) || stats_size != sizeof(ps_stats) ||
           plan_opts_size != sizeof(ps_plan_opts) || dist_config_size != sizeof(ps_dist_config))
    std::snprintf(buf, sizeof buf,
                  "struct sizes (config %zu, stats %zu, plan_opts %zu, dist_config %zu) differ from the library's "
                  "(%zu, %zu, %zu, %zu)",
                  config_size, stats_size, plan_opts_size, dist_config_size, sizeof(ps_config), sizeof(ps_stats),
                  sizeof(ps_plan_opts), sizeof(ps_dist_config));
  else
    return PS_OK;
  g_abi_error = buf;
  return PS_E_INVAL;
}

// Debug switches read at creation (host phase times, per-wave profiles: they
// change no plan).  The plan options come from ps_set_plan_opts; only A/B
// tools that also set PSAMD_AB=1 may override them from the environment.
static void read_switches(ps_engine* e) {
  if (const char* v = std::getenv("PSAMD_HOST_TIMING")) e->host_timing = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FLOOD_PROFILE")) e->flood_profile = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_CHAIN_PROFILE")) e->chain_prof_path = v;
  const char* ab = std::getenv("PSAMD_AB");
  if (!ab || std::atoi(ab) == 0) return;
  if (const char* v = std::getenv("PSAMD_TWIN")) e->twin_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_NARROW")) e->expand_opts = std::atoi(v) == 0 ? kExpandNoNarrow : 0u;
  if (const char* v = std::getenv("PSAMD_CHAIN_WORDS_LEAD"))
    e->chain_words_lead = static_cast<uint32_t>(std::min(1 << 20, std::max(0, std::atoi(v))));
  ps_plan_opts o = current_opts(e);
  if (const char* v = std::getenv("PSAMD_GPU_BUILD")) o.gpu_build = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FLOOD")) o.flood = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_PULL_PAIR"))  // 0: one k_pull launch per round
    if (std::atoi(v) == 0) o.chain_max = o.chain_max_groups = 1;
  if (const char* v = std::getenv("PSAMD_XCHG_OVERLAP")) o.xchg_overlap = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_CHAIN"))  // rounds per launch at most: 1 (k_pull only), 2 (pairs), 3..6
    o.chain_max = o.chain_max_groups =
        static_cast<uint32_t>(std::max(1, std::min(static_cast<int>(kChainLevels), std::atoi(v))));
  if (const char* v = std::getenv("PSAMD_OVERLAP")) o.overlap = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_OVERLAP_ROUNDS"))
    o.overlap_min_rounds = static_cast<uint32_t>(std::max(2, std::atoi(v)));
  if (const char* v = std::getenv("PSAMD_OVERLAP_BYTES")) o.overlap_min_bytes = std::strtoull(v, nullptr, 10);
  if (const char* v = std::getenv("PSAMD_PAD_WORDS")) o.pad_words = static_cast<uint32_t>(std::max(2, std::atoi(v)));
  if (const char* v = std::getenv("PSAMD_CHAIN_TAIL")) o.chain_tail = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_LAUNCH_BYTES")) o.launch_bytes = static_cast<uint64_t>(std::max(0.0, std::atof(v)));
  if (const char* v = std::getenv("PSAMD_CHAIN_WORDS"))
    o.chain_words = static_cast<uint32_t>(std::min(1 << 20, std::max(256, std::atoi(v))));
  if (const char* v = std::getenv("PSAMD_FLOOD_WORDS"))
    o.flood_words = static_cast<uint32_t>(std::min(1 << 16, std::max(64, std::atoi(v))));
  if (const char* v = std::getenv("PSAMD_FLOOD_SPIN_TICKS")) o.flood_spin_ticks = static_cast<uint32_t>(std::strtoul(v, nullptr, 0));
  if (const char* v = std::getenv("PSAMD_FLOOD_TOP_BYTES")) o.flood_top_bytes = std::strtoull(v, nullptr, 0);
  if (const char* v = std::getenv("PSAMD_UPLOAD_REUSE")) e->upload_reuse = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_SIG_WINDOWS")) e->sig_windows = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FUSE_REDUCE")) e->fuse_reduce = std::atoi(v) != 0;
  if (const char* v = std::getenv("PSAMD_FLOOD_MIN_ROUNDS"))
    o.flood_min_rounds = static_cast<uint32_t>(std::max(1, std::atoi(v)));
  if (const char* v = std::getenv("PSAMD_CHAIN_WAVES"))
    o.chain_waves = static_cast<uint32_t>(std::max(0, std::min(16, std::atoi(v))));
  if (!check_opts(o)) apply_opts(e, o);
}

int ps_plan_opts_default(ps_plan_opts* out) {
  if (!out) return PS_E_INVAL;
  const ps_engine fresh;  // (the member initialisers are the defaults)
  *out = current_opts(&fresh);
  return PS_OK;
}

int ps_get_plan_opts(const ps_engine* e, ps_plan_opts* out) {
  if (!e || !out) return PS_E_INVAL;
  *out = current_opts(e);
  return PS_OK;
}

int ps_set_plan_opts(ps_engine* e, const ps_plan_opts* o) {
  if (!e || !o) return PS_E_INVAL;
  if (const char* why = check_opts(*o)) return e->fail(PS_E_INVAL, why);
  if (e->infl_count) return e->fail(PS_E_STATE, "asynchronous runs pending: ps_wait first");
  const ps_plan_opts old = current_opts(e);
  apply_opts(e, *o);
  // a changed node-space build or row padding re-plans everything; the plan
  // keys cover the rest (chain lengths, words, tail, launch price, k_flood split)
  if (old.gpu_build != o->gpu_build || old.pad_words != o->pad_words) e->graph_dirty = true;
  e->pull.key.clear();
  e->pair.key.clear();
  e->flood.key.clear();
  e->chain_fail_key.clear();
  e->gate_valid = false;
  return PS_OK;
}

int ps_create(const ps_config* cfg, ps_engine** out) {
  if (!cfg || !out) return PS_E_INVAL;
  *out = nullptr;
  if (cfg->n_peers == 0 || cfg->n_topics == 0 || cfg->n_topics > 65535) return PS_E_INVAL;
  if (cfg->msg_window > kMaxWindow) return PS_E_INVAL;  // (rows of at most 2^24 words)
  auto* e = new (std::nothrow) ps_engine();
  if (!e) return PS_E_NOMEM;
  e->cfg = *cfg;
  if (!e->cfg.tree_width) e->cfg.tree_width = 2;          // pubsub.go:16
  if (!e->cfg.tree_max_width) e->cfg.tree_max_width = 5;  // pubsub.go:17
  if (!e->cfg.msg_window) e->cfg.msg_window = kDefaultWindow;
  e->cfg.msg_window = ((e->cfg.msg_window + 63) / 64) * 64;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    delete e;
    return PS_E_DEVICE;
  }
  if (cfg->device < 0 || cfg->device >= ndev || hipSetDevice(cfg->device) != hipSuccess) {
    delete e;
    return PS_E_DEVICE;
  }
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess && cus > 0)
    e->n_cus = static_cast<uint32_t>(cus);
  // resident 256-thread blocks per CU: k_expand needs 80 VGPRs / 106 SGPRs,
  // which admits 6 (MI355X_MICROARCH.md §Residency)
  e->expand_grid = e->n_cus * 6;
  // k_flood's waves must all be resident at once (its tasks wait on earlier
  // tasks): the grid stays within the occupancy the runtime reports, capped
  // at kFloodBlocksPerCu for margin (MI355X_MICROARCH.md §Residency)
  {
    int bpc = 0;
    if (flood_blocks_per_cu(&bpc) == hipSuccess && bpc > 0)
      e->flood_grid = e->n_cus * std::min<uint32_t>(static_cast<uint32_t>(bpc), kFloodBlocksPerCu);
  }
  read_switches(e);
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_run0, kStartEvent) != hipSuccess || hipEventCreate(&e->ev_run1) != hipSuccess) {
    delete e;
    return PS_E_DEVICE;
  }
  for (auto& f : e->infl) {
    void* h = nullptr;
    if (hipEventCreateWithFlags(&f.ev0, kStartEvent) != hipSuccess || hipEventCreate(&f.ev1) != hipSuccess ||
        hipHostMalloc(&h, 2 * (PS_MAX_ROUNDS + 1) * kNumCtr * 8 + 64, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess) {
      ps_destroy(e);
      return PS_E_DEVICE;
    }
    f.hs = static_cast<uint64_t*>(h);
    void* hd = nullptr;
    if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) {
      ps_destroy(e);
      return PS_E_DEVICE;
    }
    f.hs_dev = static_cast<uint64_t*>(hd);
    f.ha = f.hs + (PS_MAX_ROUNDS + 1) * kNumCtr;
    f.sig = f.hs + 2 * (PS_MAX_ROUNDS + 1) * kNumCtr;
    f.sig_dev = f.hs_dev + 2 * (PS_MAX_ROUNDS + 1) * kNumCtr;
    f.sig[0] = 0;
  }
  e->topics.resize(cfg->n_topics);
  e->live.assign(cfg->n_peers, 1);
  if (e->d_digest.ensure(8) != hipSuccess) {
    ps_destroy(e);
    return PS_E_NOMEM;
  }
  *out = e;
  return PS_OK;
}

void ps_destroy(ps_engine* e) {
  if (!e) return;
  if (e->host_only) {
    delete e;
    return;
  }
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->xstream) (void)hipStreamSynchronize(e->xstream);
  if (e->pstream) (void)hipStreamSynchronize(e->pstream);
  if (e->rstream) (void)hipStreamSynchronize(e->rstream);
  if (e->qstream) (void)hipStreamSynchronize(e->qstream);
  if (e->tstream) (void)hipStreamSynchronize(e->tstream);
  for (auto ev : e->ev_k) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : {e->ev_run0, e->ev_run1, e->ev_round, e->ev_xchg, e->ev_gate[0], e->ev_gate[1], e->ev_pre, e->ev_end,
                      e->ev_tend, e->ev_e2t})
    if (ev) (void)hipEventDestroy(ev);
  for (auto& f : e->infl) {
    if (f.ev0) (void)hipEventDestroy(f.ev0);
    if (f.ev1) (void)hipEventDestroy(f.ev1);
    if (f.hs) (void)hipHostFree(f.hs);
  }
  for (auto& g : e->stg)
    if (g.h) (void)hipHostFree(g.h);
  if (e->pairs_pinned) (void)hipHostFree(e->pairs_pinned);
  e->transport.reset();  // (a communicator before its streams)
  if (e->xstream) (void)hipStreamDestroy(e->xstream);
  if (e->pstream) (void)hipStreamDestroy(e->pstream);
  if (e->rstream) (void)hipStreamDestroy(e->rstream);
  if (e->qstream) (void)hipStreamDestroy(e->qstream);
  if (e->tstream) (void)hipStreamDestroy(e->tstream);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

const char* ps_last_error(const ps_engine* e) {
  return e ? e->err.c_str() : g_abi_error.empty() ? "null engine" : g_abi_error.c_str();
}

int ps_topic_create(ps_engine* e, uint32_t topic, uint32_t root, uint32_t w, uint32_t mw) {
  if (!e) return PS_E_INVAL;
  if (topic >= e->topics.size()) return e->fail(PS_E_RANGE, "topic id out of range");
  if (root >= e->cfg.n_peers) return e->fail(PS_E_INVAL, "root out of range");
  if (e->topics[topic].exists) return e->fail(PS_E_STATE, "topic exists");
  TopicHost& T = e->topics[topic];
  T = TopicHost{};
  T.exists = true;
  T.kind = Kind::Join;
  T.root = root;
  T.width = w ? w : e->cfg.tree_width;  // TreeOpts (pubsub.go:66-72)
  T.max_width = mw ? mw : e->cfg.tree_max_width;
  T.tree = SubscriptionTree(e->cfg.n_peers, root, T.width, T.max_width, e->cfg.seed ^ (0xA5A5A5A5ull * (topic + 1)));
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_close(ps_engine* e, uint32_t topic) {
  if (!e) return PS_E_INVAL;
  if (!topic_ok(e, topic)) return e->fail(PS_E_STATE, "no such topic");
  for (const auto& m : e->pending)
    if (m.topic == topic) return e->fail(PS_E_STATE, "topic has unsent messages");
  e->topics[topic] = TopicHost{};
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_join(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n, int32_t* status_out) {
  if (!e || (n && !peers)) return PS_E_INVAL;
  TopicHost* T = join_topic(e, topic);
  if (!T) return PS_E_STATE;
  int first = PS_OK;
  // a joiner's own line is written when it attaches, at the end of a walk
  // of ~17 dependent hops: fetched a few joins ahead (tools/probe/tree_bench)
  constexpr size_t kAhead = 8;
  for (size_t i = 0; i < std::min(n, kAhead); ++i) T->tree.prefetch_join(peers[i]);
  for (size_t i = 0; i < n; ++i) {
    if (i + kAhead < n) T->tree.prefetch_join(peers[i + kAhead]);
    int rc = T->tree.subscribe(peers[i]);
    if (status_out) status_out[i] = rc;
    if (rc && !first) {
      first = rc;
      e->err = "join of peer " + std::to_string(peers[i]) + " failed";
    }
  }
  e->graph_dirty = true;
  return first;
}

int ps_topic_leave(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n) {
  if (!e || (n && !peers)) return PS_E_INVAL;
  TopicHost* T = join_topic(e, topic);
  if (!T) return PS_E_STATE;
  int first = PS_OK;
  // leaving peers are scattered over the tree: their entries are fetched a
  // few peers ahead (two stages: the peer, then the lists it points to)
  constexpr size_t kAhead0 = 16, kAhead1 = 8;
  for (size_t i = 0; i < std::min(n, kAhead0); ++i) T->tree.prefetch_leave(peers[i], 0);
  for (size_t i = 0; i < std::min(n, kAhead1); ++i) T->tree.prefetch_leave(peers[i], 1);
  for (size_t i = 0; i < n; ++i) {
    if (i + kAhead0 < n) T->tree.prefetch_leave(peers[i + kAhead0], 0);
    if (i + kAhead1 < n) T->tree.prefetch_leave(peers[i + kAhead1], 1);
    int rc = T->tree.close_client(peers[i]);
    if (rc && !first) first = rc;
  }
  e->graph_dirty = true;
  return first;
}

int ps_topic_drop(ps_engine* e, uint32_t topic, const uint32_t* peers, size_t n) {
  if (!e || (n && !peers)) return PS_E_INVAL;
  TopicHost* T = join_topic(e, topic);
  if (!T) return PS_E_STATE;
  int first = PS_OK;
  for (size_t i = 0; i < n; ++i) {
    int rc = T->tree.close_host(peers[i]);
    if (rc && !first) first = rc;
  }
  e->graph_dirty = true;
  return first;
}

int ps_topic_set_tree(ps_engine* e, uint32_t topic, uint32_t root, const uint32_t* parent) {
  if (!e || !parent) return PS_E_INVAL;
  if (topic >= e->topics.size()) return e->fail(PS_E_RANGE, "topic id out of range");
  if (root >= e->cfg.n_peers) return e->fail(PS_E_INVAL, "root out of range");
  for (uint32_t c = 0; c < e->cfg.n_peers; ++c)
    if (parent[c] != PS_NONE && parent[c] >= e->cfg.n_peers) return e->fail(PS_E_INVAL, "parent id out of range");
  TopicHost& T = e->topics[topic];
  T = TopicHost{};
  T.exists = true;
  T.kind = Kind::Parent;
  T.root = root;
  T.parent.assign(parent, parent + e->cfg.n_peers);
  T.par_full_dirty = true;
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_set_children(ps_engine* e, uint32_t topic, uint32_t root, const uint32_t* row_ptr, const uint32_t* col) {
  if (!e || !row_ptr) return PS_E_INVAL;
  if (topic >= e->topics.size()) return e->fail(PS_E_RANGE, "topic id out of range");
  const uint32_t n = e->cfg.n_peers;
  if (root >= n) return e->fail(PS_E_INVAL, "root out of range");
  if (row_ptr[0] != 0) return e->fail(PS_E_INVAL, "row_ptr[0] != 0");
  for (uint32_t i = 0; i < n; ++i)
    if (row_ptr[i + 1] < row_ptr[i]) return e->fail(PS_E_INVAL, "row_ptr not monotone");
  if (row_ptr[n] && !col) return e->fail(PS_E_INVAL, "null col");
  for (uint32_t k = 0; k < row_ptr[n]; ++k)
    if (col[k] >= n) return e->fail(PS_E_INVAL, "child id out of range");
  TopicHost& T = e->topics[topic];
  T = TopicHost{};
  T.exists = true;
  T.kind = Kind::Children;
  T.root = root;
  T.rp.assign(row_ptr, row_ptr + n + 1);
  T.cl.assign(col, col + row_ptr[n]);
  e->graph_dirty = true;
  return PS_OK;
}

int ps_topic_get_parents(ps_engine* e, uint32_t topic, uint32_t* parent_out) {
  if (!e || !parent_out) return PS_E_INVAL;
  if (!topic_ok(e, topic)) return e->fail(PS_E_STATE, "no such topic");
  const TopicHost& T = e->topics[topic];
  std::vector<uint32_t> par;
  if (T.kind == Kind::Join) {
    T.tree.attached_parents(par);
  } else {
    // BFS tree of the given topology (first parent in BFS order)
    std::vector<uint32_t> rp, cl;
    peer_children(e, T, rp, cl);
    par.assign(e->cfg.n_peers, kNone);
    std::vector<uint8_t> vis(e->cfg.n_peers, 0);
    std::vector<uint32_t> q{T.root};
    vis[T.root] = 1;
    for (size_t i = 0; i < q.size(); ++i)
      for (uint32_t k = rp[q[i]]; k < rp[q[i] + 1]; ++k)
        if (!vis[cl[k]]) {
          vis[cl[k]] = 1;
          par[cl[k]] = q[i];
          q.push_back(cl[k]);
        }
  }
  std::copy(par.begin(), par.end(), parent_out);
  return PS_OK;
}

int ps_topic_depth(ps_engine* e, uint32_t topic, uint32_t* depth_out, uint32_t* n_nodes_out) {
  if (!e) return PS_E_INVAL;
  if (!topic_ok(e, topic)) return e->fail(PS_E_STATE, "no such topic");
  int rc = upload_graph(e);
  if (rc) return rc;
  if (depth_out) *depth_out = e->topics[topic].depth;
  if (n_nodes_out) *n_nodes_out = e->topics[topic].n_nodes;
  return PS_OK;
}

int ps_set_flags(ps_engine* e, uint32_t flags) {
  if (!e) return PS_E_INVAL;
  if (flags & ~(PS_F_RECORD_HOPS | PS_F_TIME_KERNELS | PS_F_NO_LAZY_SEEN | PS_F_COMPACT))
    return e->fail(PS_E_INVAL, "unknown flag");
  e->cfg.flags = flags;
  return PS_OK;
}

int ps_set_live(ps_engine* e, const uint8_t* live) {
  if (!e || !live) return PS_E_INVAL;
  for (uint32_t p = 0; p < e->cfg.n_peers; ++p) e->live[p] = live[p] ? 1 : 0;
  e->flags_dirty = true;
  e->live_dev_valid = false;
  return PS_OK;
}

int ps_publish_at(ps_engine* e, const uint32_t* topic_of_msg, const uint32_t* start_round, size_t n,
                  uint32_t* first) {
  if (!e || (n && !topic_of_msg)) return PS_E_INVAL;
  if (static_cast<uint64_t>(e->next_msg) + n >= 0xFFFFFFF0ull) return e->fail(PS_E_RANGE, "message id space exhausted");
  // one pass: validate and append (a failure takes the batch back out); a
  // topic is looked up only where it changes along the batch
  const size_t old = e->pending.size();
  e->pending.resize(old + n);
  RunMsg* out = e->pending.data() + old;
  const uint32_t t0 = old ? e->pending_topic0 : (n ? topic_of_msg[0] : 0u);
  bool mixed = old ? e->pending_mixed : false, nonzero = false;
  uint32_t last = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t t = topic_of_msg[i];
    if (t != last) {
      if (!topic_ok(e, t)) {
        e->pending.resize(old);
        return e->fail(PS_E_STATE, "publish to a closed topic");
      }
      last = t;
      mixed |= t != t0;
    }
    const uint32_t s0 = start_round ? start_round[i] : 0u;
    if (s0 > kMaxStartRound) {
      e->pending.resize(old);
      return e->fail(PS_E_RANGE, "start round too large");
    }
    nonzero |= s0 != 0;
    out[i] = RunMsg(t, s0);
  }
  e->pending_topic0 = t0;
  e->pending_mixed = mixed;
  e->pending_nonzero_start |= nonzero;
  if (first) *first = e->next_msg;
  e->next_msg += static_cast<uint32_t>(n);
  return PS_OK;
}

int ps_publish(ps_engine* e, const uint32_t* topic_of_msg, size_t n, uint32_t* first) {
  return ps_publish_at(e, topic_of_msg, nullptr, n, first);
}

int ps_read_hops(ps_engine* e, uint32_t msg, uint8_t* hop_per_peer) {
  if (!e || !hop_per_peer) return PS_E_INVAL;
  if (!e->have_hops) return e->fail(PS_E_NOTREADY, "no hop record (PS_F_RECORD_HOPS)");
  if (msg < e->last_first || msg >= e->last_first + e->last_n) return e->fail(PS_E_RANGE, "message not in the last run");
  const uint32_t np = e->cfg.n_peers;
  std::memcpy(hop_per_peer, e->hops.data() + static_cast<size_t>(msg - e->last_first) * np, np);
  return PS_OK;
}

int ps_read_delivered(ps_engine* e, uint32_t msg, uint8_t* out) {
  if (!e || !out) return PS_E_INVAL;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  if (const int rj = twin_join(e)) return rj;  // (the last window may have run on tstream)
  if (msg < e->last_first || msg >= e->last_first + e->last_n) return e->fail(PS_E_RANGE, "message not in the last run");
  const uint32_t i = msg - e->last_first;
  const uint32_t t = e->last_msgs[i].topic;
  const uint32_t rank = e->run_rank[i];
  if (rank < e->last_lo[t] || rank >= e->last_lo[t] + e->last_cnt[t])
    return e->fail(PS_E_NOTREADY, "message not in the last window");
  const uint32_t li = rank - e->last_lo[t];
  const uint32_t b = t < e->last_pos.size() && !e->last_pos[t].empty() ? e->last_pos[t][li] : li;
  const TopicDev& d = e->last_topics[t];
  {
    int rcm = ensure_mirrors(e);
    if (rcm) return rcm;
  }
  std::memset(out, 0, e->cfg.n_peers);
  std::vector<uint64_t> col(d.n_nodes);
  // one word per node: strided copy of this message's word column (row
  // stride W, or its group's block width when group-major)
  static const std::vector<StartGroup> kNoGroups;
  const auto& G = t < e->last_groups.size() ? e->last_groups[t] : kNoGroups;
  uint64_t stride = d.W;
  if (d.flags & kTopicGroups)
    for (const StartGroup& g : G)
      if ((b >> 6) < g.w0 + g.wn) {
        stride = g.wn;
        break;
      }
  if (d.n_nodes)
    HIP_TRY(hipMemcpy2DAsync(col.data(), 8, e->d_seen.as<uint64_t>() + phys_word(d, G, 0, b >> 6), stride * 8ull, 8,
                             d.n_nodes, hipMemcpyDeviceToHost, e->stream),
            "read seen");
  std::vector<uint8_t> gen(d.n_nodes);
  if (d.n_nodes)
    HIP_TRY(hipMemcpyAsync(gen.data(), e->d_gen.as<uint8_t>() + d.nbase, d.n_nodes, hipMemcpyDeviceToHost, e->stream),
            "read generations");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  const bool mesh = (d.flags & kTopicMesh) != 0;
  const uint64_t bit = 1ull << (b & 63);
  // the root (node 0 of the topic on the rank that owns it) is not a
  // recipient; on another rank node 0 is an ordinary node
  const uint32_t u0 = (d.flags & kTopicRootLocal) ? 1 : 0;
  for (uint32_t u = u0; u < d.n_nodes; ++u)
    if ((mesh || gen[u] == e->gen_cur) && (col[u] & bit)) out[e->node_peer[d.nbase + u]] = 1;
  return PS_OK;
}

int ps_read_peer_messages(ps_engine* e, uint32_t topic, uint32_t peer, uint32_t* msg_out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !msg_out)) return PS_E_INVAL;
  *n_out = 0;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  if (const int rj = twin_join(e)) return rj;
  if (topic >= e->topics.size() || peer >= e->cfg.n_peers) return e->fail(PS_E_RANGE, "topic or peer out of range");
  const TopicDev& d = e->last_topics[topic];
  if (!d.W || !e->last_cnt[topic]) return PS_OK;
  {
    int rcm = ensure_mirrors(e);
    if (rcm) return rcm;
  }
  // the peer's node in this topic (the root is the publisher, not a recipient):
  // a peer -> node map per topic, built once per node space
  auto& pm = e->peer_node[topic];
  if (e->peer_node_epoch.size() != e->topics.size()) e->peer_node_epoch.assign(e->topics.size(), ~0ull);
  if (e->peer_node_epoch[topic] != e->graph_epoch) {
    pm.assign(e->cfg.n_peers, kNone);
    const uint32_t u0 = (d.flags & kTopicRootLocal) ? 1 : 0;
    for (uint32_t k = u0; k < d.n_nodes; ++k) pm[e->node_peer[d.nbase + k]] = k;
    e->peer_node_epoch[topic] = e->graph_epoch;
  }
  const uint32_t u = pm[peer];
  if (u == kNone) return PS_OK;  // not subscribed (or not owned by this rank)
  std::vector<uint64_t> row(d.W);
  uint8_t g = 0;
  if (d.flags & kTopicGroups) {  // the row's blocks, one per start group
    for (const StartGroup& sg : e->last_groups[topic])
      HIP_TRY(hipMemcpyAsync(row.data() + sg.w0, e->d_seen.as<uint64_t>() + phys_word(d, e->last_groups[topic], u, sg.w0),
                             sg.wn * 8ull, hipMemcpyDeviceToHost, e->stream),
              "read seen row");
  } else {
    HIP_TRY(hipMemcpyAsync(row.data(), e->d_seen.as<uint64_t>() + d.wbase + static_cast<uint64_t>(u) * d.W, d.W * 8ull,
                           hipMemcpyDeviceToHost, e->stream),
            "read seen row");
  }
  HIP_TRY(hipMemcpyAsync(&g, e->d_gen.as<uint8_t>() + d.nbase + u, 1, hipMemcpyDeviceToHost, e->stream),
          "read generation");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  if (!(d.flags & kTopicMesh) && g != e->gen_cur) return PS_OK;  // stale row: saw nothing
  // window slot li -> message: the window holds the topic's ranks
  // [last_lo, last_lo + last_cnt)
  const uint32_t lo = e->last_lo[topic], cnt = e->last_cnt[topic];
  std::vector<std::pair<uint64_t, uint32_t>> got;  // (start round << 32 | id, id)
  for (uint32_t i = 0; i < e->last_n; ++i) {
    if (e->last_msgs[i].topic != topic) continue;
    const uint32_t r = e->run_rank[i];
    if (r < lo || r >= lo + cnt) continue;
    const uint32_t li = r - lo;
    const uint32_t b = topic < e->last_pos.size() && !e->last_pos[topic].empty() ? e->last_pos[topic][li] : li;
    if (row[b >> 6] >> (b & 63) & 1ull)
      got.emplace_back((static_cast<uint64_t>(e->last_msgs[i].start) << 32) | i, e->last_first + i);
  }
  // arrival order: paced messages by entry round, then publish order
  std::sort(got.begin(), got.end());
  *n_out = got.size();
  if (got.size() > cap) return e->fail(PS_E_RANGE, "output buffer too small");
  for (size_t k = 0; k < got.size(); ++k) msg_out[k] = got[k].second;
  return PS_OK;
}

int ps_overlapped_windows(ps_engine* e, uint64_t* count_out) {
  if (!e || !count_out) return PS_E_INVAL;
  *count_out = e->overlapped;
  return PS_OK;
}

int ps_seen_digest(ps_engine* e, uint64_t* digest_out) {
  if (!e || !digest_out) return PS_E_INVAL;
  if (!e->have_window) return e->fail(PS_E_NOTREADY, "no completed run");
  if (const int rj = twin_join(e)) return rj;
  HIP_TRY(hipMemsetAsync(e->d_digest.p, 0, 8, e->stream), "clear digest");
  HIP_TRY(launch_digest(e->d_seen.as<uint64_t>(), e->d_gen.as<uint8_t>(), e->gen_cur, e->d_node_peer.as<uint32_t>(),
                        e->d_node_topic.as<uint16_t>(),
                        (e->last_slot ? e->d_topics1 : e->d_topics).as<TopicDev>(),
                        (e->last_slot ? e->d_groups1 : e->d_groups).as<GroupDev>(),
                        e->n_nodes, e->d_digest.as<uint64_t>(), e->stream),
          "digest");
  HIP_TRY(hipMemcpyAsync(digest_out, e->d_digest.p, 8, hipMemcpyDeviceToHost, e->stream), "read digest");
  HIP_TRY(hipStreamSynchronize(e->stream), "sync");
  return PS_OK;
}

int ps_dist_unique_id(uint8_t id_out[PS_UNIQUE_ID_BYTES]) {
  if (!id_out) return PS_E_INVAL;
  return rccl_unique_id(id_out) == 0 ? PS_OK : PS_E_DEVICE;
}

int ps_dist_init(ps_engine* e, const ps_dist_config* dc, const uint8_t id[PS_UNIQUE_ID_BYTES]) {
  if (!e || !dc || !id) return PS_E_INVAL;
  if (dc->flags & PS_DIST_F_INPLACE)  // (RCCL moves records; mapped row sets are ps_dist_init_ipc's)
    return e->fail(PS_E_INVAL, "PS_DIST_F_INPLACE needs mapped row sets: ps_dist_init_ipc or the loopback");
  int rc = dist_common(e, dc);
  if (rc) return rc;
  if (dc->world == 1) return PS_OK;
  if ((rc = dist_streams(e))) return rc;
  std::string err;
  e->transport = make_rccl_transport(dc->rank, dc->world, id, &err);
  if (!e->transport) return dist_undo(e, PS_E_DEVICE, err);
  refresh_xchg_overlap(e);
  return PS_OK;
}

int ps_device_count(int32_t* out) {
  if (!out) return PS_E_INVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return PS_OK;
}

int ps_dist_ipc_id(uint8_t id_out[PS_UNIQUE_ID_BYTES]) {
  if (!id_out) return PS_E_INVAL;
  return ipc_group_id(id_out) == 0 ? PS_OK : PS_E_DEVICE;
}

int ps_dist_init_ipc(ps_engine* e, const ps_dist_config* dc, const uint8_t id[PS_UNIQUE_ID_BYTES]) {
  if (!e || !dc || !id) return PS_E_INVAL;
  int rc = dist_common(e, dc);
  if (rc) return rc;
  if (dc->world == 1) return PS_OK;
  if ((rc = dist_streams(e))) return rc;
  std::string err;
  e->transport = make_ipc_transport(dc->rank, dc->world, e->cfg.device, id, e->cfg.n_topics,
                                    (dc->flags & PS_DIST_F_COPY) != 0, (dc->flags & PS_DIST_F_INPLACE) != 0, &err);
  if (!e->transport) return dist_undo(e, PS_E_DEVICE, err);
  refresh_xchg_overlap(e);
  return PS_OK;
}

int ps_loopback_create(int32_t world, ps_loopback** out) {
  if (!out || world < 1 || world > kMaxRanks) return PS_E_INVAL;
  auto* lb = new (std::nothrow) ps_loopback{loopback_create(world)};
  if (!lb || !lb->g) {
    delete lb;
    return PS_E_NOMEM;
  }
  *out = lb;
  return PS_OK;
}

void ps_loopback_destroy(ps_loopback* lb) {
  if (!lb) return;
  loopback_destroy(lb->g);
  delete lb;
}

int ps_dist_init_loopback(ps_engine* e, const ps_dist_config* dc, ps_loopback* lb) {
  if (!e || !dc || !lb) return PS_E_INVAL;
  int rc = dist_common(e, dc);
  if (rc) return rc;
  if (dc->world == 1) return PS_OK;
  if ((rc = dist_streams(e))) return rc;
  e->transport = make_loopback_transport(lb->g, dc->rank, e->cfg.device, (dc->flags & PS_DIST_F_COPY) != 0,
                                         (dc->flags & PS_DIST_F_INPLACE) != 0);
  if (!e->transport) return dist_undo(e, PS_E_INVAL, "loopback group size != world");
  refresh_xchg_overlap(e);
  return PS_OK;
}

int ps_partition_owner(uint32_t n_peers, uint32_t root, const uint32_t* parent, uint32_t topic,
                       const ps_dist_config* dc, int32_t* owner_out) {
  if (!parent || !dc || !owner_out || root >= n_peers) return PS_E_INVAL;
  if (dc->world < 1 || dc->world > kMaxRanks) return PS_E_INVAL;
  (void)topic;
  // children lists, then the same BFS the engine uses
  std::vector<uint32_t> rp(n_peers + 1, 0), cl;
  for (uint32_t c = 0; c < n_peers; ++c)
    if (parent[c] != PS_NONE && c != root) {
      if (parent[c] >= n_peers) return PS_E_INVAL;
      rp[parent[c] + 1]++;
    }
  for (uint32_t i = 0; i < n_peers; ++i) rp[i + 1] += rp[i];
  cl.assign(rp[n_peers], 0);
  {
    std::vector<uint32_t> fill(rp.begin(), rp.end() - 1);
    for (uint32_t c = 0; c < n_peers; ++c)
      if (parent[c] != PS_NONE && c != root) cl[fill[parent[c]]++] = c;
  }
  std::vector<uint32_t> order{root}, bfs_parent{kNone}, level{0}, local(n_peers, kNone);
  local[root] = 0;
  for (size_t qi = 0; qi < order.size(); ++qi)
    for (uint32_t k = rp[order[qi]]; k < rp[order[qi] + 1]; ++k)
      if (local[cl[k]] == kNone) {
        local[cl[k]] = static_cast<uint32_t>(order.size());
        order.push_back(cl[k]);
        bfs_parent.push_back(static_cast<uint32_t>(qi));
        level.push_back(level[qi] + 1);
      }
  std::vector<int32_t> owner;
  partition_topic(order, bfs_parent, level, dc->world, dc->partition, dc->split_depth, owner);
  for (uint32_t p = 0; p < n_peers; ++p) owner_out[p] = -1;
  for (size_t u = 0; u < order.size(); ++u) owner_out[order[u]] = owner[u];
  return PS_OK;
}

// ---- planner probe (include/psengine_plan.h): host only ----------------------

int ps_plan_create(uint32_t n_peers, uint32_t n_topics, const uint32_t* roots, const uint32_t* parents,
                   const ps_dist_config* dc, ps_engine** out) {
  if (!out || !roots || !parents || n_peers == 0 || n_topics == 0 || n_topics > 65535) return PS_E_INVAL;
  *out = nullptr;
  auto* e = new (std::nothrow) ps_engine();
  if (!e) return PS_E_NOMEM;
  e->host_only = true;
  e->cfg.n_peers = n_peers;
  e->cfg.n_topics = n_topics;
  e->cfg.msg_window = kDefaultWindow;
  e->topics.resize(n_topics);
  e->live.assign(n_peers, 1);
  read_switches(e);
  e->gpu_build_on = false;
  for (uint32_t t = 0; t < n_topics; ++t) {
    int rc = ps_topic_set_tree(e, t, roots[t], parents + static_cast<size_t>(t) * n_peers);
    if (rc) {
      delete e;
      return rc;
    }
  }
  if (dc) {
    int rc = dist_common(e, dc);
    if (rc) {
      delete e;
      return rc;
    }
  }
  int rc = build_graph(e);
  if (rc) {
    delete e;
    return rc;
  }
  build_flags(e);
  e->graph_dirty = e->flags_dirty = false;
  ++e->graph_epoch;
  ++e->flags_epoch;
  *out = e;
  return PS_OK;
}

void ps_plan_destroy(ps_engine* e) {
  if (e && e->host_only) delete e;
}

int ps_plan_set_msg_window(ps_engine* e, uint32_t msg_window) {
  if (!e || !e->host_only || msg_window == 0 || msg_window > kMaxWindow) return PS_E_INVAL;
  e->cfg.msg_window = ((msg_window + 63) / 64) * 64;
  return PS_OK;
}

int ps_plan_window(ps_engine* e, const uint32_t* topic_of_msg, const uint32_t* start_round, size_t n_msgs,
                   uint32_t flags) {
  if (!e || !e->host_only || (n_msgs && !topic_of_msg)) return PS_E_INVAL;
  e->cfg.flags = flags;
  e->pending.clear();
  e->pending_nonzero_start = false;
  int rc = ps_publish_at(e, topic_of_msg, start_round, n_msgs, nullptr);
  if (rc) return rc;
  std::vector<RunMsg> msgs;
  msgs.swap(e->pending);
  e->run_zero_start = !e->pending_nonzero_start;
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  std::vector<uint32_t> off(nt + 1, 0), sorted(msgs.size());
  for (const RunMsg& m : msgs) off[m.topic + 1]++;
  for (uint32_t t = 0; t < nt; ++t) off[t + 1] += off[t];
  {
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint32_t i = 0; i < msgs.size(); ++i) sorted[fill[msgs[i].topic]++] = i;
  }
  std::vector<WinSlice> win(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    win[t].idx = sorted.data() + off[t];
    win[t].n = std::min(off[t + 1] - off[t], e->cfg.msg_window);
  }
  WindowLayout& L = e->probe;
  rc = plan_window_layout(e, msgs, win, L);
  if (rc) return rc;
  e->round_kind.clear();
  if (!L.level) return PS_OK;
  plan_pull_chunks(e, L);
  bool gch = false;
  rc = plan_ghost(e, L, &gch);
  if (rc) return rc;
  // the k_flood split a one-rank run would take (its rounds replay as pulls)
  const uint32_t first = e->world == 1 && e->flood_on && !deep_window(e, L) ? plan_flood_rounds(e, L) : 0;
  plan_pair_chunks(e, L, first);
  if (e->world > 1) annotate_chunks(e, L);
  e->round_kind = e->pair.kind;
  return PS_OK;
}

int ps_plan_get(ps_engine* e, uint32_t what, uint32_t index, uint64_t* out, size_t cap, size_t* n_out) {
  if (!e || !e->host_only || !n_out || (cap && !out)) return PS_E_INVAL;
  std::vector<uint64_t> v;
  const WindowLayout* L = e->probe.tab.empty() ? nullptr : &e->probe;
  auto chunk = [&](const PullChunk& c) {
    for (uint64_t x : {static_cast<uint64_t>(c.node_begin), static_cast<uint64_t>(c.node_end),
                       static_cast<uint64_t>(c.topic), static_cast<uint64_t>(c.W),
                       static_cast<uint64_t>(c.row0_hi) << 32 | c.row0_lo, static_cast<uint64_t>(c.e_lo),
                       static_cast<uint64_t>(c.e_hi), static_cast<uint64_t>(c.gin), static_cast<uint64_t>(c.gout),
                       static_cast<uint64_t>(c.group), static_cast<uint64_t>(c.p_lo), static_cast<uint64_t>(c.p_hi),
                       static_cast<uint64_t>(c.c_lo)})
      v.push_back(x);
  };
  switch (what) {
    case PS_PLAN_INFO:
      v = {L ? L->planned0 : 0u, e->n_nodes, e->pull.chunks.size(), e->pair.chunks.size(),
           static_cast<uint64_t>(e->world), static_cast<uint64_t>(e->rank), e->ghost.send_half, e->ghost.recv_words,
           e->ghost.segs.size(), L && L->level ? 1u : 0u, e->ship_host.size(), L && L->aligned ? 1u : 0u};
      break;
    case PS_PLAN_NODES:
      v.assign(e->node_peer.begin(), e->node_peer.end());
      break;
    case PS_PLAN_PARENT:
      v.assign(e->node_parent.begin(), e->node_parent.end());
      break;
    case PS_PLAN_GHOST_REF:
      v.assign(e->n_nodes, kNone);
      for (size_t i = 0; i < e->ghost_ref.size(); ++i) v[i] = e->ghost_ref[i];
      break;
    case PS_PLAN_TOPIC: {
      if (index >= e->topics.size()) return e->fail(PS_E_RANGE, "topic");
      const TopicHost& T = e->topics[index];
      v = {T.nbase, T.n_nodes, T.depth, T.root_local ? 1u : 0u};
      v.insert(v.end(), T.level_off.begin(), T.level_off.end());
      v.insert(v.end(), T.level_local.begin(), T.level_local.end());
      break;
    }
    case PS_PLAN_LAYOUT: {
      if (!L || index >= e->topics.size()) return e->fail(PS_E_RANGE, "topic");
      const TopicDev& d = L->tab[index];
      v = {d.W, d.wbase, d.flags, L->groups[index].size()};
      for (const StartGroup& g : L->groups[index]) v.insert(v.end(), {g.start, g.w0, g.wn});
      // level-aligned: the start groups over the packed row (start, first bit, messages)
      const auto& AG = L->split.groups;
      const size_t na = L->aligned && index < AG.size() ? AG[index].size() : 0;
      v.push_back(na);
      for (size_t i = 0; i < na; ++i) v.insert(v.end(), {AG[index][i].start, AG[index][i].b0, AG[index][i].n});
      break;
    }
    case PS_PLAN_ROUND_KIND:
      v.assign(e->round_kind.begin(), e->round_kind.end());
      break;
    case PS_PLAN_PULL: {
      const PullPlan& P = e->pull;
      if (index == 0 || index + 1 >= P.off.size()) return e->fail(PS_E_RANGE, "round");
      v = {P.off[index], P.gsplit[index], P.off[index + 1]};
      for (uint32_t c = P.off[index]; c < P.off[index + 1]; ++c) chunk(P.chunks[c]);
      break;
    }
    case PS_PLAN_PAIR: {
      const PairPlan& P = e->pair;
      if (index >= P.lo.size()) return e->fail(PS_E_RANGE, "round");
      v = {P.lo[index], P.gsplit[index], P.hi[index]};
      for (uint32_t c = P.lo[index]; c < P.hi[index]; ++c) chunk(P.chunks[c]);
      break;
    }
    case PS_PLAN_XCHG: {
      const GhostPlan& G = e->ghost;
      if (index >= G.rounds.size()) {  // one rank: nothing exchanged
        v = {0};
        break;
      }
      const GhostRound& R = G.rounds[index];
      v = {R.any ? 1u : 0u};
      for (size_t b = 0; b < R.s_off.size(); ++b) v.insert(v.end(), {R.s_off[b], R.s_len[b], R.r_off[b], R.r_len[b]});
      break;
    }
    case PS_PLAN_SEGS:
      for (const GhostSeg& S : e->ghost.segs) {
        v.push_back(S.topic);
        v.push_back(S.rw);
        for (int32_t b = 0; b < e->world; ++b) v.push_back(S.rbase[b]);
        for (int32_t b = 0; b < e->world; ++b) v.push_back(S.sbase[b]);
      }
      break;
    case PS_PLAN_SHIP:
      for (const ShipEntry& s : e->ship_host) v.insert(v.end(), {s.node, s.dst});
      break;
    case PS_PLAN_PACK: {
      const GhostPlan& G = e->ghost;
      if (index >= G.rounds.size()) break;
      for (uint32_t k = G.rounds[index].pack0; k < G.rounds[index].pack1; ++k) {
        const PackSeg& p = G.pack[k];
        v.insert(v.end(), {p.e0, p.e1, p.gseg, p.W, p.row, p.unit0});
      }
      break;
    }
    case PS_PLAN_CHAIN: {
      const PairPlan& P = e->pair;
      if (index >= P.len.size() || P.len[index] < 3) {
        v = {0};
        break;
      }
      v = {P.len[index]};
      for (uint32_t k = P.lo[index]; k < P.hi[index]; ++k) {
        const ChainChunk& c = P.chain[k];
        v.insert(v.end(), {c.node_begin, c.node_end, c.topic, c.W, static_cast<uint64_t>(c.row0_hi) << 32 | c.row0_lo,
                           c.w0, c.S, c.levels, c.r0, c.group});
        for (uint32_t f = 0; f <= kChainLevels; ++f) v.push_back(c.first[f]);
      }
      break;
    }
    default:
      return e->fail(PS_E_INVAL, "unknown plan table");
  }
  *n_out = v.size();
  if (v.size() > cap) return PS_E_RANGE;
  std::copy(v.begin(), v.end(), out);
  return PS_OK;
}

}  // extern "C"
