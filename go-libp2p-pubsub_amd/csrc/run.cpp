// run.cpp -- the round loop on the GPU (ps_run / ps_run_async / ps_wait):
// plan uploads, one window's launches on the engine's stream (level mode:
// k_flood, k_pull_pair, k_pull; N ranks: the ghost exchange on a second
// stream beside each round's locally fed chunks; compaction mode: k_expand +
// frontier compaction), counters and readbacks.  DESIGN.md §5-§7.
#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "engine.hpp"
#include "gbuild.hpp"

namespace {
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}
}  // namespace

namespace psamd {

namespace {

int upload_pull(ps_engine* e) {
  if (e->pull.version == e->pull_up) return PS_OK;
  const auto& C = e->pull.chunks;
  HIP_TRY(e->d_pull.ensure(std::max<size_t>(C.size(), 1) * sizeof(PullChunk)), "alloc pull chunks");
  if (!C.empty()) {
    HIP_TRY(hipMemcpyAsync(e->d_pull.p, C.data(), C.size() * sizeof(PullChunk), hipMemcpyHostToDevice, e->stream),
            "upload pull chunks");
    if (e->gpu_graph)  // parent ranges for the generation staging
      HIP_TRY(launch_chunk_parents(e->d_pull.as<PullChunk>(), static_cast<uint32_t>(C.size()),
                                   e->d_node_parent.as<uint32_t>(), e->stream),
              "chunk parents");
  }
  e->pull_up = e->pull.version;
  return PS_OK;
}

// *overflow: some chain chunk's level range exceeded the level tables (checked once
// per plan, with one readback): the caller replans without chains.
int upload_pair(ps_engine* e, bool* overflow) {
  *overflow = false;
  if (e->pair.version == e->pair_up) return PS_OK;
  const auto& C = e->pair.chunks;
  HIP_TRY(e->d_pp.ensure(std::max<size_t>(C.size(), 1) * sizeof(PullChunk)), "alloc pair chunks");
  if (!C.empty()) {
    HIP_TRY(hipMemcpyAsync(e->d_pp.p, C.data(), C.size() * sizeof(PullChunk), hipMemcpyHostToDevice, e->stream),
            "upload pair chunks");
    if (e->gpu_graph)
      HIP_TRY(launch_chunk_parents(e->d_pp.as<PullChunk>(), static_cast<uint32_t>(C.size()),
                                   e->d_node_parent.as<uint32_t>(), e->stream),
              "pair chunk parents");
    HIP_TRY(launch_pair_kids(e->d_pp.as<PullChunk>(), static_cast<uint32_t>(C.size()), e->d_row_ptr.as<uint32_t>(),
                             e->d_col.as<uint32_t>(), e->stream),
            "pair chunk children");
  }
  const auto& K = e->pair.chain;
  HIP_TRY(e->d_chain.ensure(std::max<size_t>(K.size(), 1) * sizeof(ChainChunk)), "alloc chain chunks");
  if (!K.empty()) {
    HIP_TRY(hipMemcpyAsync(e->d_chain.p, K.data(), K.size() * sizeof(ChainChunk), hipMemcpyHostToDevice, e->stream),
            "upload chain chunks");
    if (e->gpu_graph)
      HIP_TRY(launch_chain_parents(e->d_chain.as<ChainChunk>(), static_cast<uint32_t>(K.size()),
                                   e->d_node_parent.as<uint32_t>(), e->stream),
              "chain chunk parents");
    HIP_TRY(e->d_chain_ovf.ensure(4), "alloc chain overflow word");
    HIP_TRY(hipMemsetAsync(e->d_chain_ovf.p, 0, 4, e->stream), "clear chain overflow word");
    const uint32_t nk = static_cast<uint32_t>(K.size());
    HIP_TRY(launch_chain_ranges(e->d_chain.as<ChainChunk>(), nk, e->d_row_ptr.as<uint32_t>(), kChainCap,
                                e->d_chain_ovf.as<uint32_t>(), e->stream),
            "chain ranges");
    // the chunks' node entries: counts and their scan now, the entries once
    // the total is back (one readback with the overflow word)
    const size_t scan_bytes = chain_meta_scan_bytes(nk);
    HIP_TRY(e->d_chain_scan.ensure(std::max<size_t>(scan_bytes, 16)), "alloc chain scan");
    HIP_TRY(e->d_chain_cnt.ensure((2 * static_cast<size_t>(nk) + 2) * 4), "alloc chain counts");
    HIP_TRY(launch_chain_meta(e->d_chain.as<ChainChunk>(), nk, nullptr, nullptr, e->d_chain_cnt.as<uint32_t>(),
                              e->d_chain_scan.p, e->d_chain_scan.bytes, nullptr, false, e->stream),
            "chain entry counts");
    uint32_t back[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&back[0], e->d_chain_ovf.p, 4, hipMemcpyDeviceToHost, e->stream), "read chain overflow");
    HIP_TRY(hipMemcpyAsync(&back[1], e->d_chain_cnt.as<uint32_t>() + nk + 1 + nk, 4, hipMemcpyDeviceToHost,
                           e->stream),
            "read chain entries");
    HIP_TRY(hipStreamSynchronize(e->stream), "sync");
    if (back[0]) {
      *overflow = true;
      return PS_OK;
    }
    HIP_TRY(e->d_chain_meta.ensure(std::max<size_t>(back[1], 1) * 4), "alloc chain entries");
    HIP_TRY(launch_chain_meta(e->d_chain.as<ChainChunk>(), nk, e->d_node_parent.as<uint32_t>(),
                              e->d_node_flags.as<uint8_t>(), e->d_chain_cnt.as<uint32_t>(), nullptr, 0,
                              e->d_chain_meta.as<uint32_t>(), true, e->stream),
            "chain entries");
  }
  e->pair_up = e->pair.version;
  return PS_OK;
}

int upload_flood(ps_engine* e) {
  if (e->flood.version == e->flood_up) return PS_OK;
  const auto& TK = e->flood.tasks;
  const auto& SG = e->flood.segs;
  const size_t n = TK.size();
  HIP_TRY(e->d_flood_tasks.ensure(std::max<size_t>(n, 1) * sizeof(FloodTask)), "alloc flood tasks");
  HIP_TRY(e->d_flood_segs.ensure(std::max<size_t>(SG.size(), 1) * sizeof(FloodSeg)), "alloc flood segments");
  bool fresh = false;  // granules of a fresh allocation carry no epoch yet
  HIP_TRY(e->d_flood_gran.ensure(std::max<size_t>(e->flood.granules, 1) * 8, &fresh), "alloc flood granules");
  if (fresh) HIP_TRY(hipMemsetAsync(e->d_flood_gran.p, 0, e->d_flood_gran.bytes, e->stream), "clear granules");
  if (n) {
    HIP_TRY(hipMemcpyAsync(e->d_flood_tasks.p, TK.data(), n * sizeof(FloodTask), hipMemcpyHostToDevice, e->stream),
            "upload flood tasks");
    HIP_TRY(hipMemcpyAsync(e->d_flood_segs.p, SG.data(), SG.size() * sizeof(FloodSeg), hipMemcpyHostToDevice,
                           e->stream),
            "upload flood segments");
    HIP_TRY(launch_flood_deps(e->d_flood_tasks.as<FloodTask>(), static_cast<uint32_t>(n),
                              e->d_flood_segs.as<FloodSeg>(), e->d_node_parent.as<uint32_t>(), e->stream),
            "flood dependencies");
  }
  e->flood_up = e->flood.version;
  return PS_OK;
}

int upload_ghost(ps_engine* e) {
  const GhostPlan& G = e->ghost;
  HIP_TRY(e->d_gsegs.ensure(std::max<size_t>(G.segs.size(), 1) * sizeof(GhostSeg)), "alloc ghost segments");
  HIP_TRY(e->d_pack.ensure(std::max<size_t>(G.pack.size(), 1) * sizeof(PackSeg)), "alloc pack segments");
  HIP_TRY(e->d_send.ensure(std::max<uint64_t>(kSendBufs * G.send_half, 16) * 8), "alloc send buffer");
  HIP_TRY(e->d_recv.ensure(std::max<uint64_t>(G.recv_words, 16) * 8), "alloc recv buffer");
  if (!G.segs.empty())
    HIP_TRY(hipMemcpyAsync(e->d_gsegs.p, G.segs.data(), G.segs.size() * sizeof(GhostSeg), hipMemcpyHostToDevice,
                           e->stream),
            "upload ghost segments");
  if (!G.pack.empty())
    HIP_TRY(hipMemcpyAsync(e->d_pack.p, G.pack.data(), G.pack.size() * sizeof(PackSeg), hipMemcpyHostToDevice,
                           e->stream),
            "upload pack segments");
  return PS_OK;
}

// Host -> device copies of one window through a pinned staging slot
// (ps_engine::Staging): asynchronous for the host, stream-ordered.
struct Upload {
  void* dst;
  const void* src;
  size_t bytes;
  const DevBuf* buf;  // dst's buffer (its upload shadow), nullable
};
// With `fold` set and the copy-kernel form, nothing is launched: *fold gets
// the copies for a kernel that folds them in, and staged[i] the device-mapped
// address of upload i's staged bytes (else its destination).
}  // namespace

// A held-back reduce launched on its own (ps_wait came first, or the next
// window cannot take it into its first launch).
int flush_reduce(ps_engine* e) {
  if (!e->pend_reduce.valid) return PS_OK;
  e->pend_reduce.valid = false;
  const ReduceArgs& r = e->pend_reduce.args;
  HIP_TRY(launch_reduce_rounds(r.partials, r.desc, r.n_rounds, r.round_stats, r.host_stats, r.sig, e->stream),
          "reduce rounds");
  return PS_OK;
}

int twin_join(ps_engine* e) {
  if (!e->t_pending) return PS_OK;
  HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_tend, 0), "twin join");
  e->t_pending = false;
  return PS_OK;
}

namespace {

int stage_uploads(ps_engine* e, const Upload* ups, size_t n, hipStream_t s, StageCopy* fold = nullptr,
                  const void** staged = nullptr) {
  if (fold) *fold = StageCopy{};
  for (size_t i = 0; staged && i < n; ++i) staged[i] = ups[i].dst;
  // bytes a buffer already holds (the same slot's last upload, same
  // allocation) are not staged again: the window reads them where they lie
  // (device memory) instead of over PCIe
  bool keep[8] = {};
  for (size_t i = 0; i < n && i < 8; ++i) {
    const Upload& u = ups[i];
    if (!u.buf || !u.bytes || !e->upload_reuse) continue;
    auto& sh = e->upload_shadow[u.buf];
    if (sh.gen == u.buf->gen && sh.data.size() == u.bytes && std::memcmp(sh.data.data(), u.src, u.bytes) == 0) {
      keep[i] = true;
      continue;
    }
    sh.gen = u.buf->gen;
    sh.data.assign(static_cast<const uint8_t*>(u.src), static_cast<const uint8_t*>(u.src) + u.bytes);
  }
  size_t need = 0;
  for (size_t i = 0; i < n; ++i)
    if (!(i < 8 && keep[i])) need += (ups[i].bytes + 255) & ~size_t(255);
  if (need == 0) return PS_OK;
  // the slot of the asynchronous run being enqueued (its previous user was
  // waited for before the run slot was reused); synchronous runs start with
  // nothing in flight
  ps_engine::Staging& g = e->stg[e->defer_into ? e->defer_into - e->infl : 0];
  if (need > g.cap) {
    if (g.h) HIP_TRY(hipHostFree(g.h), "free staging");
    g.h = nullptr;
    g.cap = 0;
    const size_t cap = std::max<size_t>(need, 64 << 10);
    void* h = nullptr;
    HIP_TRY(hipHostMalloc(&h, cap, hipHostMallocMapped | hipHostMallocCoherent), "alloc staging");
    g.h = static_cast<uint8_t*>(h);
    g.cap = cap;
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, h, 0), "map staging");
    g.d = static_cast<uint8_t*>(d);
  }
  // one copy kernel for up to kStageMax arrays of whole u32 words; blits
  // otherwise
  bool kernel = n <= kStageMax;
  for (size_t i = 0; i < n; ++i) kernel = kernel && ups[i].bytes % 4 == 0;
  StageCopy c{};
  size_t off = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!ups[i].bytes || (i < 8 && keep[i])) continue;
    std::memcpy(g.h + off, ups[i].src, ups[i].bytes);
    if (kernel) {
      if (staged && fold) staged[i] = g.d + off;
      c.src[c.n] = reinterpret_cast<const uint32_t*>(g.d + off);
      c.dst[c.n] = static_cast<uint32_t*>(ups[i].dst);
      c.words[c.n++] = static_cast<uint32_t>(ups[i].bytes / 4);
    } else {
      HIP_TRY(hipMemcpyAsync(ups[i].dst, g.h + off, ups[i].bytes, hipMemcpyHostToDevice, s), "upload");
    }
    off += (ups[i].bytes + 255) & ~size_t(255);
  }
  if (kernel && fold)
    *fold = c;
  else if (kernel)
    HIP_TRY(launch_stage_copy(c, s), "stage copy");
  return PS_OK;
}

// Debug (PSAMD_FLOOD_PROFILE=1): where k_flood's waves spent the last launch.
void flood_profile_report(ps_engine* e) {
  const uint32_t nw = e->flood_prof_waves;
  std::vector<uint64_t> p(static_cast<size_t>(nw) * kFloodProf);
  if (hipMemcpy(p.data(), e->d_flood_prof.p, p.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  uint64_t t0 = ~0ull, t1 = 0, smax = 0;
  double sum[kFloodProf] = {};
  std::vector<double> ends;
  for (uint32_t w = 0; w < nw; ++w) {
    const uint64_t* q = &p[static_cast<size_t>(w) * kFloodProf];
    t0 = std::min(t0, q[0]);
    t1 = std::max(t1, q[1]);
    smax = std::max(smax, q[0]);
    for (uint32_t k = 2; k < kFloodProf; ++k) sum[k] += static_cast<double>(q[k]);
    ends.push_back(static_cast<double>(q[1]));
  }
  std::sort(ends.begin(), ends.end());
  auto us = [](double ticks) { return ticks / 100.0; };  // s_memrealtime: 100 MHz
  const double busy = sum[2] + sum[3] + sum[4] + sum[5];
  std::fprintf(stderr,
               "[psengine] k_flood profile: %u waves, span %.1f us, start skew %.1f us, ends p50 %.1f p90 %.1f "
               "max %.1f us; per wave avg: wait %.1f resolve %.1f stream %.1f publish %.1f us (%.0f%%/%.0f%%/%.0f%%/"
               "%.0f%%), %.1f tasks; waits in the last third of the rounds %.1f us\n",
               nw, us(static_cast<double>(t1 - t0)), us(static_cast<double>(smax - t0)),
               us(ends[ends.size() / 2] - t0), us(ends[ends.size() * 9 / 10] - t0), us(ends.back() - t0),
               us(sum[2] / nw), us(sum[3] / nw), us(sum[4] / nw), us(sum[5] / nw), 100 * sum[2] / busy,
               100 * sum[3] / busy, 100 * sum[4] / busy, 100 * sum[5] / busy, sum[6] / nw, us(sum[7] / nw));
}

// Debug (PSAMD_CHAIN_PROFILE=<file>): appends the last blocking window's
// k_pull_chain wave records to <file> (tools/chain_profile.py reads them):
// u64 magic, u64 launches, per launch (round, rounds, lo, gsplit, hi), u64
// chunks, then per chunk kChainProf profile words and (topic, W, S, run
// nodes << 8 | levels).
void chain_profile_dump(ps_engine* e, uint32_t planned0) {
  const auto& K = e->pair.chain;
  std::vector<uint64_t> p(K.size() * kChainProf);
  if (p.empty() || hipMemcpy(p.data(), e->d_chain_prof.p, p.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  std::vector<uint64_t> out{0x50524F4643484149ull, 0};
  for (uint32_t q = 1; q <= planned0 && q < e->round_kind.size(); ++q)
    if (e->round_kind[q] == PS_K_CHAIN) {
      out.insert(out.end(), {q, e->pair.len[q], e->pair.lo[q], e->pair.gsplit[q], e->pair.hi[q]});
      ++out[1];
    }
  out.push_back(K.size());
  for (size_t i = 0; i < K.size(); ++i) {
    out.insert(out.end(), p.begin() + i * kChainProf, p.begin() + (i + 1) * kChainProf);
    out.insert(out.end(), {K[i].topic, K[i].W, K[i].S,
                           static_cast<uint64_t>(K[i].node_end - K[i].node_begin) << 8 | K[i].levels});
  }
  if (FILE* f = std::fopen(e->chain_prof_path.c_str(), "ab")) {
    std::fwrite(out.data(), 8, out.size(), f);
    std::fclose(f);
  }
}

// Propagates one window: per topic t, win[t] lists the messages (indices into
// `msgs`) whose bits form t's block of W_t = ceil(|win[t]|/64) words.
int run_window(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<WinSlice>& win, ps_stats* st) {
  const auto t_g0 = std::chrono::steady_clock::now();
  const uint64_t epochs0 = e->graph_epoch ^ (e->flags_epoch << 32);
  if (e->graph_dirty || e->flags_dirty) {  // (the node space a twin window on tstream may still read)
    const int rj = twin_join(e);
    if (rj) return rj;
    ++e->e_seq;
  }
  int rc = upload_graph(e);
  if (rc) return rc;
  // the per-window device tables of this run's slot: a pipelined window's
  // leading launches may run beside the previous window's last ones (the
  // other slot), see `overlap` below
  const uint32_t slot = e->defer_into ? static_cast<uint32_t>(e->defer_into - e->infl) : 0u;
  DevBuf& d_topics = slot ? e->d_topics1 : e->d_topics;
  DevBuf& d_woff = slot ? e->d_woff1 : e->d_woff;
  DevBuf& d_groups = slot ? e->d_groups1 : e->d_groups;
  DevBuf& d_partials = slot ? e->d_partials1 : e->d_partials;
  DevBuf& d_seeds = slot ? e->d_seeds1 : e->d_seeds;
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const int32_t world = e->world, me = e->rank;
  const auto t_w0 = std::chrono::steady_clock::now();
  if (e->host_timing)
    std::fprintf(stderr, "[psengine] graph upload/build %.3f ms (%s)\n",
                 std::chrono::duration<double, std::milli>(t_w0 - t_g0).count(), e->gpu_graph ? "gpu" : "host");
  WindowLayout L;
  rc = plan_window_layout(e, msgs, win, L);
  if (rc) return rc;
  if (L.wtot == 0 && world == 1) return PS_OK;
  auto& tab = L.tab;
  auto& groups = L.groups;
  const uint64_t wtot = L.wtot;
  const uint32_t max_start = L.max_start, planned0 = L.planned0, round_cap = L.round_cap;
  const bool level = L.level, any_mesh = L.any_mesh, need_direct = L.need_direct;
  const auto t_w1 = std::chrono::steady_clock::now();
  const bool record = (e->cfg.flags & PS_F_RECORD_HOPS) != 0;
  HIP_TRY(e->d_seen.ensure(wtot * 8), "alloc seen");
  HIP_TRY(e->d_arr0.ensure(wtot * 8), "alloc arrivals");
  HIP_TRY(e->d_arr1.ensure(wtot * 8), "alloc arrivals");
  if (record) HIP_TRY(e->d_hop.ensure(wtot * 64 * 2), "alloc hop record");
  const uint32_t n_waves = e->expand_grid * (kBlock / 64);
  // staged + direct kernel counters side by side
  HIP_TRY(d_partials.ensure(static_cast<size_t>(2) * n_waves * kNumCtr * 8), "alloc partials");
  // per-round counter rows: the planned rounds plus slack, grown (content kept)
  // if a mesh path outlives them
  uint32_t stats_rows = std::min<uint32_t>(round_cap, std::max<uint32_t>(kMaxRoundsCap, L.max_depth + max_start + 32));
  HIP_TRY(e->d_stats.ensure(static_cast<size_t>(stats_rows + 1) * kNumCtr * 8), "alloc stats");
  HIP_TRY(e->d_apply_stats.ensure(static_cast<size_t>(stats_rows + 1) * kNumCtr * 8), "alloc apply stats");
  HIP_TRY(d_topics.ensure(tab.size() * sizeof(TopicDev)), "alloc topics");
  HIP_TRY(e->d_nfront.ensure(4), "alloc n_front");
  HIP_TRY(d_groups.ensure(std::max<size_t>(L.gtab.size(), 1) * sizeof(GroupDev)), "alloc groups");
  // word offset of virtual word w of node u's row (u relative to the topic)
  auto phys = [&](uint32_t t, uint64_t u, uint32_t w) { return phys_word(tab[t], groups[t], u, w); };

  // root injections (owned roots only), grouped by round: mask[t][round][word]
  std::vector<std::vector<uint64_t>> inj(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    const TopicDev& d = tab[t];
    if (d.W == 0 || !(d.flags & kTopicRootLocal)) continue;
    inj[t].assign(static_cast<size_t>(max_start + 1) * d.W, 0);
    if (e->run_zero_start) {  // bits 0 .. n-1 of round 0
      for (uint32_t w = 0; w < win[t].n / 64; ++w) inj[t][w] = ~0ull;
      if (win[t].n % 64) inj[t][win[t].n / 64] = (1ull << (win[t].n % 64)) - 1;
    } else {
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t b = L.pos[t].empty() ? li : L.pos[t][li];
        // (level-aligned: every message is seeded before launch round 1)
        const uint32_t r0 = L.aligned ? 0u : msgs[win[t].idx[li]].start;
        inj[t][static_cast<size_t>(r0) * d.W + (b >> 6)] |= 1ull << (b & 63);
      }
    }
  }
  std::vector<SeedDev> seeds;
  std::vector<uint32_t> seed_off(max_start + 2, 0);
  for (uint32_t r = 0; r <= max_start; ++r) {
    for (uint32_t t = 0; t < nt; ++t) {
      TopicDev& d = tab[t];
      if (r == 0) d.seed_lo = static_cast<uint32_t>(seeds.size());
      if (inj[t].empty()) continue;
      if (d.flags & kTopicGroups) {
        // group-major: the root's block of the group starting this round is
        // set whole (k_window_init zeroes block 0 only)
        for (const StartGroup& g : groups[t])
          if (g.start == r)
            for (uint32_t w = g.w0; w < g.w0 + g.wn; ++w)
              seeds.push_back(SeedDev{phys(t, 0, w), inj[t][static_cast<size_t>(r) * d.W + w], d.nbase, 1});
      } else {
        for (uint32_t w = 0; w < d.W; ++w) {
          const uint64_t m = inj[t][static_cast<size_t>(r) * d.W + w];
          if (m) seeds.push_back(SeedDev{d.wbase + w, m, d.nbase, 0});  // root = node 0
        }
      }
      if (r == 0) d.seed_n = static_cast<uint32_t>(seeds.size()) - d.seed_lo;
    }
    seed_off[r + 1] = static_cast<uint32_t>(seeds.size());
  }
  HIP_TRY(d_seeds.ensure(seeds.size() * sizeof(SeedDev)), "alloc seeds");
  const auto t_w2 = std::chrono::steady_clock::now();

  // Start rounds present per topic.  A node at BFS level d receives a
  // message started at round s in round s + d and is expanded in round
  // s + d + 1: that bounds each round's frontier (grid size) and, for the
  // multi-GPU compaction exchange, each round's cross-rank traffic exactly.
  std::vector<std::vector<uint8_t>> starts_of(nt);
  for (uint32_t t = 0; t < nt; ++t) {
    if (win[t].n == 0 || !e->topics[t].exists) continue;
    starts_of[t].assign(max_start + 1, 0);
    if (e->run_zero_start)
      starts_of[t][0] = 1;
    else
      for (uint32_t li = 0; li < win[t].n; ++li) starts_of[t][msgs[win[t].idx[li]].start] = 1;
  }
  auto round_grid = [&](uint32_t r) -> uint32_t {
    if (any_mesh) return e->expand_grid;
    uint64_t bound = 0;
    for (uint32_t t = 0; t < nt; ++t) {
      if (tab[t].W == 0) continue;
      const auto& li = e->topics[t].level_internal;
      for (uint32_t s0 = 0; s0 <= max_start; ++s0) {
        if (!starts_of[t][s0] || r < 1 + s0) continue;
        const uint32_t d = r - 1 - s0;
        if (d < li.size()) bound += li[d];
      }
    }
    const uint64_t blocks = (bound + 3) / 4;  // ~1 entry per wave at least
    return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(e->expand_grid, blocks)));
  };
  // Level mode: one rank runs the leading rounds whose rows are small
  // (latency bound) as ONE persistent k_flood launch, then k_pull_pair /
  // k_pull launches (bandwidth bound); N ranks run k_pull_pair / k_pull with
  // the ghost exchange between rounds.  PSAMD_FLOOD=0 selects per-round
  // launches on one rank too.
  // deep single-start windows: per-round launches from round 1 (their first
  // few form the prefix that may overlap the previous window)
  const bool deep = deep_window(e, L);
  const bool flood_ok = !deep && level && world == 1 && e->flood_on && !e->flood_broken && e->flood_grid > 0 &&
                        e->n_nodes < 0x80000000u;  // k_flood marks node ids with bit 31
  uint32_t flood_rounds = 0;    // rounds 1..flood_rounds: k_flood
  std::vector<uint32_t> lgrid;  // per-round launches: blocks of every round (L and G parts together)
  uint32_t n_slots = 0;         // level mode: partial counter slots of the window
  // level-aligned windows: counter rows of the reach counts after the rounds'
  const uint32_t reach_rows =
      L.aligned ? static_cast<uint32_t>(ceil_div(2ull * L.split.n_segs, static_cast<uint64_t>(kNumCtr))) : 0u;
  uint32_t reach_slot0 = 0;
  bool fresh = false;           // level mode: no plan upload this window
  if (level) {
    bool changed = plan_pull_chunks(e, L);
    if (flood_ok) {
      flood_rounds = plan_flood_rounds(e, L);
      if (flood_rounds) plan_flood_tasks(e, L, flood_rounds);
    }
    bool gch = false;
    rc = plan_ghost(e, L, &gch);
    if (rc) return rc;
    changed |= gch;
    changed |= plan_pair_chunks(e, L, flood_rounds);
    if (world > 1 && changed) annotate_chunks(e, L);
    bool chain_overflow = false;
    // (nothing re-uploaded: the plan the previous window ran, a condition of the overlap)
    fresh = e->pull.version == e->pull_up && e->pair.version == e->pair_up &&
            (!flood_rounds || e->flood.version == e->flood_up);
    if (!fresh || (world > 1 && gch)) {  // (plan tables a twin window on tstream may still read)
      if ((rc = twin_join(e))) return rc;
      ++e->e_seq;
    }
    if ((rc = upload_pull(e)) || (rc = upload_pair(e, &chain_overflow))) return rc;
    if (chain_overflow) {  // a subtree wider than the level tables: this plan runs without chains
      e->chain_fail_key = e->pair.key;
      e->pair.key.clear();
      plan_pair_chunks(e, L, flood_rounds);
      if (world > 1) annotate_chunks(e, L);
      if ((rc = upload_pair(e, &chain_overflow))) return rc;
    }
    e->round_kind = e->pair.kind;
    if (flood_rounds && (rc = upload_flood(e))) return rc;
    if (world > 1 && gch && (rc = upload_ghost(e))) return rc;
    // desc[3q..]: round q's partial slots (first, end, stride) for the reduce
    auto& desc = e->desc_host;
    desc.assign(3 * (planned0 + 2 + reach_rows), 0);
    uint32_t slot = 0;
    if (flood_rounds) {
      desc[0] = 0;  // row 0: k_flood's timeout word (slot 0)
      desc[1] = 1;
      desc[2] = 1;
      for (uint32_t q = 1; q <= flood_rounds; ++q) {
        desc[3 * q] = e->flood.slot0[q];
        desc[3 * q + 1] = e->flood.slot0[q] + e->flood.nslot[q];
        desc[3 * q + 2] = e->flood.nslot[q] ? 1 : 0;
      }
      slot = e->flood.slots;
    }
    // the launches of round q own the slots [woff[q], woff[q+1]): one per
    // block (pull) or wave (pair), at most kPullSlots; the L and G parts of
    // a round share them (counters are added)
    lgrid.assign(planned0 + 1, 0);
    auto& woff = e->woff_host;
    woff.assign(planned0 + 2, 0);
    woff[flood_rounds + 1] = slot;
    for (uint32_t q = flood_rounds + 1; q <= planned0; ++q) {
      const uint8_t kq = e->round_kind[q];
      const bool multi_round = kq == PS_K_PAIR || kq == PS_K_CHAIN;
      const uint32_t len = multi_round ? e->pair.len[q] : 1u;
      lgrid[q] = multi_round ? e->pair.hi[q] - e->pair.lo[q]  // (one one-wave workgroup per chunk)
                             : ceil_div(e->pull.gsplit[q] - e->pull.off[q], kBlock / 64) +
                                   ceil_div(e->pull.off[q + 1] - e->pull.gsplit[q], kBlock / 64);
      for (uint32_t k = q; k < q + len; ++k) {  // a multi-round launch: one slot range per round
        woff[k + 1] = woff[k] + std::min<uint32_t>(lgrid[q], multi_round ? kPairSlots : kPullSlots);
        desc[3 * k] = woff[k];
        desc[3 * k + 1] = woff[k + 1];
        desc[3 * k + 2] = 1;
      }
      for (uint32_t k = 1; k < len; ++k) lgrid[q + k] = 0;
      q += len - 1;
    }
    n_slots = woff[planned0 + 1];
    // level-aligned: the reach counts (2 per (topic, level) segment, kNumCtr
    // per slot) as pseudo-slots after the rounds', one reduce row each
    reach_slot0 = n_slots;
    for (uint32_t j = 0; j < reach_rows; ++j) {
      desc[3 * (planned0 + 1 + j)] = n_slots + j;
      desc[3 * (planned0 + 1 + j) + 1] = n_slots + j + 1;
      desc[3 * (planned0 + 1 + j) + 2] = 1;
    }
    n_slots += reach_rows;
    fresh = fresh && !chain_overflow;
    HIP_TRY(d_partials.ensure(static_cast<size_t>(std::max<uint32_t>(n_slots, 1)) * kNumCtr * 8),
            "alloc level partials");
    HIP_TRY(d_woff.ensure(desc.size() * 4), "alloc reduce descriptors");
  }
  // compaction mode on N ranks: cross-rank capacities (items = node words)
  // per round: cap[r][from*world+to]
  std::vector<std::vector<uint64_t>> cap;
  if (world > 1 && !level) {
    uint64_t max_send = 0, max_recv = 0;
    cap.assign(planned0 + 1, std::vector<uint64_t>(static_cast<size_t>(world) * world, 0));
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicHost& T = e->topics[t];
      if (starts_of[t].empty()) continue;
      const uint64_t Wt = L.wglob[t];
      for (const auto& c : T.cross)
        for (uint32_t s0 = 0; s0 <= max_start; ++s0) {
          const uint32_t r = c.level + 1 + s0;
          if (starts_of[t][s0] && r <= planned0) cap[r][c.from * world + c.to] += c.count * Wt;
        }
    }
    for (uint32_t r = 1; r <= planned0; ++r) {
      uint64_t sb = 0, rb = 0;
      for (int32_t q = 0; q < world; ++q) {
        if (cap[r][me * world + q]) sb += kRegionHeader + cap[r][me * world + q] * sizeof(XItem);
        if (cap[r][q * world + me]) rb += kRegionHeader + cap[r][q * world + me] * sizeof(XItem);
      }
      max_send = std::max(max_send, sb);
      max_recv = std::max(max_recv, rb);
    }
    HIP_TRY(e->d_send.ensure(max_send), "alloc send regions");
    HIP_TRY(e->d_recv.ensure(max_recv), "alloc recv regions");
  }

  const bool flood = flood_rounds > 0;
  const uint32_t mode = flood ? PS_MODE_FLOOD : level ? PS_MODE_LEVEL_PULL : PS_MODE_COMPACT;
  const auto t_w3 = std::chrono::steady_clock::now();
  hipStream_t s = e->stream;
  // the prefix (deep windows): leading launches of at most 1/64 of the
  // window's row bytes, rounds 1..pre_P, followed by a launch starting at
  // round pre_P + 1 (the gate) and at least one more
  uint32_t pre_P = 0;
  uint64_t total = 0;  // the window's row bytes
  if (level)
    for (uint32_t q = 1; q <= planned0 && q < e->pull.bytes.size(); ++q) total += e->pull.bytes[q];
  // deep windows of at least overlap_min_bytes alternate between the two row
  // sets (engine.hpp, twin windows): a window's prefix then writes no row its
  // predecessor's last launch still reads, so the prefix may hold every
  // launch but the last (the gate: recorded before that launch)
  const bool alt_plan = e->twin_on && level && world == 1 && deep && flood_rounds == 0 &&
                        total >= e->overlap_min_bytes;
  if (deep && flood_rounds == 0) {
    std::vector<std::pair<uint32_t, uint32_t>> ls;  // launches: (first round, last round)
    for (uint32_t q = 1; q <= planned0; ++q) {
      const uint8_t k = e->round_kind[q];
      if (k != PS_K_PULL && k != PS_K_PAIR && k != PS_K_CHAIN) continue;
      const uint32_t len = k == PS_K_PULL ? 1u : e->pair.len[q];
      ls.emplace_back(q, q + len - 1);
    }
    uint64_t acc = 0;
    for (size_t i = 0; i + 2 < ls.size(); ++i) {
      uint64_t b = 0;
      for (uint32_t q = ls[i].first; q <= ls[i].second && q < e->pull.bytes.size(); ++q) b += e->pull.bytes[q];
      if (acc + b > total / 64 || ls[i + 1].first != ls[i].second + 1) break;
      acc += b;
      pre_P = ls[i].second;
    }
    // alternating row sets (below): every launch but the last is the prefix
    // -- nothing the predecessor's last launch reads is written by it
    if (alt_plan && ls.size() >= 2) {
      bool contiguous = true;
      for (size_t i = 0; i + 1 < ls.size(); ++i) contiguous = contiguous && ls[i + 1].first == ls[i].second + 1;
      if (contiguous) pre_P = ls[ls.size() - 2].second;
    }
  }
  // level-aligned: the (topic, level) pieces of k_level_reach, levels <= P
  // first (they are counted before the gate launch: a pipelined successor's
  // prefix may restamp those levels' generation bytes beside this window's
  // remaining launches), cached per node space, active topic set and P
  uint32_t reach_a = 0;  // pieces of levels <= pre_P
  bool reach_up = false;  // the pieces were uploaded for this window
  if (L.aligned) {
    std::vector<uint64_t> key{e->graph_epoch, pre_P};
    for (uint32_t t = 0; t < nt; ++t) key.push_back(L.split.seg_lo[t]);
    if (key != e->reach_key) {
      if ((rc = twin_join(e))) return rc;
      ++e->e_seq;
      reach_up = true;
      std::vector<ReachPiece>& pc = e->reach_host;
      pc.clear();
      for (int part = 0; part < 2; ++part) {
        for (uint32_t t = 0; t < nt; ++t) {
          if (L.split.seg_lo[t] == kNone) continue;
          const TopicHost& T = e->topics[t];
          for (uint32_t dl = 0; dl < L.split.seg_n[t]; ++dl) {
            if ((dl <= pre_P) != (part == 0)) continue;
            for (uint32_t u = T.level_off[dl]; u < T.level_off[dl + 1]; u += kReachPiece)
              pc.push_back(ReachPiece{L.split.seg_lo[t] + dl, T.nbase + u,
                                      T.nbase + std::min<uint32_t>(u + kReachPiece, T.level_off[dl + 1]), t});
          }
        }
        if (part == 0) e->reach_a = static_cast<uint32_t>(pc.size());
      }
      HIP_TRY(e->d_reach.ensure(std::max<size_t>(pc.size(), 1) * sizeof(ReachPiece)), "alloc reach pieces");
      if (!pc.empty())
        HIP_TRY(hipMemcpyAsync(e->d_reach.p, pc.data(), pc.size() * sizeof(ReachPiece), hipMemcpyHostToDevice,
                               e->stream),
                "upload reach pieces");
      e->n_reach = static_cast<uint32_t>(pc.size());
      e->reach_key = key;
    }
    reach_a = e->reach_a;
  }
  // every single-rank tree window may overlap its window init (pre_P = 0:
  // the gate is the predecessor's first launch, the last one reading the
  // root rows the init rewrites); deep windows also their leading launches
  // (windows of under 512 MB: the stream hand-offs cost more than the init
  // they hide -- cfg2 0.066 -> 0.068-0.073 ms/step, cfg4 0.4536 -> 0.4502)
  // (a shallow window -- k_flood leading rounds, nothing but its init to hide
  // -- ends signalled instead: its events cost more than the init, cfg4
  // 0.4472-0.4479 -> 0.4421-0.4425 ms/step, profiles/r04/ab/shallow_signalled.log)
  // a twin window (engine.hpp): its plan is on the device already, it ends
  // signalled, and nothing of it needs the stream order of `stream`.  Only
  // windows under overlap_min_bytes: a small window is latency bound and its
  // twin fills the chip (cfg2 0.0486 -> 0.0358 ms/step); two bandwidth-bound
  // windows side by side only share HBM and the MALL (paced cfg3 1.058 vs
  // 1.015, cfg4 0.4437 vs 0.4432 ms/step: profiles/r05/ab/twin_*.json) --
  // those keep the prefix overlap
  const bool twin = e->twin_on && e->sig_windows && level && world == 1 && !any_mesh && !record &&
                    !(e->cfg.flags & (PS_F_NO_LAZY_SEEN | PS_F_TIME_KERNELS)) && flood_rounds == 0 &&
                    e->defer_last && e->defer_into && planned0 <= PS_MAX_ROUNDS && fresh && !reach_up &&
                    e->chain_prof_path.empty() && total < e->overlap_min_bytes;
  const bool pcap = !twin && e->overlap_on && level && world == 1 && !any_mesh && !record && !L.multi &&
                    !(e->cfg.flags & (PS_F_NO_LAZY_SEEN | PS_F_TIME_KERNELS)) && total >= e->overlap_min_bytes && deep;
  // this window into the row set the last one did not write (cleared on s
  // when newly allocated)
  auto switch_sets = [&](bool* fresh_gen = nullptr) -> int {
    const size_t gen_bytes = e->d_gen.bytes;
    e->swap_row_sets();
    HIP_TRY(e->d_seen.ensure(wtot * 8), "alloc seen");
    HIP_TRY(e->d_arr0.ensure(wtot * 8), "alloc arrivals");
    HIP_TRY(e->d_arr1.ensure(wtot * 8), "alloc arrivals");
    bool gfresh = false;
    HIP_TRY(e->d_gen.ensure(gen_bytes, &gfresh), "alloc generations");
    if (gfresh) {
      HIP_TRY(hipMemsetAsync(e->d_gen.p, 0, e->d_gen.bytes, s), "clear generations");
      e->gen_cur = 0;
    }
    if (fresh_gen) *fresh_gen = gfresh;
    return PS_OK;
  };
  if (!twin) {
    if ((rc = twin_join(e))) return rc;  // (it reuses the last window's row set)
    ++e->e_seq;
  } else {
    if (e->pend_reduce.valid && (rc = flush_reduce(e))) return rc;
    ++e->overlapped;  // (ps_overlapped_windows: it may run beside its predecessor)
    // the stream the last window did not run on, and the row set it did not write
    if (!e->tstream) {
      HIP_TRY(hipStreamCreateWithFlags(&e->tstream, hipStreamNonBlocking), "twin stream");
      HIP_TRY(hipEventCreateWithFlags(&e->ev_tend, kStreamEvent), "twin events");
      HIP_TRY(hipEventCreateWithFlags(&e->ev_e2t, kStreamEvent), "twin events");
    }
    s = e->last_win_stream == e->stream ? e->tstream : e->stream;
    if (s == e->tstream && e->t_seq != e->e_seq) {  // shared state `stream` changed since tstream last followed it
      HIP_TRY(hipEventRecord(e->ev_e2t, e->stream), "event");
      HIP_TRY(hipStreamWaitEvent(s, e->ev_e2t, 0), "twin wait");
      e->t_seq = e->e_seq;
    }
    if ((rc = switch_sets())) return rc;
  }
  const bool alt_sets = pcap && alt_plan;
  bool sets_fresh = false;  // (the other set's generation bytes were just cleared on `stream`)
  if (alt_sets && (rc = switch_sets(&sets_fresh))) return rc;
  if (pcap && !e->pstream) {  // (created on first use: multi-rank engines never need them)
    HIP_TRY(hipStreamCreateWithFlags(&e->pstream, hipStreamNonBlocking), "prefix stream");
    for (hipEvent_t* ev : {&e->ev_gate[0], &e->ev_gate[1], &e->ev_pre})
      HIP_TRY(hipEventCreateWithFlags(ev, kStreamEvent), "overlap events");
  }
  std::vector<uint64_t> gkey;
  if (pcap)
    gkey = {e->pull.version, e->pair.version, e->flood.version, e->graph_epoch, e->flags_epoch, pre_P,
            flood_rounds, wtot, planned0};
  const bool overlap = pcap && fresh && !sets_fresh && e->defer_into && e->gate_valid && e->gate_slot != slot &&
                       e->gate_key == gkey && epochs0 == (e->graph_epoch ^ (e->flags_epoch << 32)) &&
                       e->gen_cur + 1 <= 255 && level && !any_mesh &&
                       !(e->cfg.flags & (PS_F_NO_LAZY_SEEN | PS_F_TIME_KERNELS));
  e->gate_valid = false;  // (this window records its own gate below)
  // the window's effective plan (ps_stats diagnostics)
  st->prefix_rounds = pcap ? pre_P : 0;
  st->overlapped += (overlap || twin) ? 1 : 0;
  st->xchg_path = PS_XCHG_NONE;
  st->plan_max_rounds = 1;
  if (level)
    for (uint32_t q = flood_rounds + 1; q <= planned0 && q < e->pair.len.size(); ++q)
      st->plan_max_rounds = std::max(st->plan_max_rounds, e->pair.len[q]);
  if (overlap) {
    HIP_TRY(hipStreamWaitEvent(e->pstream, e->ev_gate[e->gate_slot], 0), "wait for the previous gate");
    s = e->pstream;
    ++e->overlapped;
  }
  // the window's first kernel also copies the staged uploads, applies the
  // round-0 seeds of tree roots and clears the pull partial slots (level
  // mode without meshes; the eager seen clear below would erase the seeds)
  const bool fold = level && !any_mesh && !(e->cfg.flags & PS_F_NO_LAZY_SEEN);
  WindowStart ws{};
  const void* staged[4] = {nullptr, nullptr, nullptr, nullptr};
  {
    const Upload ups[4] = {{d_topics.p, tab.data(), tab.size() * sizeof(TopicDev), &d_topics},
                           {d_seeds.p, seeds.data(), seeds.size() * sizeof(SeedDev), &d_seeds},
                           {d_woff.p, e->desc_host.data(), level ? e->desc_host.size() * 4 : 0, &d_woff},
                           {d_groups.p, L.gtab.data(), L.gtab.size() * sizeof(GroupDev), &d_groups}};
    const int rcu = stage_uploads(e, ups, 4, s, fold ? &ws.copy : nullptr, staged);
    if (rcu) return rcu;
  }
  if (fold) {
    if (seed_off[1] > 0) ws.seeds = static_cast<const SeedDev*>(staged[1]);
    ws.zero = d_partials.as<uint64_t>();
    ws.zero_words = static_cast<uint64_t>(n_slots) * kNumCtr;
  }
  const bool seeds0_done = ws.seeds != nullptr;
  const bool partials_done = ws.zero != nullptr;
  // a pipelined one-rank window on the main stream alone ends with a pinned
  // flag and timestamps instead of events (ps_wait polls the flag): no event
  // record between consecutive windows
  const bool sigwin = e->sig_windows && e->defer_last && e->defer_into && level && world == 1 && !record &&
                      !(e->cfg.flags & PS_F_TIME_KERNELS) && !pcap && planned0 <= PS_MAX_ROUNDS;
  e->defer_into_signalled = false;
  if (sigwin)
    ws.t0 = e->defer_into->sig_dev + 1;
  else
    HIP_TRY(hipEventRecord(e->ev_run0, s), "event");
  const auto t_first = std::chrono::steady_clock::now();
  // new window generation: every tree row from older windows becomes stale
  if (++e->gen_cur > 255) {
    HIP_TRY(hipMemsetAsync(e->d_gen.p, 0, e->d_gen.bytes, s), "clear generations");
    e->gen_cur = 1;
  }
  // the previous window's held-back reduce: in this launch when both run on
  // the main stream, else on its own first
  const bool turn = e->pend_reduce.valid && fold && s == e->stream && nt > 0;
  if (e->pend_reduce.valid && !turn) {
    const int rcf = flush_reduce(e);
    if (rcf) return rcf;
  }
  if (turn) {
    e->pend_reduce.valid = false;
    HIP_TRY(launch_window_turn(e->pend_reduce.args, static_cast<const TopicDev*>(staged[0]), nt,
                               e->d_seen.as<uint64_t>(), e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>(),
                               e->d_gen.as<uint8_t>(), e->gen_cur, any_mesh, ws, s),
            "reduce + window init");
  } else {
    HIP_TRY(launch_window_init(static_cast<const TopicDev*>(fold ? staged[0] : d_topics.p), nt,
                               e->d_seen.as<uint64_t>(), e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>(),
                               e->d_gen.as<uint8_t>(), e->gen_cur, any_mesh, ws, s),
            "window init");
  }
  if (e->n_remote_fed && !level)
    HIP_TRY(launch_init_nodes(e->d_remote_fed.as<uint32_t>(), e->n_remote_fed, e->d_node_topic.as<uint16_t>(),
                              d_topics.as<TopicDev>(), e->d_seen.as<uint64_t>(), e->d_arr0.as<uint64_t>(),
                              e->d_arr1.as<uint64_t>(), e->d_gen.as<uint8_t>(), e->gen_cur, !level, s),
            "init remote-fed rows");
  if (e->cfg.flags & PS_F_NO_LAZY_SEEN) {
    // eager variant: clear every row and mark every node current, so the
    // expand kernel reads each child's seen word before it tests and sets it
    HIP_TRY(hipMemsetAsync(e->d_seen.p, 0, wtot * 8, s), "clear seen");
    HIP_TRY(hipMemsetAsync(e->d_gen.p, static_cast<int>(e->gen_cur), e->d_gen.bytes, s), "stamp generations");
  }
  if (record) HIP_TRY(hipMemsetAsync(e->d_hop.p, 0xFF, wtot * 64 * 2, s), "clear hop record");
  if (world > 1)  // (level mode: stays zero; the pull kernels count every delivery)
    HIP_TRY(hipMemsetAsync(e->d_apply_stats.p, 0, static_cast<size_t>(planned0 + 1) * kNumCtr * 8, s),
            "clear apply stats");

  ExpandArgs a{};
  bool cprof = false;               // debug: chain launches profiled (PSAMD_CHAIN_PROFILE)
  bool host_stats_written = false;  // the reduce wrote the deferred slot's pinned rows
  bool reduce_side = false;         // ... on e->rstream (the window's end event goes there)
  a.frontier = e->d_frontier.as<uint32_t>();
  a.opts = e->expand_opts;
  a.n_front = e->d_nfront.as<uint32_t>();
  a.row_ptr = e->d_row_ptr.as<uint32_t>();
  a.col = e->d_col.as<uint32_t>();
  a.node_topic = e->d_node_topic.as<uint16_t>();
  a.node_flags = e->d_node_flags.as<uint8_t>();
  a.topics = d_topics.as<TopicDev>();
  a.seen = e->d_seen.as<uint64_t>();
  a.gen = e->d_gen.as<uint8_t>();
  a.gen_cur = e->gen_cur;
  a.next_flag = e->d_flags.as<uint8_t>();
  a.blk_flag = e->d_blk.as<uint8_t>();
  a.hop_rec = record ? e->d_hop.as<uint16_t>() : nullptr;
  a.send = e->d_send.as<uint8_t>();
  uint64_t* const partials = d_partials.as<uint64_t>();
  uint64_t* arr[2] = {e->d_arr0.as<uint64_t>(), e->d_arr1.as<uint64_t>()};
  uint64_t* stats = e->d_stats.as<uint64_t>();
  const bool timed = (e->cfg.flags & PS_F_TIME_KERNELS) != 0;

  auto seed_round = [&](uint32_t r, uint64_t* into) -> hipError_t {
    if (r > max_start) return hipSuccess;
    return launch_seed(d_seeds.as<SeedDev>(), seed_off[r], seed_off[r + 1], into, a.seen,
                       level ? nullptr : a.next_flag, level ? nullptr : a.blk_flag, s);
  };
  auto compact = [&](uint32_t r, uint32_t waves_r) -> hipError_t {
    hipError_t x = launch_flag_count(a.next_flag, a.blk_flag, e->n_pad, e->d_wgcount.as<uint32_t>(), partials,
                                     waves_r, r ? stats + r * kNumCtr : nullptr, s);
    if (x != hipSuccess) return x;
    return launch_flag_compact(a.next_flag, a.blk_flag, e->n_pad, e->d_wgcount.as<uint32_t>(),
                               e->d_frontier.as<uint32_t>(), e->d_nfront.as<uint32_t>(), s);
  };
  // compaction mode on N ranks, round r: region layout, header reset, exchange, apply
  std::vector<uint64_t> s_off(world, 0), s_len(world, 0), r_off(world, 0), r_len(world, 0);
  auto layout = [&](uint32_t r) -> bool {
    if (world <= 1 || r > planned0 || cap.empty()) return false;
    uint64_t so = 0, ro = 0;
    bool any = false;
    for (int32_t q = 0; q < world; ++q) {
      const uint64_t cs = cap[r][me * world + q], cr = cap[r][q * world + me];
      s_off[q] = so;
      s_len[q] = cs ? kRegionHeader + cs * sizeof(XItem) : 0;
      so += s_len[q];
      r_off[q] = ro;
      r_len[q] = cr ? kRegionHeader + cr * sizeof(XItem) : 0;
      ro += r_len[q];
      for (int32_t z = 0; z < world; ++z) any |= cap[r][q * world + z] != 0;
    }
    for (int32_t q = 0; q < world && q < kMaxRanks; ++q) a.send_off[q] = s_off[q];
    return any;  // the same verdict on every rank
  };

  uint32_t planned = planned0;
  uint32_t r = 0;
  size_t ev_used = 0;
  std::vector<uint32_t> ev_round;  // round of every timed launch pair
  uint32_t launches = 0;
  auto time_mark = [&](bool begin) -> hipError_t {
    if (!timed) return hipSuccess;
    if (begin) ev_round.push_back(r);
    if (begin && ev_used + 2 > e->ev_k.size()) {
      hipEvent_t x, y;
      hipError_t c = hipEventCreate(&x);
      if (c == hipSuccess) c = hipEventCreate(&y);
      if (c != hipSuccess) return c;
      e->ev_k.push_back(x);
      e->ev_k.push_back(y);
    }
    const hipError_t c = hipEventRecord(e->ev_k[ev_used + (begin ? 0 : 1)], s);
    if (!begin) ev_used += 2;
    return c;
  };
  // compaction mode: all-to-allv of this round's send regions, then the apply kernel
  auto xchg = [&](uint32_t rr) -> int {
    std::string xerr;
    hipError_t xe = e->transport->exchange(a.send, s_off, s_len, e->d_recv.as<uint8_t>(), r_off, r_len, s, &xerr);
    if (xe != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
    st->xchg_path = PS_XCHG_COPY;
    st->xchg_rounds += 1;
    for (const uint64_t n : r_len) st->xchg_bytes += n;
    ApplyArgs ap{};
    ap.recv = e->d_recv.as<uint8_t>();
    ap.world = static_cast<uint32_t>(world);
    ap.cap_pre[0] = 0;
    for (int32_t q = 0; q < world; ++q) {
      ap.recv_off[q] = r_off[q];
      ap.cap_pre[q + 1] = ap.cap_pre[q] + cap[rr][q * world + me];
    }
    ap.node_topic = a.node_topic;
    ap.node_flags = a.node_flags;
    ap.topics = a.topics;
    ap.seen = a.seen;
    ap.a_next = a.a_next;
    ap.next_flag = level ? nullptr : a.next_flag;
    ap.blk_flag = level ? nullptr : a.blk_flag;
    ap.hop_rec = a.hop_rec;
    ap.stats = e->d_apply_stats.as<uint64_t>() + static_cast<size_t>(rr) * kNumCtr;
    ap.gen = level ? a.gen : nullptr;
    ap.gen_cur = a.gen_cur;
    HIP_TRY(launch_apply(ap, rr, record, s), "apply");
    return PS_OK;
  };
  if (level) {
    // static frontier, counters reduced once per window
    if (!partials_done)  // blocks / waves add into shared partial slots
      HIP_TRY(hipMemsetAsync(partials, 0, static_cast<size_t>(n_slots) * kNumCtr * 8, s), "clear partials");
    if (!seeds0_done) HIP_TRY(seed_round(0, arr[0]), "seed");
    // k_flood, start groups or pair launches: every root row is seeded up
    // front into arr[0] (and seen: k_flood reads parent rows from there), the
    // blocks of later start rounds included -- a block is read only in its
    // own rounds
    bool pairs = false;
    for (uint32_t q = 1; q <= planned0; ++q) pairs |= e->round_kind[q] == PS_K_PAIR || e->round_kind[q] == PS_K_CHAIN;
    const bool upfront = flood || L.multi || pairs;  // (a pair launch's plain level-1 runs read roots)
    if (upfront && max_start > 0)
      HIP_TRY(launch_seed(d_seeds.as<SeedDev>(), seed_off[1], seed_off[max_start + 1], arr[0], a.seen, nullptr,
                          nullptr, s),
              "seed");
    if (flood) {
      if (s != e->stream) {  // (pre_P = 0) the window init is enqueued: k_flood follows it on the main stream
        HIP_TRY(hipEventRecord(e->ev_pre, s), "event");
        s = e->stream;
        HIP_TRY(hipStreamWaitEvent(s, e->ev_pre, 0), "prefix join");
      }
      FloodArgs fa{};
      fa.tasks = e->d_flood_tasks.as<FloodTask>();
      fa.segs = e->d_flood_segs.as<FloodSeg>();
      fa.node_parent = e->d_node_parent.as<uint32_t>();
      fa.node_flags = a.node_flags;
      fa.topics = a.topics;
      fa.seen = a.seen;
      fa.gen = a.gen;
      fa.hop_rec = a.hop_rec;
      fa.granules = e->d_flood_gran.as<uint64_t>();
      fa.partials = partials;
      fa.err = reinterpret_cast<uint32_t*>(partials);  // slot 0, reduced into row 0
      fa.n_tasks = static_cast<uint32_t>(e->flood.tasks.size());
      if (++e->flood_epoch == 0) ++e->flood_epoch;  // granules of older launches carry older epochs
      fa.epoch = e->flood_epoch;
      fa.gen_cur = a.gen_cur;
      fa.spin_ticks = e->flood_spin_ticks;
      const uint32_t flood_blocks = std::min<uint32_t>(e->flood_grid, ceil_div(fa.n_tasks, kBlock / 64));
      if (e->flood_profile) {
        HIP_TRY(e->d_flood_prof.ensure(static_cast<size_t>(flood_blocks) * 4 * kFloodProf * 8), "alloc flood profile");
        fa.prof = e->d_flood_prof.as<uint64_t>();
        fa.prof_split = flood_rounds * 2 / 3;
        e->flood_prof_waves = flood_blocks * 4;
      }
      r = 1;  // the per-round kernel times of a timed run go to round 1
      HIP_TRY(time_mark(true), "event");
      ++launches;
      HIP_TRY(launch_flood(fa, flood_blocks, record, s), "flood");
      HIP_TRY(time_mark(false), "event");
    }
    PullArgs pa{};
    pa.node_parent = e->d_node_parent.as<uint32_t>();
    pa.node_flags = a.node_flags;
    pa.topics = a.topics;
    pa.seen = a.seen;
    pa.gen = a.gen;
    pa.hop_rec = a.hop_rec;
    pa.gen_cur = a.gen_cur;
    pa.ghost_ref = world > 1 ? e->d_ghost_ref.as<uint32_t>() : nullptr;
    pa.gsegs = e->d_gsegs.as<GhostSeg>();
    pa.chain_meta = e->d_chain_meta.as<uint32_t>();
    if (e->inplace && e->rrows_dirty) {  // (the owners' row sets, from the ghost plan's exchange)
      HIP_TRY(e->d_rrows.ensure(kMaxRanks * sizeof(RankRows)), "alloc rank rows");
      HIP_TRY(hipMemcpyAsync(e->d_rrows.p, e->rrows_host.data(), kMaxRanks * sizeof(RankRows), hipMemcpyHostToDevice,
                             e->stream),
              "upload rank rows");
      e->rrows_dirty = false;
    }
    pa.rrows = e->inplace ? e->d_rrows.as<RankRows>() : nullptr;
    pa.recv = e->d_recv.as<uint64_t>();
    for (int32_t q = 0; q < kMaxRanks; ++q) pa.rsrc[q] = pa.recv;
    const bool zero_copy = world > 1 && e->transport->zero_copy();
    std::vector<const uint8_t*> peer_region;
    pa.ship = world > 1 ? e->d_ship.as<ShipEntry>() : nullptr;
    pa.send = e->d_send.as<uint64_t>();
    pa.all_current = (e->cfg.flags & PS_F_NO_LAZY_SEEN) ? 1u : 0u;
    // debug: the chain launches' per-wave profile (blocking windows only)
    cprof = !e->chain_prof_path.empty() && !(e->defer_last && e->defer_into) && !e->pair.chain.empty();
    if (cprof) HIP_TRY(e->d_chain_prof.ensure(e->pair.chain.size() * kChainProf * 8), "alloc chain profile");
    // zero copy: the launches of round r ship into send part (r + 1) %
    // kSendBufs, which the readers of round r + 1 - kSendBufs may still hold
    auto reuse = [&](uint32_t q) -> int {
      if (!zero_copy || q < 1 || q >= e->ghost.rounds.size() || !e->ghost.rounds[q].any) return PS_OK;
      std::string xerr;
      if (e->transport->reuse(s, q, &xerr) != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
      return PS_OK;
    };
    static_assert(kSendBufs == 3, "reuse() below waits kSendBufs - 1 rounds back");
    bool gate_done = false;
    bool reach_a_done = false;
    for (r = flood_rounds + 1; r <= planned0; ++r) {
      if (!twin && s != e->stream && r > pre_P) {  // the prefix is enqueued: the rest follows it on the main stream
        HIP_TRY(hipEventRecord(e->ev_pre, s), "event");
        s = e->stream;
        HIP_TRY(hipStreamWaitEvent(s, e->ev_pre, 0), "prefix join");
      }
      // levels <= P counted before the gate (alternating row sets: no successor
      // restamps them, the whole pass runs beside the next window, below)
      if (L.aligned && !alt_sets && r == pre_P + 1 && reach_a && !reach_a_done) {
        HIP_TRY(launch_level_reach(e->d_reach.as<ReachPiece>(), reach_a, a.gen, a.gen_cur, a.node_flags, a.topics,
                                   a.seen, L.split.eager, partials + static_cast<size_t>(reach_slot0) * kNumCtr, s),
                "level reach (prefix levels)");
        reach_a_done = true;
      }
      // the gate launch is enqueued (alternating sets: the gate is recorded
      // before the window's last launch)
      if (pcap && !gate_done && r > (alt_sets ? pre_P : pre_P + 1)) {
        HIP_TRY(hipEventRecord(e->ev_gate[slot], e->stream), "event");
        e->gate_valid = true;
        e->gate_slot = slot;
        e->gate_key = gkey;
        gate_done = true;
      }
      if (r >= 3)
        if (const int rc = reuse(r - 2)) return rc;
      const uint8_t kind = e->round_kind[r];
      if (kind == PS_K_PAIR2 || kind == PS_K_CHAIN2) continue;  // written by the launch of an earlier round
      a.a_cur = upfront ? arr[0] : arr[(r - 1) & 1];
      a.a_next = arr[r & 1];
      pa.a_cur = a.a_cur;
      // N ranks: this round's records (rows the last round wrote; the
      // seeded roots' packed now) go to the ranks owning their children on
      // the exchange stream, while this round's locally fed chunks run; the
      // ghost-fed chunks wait for the exchange
      const bool xr = world > 1 && r < e->ghost.rounds.size() && e->ghost.rounds[r].any;
      hipStream_t xs = e->xchg_overlap ? e->xstream : s;
      if (xr) {
        const GhostRound& R = e->ghost.rounds[r];
        if (R.pack1 > R.pack0)
          HIP_TRY(launch_pack(e->d_ship.as<ShipEntry>(), e->d_pack.as<PackSeg>() + R.pack0, R.pack1 - R.pack0,
                              R.pack_units, e->d_gsegs.as<GhostSeg>(), a.seen, e->d_send.as<uint64_t>(), s),
                  "pack");
        if (xs != s) {
          HIP_TRY(hipEventRecord(e->ev_round, s), "event");
          HIP_TRY(hipStreamWaitEvent(xs, e->ev_round, 0), "exchange wait");
        }
        std::string xerr;
        st->xchg_path = e->inplace ? PS_XCHG_IN_PLACE : zero_copy ? PS_XCHG_ZERO_COPY : PS_XCHG_COPY;
        st->xchg_rounds += 1;
        st->xchg_bytes += R.rec_bytes;
        const uint8_t* sb = e->d_send.as<uint8_t>() + (r % kSendBufs) * e->ghost.send_half * 8;
        if (zero_copy) {
          // the ghost-fed nodes read each source's region in place: rsrc[a] is
          // offset so that the receive-side record bases (rbase) apply
          const hipError_t xe = e->transport->exchange_zc(sb, R.s_off, peer_region, xs, &xerr);
          if (xe != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
          for (int32_t q = 0; q < world && q < kMaxRanks; ++q)
            if (q != me && peer_region[q])
              pa.rsrc[q] = reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(peer_region[q]) -
                                                             R.r_off[q]);
        } else {
          const hipError_t xe = e->transport->exchange(sb, R.s_off, R.s_len, e->d_recv.as<uint8_t>(), R.r_off,
                                                       R.r_len, xs, &xerr);
          if (xe != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
        }
        if (xs != s) HIP_TRY(hipEventRecord(e->ev_xchg, xs), "event");
      }
      if (!lgrid[r] && !xr) {
        if (!upfront) HIP_TRY(seed_round(r, a.a_next), "seed");  // (messages starting this round)
        continue;
      }
      const bool pair = kind == PS_K_PAIR;
      if (kind == PS_K_CHAIN) {  // rounds r .. r + len - 1 in one launch (one rank, or no exchange inside)
        const uint32_t len = e->pair.len[r];
        const uint32_t last = r + len - 1;
        const bool ntc = last == planned0 || (last < e->pull.bytes.size() && e->pull.bytes[last] >= ps_engine::kNtBytes);
        pa.slot_mod = kPairSlots;
        pa.row_ptr = e->d_row_ptr.as<uint32_t>();
        for (uint32_t k = 0; k < kChainLevels; ++k)
          pa.partials_r[k] = k < len ? partials + static_cast<size_t>(e->woff_host[r + k]) * kNumCtr : nullptr;
        HIP_TRY(time_mark(true), "event");
        ++launches;
        uint64_t* const prof = cprof ? e->d_chain_prof.as<uint64_t>() : nullptr;
        pa.prof = prof ? prof + static_cast<size_t>(e->pair.lo[r]) * kChainProf : nullptr;
        HIP_TRY(launch_pull_chain(pa, e->d_chain.as<ChainChunk>() + e->pair.lo[r], e->pair.gsplit[r] - e->pair.lo[r],
                                  r, record, ntc, false, e->chain_nt, e->chain_waves, s),
                "pull chain");
        pa.prof = prof ? prof + static_cast<size_t>(e->pair.gsplit[r]) * kChainProf : nullptr;
        HIP_TRY(launch_pull_chain(pa, e->d_chain.as<ChainChunk>() + e->pair.gsplit[r],
                                  e->pair.hi[r] - e->pair.gsplit[r], r, record, ntc, true, e->chain_nt,
                                  e->chain_waves, s),
                "pull chain (column slices)");
        pa.prof = nullptr;
        HIP_TRY(time_mark(false), "event");
        if (xr) HIP_TRY(hipStreamWaitEvent(s, e->ev_xchg, 0), "exchange join");  // (never: chains skip exchange rounds)
        continue;
      }
      // rows nobody re-reads while they can still sit in the 256 MB MALL
      // (large rounds and the last round) store non-temporally
      const uint32_t rw = pair ? r + 1 : r;  // the round whose rows the next launch reads
      const bool nt = rw < e->pull.bytes.size() && (e->pull.bytes[rw] >= ps_engine::kNtBytes || rw == planned0);
      pa.partials = partials + static_cast<size_t>(e->woff_host[r]) * kNumCtr;
      pa.slot_mod = pair ? kPairSlots : kPullSlots;
      if (pair) pa.partials2 = partials + static_cast<size_t>(e->woff_host[r + 1]) * kNumCtr;
      // the locally fed part, then (after the exchange) the ghost-fed part;
      // without the overlap (PSAMD_XCHG_OVERLAP=0) one launch after the exchange
      const bool split = xs != s;
      for (int part = split ? 0 : 1; part < 2; ++part) {
        if (part == 1 && xr && split) HIP_TRY(hipStreamWaitEvent(s, e->ev_xchg, 0), "exchange join");
        uint32_t c0, c1;
        if (pair) {
          c0 = part ? (split ? e->pair.gsplit[r] : e->pair.lo[r]) : e->pair.lo[r];
          c1 = part ? e->pair.hi[r] : e->pair.gsplit[r];
        } else {
          c0 = part ? (split ? e->pull.gsplit[r] : e->pull.off[r]) : e->pull.off[r];
          c1 = part ? e->pull.off[r + 1] : e->pull.gsplit[r];
        }
        if (c1 <= c0) continue;
        HIP_TRY(time_mark(true), "event");
        ++launches;
        if (pair) {
          HIP_TRY(launch_pull_pair(pa, e->d_pp.as<PullChunk>() + c0, c1 - c0, c1 - c0, r, record, nt, s),
                  "pull pair");
        } else {
          // one rank: big rounds at 5 blocks per CU (+6 %); N ranks keep full
          // residency (4 loopback ranks on one GPU: 6.49 -> 7.13 ms capped)
          HIP_TRY(launch_pull(pa, e->d_pull.as<PullChunk>() + c0, c1 - c0, ceil_div(c1 - c0, kBlock / 64), r,
                              record, nt, world == 1, s),
                  "pull");
        }
        HIP_TRY(time_mark(false), "event");
      }
      if (xr && zero_copy) {  // the sources' regions of round r: read once the launches above end
        std::string xerr;
        if (e->transport->consumed(s, r, &xerr) != hipSuccess) return e->fail(PS_E_DEVICE, xerr);
      }
      if (!upfront) HIP_TRY(seed_round(r, a.a_next), "seed");
    }
    if (!twin && s != e->stream) {  // (a prefix never ends a window; kept safe)
      HIP_TRY(hipEventRecord(e->ev_pre, s), "event");
      s = e->stream;
      HIP_TRY(hipStreamWaitEvent(s, e->ev_pre, 0), "prefix join");
    }
    // the window's last two exchange rounds: before the next window writes
    if (planned0 >= 2)
      if (const int rc = reuse(planned0 - 1)) return rc;
    if (const int rc = reuse(planned0)) return rc;
    r = planned0;
    // a deferred window's counters go straight into its pinned rows
    const bool direct = e->defer_last && e->defer_into && !record && !timed && r <= PS_MAX_ROUNDS &&
                        (world == 1 || planned0 <= PS_MAX_ROUNDS);
    host_stats_written = direct;
    // a pipelined window's reduce runs on its own stream, beside the next
    // window's first launches (its partial slots and descriptors are this
    // slot's; ps_wait waits for it through the window's end event)
    hipStream_t rs = s;
    if (direct && world == 1 && !sigwin) {  // (the next window's launches never wait for it)
      if (!e->rstream) HIP_TRY(hipStreamCreateWithFlags(&e->rstream, hipStreamNonBlocking), "reduce stream");
      if (!e->ev_end) HIP_TRY(hipEventCreateWithFlags(&e->ev_end, kStreamEvent), "reduce event");
      HIP_TRY(hipEventRecord(e->ev_end, s), "event");
      HIP_TRY(hipStreamWaitEvent(e->rstream, e->ev_end, 0), "reduce wait");
      rs = e->rstream;
    }
    reduce_side = rs != s;
    // level-aligned: each (topic, level)'s reached and frontier nodes, for
    // the per-round split (into the pseudo-slots after the rounds'); with
    // alternating row sets on the reduce's stream, beside the next window
    // (its generation bytes are the other set's)
    if (L.aligned && e->n_reach) {
      const uint32_t from = reach_a_done ? reach_a : 0u;
      HIP_TRY(launch_level_reach(e->d_reach.as<ReachPiece>() + from, e->n_reach - from, a.gen, a.gen_cur,
                                 a.node_flags, a.topics, a.seen, L.split.eager,
                                 partials + static_cast<size_t>(reach_slot0) * kNumCtr,
                                 alt_sets && reduce_side ? rs : s),
              "level reach");
    }
    // a signalled window: the reduce's last block raises its flag
    WindowSignal wsig{};
    if (sigwin && direct && !reduce_side && (s == e->stream || twin)) {
      if (!e->d_sigctr.p) {  // (one counter per slot, a line apart: twin windows reduce side by side)
        HIP_TRY(e->d_sigctr.ensure(256), "alloc window counter");
        HIP_TRY(hipMemsetAsync(e->d_sigctr.p, 0, 256, s), "clear window counter");
        if (s != e->stream) HIP_TRY(hipStreamSynchronize(s), "sync");  // (before `stream`'s windows use it)
      }
      wsig.flag = e->defer_into->sig_dev;
      wsig.ctr = e->d_sigctr.as<uint32_t>() + 32 * slot;
      wsig.seq = ++e->sig_seq;
      e->defer_into->seq = wsig.seq;
    }
    // (beside other windows it writes only the slot's pinned rows, not the shared device rows)
    if (wsig.flag && e->fuse_reduce && planned0 > 0 && !twin) {
      // held back for the next window's first launch (k_window_turn); only
      // this slot's buffers and the pinned rows: the shared device stats rows
      // may be reallocated by then, and nobody reads a deferred window's
      e->pend_reduce.valid = true;
      e->pend_reduce.owner = e->defer_into;
      e->pend_reduce.args =
          ReduceArgs{partials, d_woff.as<uint32_t>(), planned0 + reach_rows, nullptr, e->defer_into->hs_dev, wsig};
    } else {
      // (twin windows reduce side by side: neither writes the shared device rows)
      HIP_TRY(launch_reduce_rounds(partials, d_woff.as<uint32_t>(), planned0 + reach_rows,
                                   (reduce_side || twin) ? nullptr : stats,
                                   direct ? e->defer_into->hs_dev : nullptr, wsig, rs),
              "reduce rounds");
    }
    e->defer_into_signalled = wsig.flag != nullptr;
    if (twin && s == e->tstream) {  // (for twin_join)
      HIP_TRY(hipEventRecord(e->ev_tend, s), "event");
      e->t_pending = true;
    }
  } else {
    e->round_kind.clear();  // (accumulate_window: every round k_expand)
    uint32_t* ext[2] = {nullptr, nullptr};
    if (world == 1) {  // (ghost-fed rows arrive whole: N ranks keep whole rows)
      HIP_TRY(e->d_ext0.ensure(static_cast<size_t>(e->n_pad) * 4), "alloc extents");
      HIP_TRY(e->d_ext1.ensure(static_cast<size_t>(e->n_pad) * 4), "alloc extents");
      ext[0] = e->d_ext0.as<uint32_t>();
      ext[1] = e->d_ext1.as<uint32_t>();
    }
    HIP_TRY(seed_round(0, arr[0]), "seed");
    HIP_TRY(compact(0, 0), "compact");
    while (true) {
      for (; r < planned && r < round_cap;) {
        ++r;
        a.a_cur = arr[(r - 1) & 1];
        a.a_next = arr[r & 1];
        a.ext_cur = ext[(r - 1) & 1];
        a.ext_next = ext[r & 1];
        const bool xr = layout(r);
        if (xr)
          for (int32_t q = 0; q < world; ++q)
            if (s_len[q]) HIP_TRY(hipMemsetAsync(a.send + s_off[q], 0, kRegionHeader, s), "reset header");
        HIP_TRY(time_mark(true), "event");
        ++launches;
        const uint32_t grid_r = r <= planned0 ? round_grid(r) : e->expand_grid;
        a.partials = partials;
        HIP_TRY(launch_expand(a, r, record, grid_r, s), "expand");
        uint32_t waves_r = grid_r * (kBlock / 64);
        if (need_direct) {
          a.partials = partials + static_cast<size_t>(waves_r) * kNumCtr;
          HIP_TRY(launch_expand_direct(a, r, record, e->expand_grid, s), "expand direct");
          waves_r += n_waves;
        }
        HIP_TRY(time_mark(false), "event");
        if (xr) {
          const int rc3 = xchg(r);
          if (rc3) return rc3;
        }
        HIP_TRY(seed_round(r, a.a_next), "seed");
        HIP_TRY(compact(r, waves_r), "compact");
      }
      uint32_t left = 0;
      HIP_TRY(hipMemcpyAsync(&left, e->d_nfront.p, 4, hipMemcpyDeviceToHost, s), "read frontier");
      HIP_TRY(hipStreamSynchronize(s), "sync");
      if (left == 0 || r >= round_cap) {
        if (left) return e->fail(PS_E_STATE, "propagation did not converge");
        break;
      }
      if (world > 1) return e->fail(PS_E_STATE, "multi-GPU frontier outlived the planned rounds");
      planned = r + 8;  // live mask lengthened a mesh path beyond the BFS depth
      if (planned + 1 > stats_rows) {  // grow the round rows, keeping the counted ones
        const uint32_t rows = std::min<uint32_t>(round_cap, std::max(planned + 1, 2 * stats_rows));
        DevBuf grown;
        HIP_TRY(grown.ensure(static_cast<size_t>(rows + 1) * kNumCtr * 8), "grow stats");
        HIP_TRY(hipMemcpyAsync(grown.p, e->d_stats.p, static_cast<size_t>(stats_rows + 1) * kNumCtr * 8,
                               hipMemcpyDeviceToDevice, s),
                "keep stats");
        HIP_TRY(hipStreamSynchronize(s), "sync");
        std::swap(grown.p, e->d_stats.p);
        std::swap(grown.bytes, e->d_stats.bytes);
        stats = e->d_stats.as<uint64_t>();
        stats_rows = rows;
      }
    }
  }
  const bool defer = e->defer_last && e->defer_into && !record && !timed && r <= PS_MAX_ROUNDS &&
                     (world == 1 || planned0 <= PS_MAX_ROUNDS);  // the pinned slots hold PS_MAX_ROUNDS + 1 rows
  e->last_win_stream = s;
  if (!defer) HIP_TRY(hipEventRecord(e->ev_run1, s), "event");
  const auto t_enq = std::chrono::steady_clock::now();
  auto remember = [&]() {
    // the last window, for ps_read_delivered / ps_read_peer_messages / ps_seen_digest
    e->last_topics = tab;
    for (uint32_t t = 0; t < nt; ++t) {
      e->last_cnt[t] = tab[t].W ? win[t].n : 0;
      e->last_lo[t] = win[t].n ? e->run_rank[win[t].idx[0]] : 0;
    }
    e->last_pos.swap(L.pos);
    e->last_groups.swap(L.groups);
    e->have_window = true;
    e->last_slot = slot;
  };
  if (defer) {
    // asynchronous run: the counters follow the kernels on the stream into
    // pinned memory (level mode: written there by the reduce itself); the
    // window's end event marks their arrival; ps_wait accumulates them
    ps_engine::Inflight& f = *e->defer_into;
    if (!host_stats_written)
      HIP_TRY(hipMemcpyAsync(f.hs, stats, static_cast<size_t>(r + 1 + reach_rows) * kNumCtr * 8,
                             hipMemcpyDeviceToHost, s),
              "read stats");
    if (world > 1)
      HIP_TRY(hipMemcpyAsync(f.ha, e->d_apply_stats.p, static_cast<size_t>(planned0 + 1) * kNumCtr * 8,
                             hipMemcpyDeviceToHost, s),
              "read apply stats");
    f.signalled = e->defer_into_signalled;  // (its flag rises with the reduce)
    if (!f.signalled) HIP_TRY(hipEventRecord(e->ev_run1, reduce_side ? e->rstream : s), "event");
    f.deferred = true;
    f.planned0 = planned0;
    f.true_rounds = L.aligned ? L.true_rounds : 0u;
    if (L.aligned)
      f.split = L.split;
    else
      f.split.n_segs = 0;
    f.world = world;
    f.r = r;
    f.launches = launches;
    f.mode = mode;
    f.flood_rounds = flood_rounds;
    f.kinds = e->round_kind;
    f.stream = s;
    remember();
    if (e->host_timing) {
      auto ms = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
      std::fprintf(stderr, "[psengine] async window: plan %.3f ms (run->window %.3f, topics %.3f, seeds %.3f, "
                   "schedule %.3f, uploads %.3f), enqueue %.3f ms, prefix P %u%s\n",
                   ms(e->t_run0, t_first), ms(e->t_run0, t_w0), ms(t_w0, t_w1), ms(t_w1, t_w2), ms(t_w2, t_w3),
                   ms(t_w3, t_first), ms(t_first, t_enq), pre_P, overlap ? " (beside the previous window)" : "");
    }
    return PS_OK;
  }
  HIP_TRY(hipEventSynchronize(e->ev_run1), "sync");
  const auto t_sync = std::chrono::steady_clock::now();
  const ps_stats keep = *st;  // a k_flood timeout re-runs the window from these stats
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e->ev_run0, e->ev_run1), "elapsed");
  st->run_ms += ms;
  for (size_t i = 0; i < ev_used; i += 2) {
    float k = 0.f;
    HIP_TRY(hipEventElapsedTime(&k, e->ev_k[i], e->ev_k[i + 1]), "elapsed");
    st->expand_ms += k;
    const size_t q = ev_round[i / 2];  // round of this launch
    if (q < PS_MAX_ROUNDS) st->expand_ms_per_round[q] += k;
  }
  std::vector<uint64_t> hs(static_cast<size_t>(r + 1 + reach_rows) * kNumCtr), ha;
  HIP_TRY(hipMemcpyAsync(hs.data(), stats, hs.size() * 8, hipMemcpyDeviceToHost, s), "read stats");
  if (world > 1) {
    ha.resize(static_cast<size_t>(planned0 + 1) * kNumCtr);
    HIP_TRY(hipMemcpyAsync(ha.data(), e->d_apply_stats.p, ha.size() * 8, hipMemcpyDeviceToHost, s),
            "read apply stats");
  }
  HIP_TRY(hipStreamSynchronize(s), "sync");
  if (mode == PS_MODE_FLOOD && e->flood_profile && e->flood_prof_waves) flood_profile_report(e);
  if (cprof) chain_profile_dump(e, planned0);
  if (std::string why; L.aligned && !split_aligned_window(st, hs.data(), r, L.true_rounds, L.split, &why))
    return e->fail(PS_E_DEVICE, "level-aligned window: reach counts disagree with the per-level counters (" + why + ")");
  if (!accumulate_window(st, hs.data(), ha.data(), r, planned0, mode, flood_rounds, launches, world,
                         e->round_kind, !L.aligned)) {
    // a k_flood dependency wait timed out (its waves were not all resident:
    // another engine or process shares the GPU): this window's rows are
    // incomplete.  Run the same window again with per-round launches under a
    // fresh generation, and keep those from now on.
    e->flood_broken = true;
    *st = keep;
    if (e->host_timing) std::fprintf(stderr, "[psengine] k_flood timed out: window re-run per round\n");
    return run_window(e, msgs, win, st);
  }
  if (e->host_timing) {
    auto ms2 = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    std::fprintf(stderr, "[psengine] window: plan %.3f ms (run->window %.3f, topics %.3f, seeds %.3f, "
                 "schedule %.3f, uploads %.3f), enqueue %.3f ms, wait %.3f ms, tail %.3f ms\n",
                 ms2(e->t_run0, t_first), ms2(e->t_run0, t_w0), ms2(t_w0, t_w1), ms2(t_w1, t_w2), ms2(t_w2, t_w3),
                 ms2(t_w3, t_first), ms2(t_first, t_enq), ms2(t_enq, t_sync),
                 ms2(t_sync, std::chrono::steady_clock::now()));
  }
  if (record) {
    {
      int rcm = ensure_mirrors(e);
      if (rcm) return rcm;
    }
    std::vector<uint16_t> hr(wtot * 64);
    if (!hr.empty()) {
      HIP_TRY(hipMemcpyAsync(hr.data(), e->d_hop.p, hr.size() * 2, hipMemcpyDeviceToHost, s), "read hops");
      HIP_TRY(hipStreamSynchronize(s), "sync");
    }
    const uint32_t np = e->cfg.n_peers;
    for (uint32_t t = 0; t < nt; ++t) {
      const TopicDev& d = tab[t];
      if (d.W == 0) continue;
      for (uint32_t li = 0; li < win[t].n; ++li) {
        const uint32_t mi = win[t].idx[li];
        const uint32_t s0 = L.aligned ? 0u : msgs[mi].start;  // (level-aligned: the record holds the level)
        const uint32_t b = L.pos[t].empty() ? li : L.pos[t][li];
        uint8_t* row = e->hops.data() + static_cast<size_t>(mi) * np;
        for (uint32_t u = 0; u < d.n_nodes; ++u) {
          const uint16_t v = hr[phys(t, u, b >> 6) * 64 + (b & 63)];
          // hop = round - start round, saturated at 254 (0xFF: not delivered)
          if (v != kHopRecNone) row[e->node_peer[d.nbase + u]] = static_cast<uint8_t>(std::min<uint32_t>(v - s0, 254u));
        }
      }
    }
  }
  remember();
  return PS_OK;
}

// Messages of one phase (per topic, a slice of the run's topic-sorted index
// array), split into windows of at most msg_window messages per topic.
int run_phase(ps_engine* e, const std::vector<RunMsg>& msgs, const std::vector<WinSlice>& per, ps_stats* st) {
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  const uint32_t cap = e->cfg.msg_window;
  uint32_t n_win = 0;
  for (const auto& v : per) n_win = std::max(n_win, (v.n + cap - 1) / cap);
  std::vector<WinSlice> win(nt);
  for (uint32_t k = 0; k < n_win; ++k) {
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t lo = k * cap;
      win[t].idx = per[t].idx + std::min(lo, per[t].n);
      win[t].n = lo < per[t].n ? std::min(cap, per[t].n - lo) : 0;
    }
    e->defer_last = e->defer_phase && k + 1 == n_win;
    int rc = run_window(e, msgs, win, st);
    e->defer_last = false;
    if (rc) return rc;
  }
  return PS_OK;
}

}  // namespace

// Counters of one window (rows r x kNumCtr, apply rows for multi-GPU) into
// the run's stats.  Returns false when a k_flood dependency wait timed out
// (its timeout word is folded into row 0).
bool accumulate_window(ps_stats* st, const uint64_t* hs, const uint64_t* ha, uint32_t r, uint32_t planned0,
                       uint32_t mode, uint32_t flood_rounds, uint32_t launches, int32_t world,
                       const std::vector<uint8_t>& kinds, bool by_round) {
  const bool pull = mode == PS_MODE_LEVEL_PULL || mode == PS_MODE_FLOOD;
  std::memset(st->round_kernel, 0, sizeof(st->round_kernel));
  for (uint32_t q = 1; q <= r; ++q) {
    const uint8_t kind = q < kinds.size() ? kinds[q] : static_cast<uint8_t>(pull ? PS_K_PULL : PS_K_EXPAND);
    const uint64_t* c = &hs[static_cast<size_t>(q) * kNumCtr];
    const uint64_t app_d = (world > 1 && q <= planned0) ? ha[static_cast<size_t>(q) * kNumCtr + kCtrDeliveries] : 0;
    const uint64_t app_u = (world > 1 && q <= planned0) ? ha[static_cast<size_t>(q) * kNumCtr + kCtrDuplicates] : 0;
    st->deliveries += c[kCtrDeliveries] + app_d;
    st->duplicates += c[kCtrDuplicates] + app_u;
    st->frontier_entries += c[kCtrEntries];
    st->child_visits += c[kCtrChildren];
    st->edge_words += c[kCtrSeenWrites];
    // algorithmic bytes of the expand kernel (DESIGN.md §5.1 byte model):
    // per entry frontier id 4 + topic 2 + row_ptr pair 8 + first child 4;
    // per entry word the arrival read 8 (+ 8 when cleared); per child its
    // flag byte + generation read/write (tree) or col id 4 (mesh); per
    // seen read / seen write / arrival write 8.
    uint64_t b;
    if (pull)  // pull model: per node parent id 4 + flag 1 + parent generation 1 (k_flood:
               // + its own generation 1, the seen test; the second round of a k_pull_pair
               // launch: no parent generation, its parents' reach and rows are in LDS),
               // per reached node its generation write 1; parent rows read once (from
               // HBM: none in a pair's second round); rows written
      b = c[kCtrChildren] * (kind == PS_K_FLOOD ? 7 : (kind == PS_K_PAIR2 || kind == PS_K_CHAIN2) ? 5 : 6) +
          c[kCtrMeshChildren] * 1 +
          c[kCtrEntryWords] * 8 + c[kCtrSeenWrites] * 8;
    else
      b = c[kCtrEntries] * 18 + c[kCtrEntryWords] * 8 + c[kCtrClearWords] * 8 + c[kCtrChildren] * 3 +
          c[kCtrMeshChildren] * 4 + c[kCtrSeenReads] * 8 + c[kCtrSeenWrites] * 8 + c[kCtrArrivalWrites] * 8;
    st->expand_bytes += b;
    if (q < PS_MAX_ROUNDS) {
      st->round_kernel[q] = kind;
      st->expand_bytes_per_round[q] += b;
      if (by_round) {  // (level-aligned windows: split_aligned_window)
        st->deliveries_per_round[q] += c[kCtrDeliveries] + app_d;
        st->frontier_per_round[q] += static_cast<uint32_t>(c[kCtrEntries]);
      }
    }
  }
  st->rounds += by_round ? r : 0;
  st->level_aligned = by_round ? 0u : 1u;
  st->expand_launches += launches;
  st->expand_mode = mode;
  st->flood_rounds = flood_rounds;
  st->windows += 1;
  return mode != PS_MODE_FLOOD || hs[kCtrDeliveries] == 0;
}

// A level-aligned window: row d (1 .. r) holds the
// kernels' counters of BFS level d over every topic; the reach rows after
// them, per (topic, level) segment, the reached nodes and the frontier
// nodes.  Level d of topic t delivers each message of group g (start s_g,
// n_g messages) to every reached node in round s_g + d -- the reached node
// holds its root's row, every message of the topic -- and expands the
// frontier nodes of level d - 1 in that round.  Both are checked, level by
// level, against the kernels' own popcounts and parent counts first.
bool split_aligned_window(ps_stats* st, const uint64_t* hs, uint32_t r, uint32_t true_rounds,
                          const AlignedSplit& sp, std::string* why) {
  const uint64_t* reach = hs + static_cast<size_t>(r + 1) * kNumCtr;  // 2 per segment
  const uint32_t nt = static_cast<uint32_t>(sp.seg_lo.size());
  std::vector<uint64_t> deliv(r + 1, 0), front(r + 1, 0);
  for (uint32_t t = 0; t < nt; ++t) {
    if (sp.seg_lo[t] == kNone) continue;
    uint64_t n_msgs = 0;
    for (const AlignedGroup& g : sp.groups[t]) n_msgs += g.n;
    for (uint32_t d = 1; d < sp.seg_n[t] && d <= r; ++d) {
      const uint64_t reached = reach[2 * (sp.seg_lo[t] + d)], fr = reach[2 * (sp.seg_lo[t] + d - 1) + 1];
      deliv[d] += reached * n_msgs;
      front[d] += fr;
      for (const AlignedGroup& g : sp.groups[t]) {
        const uint32_t rt = g.start + d;
        if (rt < PS_MAX_ROUNDS) {
          st->deliveries_per_round[rt] += reached * g.n;
          st->frontier_per_round[rt] += static_cast<uint32_t>(fr);
        }
      }
    }
  }
  bool ok = true;
  for (uint32_t d = 1; d <= r; ++d) {
    const uint64_t* c = &hs[static_cast<size_t>(d) * kNumCtr];
    // (eager seen, PS_F_NO_LAZY_SEEN: every generation is stamped up front and
    // the level kernels count parents by their own reach tests -- k_flood's
    // granules, the pull kernels' stamps -- so only the deliveries compare)
    if (c[kCtrDeliveries] != deliv[d] || (!sp.eager && c[kCtrEntries] != front[d])) {
      if (ok && why)
        *why = "level " + std::to_string(d) + ": deliveries " + std::to_string(c[kCtrDeliveries]) + " vs " +
               std::to_string(deliv[d]) + ", frontier " + std::to_string(c[kCtrEntries]) + " vs " +
               std::to_string(front[d]);
      ok = false;
    }
  }
  st->rounds += true_rounds;
  return ok;
}

// ps_run's body.  may_defer: the last window of the final phase may leave its
// counters on the stream (ps_run_async); *stp is completed by ps_wait then.
int run_body(ps_engine* e, ps_stats* stp, bool may_defer) {
  const auto t_host0 = std::chrono::steady_clock::now();
  e->t_run0 = t_host0;
  ps_stats& st = *stp;
  if (hipSetDevice(e->cfg.device) != hipSuccess) return e->fail(PS_E_DEVICE, "hipSetDevice");
  e->last_msgs.clear();
  e->last_msgs.swap(e->pending);
  e->run_zero_start = !e->pending_nonzero_start;
  e->pending_nonzero_start = false;
  const std::vector<RunMsg>& msgs = e->last_msgs;
  const uint32_t nmsg = static_cast<uint32_t>(msgs.size());
  e->last_first = e->next_msg - nmsg;
  e->last_n = nmsg;
  e->have_hops = false;
  e->have_window = false;
  const bool record = (e->cfg.flags & PS_F_RECORD_HOPS) != 0;
  if (record) {
    const uint64_t bytes = static_cast<uint64_t>(nmsg) * e->cfg.n_peers;
    if (bytes > (8ull << 30)) return e->fail(PS_E_NOMEM, "hop record larger than 8 GiB");
    e->hops.assign(bytes, PS_HOP_NONE);
  }
  const uint32_t nt = static_cast<uint32_t>(e->topics.size());
  // one counting sort: message indices grouped by topic, publish order kept
  // (a batch of one topic: the identity, kept from the last such run)
  auto& off = e->run_topic_off;
  off.assign(nt + 1, 0);
  if (nmsg && !e->pending_mixed) {
    for (uint32_t t = e->pending_topic0 + 1; t <= nt; ++t) off[t] = nmsg;
    if (e->run_iota_n != nmsg) {
      e->run_sorted.resize(nmsg);
      e->run_rank.resize(nmsg);
      for (uint32_t i = 0; i < nmsg; ++i) e->run_sorted[i] = e->run_rank[i] = i;
      e->run_iota_n = nmsg;
    }
  } else {
    e->run_iota_n = 0;
    for (uint32_t i = 0; i < nmsg; ++i) off[msgs[i].topic + 1]++;
    for (uint32_t t = 0; t < nt; ++t) off[t + 1] += off[t];
    e->run_sorted.resize(nmsg);
    e->run_rank.resize(nmsg);
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint32_t i = 0; i < nmsg; ++i) {
      const uint32_t t = msgs[i].topic;
      e->run_rank[i] = fill[t] - off[t];
      e->run_sorted[fill[t]++] = i;
    }
  }
  e->pending_mixed = false;
  e->last_lo.assign(nt, 0);
  e->last_cnt.assign(nt, 0);
  std::vector<uint32_t> head(nt, 0);
  auto slice = [&](uint32_t t, uint32_t from, uint32_t n) {
    WinSlice w;
    w.idx = e->run_sorted.data() + off[t] + from;
    w.n = n;
    return w;
  };
  // Abruptly dropped hosts: the first message through the failed edge is lost
  // below it, then the parent repairs (subtree.go:333-351): that message runs
  // on its own over the current tree, the rest over the repaired one.
  while (true) {
    std::vector<WinSlice> solo(nt);
    bool any = false;
    for (uint32_t t = 0; t < nt; ++t) {
      TopicHost& T = e->topics[t];
      const uint32_t cnt = off[t + 1] - off[t];
      if (T.exists && T.kind == Kind::Join && T.tree.has_pending_failures() && head[t] < cnt) {
        solo[t] = slice(t, head[t], 1);
        head[t]++;
        any = true;
      }
    }
    if (!any) break;
    int rc = run_phase(e, msgs, solo, &st);
    if (rc) return rc;
    for (uint32_t t = 0; t < nt; ++t)
      if (solo[t].n) {
        e->topics[t].tree.after_message();
        e->graph_dirty = true;
      }
  }
  {
    std::vector<WinSlice> rest(nt);
    bool any = false;
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t cnt = off[t + 1] - off[t];
      rest[t] = slice(t, head[t], cnt - head[t]);
      any |= rest[t].n > 0;
    }
    // the prune's questions, asked with this phase's rebuild (graph.cpp)
    e->early_q.clear();
    if (any && e->graph_dirty && e->gpu_build_on)
      for (uint32_t t = 0; t < nt; ++t) {
        TopicHost& T = e->topics[t];
        if (!(T.exists && T.kind == Kind::Join && rest[t].n && T.tree.parts_only_pass())) continue;
        ps_engine::EarlyQuery q;
        q.topic = t;
        q.peers = T.tree.part_parents();
        if (!q.peers.empty()) e->early_q.push_back(std::move(q));
      }
    if (any) {
      e->defer_phase = may_defer && !record;
      int rc = run_phase(e, msgs, rest, &st);
      e->defer_phase = false;
      if (rc) return rc;
    }
  }
  // lazy prune of Part'ed children at every forwarding node (subtree.go:326-331)
  const auto t_am = std::chrono::steady_clock::now();
  const bool gpu_reach = e->gpu_graph && !e->graph_dirty;  // the node space the messages ran on
  for (uint32_t t = 0; t < nt; ++t) {
    TopicHost& T = e->topics[t];
    if (T.exists && T.kind == Kind::Join && head[t] < off[t + 1] - off[t] && T.tree.needs_message_pass()) {
      // on a GPU-built node space the message's reach is a lookup there (a
      // host walk to the root per Part'ed parent costs ~0.2 us each)
      SubscriptionTree::ReachQuery q = [e, &T](const std::vector<uint32_t>& peers, std::vector<uint8_t>& outv) -> int {
        const uint32_t k = static_cast<uint32_t>(peers.size());
        if (!k) return PS_OK;
        for (const ps_engine::EarlyQuery& eq : e->early_q)  // answered with the rebuild
          if (eq.ready && eq.topic == static_cast<uint32_t>(&T - e->topics.data()) && eq.peers.size() == k &&
              std::equal(peers.begin(), peers.end(), eq.peers.begin())) {
            outv = eq.out;
            if (e->host_timing) std::fprintf(stderr, "[psengine] prune reach query: %u parents, from the rebuild\n", k);
            return PS_OK;
          }
        // (its own stream: the GPU build ended with a stream sync, so the node
        // space it reads is complete; the window's kernels need not finish)
        if (!e->qstream) HIP_TRY(hipStreamCreateWithFlags(&e->qstream, hipStreamNonBlocking), "query stream");
        hipStream_t qs = e->qstream;
        HIP_TRY(e->d_query.ensure(static_cast<size_t>(k) * 4 + k + 16), "alloc reach query");
        uint32_t* dp = e->d_query.as<uint32_t>();
        uint8_t* dout = reinterpret_cast<uint8_t*>(dp + k);
        HIP_TRY(hipMemcpyAsync(dp, peers.data(), static_cast<size_t>(k) * 4, hipMemcpyHostToDevice, qs),
                "upload reach query");
        const size_t toff = static_cast<size_t>(&T - e->topics.data()) * e->cfg.n_peers;
        HIP_TRY(launch_reach_query(dp, k, e->cfg.n_peers, e->d_tpar.as<uint32_t>() + toff,
                                   e->d_orph.as<uint8_t>() + toff, T.tree.root(), dout, qs),
                "reach query");
        HIP_TRY(hipMemcpyAsync(outv.data(), dout, k, hipMemcpyDeviceToHost, qs), "read reach query");
        HIP_TRY(hipStreamSynchronize(qs), "sync");
        if (e->host_timing)
          std::fprintf(stderr, "[psengine] prune reach query: %u parents, done at %.3f ms\n", k,
                       std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - e->t_run0).count());
        return PS_OK;
      };
      int rc = T.tree.after_message(gpu_reach ? &q : nullptr);
      if (rc) return rc;
      e->graph_dirty = true;
    }
  }
  e->early_q.clear();
  e->have_hops = record;
  if (e->host_timing)
    std::fprintf(stderr, "[psengine] after-message prune %.3f ms (started at %.3f ms)\n",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_am).count(),
                 std::chrono::duration<double, std::milli>(t_am - e->t_run0).count());
  st.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_host0).count();
  return PS_OK;
}

}  // namespace psamd

using namespace psamd;

extern "C" {

int ps_run(ps_engine* e, ps_stats* out) {
  if (!e) return PS_E_INVAL;
  if (e->host_only) return e->fail(PS_E_STATE, "planner probe: no device");
  if (e->infl_count) return e->fail(PS_E_STATE, "asynchronous runs pending: ps_wait first");
  ps_stats st{};
  const int rc = run_body(e, &st, false);
  if (rc) {
    e->upload_shadow.clear();  // (a failed window's staged copies may not have run)
    return rc;
  }
  if (out) *out = st;
  return PS_OK;
}

int ps_run_async(ps_engine* e) {
  if (!e) return PS_E_INVAL;
  if (e->host_only) return e->fail(PS_E_STATE, "planner probe: no device");
  if (e->infl_count >= 2) return e->fail(PS_E_STATE, "two runs in flight: ps_wait first");
  ps_engine::Inflight& f = e->infl[(e->infl_head + e->infl_count) % 2];
  f.st = ps_stats{};
  f.deferred = false;
  f.stream = nullptr;
  hipEvent_t ev0 = e->ev_run0, ev1 = e->ev_run1;
  e->ev_run0 = f.ev0;  // this run's window events belong to its slot
  e->ev_run1 = f.ev1;
  e->defer_into = &f;
  const int rc = run_body(e, &f.st, true);
  e->ev_run0 = ev0;
  e->ev_run1 = ev1;
  e->defer_into = nullptr;
  if (rc) {
    // a failed window may have left its init and prefix on pstream or a
    // reduce on rstream: drain every stream, and let no later window start
    // beside a gate this one recorded
    (void)hipStreamSynchronize(e->stream);
    for (hipStream_t x : {e->pstream, e->rstream, e->xstream, e->tstream})
      if (x) (void)hipStreamSynchronize(x);
    e->t_pending = false;
    e->gate_valid = false;
    e->upload_shadow.clear();  // (a failed window's staged copies may not have run)
    if (e->pend_reduce.owner == &f) e->pend_reduce.valid = false;  // (its window failed: nobody waits for it)
    return rc;
  }
  ++e->infl_count;
  return PS_OK;
}

int ps_wait(ps_engine* e, ps_stats* out) {
  if (!e) return PS_E_INVAL;
  if (!e->infl_count) return e->fail(PS_E_NOTREADY, "no asynchronous run pending");
  ps_engine::Inflight& f = e->infl[e->infl_head];
  e->infl_head = (e->infl_head + 1) % 2;
  --e->infl_count;
  if (e->pend_reduce.valid && e->pend_reduce.owner == &f) {
    const int rc = flush_reduce(e);
    if (rc) return rc;
  }
  if (f.deferred && f.signalled) {
    // poll the window's flag (pinned, written after its reduce); a stream
    // that has drained or failed without it is an error, not a hang
    const volatile uint64_t* flag = f.sig;
    // Back-off: pause-spin for the first ~50 us (a cfg2 window
    // is ~50 us: a sleep's timer slack would cost a step), then yield the
    // core between polls, and past 2 ms sleep 20 us per poll -- a caller
    // publishing the next batch from another thread is not starved
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0; *flag != f.seq; ++spin) {
      cpu_relax();
      if ((spin & 255) == 255) {
        const hipError_t q = hipStreamQuery(f.stream ? f.stream : e->stream);
        if (q != hipSuccess && q != hipErrorNotReady) return e->fail(PS_E_DEVICE, "window: stream failed");
        if (q == hipSuccess && *flag != f.seq) return e->fail(PS_E_DEVICE, "window: completion flag missing");
        const auto us =
            std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
        if (us > 2000)
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        else if (us > 50)
          std::this_thread::yield();
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const volatile uint64_t* t = f.sig;
    f.st.run_ms += static_cast<double>(t[2] - t[1]) * 1e-5;  // (s_memrealtime: 100 MHz)
  } else if (f.deferred) {
    HIP_TRY(hipEventSynchronize(f.ev1), "sync");
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, f.ev0, f.ev1), "elapsed");
    f.st.run_ms += ms;
  }
  if (f.deferred) {
    f.deferred = false;
    const bool aligned = f.split.n_segs > 0;
    if (std::string why; aligned && !split_aligned_window(&f.st, f.hs, f.r, f.true_rounds, f.split, &why))
      return e->fail(PS_E_DEVICE, "level-aligned window: reach counts disagree with the per-level counters (" + why +
                                      ")");
    if (!accumulate_window(&f.st, f.hs, f.ha, f.r, f.planned0, f.mode, f.flood_rounds, f.launches, f.world,
                           f.kinds, !aligned)) {
      e->flood_broken = true;
      return e->fail(PS_E_DEVICE, "k_flood: a dependency wait timed out (waves not co-resident?); "
                                  "per-round launches from now on");
    }
  }
  if (out) *out = f.st;
  return PS_OK;
}

}  // extern "C"
