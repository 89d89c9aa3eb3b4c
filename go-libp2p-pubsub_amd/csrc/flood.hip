// flood.hip -- k_flood: every round of a single-start tree window in ONE
// persistent launch.
//
// Reference: the recursive flood of subtree.forwardMessage (subtree.go:319-354)
// driven hop by hop by client.processMessages (client.go:100-132): round q
// delivers to BFS level q - s_t of every active topic t.  A node's row of
// 64-message words receives, in its round, its parent's row of the previous
// round -- if the parent was reached this window and the node is live (the
// dead child is skipped, subtree.go:326-331) -- through the seen test-and-set
// new = row(parent) & ~seen(node), seen(node) |= new, where a node whose
// generation byte is stale has seen nothing yet (lazy reset).
//
// Per-round launches (k_pull) separate the rounds by kernel boundaries.  Here
// the rounds are ordered by dataflow inside one launch:
//   * the host cuts every level of every topic into tasks (a run of at most
//     64 consecutive nodes of one level, about kFloodWords row words), listed
//     level by level: a topological order of "reads the rows the previous
//     round wrote";
//   * wave g of the G co-resident waves runs tasks g, g + G, g + 2G, ... in
//     order.  A task's lanes poll the granules of their parents -- 8-B words
//     {epoch, reach bits} its parents' tasks published -- until every one
//     carries this launch's epoch: that is both the dependency wait and the
//     frontier test (parent reached this window), in one load;
//   * the task then pulls the parents' rows, stores its own rows, and once
//     they have drained publishes its own granules.
// Hand-off (MI355X_MICROARCH.md §Workgroup dispatch... Valid forms; Guideline
// 16 R1/R2): rows are stored write-through (sc1 buffer stores) and drained
// before the granule store; granules are single 8-B agent-scope stores (data
// and tag together); every load of a handed-off byte is an sc1 load.  No
// fence, correct for any placement.
// Deadlock freedom: every dependency points to an earlier task, and the grid
// never exceeds the resident capacity, so the wave holding the earliest
// unfinished task always runs.  Every wait is bounded: a timeout sets *err
// (read back with the round counters) and the launch still completes.
#include "devutil.hpp"
#include "kernels.hpp"

namespace psamd {
namespace {

using namespace dev;


__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// The task record, wave-uniform (scalar registers: buffer descriptors built
// from it stay scalar, no per-lane loops).
__device__ __forceinline__ FloodTask uniform(FloodTask t) {
  t.nb = rfl(t.nb);
  t.ne = rfl(t.ne);
  t.topic = rfl(t.topic);
  t.round = rfl(t.round);
  t.slot0 = rfl(t.slot0);
  t.nslot = rfl(t.nslot);
  t.g_own = rfl(t.g_own);
  t.gsz = rfl(t.gsz);
  t.p_lo = rfl(t.p_lo);
  t.p_hi = rfl(t.p_hi);
  t.pg_lo = rfl(t.pg_lo);
  t.pnode0 = rfl(t.pnode0);
  t.pgsz = rfl(t.pgsz);
  return t;
}

__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Row kk = i / W and word r of word i of the run (float estimate, off by at
// most one; i < 2^24).
__device__ __forceinline__ void split_word(uint32_t i, float rw, uint32_t W, int32_t& kk, int32_t& r) {
  kk = static_cast<int32_t>(static_cast<float>(i) * rw);
  r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(W);
  const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(W);
  kk += hi - lo;
  r += (lo - hi) * static_cast<int32_t>(W);
}

// Stream, even W: the task's rows as one output stream of 16-B word pairs
// (rows and pairs 16-B aligned), each pair loaded from the parent row it
// receives.  8 loads in flight per lane, then 8 stores; a skipped node's pair
// and a lane past the end use an out-of-range offset (load 0, store dropped):
// no branches, so the compiler counts vmcnt exactly.
template <bool kRecord>
__device__ __forceinline__ void flood_stream_even(const FloodArgs& a, uint64_t* out_row, uint32_t total,
                                                  uint32_t W, __amdgpu_buffer_rsrc_t in, uint32_t pbase,
                                                  const uint32_t* src, uint32_t lane, uint32_t round,
                                                  PullCtr& c) {
  constexpr uint32_t kU = 8;
  const __amdgpu_buffer_rsrc_t out = rsrc(out_row, total * 8u);
  const float rw = 1.0f / static_cast<float>(W);
  for (uint32_t i0 = 0; i0 < total; i0 += kU * 128) {
    uint4 v[kU];
    uint32_t so[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t i = i0 + u * 128 + 2 * lane;
      int32_t kk, r;
      split_word(i < total ? i : total - 2, rw, W, kk, r);
      const uint32_t p = i < total ? src[kk] : kNoneNode;
      const bool go = p != kNoneNode;
      v[u] = ld16_sc1(in, go ? ((p - pbase) * W + static_cast<uint32_t>(r)) * 8u : kOutOfRange);
      so[u] = go ? i * 8u : kOutOfRange;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      st16_sc1(out, so[u], v[u]);
      const bool own = so[u] != kOutOfRange;
      c.deliv += own ? popc4(v[u]) : 0u;
      c.sw += own ? 2u : 0u;
      if constexpr (kRecord) {
        if (own) {
          const uint64_t cw = (out_row - a.seen) + so[u] / 8u;
          record_word(a.hop_rec, cw, static_cast<uint64_t>(v[u].y) << 32 | v[u].x, round);
          record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(v[u].w) << 32 | v[u].z, round);
        }
      }
    }
  }
}

// Stream, odd W: 16-B stores over the run's 16-B aligned word pairs; a pair
// may straddle two rows, so its two words are loaded separately (8 B each,
// from each node's own source).  A head word (run not 16-B aligned) and a
// tail word go as 8-B stores by lanes 0 and 1.  A pair with one skipped half
// stores 0 there: a skipped node's row is stale (generation not stamped),
// so what it holds is never read.
template <bool kRecord>
__device__ __forceinline__ void flood_stream_odd(const FloodArgs& a, uint64_t* out_row, uint32_t total,
                                                 uint32_t W, __amdgpu_buffer_rsrc_t in, uint32_t pbase,
                                                 const uint32_t* src, uint32_t lane, uint32_t round,
                                                 PullCtr& c) {
  constexpr uint32_t kU = 8;
  const __amdgpu_buffer_rsrc_t out = rsrc(out_row, total * 8u);
  const uint32_t head = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out_row) >> 3) & 1u;
  const float rw = 1.0f / static_cast<float>(W);
  auto at = [&](uint32_t i, bool& go) -> uint32_t {  // source byte offset of word i (or out of range)
    int32_t kk, r;
    split_word(i, rw, W, kk, r);
    const uint32_t p = src[kk];
    go = p != kNoneNode;
    return go ? ((p - pbase) * W + static_cast<uint32_t>(r)) * 8u : kOutOfRange;
  };
  const uint32_t body = total - head;
  if (lane < 2 && (lane == 0 ? head : (body & 1u))) {
    const uint32_t i = lane == 0 ? 0u : total - 1;
    bool g;
    const uint64_t v = ld8_sc1(in, at(i, g));
    st8_sc1(out, g ? i * 8u : kOutOfRange, v);
    c.deliv += g ? __popcll(v) : 0u;
    c.sw += g;
    if constexpr (kRecord)
      if (g) record_word(a.hop_rec, (out_row - a.seen) + i, v, round);
  }
  const uint32_t np = body >> 1;
  for (uint32_t j0 = 0; j0 < np; j0 += kU * 64) {
    uint64_t lo[kU], hi[kU];
    bool glo[kU], ghi[kU];
    uint32_t so[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t j = j0 + u * 64 + lane;
      const bool mine = j < np;
      const uint32_t i = head + 2 * (mine ? j : np - 1);
      const uint32_t olo = at(i, glo[u]);
      const uint32_t ohi = at(i + 1, ghi[u]);
      glo[u] = glo[u] && mine;
      ghi[u] = ghi[u] && mine;
      lo[u] = ld8_sc1(in, glo[u] ? olo : kOutOfRange);
      hi[u] = ld8_sc1(in, ghi[u] ? ohi : kOutOfRange);
      so[u] = (glo[u] || ghi[u]) ? i * 8u : kOutOfRange;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      st16_sc1(out, so[u], uint4{static_cast<uint32_t>(lo[u]), static_cast<uint32_t>(lo[u] >> 32),
                                 static_cast<uint32_t>(hi[u]), static_cast<uint32_t>(hi[u] >> 32)});
      c.deliv += (glo[u] ? __popcll(lo[u]) : 0u) + (ghi[u] ? __popcll(hi[u]) : 0u);
      c.sw += static_cast<uint32_t>(glo[u]) + static_cast<uint32_t>(ghi[u]);
      if constexpr (kRecord) {
        if (so[u] != kOutOfRange) {
          const uint64_t cw = (out_row - a.seen) + so[u] / 8u;
          if (glo[u]) record_word(a.hop_rec, cw, lo[u], round);
          if (ghi[u]) record_word(a.hop_rec, cw + 1, hi[u], round);
        }
      }
    }
  }
}

// Wide path, word by word: a parent range too wide for 32-bit buffer
// offsets.  8-B agent-scope accesses (sc1).
template <bool kRecord>
__device__ void flood_stream_wide(const FloodArgs& a, uint64_t* out_row, uint32_t total, uint32_t W,
                                  const uint64_t* prow, uint32_t pbase, const uint32_t* src, uint32_t lane,
                                  uint32_t round, PullCtr& c) {
  for (uint32_t i = lane; i < total; i += 64) {
    const uint32_t kk = i / W, r = i - kk * W;
    const uint32_t p = src[kk];
    if (p == kNoneNode) continue;
    const uint64_t m = ld_agent64(prow + static_cast<uint64_t>(p - pbase) * W + r);
    __hip_atomic_store(out_row + i, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c.deliv += __popcll(m);
    c.sw += 1;
    if constexpr (kRecord) record_word(a.hop_rec, (out_row - a.seen) + i, m, round);
  }
}

// One round's counters of this wave into the round's partial slots (zeroed
// per window); no block barrier, so waves stay independent.
__device__ __forceinline__ void flood_flush(const FloodArgs& a, PullCtr& c, uint32_t slot, uint32_t lane) {
  const uint64_t v7[7] = {wave_sum_u64(c.deliv),   wave_sum_u64(c.sw),      wave_sum_u64(c.kids),
                          wave_sum_u64(c.reached), wave_sum_u64(c.parents), wave_sum_u64(c.pwords),
                          wave_sum_u64(c.dup)};
  const uint64_t v = lane < kNumCtr ? pull_ctr_pick(v7, lane) : 0;
  if (v)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.partials + static_cast<uint64_t>(slot) * kNumCtr + lane),
              static_cast<unsigned long long>(v));
  c = PullCtr{};
}

template <bool kRecord>
__global__ __launch_bounds__(kBlock, kFloodBlocksPerCu) void k_flood(FloodArgs a) {
  __shared__ uint32_t src_lds[kBlock / 64][kFloodMaxNodes];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * (kBlock / 64) + wid;
  uint32_t* src = src_lds[wid];
  const uint32_t cur = a.gen_cur & 0xFF;
  PullCtr c;
  uint32_t slot = kNoneNode, round = 0;
  uint64_t pf[kFloodProf] = {0, 0, 0, 0, 0, 0, 0, 0};  // debug profile (a.prof)
  auto stamp = [&]() -> uint64_t { return a.prof ? __builtin_amdgcn_s_memrealtime() : 0; };
  uint64_t t_a = stamp();
  pf[0] = t_a;
  // static round robin over the list (topological order): wave g runs tasks
  // g, g + nw, ...; every wave is resident (grid <= occupancy), so the
  // earliest unfinished task always has its parents done
  const uint32_t nw = gridDim.x * (kBlock / 64);
  FloodTask T = uniform(a.tasks[wave < a.n_tasks ? wave : 0]);
  // the previous task's granules, published once its row stores are known
  // to have drained (see below)
  uint64_t pend_val = 0;
  uint32_t pend_at = kNoneNode;
  for (uint32_t ti = wave; ti < a.n_tasks; ti += nw) {
    if (T.round != round) {  // tasks come level by level: a wave's rounds only grow
      if (slot != kNoneNode) flood_flush(a, c, slot, lane);
      round = T.round;
      slot = T.slot0 + wave % T.nslot;
    }
    const uint32_t nk = T.ne - T.nb;
    // this task's nodes, one per lane (static data: loaded before the wait)
    // (unconditional loads, lanes past the run re-read its last node: no
    // branch, so nothing waits for them before the poll)
    const bool in = lane < nk;
    const uint32_t me = T.nb + (in ? lane : nk - 1);
    const uint32_t p = a.node_parent[me];
    const uint32_t f = a.node_flags[me];
    uint32_t prev = kNoneNode;
    const TopicDev D = a.topics[T.topic];
    const FloodSeg S = a.segs[T.seg];
    // the next task's record, consumed after this one
    const FloodTask Tn = a.tasks[ti + nw < a.n_tasks ? ti + nw : ti];
    if (lane == 0 && T.nb > 0) prev = a.node_parent[T.nb - 1];
    // The previous task's row stores were issued before these loads; the
    // vector-memory counter retires in issue order, so once the parent id
    // loaded above is in a register every older store has drained: publish
    // the previous task's granules now (its drain overlapped these loads).
    {
      const uint32_t p_used = __builtin_amdgcn_readfirstlane(p);  // waits for the load of p
      asm volatile("; publish after p %0" ::"s"(p_used) : "memory");
      if (pend_at != kNoneNode)
        __hip_atomic_store(a.granules + pend_at, pend_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pend_at = kNoneNode;
    }
    // round - 1's granules of the parents: the dependency wait and the
    // frontier test (parent reached this window) in one load
    bool up = false;
    if (T.pg_lo == kNoneNode) {
      up = in;  // level 1: the parent is the topic root, seeded this window
    } else {
      const uint32_t rel = in ? p - T.pnode0 : T.p_lo - T.pnode0;
      const uint64_t* gp = a.granules + T.pg_lo + (rel / T.pgsz - (T.p_lo - T.pnode0) / T.pgsz);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t g = 0;
      bool have = !in;
      for (;;) {
        if (!have) {
          g = ld_agent64(gp);
          have = static_cast<uint32_t>(g >> 32) == a.epoch;
        }
        if (__all(have)) break;
        const uint64_t waited = __builtin_amdgcn_s_memrealtime() - t0;
        if (waited > a.spin_ticks || (waited > 1000000u && ld_agent(a.err) != 0)) {
          if (lane == 0) atomicOr(a.err, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      up = in && ((g >> (rel % T.pgsz)) & 1u);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the row loads below the poll
    uint64_t t_b = stamp();
    pf[2] += t_b - t_a;
    const uint32_t W = rfl(S.W), nbase = rfl(D.nbase);
    const uint64_t row0 = static_cast<uint64_t>(rfl(static_cast<uint32_t>(S.row0 >> 32))) << 32 |
                          rfl(static_cast<uint32_t>(S.row0));
    const uint64_t base = row0 - static_cast<uint64_t>(nbase) * W;
    // resolve: the parent whose row each node receives.  Every row (block)
    // is written once per window -- a node is reached once per start group
    // -- so it is fresh: new = row(parent) & ~0, written whole.
    const bool ok = up && (f & kNodeLive);
    if (in) src[lane] = ok ? p : kNoneNode;
    {
      uint32_t pv = static_cast<uint32_t>(__shfl_up(static_cast<int>(p), 1, 64));
      if (lane == 0) pv = T.nb > nbase ? prev : kNoneNode;
      c.kids += in;
      c.reached += ok;
      if (up && p != pv) {  // a reached parent counts once, at its first child
        c.parents += 1;
        c.pwords += W;
      }
    }
    if (a.prof) {
      const uint64_t t = stamp();
      pf[3] += t - t_b;
      t_b = t;
    }
    // stream the rows
    const uint32_t total = nk * W;
    uint64_t* out_row = a.seen + base + static_cast<uint64_t>(T.nb) * W;
    const uint64_t* prow = a.seen + base + static_cast<uint64_t>(T.p_lo) * W;
    const uint64_t span = static_cast<uint64_t>(T.p_hi - T.p_lo + 1) * W * 8;
    if (span >= kOutOfRange) {  // parent range too wide for 32-bit buffer offsets
      flood_stream_wide<kRecord>(a, out_row, total, W, prow, T.p_lo, src, lane, T.round, c);
    } else {
      const __amdgpu_buffer_rsrc_t rin = rsrc(prow, static_cast<uint32_t>(span));
      if (W & 1u)
        flood_stream_odd<kRecord>(a, out_row, total, W, rin, T.p_lo, src, lane, T.round, c);
      else
        flood_stream_even<kRecord>(a, out_row, total, W, rin, T.p_lo, src, lane, T.round, c);
    }
    // the node's generation (read by later windows and the readbacks only)
    if (ok) a.gen[T.nb + lane] = static_cast<uint8_t>(cur);
    const uint64_t reach = __ballot(ok);
    const uint64_t t_c = stamp();
    pf[4] += t_c - t_b;
    if (a.prof && T.round > a.prof_split) pf[7] += t_b - t_a;  // waits of the later rounds
    // publish: the granules wait until every row store of this task has
    // reached the device-coherent level -- at the next task's first load, or
    // below for a wave's last task
    const uint32_t ng = (nk + T.gsz - 1) / T.gsz;
    if (lane < ng) {
      const uint64_t bits = (reach >> (lane * T.gsz)) & (T.gsz >= 64 ? ~0ull : (1ull << T.gsz) - 1ull);
      pend_val = static_cast<uint64_t>(a.epoch) << 32 | bits;
      pend_at = T.g_own + lane;
    }
    asm volatile("" ::: "memory");  // the next task's loads stay behind this task's stores
    T = uniform(Tn);
    t_a = stamp();
    pf[5] += t_a - t_c;
    pf[6] += 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (pend_at != kNoneNode)
    __hip_atomic_store(a.granules + pend_at, pend_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (slot != kNoneNode) flood_flush(a, c, slot, lane);
  if (a.prof && lane == 0) {
    pf[1] = stamp();
    for (uint32_t k = 0; k < kFloodProf; ++k) a.prof[static_cast<uint64_t>(wave) * kFloodProf + k] = pf[k];
  }
}

// Parents of every task (p_lo / p_hi from the node space) and the granules
// of the parent level that hold them.
__global__ __launch_bounds__(kBlock) void k_flood_deps(FloodTask* __restrict__ tasks, uint32_t n,
                                                       const FloodSeg* __restrict__ segs,
                                                       const uint32_t* __restrict__ node_parent) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  FloodTask t = tasks[i];
  t.p_lo = node_parent[t.nb];
  t.p_hi = node_parent[t.ne - 1];
  if (t.pseg == kNoneNode) {
    t.pg_lo = kNoneNode;
  } else {
    const FloodSeg s = segs[t.pseg];
    // a parent outside its level could only mis-order, never index outside
    // the granules (clamped)
    const uint32_t nodes = s.nodes;
    const uint32_t lo = t.p_lo >= s.node0 ? min(t.p_lo - s.node0, nodes - 1) : 0u;
    if (t.p_hi < t.p_lo || t.p_hi - s.node0 >= nodes) t.p_hi = s.node0 + nodes - 1;
    t.p_lo = s.node0 + lo;
    t.pg_lo = s.gbase + lo / s.gsz;
    t.pnode0 = s.node0;
    t.pgsz = s.gsz;
  }
  tasks[i] = t;
}

}  // namespace

hipError_t launch_flood(const FloodArgs& a, uint32_t grid, bool record, hipStream_t s) {
  if (a.n_tasks == 0 || grid == 0) return hipSuccess;
  if (record)
    hipLaunchKernelGGL((k_flood<true>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((k_flood<false>), dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_flood_deps(FloodTask* tasks, uint32_t n, const FloodSeg* segs, const uint32_t* node_parent,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_flood_deps, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, tasks, n, segs,
                     node_parent);
  return hipGetLastError();
}

// Resident k_flood blocks per CU (both instances; the smaller bounds the grid).
hipError_t flood_blocks_per_cu(int* out) {
  int a = 0, b = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, k_flood<false>, kBlock, 0);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_flood<true>, kBlock, 0);
  *out = a < b ? a : b;
  return e;
}

}  // namespace psamd
