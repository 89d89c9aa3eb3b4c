// flood.hip -- k_flood: every round of a single-start tree window in ONE
// persistent launch.
//
// Reference: the recursive flood of subtree.forwardMessage (subtree.go:319-354)
// driven hop by hop by client.processMessages (client.go:100-132): round q
// delivers to BFS level q - s_t of every active topic t.  A node's row of
// 64-message words receives, in its round, its parent's row of the previous
// round -- if the parent was reached this window (its generation byte was
// stamped by the round that delivered to it) and the node is live (the dead
// child is skipped, subtree.go:326-331) -- through the seen test-and-set
// new = row(parent) & ~seen(node), seen(node) |= new, where a node whose
// generation is stale has seen nothing yet (lazy reset).
//
// Per-level launches (k_pull) separate the rounds by kernel boundaries.  Here
// the rounds are ordered by dataflow inside one launch:
//   * the host cuts every level of every topic into tasks (a contiguous node
//     run of one level, about kFloodWords row words), listed level by level: a
//     topological order of "reads the rows the previous round wrote";
//   * wave g of the G co-resident waves runs tasks g, g + G, g + 2G, ... in
//     order.  A task first waits until every task writing its parents' rows
//     has published done[task] == epoch, then pulls those rows;
//   * a task publishes once its own rows and generation bytes have drained.
// Hand-off (MI355X_MICROARCH.md §Workgroup dispatch... Valid forms; Guideline
// 16 R1): rows are stored write-through (sc1 buffer stores), generation bytes
// and the done word by agent-scope relaxed stores (sc1), and every load of a
// handed-off byte is an sc1 load -- no fence, correct for any placement.
// Deadlock freedom: every dependency points to an earlier task, and the grid
// never exceeds the resident capacity, so the wave holding the earliest
// unfinished task always runs.  Every wait is bounded: a timeout sets *err
// (read back with the round counters) and the launch still completes.
#include "devutil.hpp"
#include "kernels.hpp"

namespace psamd {
namespace {

using namespace dev;

constexpr uint32_t kMergeBit = 0x80000000u;  // src[]: the node already holds rows of this window

// Waits until done[lo..hi] == epoch (relaxed sc1 polls, s_sleep back-off).
// Bounded: past spin_ticks the wait sets *err and gives up; a wait longer
// than 10 ms also gives up once another wave has set *err, so a launch whose
// waves were not all resident drains in about one timeout.
__device__ __forceinline__ bool flood_wait(const FloodArgs& a, uint32_t lo, uint32_t hi, uint32_t lane) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ok = true;
    for (uint32_t d = lo + lane; d <= hi; d += 64) ok &= ld_agent(a.done + d) == a.epoch;
    if (__all(ok)) return true;
    const uint64_t waited = __builtin_amdgcn_s_memrealtime() - t0;
    if (waited > a.spin_ticks || (waited > 1000000u && ld_agent(a.err) != 0)) {
      if (lane == 0) atomicOr(a.err, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// The task record, wave-uniform (scalar registers: buffer descriptors built
// from it stay scalar, no per-lane loops).
__device__ __forceinline__ FloodTask load_task(const FloodTask* p) {
  FloodTask t = *p;
  t.nb = rfl(t.nb);
  t.ne = rfl(t.ne);
  t.p_lo = rfl(t.p_lo);
  t.p_hi = rfl(t.p_hi);
  t.dep_lo = rfl(t.dep_lo);
  t.dep_hi = rfl(t.dep_hi);
  t.topic = rfl(t.topic);
  t.round = rfl(t.round);
  t.slot0 = rfl(t.slot0);
  t.nslot = rfl(t.nslot);
  return t;
}

__device__ __forceinline__ uint8_t ld_agent_u8(const uint8_t* p) {
  return __hip_atomic_load(const_cast<uint8_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Phase 1 for the task's nodes: src[j] = the parent whose row node nb + j
// receives (| kMergeBit when the node already holds messages of this window),
// or kNoneNode (parent not reached, or node not live).  Reached nodes get
// their generation stamped (sc1: their children read it).  Returns whether
// some node needs the merging path.
__device__ __forceinline__ bool flood_resolve(const FloodArgs& a, const FloodTask& T, uint32_t nbase,
                                              uint32_t W, uint32_t* src, uint8_t* genl, uint32_t lane,
                                              uint32_t cur, PullCtr& c) {
  const uint32_t nk = T.ne - T.nb;
  // the parents' generation bytes, staged as whole dwords when the range is short
  const bool staged = T.p_hi - T.p_lo < kFloodMaxNodes;
  const uint32_t g0 = T.p_lo & ~3u;
  if (staged) {
    const uint32_t nd = (((T.p_hi + 4u) & ~3u) - g0) >> 2;
    for (uint32_t d = lane; d < nd; d += 64)
      reinterpret_cast<uint32_t*>(genl)[d] = ld_agent(reinterpret_cast<const uint32_t*>(a.gen + g0) + d);
  }
  bool merge = false;
  for (uint32_t j0 = 0; j0 < nk; j0 += 64) {
    const uint32_t j = j0 + lane;
    const bool in = j < nk;
    uint32_t p = kNoneNode, f = 0, own = 0;
    if (in) {
      p = a.node_parent[T.nb + j];
      f = a.node_flags[T.nb + j];
      own = a.gen[T.nb + j];  // only this wave writes this byte in this launch
    }
    uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(p), 1, 64));
    if (lane == 0) prev = T.nb + j0 > nbase ? a.node_parent[T.nb + j0 - 1] : kNoneNode;
    bool up = in && p >= T.p_lo && p <= T.p_hi;  // (kNoneNode fails the range)
    if (up) up = (staged ? genl[p - g0] : ld_agent_u8(a.gen + p)) == cur;
    const bool ok = up && (f & kNodeLive);
    const bool fresh = own != cur;
    if (in) src[j] = ok ? (p | (fresh ? 0u : kMergeBit)) : kNoneNode;
    if (ok) st_agent(a.gen + T.nb + j, static_cast<uint8_t>(cur));
    merge |= ok && !fresh;
    c.kids += in;
    c.reached += ok;
    if (up && p != prev) {  // a reached parent counts once, at its first child
      c.parents += 1;
      c.pwords += W;
    }
  }
  return __any(merge);
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

// Phase 2, even W: the task's rows as one output stream of 16-B word pairs
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

// Phase 2, odd W: 16-B stores over the run's 16-B aligned word pairs; a pair
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

// Merging path, word by word: a node that already holds messages of this
// window (never on a tree whose window messages share one start round, kept
// exact anyway: new = parent & ~own, the duplicates counted), or a parent
// range too wide for 32-bit buffer offsets.  8-B agent-scope accesses (sc1).
template <bool kRecord>
__device__ void flood_stream_merge(const FloodArgs& a, uint64_t* out_row, uint32_t total, uint32_t W,
                                   const uint64_t* prow, uint32_t pbase, const uint32_t* src, uint32_t lane,
                                   uint32_t round, PullCtr& c) {
  for (uint32_t i = lane; i < total; i += 64) {
    const uint32_t kk = i / W, r = i - kk * W;
    const uint32_t s = src[kk];
    if (s == kNoneNode) continue;
    const uint32_t p = s & ~kMergeBit;
    const uint64_t m = __hip_atomic_load(const_cast<uint64_t*>(prow) + static_cast<uint64_t>(p - pbase) * W + r,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t* o = out_row + i;
    const uint64_t own = (s & kMergeBit) ? __hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const uint64_t nm = m & ~own;
    __hip_atomic_store(o, own | nm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c.deliv += __popcll(nm);
    c.dup += __popcll(m & own);
    c.sw += 1;
    if constexpr (kRecord) record_word(a.hop_rec, (out_row - a.seen) + i, nm, round);
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
  __shared__ uint32_t gen_lds[kBlock / 64][kFloodMaxNodes / 4 + 2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * (kBlock / 64) + wid;
  const uint32_t nw = gridDim.x * (kBlock / 64);
  uint32_t* src = src_lds[wid];
  uint8_t* genl = reinterpret_cast<uint8_t*>(gen_lds[wid]);
  const uint32_t cur = a.gen_cur & 0xFF;
  PullCtr c;
  uint32_t slot = kNoneNode, round = 0;
  for (uint32_t ti = wave; ti < a.n_tasks; ti += nw) {
    const FloodTask T = load_task(a.tasks + ti);
    if (T.round != round) {  // tasks come level by level: a wave's rounds only grow
      if (slot != kNoneNode) flood_flush(a, c, slot, lane);
      round = T.round;
      slot = T.slot0 + wave % T.nslot;
    }
    // round - 1 must have written the parents' rows: wait for their tasks
    if (T.dep_lo != kNoneNode) (void)flood_wait(a, T.dep_lo, T.dep_hi, lane);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
    const TopicDev D = a.topics[T.topic];
    const uint32_t W = rfl(D.W), nbase = rfl(D.nbase);
    const uint64_t wbase = static_cast<uint64_t>(rfl(static_cast<uint32_t>(D.wbase >> 32))) << 32 |
                           rfl(static_cast<uint32_t>(D.wbase));
    const uint64_t base = wbase - static_cast<uint64_t>(nbase) * W;
    const uint32_t total = (T.ne - T.nb) * W;
    const bool merge = flood_resolve(a, T, nbase, W, src, genl, lane, cur, c);
    uint64_t* out_row = a.seen + base + static_cast<uint64_t>(T.nb) * W;
    const uint64_t* prow = a.seen + base + static_cast<uint64_t>(T.p_lo) * W;
    const uint64_t span = static_cast<uint64_t>(T.p_hi - T.p_lo + 1) * W * 8;
    if (merge || span >= kOutOfRange) {
      flood_stream_merge<kRecord>(a, out_row, total, W, prow, T.p_lo, src, lane, T.round, c);
    } else {
      const __amdgpu_buffer_rsrc_t in = rsrc(prow, static_cast<uint32_t>(span));
      if (W & 1u)
        flood_stream_odd<kRecord>(a, out_row, total, W, in, T.p_lo, src, lane, T.round, c);
      else
        flood_stream_even<kRecord>(a, out_row, total, W, in, T.p_lo, src, lane, T.round, c);
    }
    // publish: every row and generation store of this wave has reached the
    // device-coherent level before the done word does
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) st_agent(a.done + ti, a.epoch);
  }
  if (slot != kNoneNode) flood_flush(a, c, slot, lane);
}

// Parents and dependencies of every task: p_lo / p_hi from the node space,
// and the tasks of the previous level that write them (FloodTask::dep_lo
// holds that level's segment until then).
__global__ __launch_bounds__(kBlock) void k_flood_deps(FloodTask* __restrict__ tasks, uint32_t n,
                                                       const FloodSeg* __restrict__ segs,
                                                       const uint32_t* __restrict__ node_parent) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  FloodTask t = tasks[i];
  t.p_lo = node_parent[t.nb];
  t.p_hi = node_parent[t.ne - 1];
  if (t.dep_lo != kNoneNode) {
    const FloodSeg s = segs[t.dep_lo];
    // (clamped to the segment: a malformed parent can only mis-order, never
    // index outside the done words)
    const uint32_t last = s.n_tasks - 1;
    t.dep_lo = s.task0 + min(last, (t.p_lo >= s.node0 ? t.p_lo - s.node0 : 0u) / s.per);
    t.dep_hi = s.task0 + min(last, (t.p_hi >= s.node0 ? t.p_hi - s.node0 : 0u) / s.per);
  }
  tasks[i] = t;
}

}  // namespace

hipError_t launch_flood(const FloodArgs& a, uint32_t grid, bool record, hipStream_t s) {
  if (a.n_tasks == 0 || grid == 0) return hipSuccess;
  if (record)
    hipLaunchKernelGGL(k_flood<true>, dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL(k_flood<false>, dim3(grid), dim3(kBlock), 0, s, a);
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
