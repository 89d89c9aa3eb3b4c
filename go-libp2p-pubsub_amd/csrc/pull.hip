// pull.hip -- level-mode pull kernels: k_pull
// (one round, child-parallel), k_pull_pair (two rounds, the second from LDS),
// and the multi-GPU ghost records they ship (k_pack for the roots).
// Reference: subtree.forwardMessage (subtree.go:319-354) and
// client.processMessages (client.go:100-132).
#include <algorithm>
#include <cstddef>

#include <hipcub/hipcub.hpp>

#include "devutil.hpp"
#include "kernels.hpp"

namespace psamd {

namespace {

using namespace dev;

// LDS-DMA: lane i copies N bytes from its own global address into
// lds_base + i * N (lds_base wave-uniform); no VGPR destination, counted on
// vmcnt like a load.
#define PSAMD_DMA(g, lds_base, N)                                                        \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g), \
                                   (__attribute__((address_space(3))) void*)(lds_base), N, 0, 0)
// ------------------------------------------------------------------ pull ---
// Level mode, pull direction, one launch per round (multi-GPU windows, whose
// rounds are separated by the frontier exchange; PSAMD_FLOOD=0 on one GPU).
// In a single-start tree window a node of BFS level d receives, in round
// s + d, exactly its parent's row -- if the parent was reached this window
// (generation current) and the node is live -- and it is fresh (it has seen
// nothing this window), so the seen test-and-set is new = row(parent) & ~0
// and the whole row is written.  A wave owns a contiguous run of next-level
// nodes, whose rows form one contiguous output stream:
//   phase 1  resolves each node's source into a wave-private LDS table: its
//            parent if the parent is in the frontier (generation current) and
//            the node is live, else none; the node's generation is stamped;
//   phase 2  streams the run's rows in order with 16-B stores (8-B for odd
//            W), each lane's load taken from its node's parent row (siblings
//            read the same parent row: L2 hits).  Loads are unconditional (a
//            skipped node reads its own row) so the unrolled body keeps
//            several in flight.
// Counters: deliveries, seen writes, nodes visited, nodes reached, parents
// expanded (a reached parent counts at its first child) and their row words.
struct PullVec {
  bool go;
  uint4 v;
};

// Counters of the pull kernels, two forms: PullCtr (devutil.hpp) counts per
// lane, as k_pull's block reduction wants; WaveCtr keeps one per-lane
// delivery sum and counts everything else wave-uniformly (ballots: scalar
// registers), which k_pull_pair's persistent waves carry across chunks for
// two rounds without the vector registers per-lane counters would take.
struct WaveCtr {
  uint32_t deliv = 0;                      // per lane, folded into dsum per sub-run
  uint32_t kids = 0, reached = 0, parents = 0;  // wave-uniform
  uint64_t sw = 0, pwords = 0;             // wave-uniform: words written, parent words read
  uint64_t dsum = 0;                       // wave-uniform: folded deliveries
};
// The per-lane delivery count into the 64-bit wave total: after each sub-run
// of at most kPairKids rows (<= 2^24 bits), so neither the lane counts nor
// the sum over a wide run's children (f * W * 64 bits) wrap.
__device__ __forceinline__ void ctr_fold(WaveCtr& c) {
  c.dsum += __builtin_amdgcn_readfirstlane(__reduce_add_sync(~0ull, c.deliv));  // (a sub-run: < 2^32)
  c.deliv = 0;
}
// One batch of (up to 64) nodes: visited (in), reached (ok), a reached
// parent's first child (par); W_sw row words written per reached node,
// W_pw parent row words read per counted parent.
__device__ __forceinline__ void ctr_nodes(PullCtr& c, bool in, bool ok, bool par, uint32_t, uint32_t W_pw) {
  c.kids += in;
  c.reached += ok;
  if (par) {
    c.parents += 1;
    c.pwords += W_pw;
  }
}
__device__ __forceinline__ void ctr_nodes(WaveCtr& c, bool in, bool ok, bool par, uint32_t W_sw, uint32_t W_pw) {
  c.kids += __popcll(__ballot(in));
  const uint32_t r = __popcll(__ballot(ok));
  c.reached += r;
  c.sw += static_cast<uint64_t>(r) * W_sw;
  const uint32_t p = __popcll(__ballot(par));
  c.parents += p;
  c.pwords += static_cast<uint64_t>(p) * W_pw;
}
// One lane's stored unit: its delivered bits, and (PullCtr) its words.
__device__ __forceinline__ void ctr_unit(PullCtr& c, bool own, uint32_t pop, uint32_t words) {
  c.deliv += own ? pop : 0u;
  c.sw += own ? words : 0u;
}
__device__ __forceinline__ void ctr_unit(WaveCtr& c, bool own, uint32_t pop, uint32_t) { c.deliv += own ? pop : 0u; }

// Chunk constants: row of node u = base + u * W (a start group's block row
// for kTopicGroups topics).
struct PullTopic {
  uint64_t base;
  uint32_t W, nbase, root;
};

// The record base of source rank r (a per-lane value: a select chain over the
// kernel arguments, not an indexed copy of them in scratch)
__device__ __forceinline__ const uint64_t* rank_base(const PullArgs& a, uint32_t r) {
  const uint64_t* b = a.rsrc[0];
#pragma unroll
  for (uint32_t k = 1; k < kMaxRanks; ++k) b = r == k ? a.rsrc[k] : b;
  return b;
}

// Phase 1 for the nodes [nb, nb + nk) of one level: src[j] = the address of
// the row node nb + j copies (its parent's row: the root's arrival row, a
// seen row, or -- multi-GPU -- a ghost row in the receive buffer), or 0.  The
// parents of a run are consecutive node ids [p_lo, p_hi] (BFS numbering):
// their generation bytes are staged into LDS by loads issued together with
// the nodes' own metadata, so phase 1 costs one memory round trip.
template <class Ctr>
__device__ __forceinline__ void pull_resolve(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t nk,
                                             uint32_t p_lo, uint32_t p_hi, uint64_t* src, uint8_t* genl,
                                             uint32_t lane, uint32_t cur, Ctr& c, uint32_t gin,
                                             uint32_t stage_cap = kPullMaxKids) {
  uint32_t g0 = 0;
  const bool staged = p_lo != kNoneNode && p_hi - p_lo < stage_cap;  // genl holds stage_cap + 8 bytes
  if (staged) {
    g0 = p_lo & ~3u;
    const uint32_t nd = ((p_hi + 4u) & ~3u) - g0;  // bytes, whole dwords
    const uint32_t* gsrc = reinterpret_cast<const uint32_t*>(a.gen + g0);
    for (uint32_t d = lane; 4 * d < nd; d += 64) reinterpret_cast<uint32_t*>(genl)[d] = gsrc[d];
  }
  for (uint32_t j0 = 0; j0 < nk; j0 += 64) {
    const uint32_t j = j0 + lane;
    const bool in = j < nk;
    uint32_t p = kNoneNode, f = 0;
    if (in) {
      p = a.node_parent[nb + j];
      f = a.node_flags[nb + j];
    }
    // lane 0: the previous node's parent (and ghost reference), issued with
    // the group's own loads -- not a second round trip after them
    const uint32_t q = nb + j0;
    uint32_t pm = kNoneNode, gm = kNoneNode;
    if (lane == 0 && q > P.nbase) {
      pm = a.node_parent[q - 1];
      if (gin != kNoneNode) gm = a.ghost_ref[q - 1];
    }
    bool up = false;  // the parent was reached this window
    uint64_t row = 0;
    uint32_t pid = p;  // the parent's identity for the once-per-parent count
    if (in && p != kNoneNode) {
      up = (staged ? genl[p - g0] : a.gen[p]) == cur;
      row = reinterpret_cast<uint64_t>((p == P.root ? a.a_cur : a.seen) + P.base + static_cast<uint64_t>(p) * P.W);
    } else if (in && gin != kNoneNode) {  // parent on another rank: its record arrived this round
      const uint32_t g = a.ghost_ref[nb + j];
      if (g != kNoneNode) {
        const GhostSeg* S = a.gsegs + gin;
        const uint32_t src_rank = g >> kRemoteRankShift, k = g & kRemoteIdMask;
        if (S->flags & kSegInPlace) {
          // the parent's own row at its owner (k: its topic-relative id
          // there), reached iff the owner stamped it this window
          const RankRows R = a.rrows[src_rank];
          row = reinterpret_cast<uint64_t>(R.seen + S->rbase[src_rank] + static_cast<uint64_t>(k) * S->rw);
          up = R.gen[S->gbase[src_rank] + k] == cur;
        } else {
          const uint64_t* rec = rank_base(a, src_rank) + S->rbase[src_rank] + static_cast<uint64_t>(k) * S->rw;
          up = rec[0] != 0;  // an unreached parent's record starts with a zero word
          row = reinterpret_cast<uint64_t>(rec);
        }
        pid = 0x80000000u | g;
      }
    }
    uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(pid), 1, 64));
    if (lane == 0) prev = pm != kNoneNode ? pm : gm != kNoneNode ? 0x80000000u | gm : kNoneNode;
    const bool ok = up && (f & kNodeLive);
    if (in) src[j] = ok ? row : 0ull;
    if (ok) a.gen[nb + j] = static_cast<uint8_t>(cur);
    ctr_nodes(c, in, ok, up && pid != prev, P.W, P.W);
  }
}

// row store of the pull stream: plain, or non-temporal (`nt`: rows nobody
// re-reads soon)
template <bool kNT>
__device__ __forceinline__ void store_row16(uint64_t* p, const uint4& v) {
  if constexpr (kNT) {
    u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}
template <bool kNT>
__device__ __forceinline__ void store_row8(uint64_t* p, uint64_t v) {
  if constexpr (kNT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Phase 2: the rows of nodes [nb, nb + nk) as one output stream, each lane's
// load from the row its node copies (src[], kNoneNode = skip).  8 loads in
// flight, then 8 stores, unconditional and branch-free (a skipped lane writes
// its own row back unchanged, a lane past the run's end stores the run's last
// pair again with the value its owner stores), so the compiler counts vmcnt
// exactly instead of draining at branches.  kLds (k_pull_pair): every word
// also goes to lrows[i], the run's rows in LDS for its children.
template <bool kRecord, bool kNT, bool kLds = false, class Ctr = PullCtr>
__device__ __forceinline__ void pull_stream(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t nk,
                                            const uint64_t* src, uint32_t lane, uint32_t round, Ctr& c,
                                            uint64_t* lrows = nullptr) {
  constexpr uint32_t kU = 8;
  const uint32_t W = P.W;
  const uint64_t base = P.base;
  const uint32_t total = nk * W;
  uint64_t* const out = a.seen + base + static_cast<uint64_t>(nb) * W;
  const float rw = 1.0f / static_cast<float>(W);
  // row kk = i / W and word r of the run, branch-free (float estimate off by
  // at most one; i < 2^24)
  auto split = [&](uint32_t i, int32_t& kk, int32_t& r) {
    kk = static_cast<int32_t>(static_cast<float>(i) * rw);
    r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(W);
    const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(W);
    kk += hi - lo;
    r += (lo - hi) * static_cast<int32_t>(W);
  };
  if (!(W & 1u)) {
    // even W: every row 16-B aligned, a 2-word pair never straddles rows
    auto one = [&](uint32_t i) {
      int32_t kk, r;
      split(i, kk, r);
      const uint64_t row = src[kk];
      const bool go = row != 0;
      const uint64_t* s = go ? reinterpret_cast<const uint64_t*>(row) + r : out + i;
      return PullVec{go, *reinterpret_cast<const uint4*>(s)};
    };
    // the stream starts h words before the run, at a 128-B line, so every
    // 1-KB wave store covers whole lines (lanes before the run store its
    // first pair again, with the value its owner stores)
    const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;
    for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 128) {
      PullVec x[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t i = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
        x[u] = one(i < 0 ? 0u : (static_cast<uint32_t>(i) < total ? static_cast<uint32_t>(i) : total - 2));
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
        const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
        const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 2);
        if constexpr (kRecord) {
          if (x[u].go && inr) {
            *reinterpret_cast<uint4*>(out + i) = x[u].v;
            const uint64_t cw = (out - a.seen) + i;
            record_word(a.hop_rec, cw, static_cast<uint64_t>(x[u].v.y) << 32 | x[u].v.x, round);
            record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(x[u].v.w) << 32 | x[u].v.z, round);
          }
        } else {
          store_row16<kNT>(out + i, x[u].v);
        }
        if constexpr (kLds) *reinterpret_cast<uint4*>(lrows + i) = x[u].v;  // (i clamped: its owner's value)
        const bool own = x[u].go && inr;
        ctr_unit(c, own, popc4(x[u].v), 2u);
      }
    }
  } else {
    // odd W: one word (8 B) per lane, the same pipeline
    const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;  // line-aligned start
    for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 64) {
      uint64_t m[kU];
      bool go[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
        // before the run: its first word again; past the end: its last word again
        const uint32_t ic = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 1);
        int32_t kk, r;
        split(ic, kk, r);
        const uint64_t row = src[kk];
        go[u] = row != 0;
        const uint64_t* s = go[u] ? reinterpret_cast<const uint64_t*>(row) + r : out + ic;
        m[u] = *s;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
        const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
        const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 1);
        if constexpr (kRecord) {
          if (go[u] && inr) {
            out[i] = m[u];
            record_word(a.hop_rec, (out - a.seen) + i, m[u], round);
          }
        } else {
          store_row8<kNT>(out + i, m[u]);
        }
        if constexpr (kLds) lrows[i] = m[u];
        const bool own = go[u] && inr;
        ctr_unit(c, own, __popcll(m[u]), 1u);
      }
    }
  }
}

// Multi-GPU: the chunk's nodes that are ghost parents next round ship their
// rows now, as records in the send buffer (GhostSeg gout: record k to rank b
// at sbase[b] + k * W), from the rows they copied (src[]: L2-resident, just
// read): one pass over the records, 16-B units for even W.  An unreached
// node's record gets a zero first word.  Replaces a separate pack launch that
// re-read the rows from HBM.
__device__ __forceinline__ void pull_ship(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t e_lo,
                                          uint32_t e_hi, uint32_t gout, const uint64_t* src, uint32_t lane) {
  const GhostSeg* S = a.gsegs + gout;
  const bool pairs = !(P.W & 1u);
  const uint32_t per = pairs ? P.W >> 1 : P.W;
  const uint32_t total = (e_hi - e_lo) * per;
  const float rp = 1.0f / static_cast<float>(per);
  // unit i -> (entry k, unit r of its record), branch-free (float estimate
  // off by at most one; i < 2^24), instead of an integer division per unit
  auto split = [&](uint32_t i, uint32_t& k, uint32_t& r) {
    int32_t kk = static_cast<int32_t>(static_cast<float>(i) * rp);
    int32_t rr = static_cast<int32_t>(i) - kk * static_cast<int32_t>(per);
    const int32_t lo = rr < 0, hi = rr >= static_cast<int32_t>(per);
    kk += hi - lo;
    rr += (lo - hi) * static_cast<int32_t>(per);
    k = static_cast<uint32_t>(kk);
    r = static_cast<uint32_t>(rr);
  };
  // kU units in flight per lane: the entry, source and row loads of all of
  // them before their stores (one dependent chain per unit, overlapped)
  constexpr uint32_t kU = 4;
  for (uint32_t i0 = lane; i0 < total; i0 += 64 * kU) {
    uint4 v[kU];
    uint64_t* dst[kU];
    bool live[kU], head[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t i = i0 + 64 * u;
      live[u] = false;
      head[u] = false;
      dst[u] = nullptr;
      v[u] = uint4{0, 0, 0, 0};
      if (i < total) {
        uint32_t k, r;
        split(i, k, r);
        const ShipEntry E = a.ship[e_lo + k];
        const uint64_t row = src[E.node - nb];
        const uint32_t w = pairs ? 2 * r : r;
        dst[u] = a.send + S->sbase[E.dst >> kRemoteRankShift] + static_cast<uint64_t>(E.dst & kRemoteIdMask) * P.W + w;
        head[u] = r == 0;
        live[u] = row != 0;
        if (live[u]) {
          const uint64_t* s = reinterpret_cast<const uint64_t*>(row) + w;
          if (pairs) {
            v[u] = *reinterpret_cast<const uint4*>(s);
          } else {
            const uint64_t x = *s;
            v[u].x = static_cast<uint32_t>(x);
            v[u].y = static_cast<uint32_t>(x >> 32);
          }
        }
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      if (!dst[u]) continue;
      if (!live[u]) {  // an unreached parent's record: a zero first word
        if (head[u]) dst[u][0] = 0;
        continue;
      }
      if (pairs)
        *reinterpret_cast<uint4*>(dst[u]) = v[u];
      else
        dst[u][0] = static_cast<uint64_t>(v[u].y) << 32 | v[u].x;
    }
  }
}

// The block's counters of one launch into partial slot `slot` (blocks share
// a slot: slots are zeroed per window).
__device__ __forceinline__ void pull_flush(const PullCtr& c, uint64_t* partials, uint64_t slot, uint32_t lane,
                                           uint32_t wid) {
  __shared__ uint64_t red[kBlock / 64][7];
  const uint64_t v7[7] = {wave_sum_u64(c.deliv),   wave_sum_u64(c.sw),      wave_sum_u64(c.kids),
                          wave_sum_u64(c.reached), wave_sum_u64(c.parents), wave_sum_u64(c.pwords),
                          wave_sum_u64(c.dup)};
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) red[wid][q] = v7[q];
  __syncthreads();
  if (threadIdx.x < kNumCtr) {
    uint64_t t[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < kBlock / 64; ++w)
#pragma unroll
      for (int q = 0; q < 7; ++q) t[q] += red[w][q];
    const uint64_t v = pull_ctr_pick(t, threadIdx.x);
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(partials + slot * kNumCtr + threadIdx.x),
                     static_cast<unsigned long long>(v));
  }
}

// (Capping the big rounds' residency through the register allocation, as
// k_pull_chain does, measured no gain: profiles/r04/ab/pull_simd.log.)
template <bool kRecord, bool kNT>
__global__ __launch_bounds__(kBlock) void k_pull(PullArgs a, const PullChunk* __restrict__ chunks,
                                                 uint32_t n_chunks, uint32_t round) {
  __shared__ uint64_t src_lds[kBlock / 64][kPullMaxKids];
  __shared__ uint32_t gen_lds[kBlock / 64][kPullMaxKids / 4 + 2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * (kBlock / 64) + wid;
  uint64_t* src = src_lds[wid];
  uint8_t* genl = reinterpret_cast<uint8_t*>(gen_lds[wid]);
  const uint32_t cur = a.gen_cur & 0xFF;
  PullCtr c;
  if (wave < n_chunks) {  // one chunk per wave
    const PullChunk ch = chunks[wave];
    const TopicDev T = a.topics[ch.topic];
    PullTopic P;
    P.W = ch.W;
    P.nbase = T.nbase;
    P.base = (static_cast<uint64_t>(ch.row0_hi) << 32 | ch.row0_lo) - static_cast<uint64_t>(T.nbase) * ch.W;
    P.root = (T.flags & kTopicRootLocal) ? T.nbase : kNoneNode;
    const uint32_t n1 = ch.node_end - ch.node_begin;
    // LDS ops of a wave are processed in order: the table written in phase 1
    // is visible to the reads that follow
    pull_resolve(a, P, ch.node_begin, n1, ch.p_lo, ch.p_hi, src, genl, lane, cur, c, ch.gin);
    pull_stream<kRecord, kNT>(a, P, ch.node_begin, n1, src, lane, round, c);
    if (ch.e_hi > ch.e_lo) pull_ship(a, P, ch.node_begin, ch.e_lo, ch.e_hi, ch.gout, src, lane);
  }
  pull_flush(c, a.partials, blockIdx.x % a.slot_mod, lane, wid);
}

// k_pull_pair: rounds q and q + 1 in one launch (one rank).
// A wave writes a run of level-d nodes as k_pull does (phase A: round q, the
// parents' rows from HBM, reach decided from this window's generation
// bytes), keeping the rows it writes in LDS, and then every child of the run
// (phase B: round q + 1, level d + 1 -- the children of a BFS-numbered run
// are consecutive ids): a child copies its parent's row as round q left it,
// read from LDS instead of HBM, if the parent was reached and the child is
// live, and stamps its generation.  No other wave writes those parents or
// reads those children, so the launch needs no cross-wave ordering.
//
// Phase B, one sub-run of at most kPairKids children: resolve into ctab (the
// LDS word offset of the parent's row, or kPairWords: a zero pair, so an
// unreached child's row is written with zeros -- stale under its old
// generation byte, so never read), then one line-aligned output stream with
// the phase-A pipeline.
// The first sub-run's parent ids and flags arrive prefetched (pf_p, pf_f:
// loaded with phase A's metadata, one memory round trip for both).
template <bool kRecord, bool kNT, uint32_t kWords>
__device__ __forceinline__ void pair_kids(const PullArgs& a, const PullTopic& P, uint32_t nb, uint32_t n1,
                                          uint32_t c_lo, uint32_t c_hi, const uint64_t* reach,
                                          const uint64_t* lrows, uint32_t* ctab, uint32_t lane, uint32_t round,
                                          const uint32_t* pf_p, const uint32_t* pf_f, WaveCtr& c) {
  constexpr uint32_t kU = 8;
  constexpr uint32_t kZero = kWords;
  const uint32_t W = P.W;
  const uint32_t cur = a.gen_cur & 0xFF;
  const float rw = 1.0f / static_cast<float>(W);
  auto split = [&](uint32_t i, int32_t& kk, int32_t& r) {
    kk = static_cast<int32_t>(static_cast<float>(i) * rw);
    r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(W);
    const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(W);
    kk += hi - lo;
    r += (lo - hi) * static_cast<int32_t>(W);
  };
  for (uint32_t k0 = c_lo; k0 < c_hi; k0 += kPairKids) {
    const uint32_t nk = min(kPairKids, c_hi - k0);
#pragma unroll
    for (uint32_t s = 0; s < kPairKids / 64; ++s) {
      const uint32_t j0 = s * 64;
      if (j0 >= nk) break;
      const uint32_t j = j0 + lane;
      const bool in = j < nk;
      uint32_t p = kNoneNode, f = 0;
      if (k0 == c_lo) {
        p = in ? pf_p[s] : kNoneNode;
        f = pf_f[s];
      } else if (in) {
        p = a.node_parent[k0 + j];
        f = a.node_flags[k0 + j];
      }
      const uint32_t kp = p - nb;  // the parent's place in the run
      const bool up = in && kp < n1 && ((a.all_current & 1u) || ((reach[kp >> 6] >> (kp & 63)) & 1ull));
      const bool ok = up && (f & kNodeLive);
      if (in) ctab[j] = ok ? kp * W : kZero;
      if (ok) a.gen[k0 + j] = static_cast<uint8_t>(cur);
      uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(p), 1, 64));
      if (lane == 0) prev = k0 + j0 > P.nbase ? a.node_parent[k0 + j0 - 1] : kNoneNode;
      ctr_nodes(c, in, ok, up && p != prev, W, 0u);  // (parent rows from LDS: no parent words read)
    }
    const uint32_t total = nk * W;
    uint64_t* const out = a.seen + P.base + static_cast<uint64_t>(k0) * W;
    const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;
    if (!(W & 1u)) {
      for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 128) {
        uint4 x[kU];
        bool go[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
          const uint32_t i = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 2);
          int32_t kk, r;
          split(i, kk, r);
          const uint32_t off = ctab[kk];
          go[u] = off != kZero;
          x[u] = *reinterpret_cast<const uint4*>(lrows + (go[u] ? off + r : kZero));
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
          const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
          const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 2);
          if constexpr (kRecord) {
            if (go[u] && inr) {
              *reinterpret_cast<uint4*>(out + i) = x[u];
              const uint64_t cw = (out - a.seen) + i;
              record_word(a.hop_rec, cw, static_cast<uint64_t>(x[u].y) << 32 | x[u].x, round);
              record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(x[u].w) << 32 | x[u].z, round);
            }
          } else {
            store_row16<kNT>(out + i, x[u]);
          }
          const bool own = go[u] && inr;
          ctr_unit(c, own, popc4(x[u]), 2u);
        }
      }
    } else {
      for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 64) {
        uint64_t m[kU];
        bool go[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
          const uint32_t i = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 1);
          int32_t kk, r;
          split(i, kk, r);
          const uint32_t off = ctab[kk];
          go[u] = off != kZero;
          m[u] = lrows[go[u] ? off + r : kZero];
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
          const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
          const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
          const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 1);
          if constexpr (kRecord) {
            if (go[u] && inr) {
              out[i] = m[u];
              record_word(a.hop_rec, (out - a.seen) + i, m[u], round);
            }
          } else {
            store_row8<kNT>(out + i, m[u]);
          }
          const bool own = go[u] && inr;
          ctr_unit(c, own, __popcll(m[u]), 1u);
        }
      }
    }
    ctr_fold(c);
  }
}

__device__ __forceinline__ void ctr_add(WaveCtr& d, const WaveCtr& s) {
  d.deliv += s.deliv;  // (one phase-A run: <= kPairWords * 64 bits, folded below)
  d.dsum += s.dsum;
  d.sw += s.sw;
  d.kids += s.kids;
  d.reached += s.reached;
  d.parents += s.parents;
  d.pwords += s.pwords;
}

// Counters of a wave (two rounds) added with its own atomics: no block
// reduction, so no barrier.
__device__ __forceinline__ void pull_flush_wave(const WaveCtr& c, uint64_t* partials, uint64_t slot, uint32_t lane) {
  const uint64_t v7[7] = {c.dsum + __reduce_add_sync(~0ull, c.deliv), c.sw, c.kids, c.reached, c.parents,
                          c.pwords, 0ull};
  if (lane < kNumCtr) {
    const uint64_t v = pull_ctr_pick(v7, lane);
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(partials + slot * kNumCtr + lane),
                     static_cast<unsigned long long>(v));
  }
}

// One wave per workgroup, one chunk per wave (grid = n_chunks; the loop
// only guards a smaller grid).  A chunk's two phases take longer when its
// run has more children: one-wave workgroups never wait for siblings (a
// 4-wave block's barrier held its LDS behind the slowest chunk: cfg3 (18,19)
// 583 -> 549 us).  Persistent waves looping over chunks measured slower at
// every grid tried (resident grid 700 us, 8192 waves 588 us, one chunk per
// wave 543 us): a wave's chunks run back to back, each paying its round
// trips, where fresh waves overlap them.
template <bool kRecord, bool kNT2>
__global__ __launch_bounds__(64) void k_pull_pair(PullArgs a, const PullChunk* __restrict__ chunks,
                                                  uint32_t n_chunks, uint32_t round) {
  __shared__ uint64_t rows[kPairWords + 2];  // + the zero pair
  __shared__ uint64_t src[kPairPar];         // phase A sources, then phase B's ctab
  __shared__ uint32_t gen_lds[kPairPar / 4 + 2];
  __shared__ uint64_t reach[kPairPar / 64];
  static_assert(kPairKids * 4 <= kPairPar * 8, "ctab fits the source table");
  const uint32_t lane = threadIdx.x;
  uint8_t* genl = reinterpret_cast<uint8_t*>(gen_lds);
  const uint32_t cur = a.gen_cur & 0xFF;
  if (lane < 2) rows[kPairWords + lane] = 0;
  WaveCtr c, c2;
  for (uint32_t ci = blockIdx.x; ci < n_chunks; ci += gridDim.x) {
    const PullChunk ch = chunks[ci];
    const TopicDev T = a.topics[ch.topic];
    PullTopic P;
    P.W = ch.W;
    P.nbase = T.nbase;
    P.base = (static_cast<uint64_t>(ch.row0_hi) << 32 | ch.row0_lo) - static_cast<uint64_t>(T.nbase) * ch.W;
    P.root = (T.flags & kTopicRootLocal) ? T.nbase : kNoneNode;
    const uint32_t n1 = ch.node_end - ch.node_begin;  // <= kPairPar, n1 * W <= kPairWords (host plan)
    const bool late = ch.c_lo == kNoneNode;           // a level-1 run of round q + 1
    // the first children's metadata, issued ahead of phase A's own
    uint32_t pf_p[kPairKids / 64], pf_f[kPairKids / 64];
    const uint32_t nk0 = late ? 0u : min(kPairKids, ch.c_hi - ch.c_lo);
#pragma unroll
    for (uint32_t s = 0; s < kPairKids / 64; ++s) {
      const uint32_t j = s * 64 + lane;
      pf_p[s] = j < nk0 ? a.node_parent[ch.c_lo + j] : kNoneNode;
      pf_f[s] = j < nk0 ? a.node_flags[ch.c_lo + j] : 0u;
    }
    WaveCtr ca;
    pull_resolve(a, P, ch.node_begin, n1, ch.p_lo, ch.p_hi, src, genl, lane, cur, ca, ch.gin, kPairPar);
    for (uint32_t j0 = 0; j0 < n1; j0 += 64) {
      const uint64_t b = __ballot(j0 + lane < n1 && src[j0 + lane] != 0);
      if (lane == 0) reach[j0 >> 6] = b;
    }
    pull_stream<kRecord, true, true>(a, P, ch.node_begin, n1, src, lane, round + (late ? 1 : 0), ca, rows);
    ctr_fold(ca);
    // src (u64 sources) and ctab (u32 offsets) share the LDS table: no memory
    // access may move across the switch from one view to the other
    asm volatile("" ::: "memory");
    if (late) {
      ctr_add(c2, ca);
    } else {
      ctr_add(c, ca);
      if (ch.c_hi > ch.c_lo)
        pair_kids<kRecord, kNT2, kPairWords>(a, P, ch.node_begin, n1, ch.c_lo, ch.c_hi, reach, rows,
                                             reinterpret_cast<uint32_t*>(src), lane, round + 1, pf_p, pf_f, c2);
    }
    asm volatile("" ::: "memory");
  }
  pull_flush_wave(c, a.partials, blockIdx.x % a.slot_mod, lane);
  pull_flush_wave(c2, a.partials2, blockIdx.x % a.slot_mod, lane);
}

// Children ranges of the pair chunks (GPU or host node space alike).
__global__ __launch_bounds__(kBlock) void k_pair_kids(PullChunk* __restrict__ chunks, uint32_t n,
                                                      const uint32_t* __restrict__ row_ptr,
                                                      const uint32_t* __restrict__ col) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  PullChunk& c = chunks[i];
  if (c.c_lo == kNoneNode) return;
  const uint32_t rb = row_ptr[c.node_begin], re = row_ptr[c.node_end];
  c.c_lo = re > rb ? col[rb] : 0u;
  c.c_hi = re > rb ? col[re - 1] + 1u : 0u;
}

// Multi-GPU level mode: the topic roots' records of a round (the roots are
// seeded, so always reached).  Thread i of the flattened stream copies unit i
// of one record -- a 16-B word pair for even W, one word for odd W: segment
// (one root, constant W) by a short scan, entry = offset / units per row.
__global__ __launch_bounds__(kBlock) void k_pack(const ShipEntry* __restrict__ ship,
                                                 const PackSeg* __restrict__ segs, uint32_t n_segs,
                                                 uint64_t total, const GhostSeg* __restrict__ gsegs,
                                                 const uint64_t* __restrict__ seen, uint64_t* __restrict__ send) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < total;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    uint32_t k = 0;
    while (k + 1 < n_segs && segs[k + 1].unit0 <= i) ++k;
    const PackSeg S = segs[k];
    const bool pairs = !(S.W & 1u);
    const uint32_t per = pairs ? S.W >> 1 : S.W;  // units per row
    const uint32_t o = static_cast<uint32_t>(i - S.unit0);
    const uint32_t e = S.e0 + o / per;
    const uint32_t w = (o - (e - S.e0) * per) << (pairs ? 1 : 0);
    const ShipEntry E = ship[e];
    uint64_t* rec = send + gsegs[S.gseg].sbase[E.dst >> kRemoteRankShift] +
                    static_cast<uint64_t>(E.dst & kRemoteIdMask) * S.W;
    const uint64_t* row = seen + S.row + w;
    if (pairs)
      *reinterpret_cast<uint4*>(rec + w) = *reinterpret_cast<const uint4*>(row);
    else
      rec[w] = *row;
  }
}

// GPU-built node spaces have no host mirror of node_parent: the chunks'
// parent ranges (k_pull's generation staging) are filled in on the device.
__global__ __launch_bounds__(kBlock) void k_chunk_parents(PullChunk* __restrict__ chunks, uint32_t n,
                                                          const uint32_t* __restrict__ node_parent) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  PullChunk& c = chunks[i];
  if (c.node_end <= c.node_begin) return;
  c.p_lo = node_parent[c.node_begin];
  c.p_hi = node_parent[c.node_end - 1];
}

// ------------------------------------------------------------- pull chain ---
// k_pull_chain: rounds q .. q + L - 1 in one launch (one
// rank, or rounds that exchange nothing).  A wave owns a run of level-d nodes
// and a column slice [w0, w0 + S) of their rows (S = W unless the rows are
// wider than the stage).  Level 0 (round q + r0): the run resolves its
// parents from this window's generation bytes, as k_pull does, and streams
// their rows from HBM into its own rows and the LDS stage.  Level k >= 1
// (round q + r0 + k): the run's descendants of that level, the contiguous
// ids [lo[k], hi[k]) (k_chain_ranges), in sub-runs of kChainKids: a node
// copies its parent's row as the level above wrote it -- if the parent was
// reached and the node is live -- and the level above wrote the row of its
// stage slot, so each node's entry in the level table is that slot
// (kChainNone: unreached).  No level below the run reads a row from HBM, and
// every level's rows form one contiguous output stream (S = W).  An
// unreached node's row is written with zeros (stale under its old generation
// byte, never read).  Slices are independent (a row is copied word for
// word), so the waves of one run's slices agree on every reach decision;
// only the slice-0 wave stamps generations and counts nodes.
struct ChainStep {
  uint64_t base;   // row of node u = base + u * W (+ w0)
  uint32_t W, w0, S, nbase;
  bool slice0;
};

// The element split of a slice stream: element i of a run of nodes with S
// words each -> (node kk, word r), branch-free (float estimate off by at most
// one; i < 2^24).
__device__ __forceinline__ void chain_split(uint32_t i, float rs, uint32_t S, int32_t& kk, int32_t& r) {
  kk = static_cast<int32_t>(static_cast<float>(i) * rs);
  r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(S);
  const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(S);
  kk += hi - lo;
  r += (lo - hi) * static_cast<int32_t>(S);
}

// Column slices (S < W): streams nk nodes' slices [y0, y0 + nk): element
// (kk, r) = source slot tab[kk] (LDS offset into `stage`, kZero: zeros)
// + r -- or, level 0, the parent row address src64[kk] (0: rewrite the
// node's own words) -- into the node's row in HBM and, when dst !=
// kNoneNode, the stage at dst + kk * S + r.  16-B units (even S) or words;
// lanes past the end repeat the last unit.
template <bool kRecord, bool kNT, bool kFromHbm, uint32_t kZero>
__device__ __forceinline__ void chain_stream(const PullArgs& a, const ChainStep& C, uint32_t y0, uint32_t nk,
                                             const uint32_t* tab, const uint64_t* src64, uint64_t* stage,
                                             uint32_t dst, uint32_t lane, uint32_t round, WaveCtr& c) {
  constexpr uint32_t kU = 8;
  const uint32_t S = C.S, W = C.W;
  const uint32_t total = nk * S;
  if (total == 0) return;
  uint64_t* const out = a.seen + C.base + static_cast<uint64_t>(y0) * W + C.w0;
  const float rs = 1.0f / static_cast<float>(S);
  if (!(S & 1u)) {
    for (uint32_t i0 = 0; i0 < total; i0 += kU * 128) {
      uint4 x[kU];
      bool go[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t is = i0 + u * 128 + 2 * lane;
        const uint32_t i = is < total ? is : total - 2;
        int32_t kk, r;
        chain_split(i, rs, S, kk, r);
        const uint64_t* q;
        if constexpr (kFromHbm) {
          const uint64_t row = src64[kk];
          go[u] = row != 0;
          q = go[u] ? reinterpret_cast<const uint64_t*>(row) + C.w0 + r : out + static_cast<uint64_t>(kk) * W + r;
        } else {
          const uint32_t off = tab[kk];
          go[u] = off != kZero;
          q = stage + (go[u] ? off + r : kZero);
        }
        x[u] = *reinterpret_cast<const uint4*>(q);
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t is = i0 + u * 128 + 2 * lane;
        const bool inr = is < total;
        const uint32_t i = inr ? is : total - 2;
        int32_t kk, r;
        chain_split(i, rs, S, kk, r);
        uint64_t* o = out + static_cast<uint64_t>(kk) * W + r;
        if constexpr (kRecord) {
          if (go[u] && inr) {
            *reinterpret_cast<uint4*>(o) = x[u];
            const uint64_t cw = o - a.seen;
            record_word(a.hop_rec, cw, static_cast<uint64_t>(x[u].y) << 32 | x[u].x, round);
            record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(x[u].w) << 32 | x[u].z, round);
          } else if (!kFromHbm && inr) {
            *reinterpret_cast<uint4*>(o) = x[u];  // (zeros of an unreached node)
          }
        } else {
          store_row16<kNT>(o, x[u]);
        }
        if (dst != kNoneNode) *reinterpret_cast<uint4*>(stage + dst + kk * S + r) = x[u];
        ctr_unit(c, go[u] && inr, popc4(x[u]), 2u);
      }
    }
  } else {
    for (uint32_t i0 = 0; i0 < total; i0 += kU * 64) {
      uint64_t m[kU];
      bool go[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t is = i0 + u * 64 + lane;
        const uint32_t i = is < total ? is : total - 1;
        int32_t kk, r;
        chain_split(i, rs, S, kk, r);
        const uint64_t* q;
        if constexpr (kFromHbm) {
          const uint64_t row = src64[kk];
          go[u] = row != 0;
          q = go[u] ? reinterpret_cast<const uint64_t*>(row) + C.w0 + r : out + static_cast<uint64_t>(kk) * W + r;
        } else {
          const uint32_t off = tab[kk];
          go[u] = off != kZero;
          q = stage + (go[u] ? off + r : kZero);
        }
        m[u] = *q;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const uint32_t is = i0 + u * 64 + lane;
        const bool inr = is < total;
        const uint32_t i = inr ? is : total - 1;
        int32_t kk, r;
        chain_split(i, rs, S, kk, r);
        uint64_t* o = out + static_cast<uint64_t>(kk) * W + r;
        if constexpr (kRecord) {
          if (go[u] && inr) {
            *o = m[u];
            record_word(a.hop_rec, o - a.seen, m[u], round);
          } else if (!kFromHbm && inr) {
            *o = m[u];
          }
        } else {
          store_row8<kNT>(o, m[u]);
        }
        if (dst != kNoneNode) stage[dst + kk * S + r] = m[u];
        ctr_unit(c, go[u] && inr, static_cast<uint32_t>(__popcll(m[u])), 1u);
      }
    }
  }
}

// Whole rows (S = W): the nodes [y0, y0 + nk) as one line-aligned output
// stream from the stage (ctab[kk]: the stage offset of node kk's source row,
// kZero: the zero pair), k_pull's 8-in-flight pipeline with LDS sources.
template <bool kRecord, bool kNT, uint32_t kZero>
__device__ __forceinline__ void stage_stream(const PullArgs& a, uint64_t* out, uint32_t nk, uint32_t W,
                                             const uint32_t* ctab, const uint64_t* lrows, uint32_t lane,
                                             uint32_t round, WaveCtr& c) {
  constexpr uint32_t kU = 8;
  const float rw = 1.0f / static_cast<float>(W);
  auto split = [&](uint32_t i, int32_t& kk, int32_t& r) {
    kk = static_cast<int32_t>(static_cast<float>(i) * rw);
    r = static_cast<int32_t>(i) - kk * static_cast<int32_t>(W);
    const int32_t lo = r < 0, hi = r >= static_cast<int32_t>(W);
    kk += hi - lo;
    r += (lo - hi) * static_cast<int32_t>(W);
  };
  const uint32_t total = nk * W;
  const uint32_t h = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(out) & 127) >> 3;
  if (!(W & 1u)) {
    for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 128) {
      uint4 x[kU];
      bool go[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
        const uint32_t i = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 2);
        int32_t kk, r;
        split(i, kk, r);
        const uint32_t off = ctab[kk];
        go[u] = off != kZero;
        x[u] = *reinterpret_cast<const uint4*>(lrows + (go[u] ? off + r : kZero));
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 128 + 2 * lane) - static_cast<int32_t>(h);
        const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
        const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 2);
        if constexpr (kRecord) {
          if (go[u] && inr) {
            *reinterpret_cast<uint4*>(out + i) = x[u];
            const uint64_t cw = (out - a.seen) + i;
            record_word(a.hop_rec, cw, static_cast<uint64_t>(x[u].y) << 32 | x[u].x, round);
            record_word(a.hop_rec, cw + 1, static_cast<uint64_t>(x[u].w) << 32 | x[u].z, round);
          } else if (inr) {
            *reinterpret_cast<uint4*>(out + i) = x[u];  // (zeros of an unreached node)
          }
        } else {
          store_row16<kNT>(out + i, x[u]);
        }
        ctr_unit(c, go[u] && inr, popc4(x[u]), 2u);
      }
    }
  } else {
    for (uint32_t i0 = 0; i0 < total + h; i0 += kU * 64) {
      uint64_t m[kU];
      bool go[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
        const uint32_t i = is < 0 ? 0u : (static_cast<uint32_t>(is) < total ? static_cast<uint32_t>(is) : total - 1);
        int32_t kk, r;
        split(i, kk, r);
        const uint32_t off = ctab[kk];
        go[u] = off != kZero;
        m[u] = lrows[go[u] ? off + r : kZero];
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) {
        const int32_t is = static_cast<int32_t>(i0 + u * 64 + lane) - static_cast<int32_t>(h);
        const bool inr = is >= 0 && static_cast<uint32_t>(is) < total;
        const uint32_t i = is < 0 ? 0u : (inr ? static_cast<uint32_t>(is) : total - 1);
        if constexpr (kRecord) {
          if (go[u] && inr) {
            out[i] = m[u];
            record_word(a.hop_rec, (out - a.seen) + i, m[u], round);
          } else if (inr) {
            out[i] = m[u];
          }
        } else {
          store_row8<kNT>(out + i, m[u]);
        }
        ctr_unit(c, go[u] && inr, static_cast<uint32_t>(__popcll(m[u])), 1u);
      }
    }
  }
}

// Levels 1 .. levels - 1 of a chain chunk, as metadata preloaded into
// registers: per node its parent's index in the level above (relative to that
// level's first node, < kChainCap) and its live flag, in 16 bits, two nodes
// per register -- kMetaSlots slots of 64 nodes per batch, the levels one
// after the other, each from a slot boundary.  The first batch is issued at
// the wave's start, beside level 0's loads, so the level loop issues no
// global load at all: gfx950 counts loads and stores on one in-order counter
// (vmcnt), and a load issued behind a level's row stores could be consumed
// only once those stores had drained -- which the previous form (each
// sub-run's ids loaded before the sub-run above streamed, and a per-group
// load of the previous node's parent for the counters) paid at every level
// (profiles/r04/chain_prof_*: 5 us fixed + 4.9 us per 8-KB row-kword per wave).
constexpr uint32_t kMetaSlots = 16;      // 64-node slots per batch: 1,024 nodes
constexpr int kWaitVmcnt0 = 0x0F70;      // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding)
constexpr uint32_t kMetaNone = 0xFFFFu;  // no node at the lane's position
constexpr uint32_t kMetaLive = 0x4000u;  // the node is live (below: the parent's index)
struct ChainMeta {
  uint32_t w[kMetaSlots / 2];  // slot i in half i & 1 of w[i / 2]
  uint32_t g0;                 // the batch's first global slot
};

// Walks the metadata slots (64 nodes of a chunk's levels 0 .., each level
// from a slot boundary) level by level: the level k of slot g, its first slot
// kb, its slot count ns, its node range [lo, hi) and the first node plo of the
// level above (level 0: the run's first parent).  Wave-uniform; no loop per
// slot, so the callers' slot loops unroll.  (A level with no node ends the
// walk: every deeper level is empty too.)
struct MetaCursor {
  uint32_t k, kb, ns, lo, hi, plo;
  uint32_t mb;  // the level's first entry in the chunk's chain_meta entries
  __device__ __forceinline__ void enter(const ChainChunk* cp, uint32_t levels) {
    if (k >= levels) return;
    plo = lo;
    mb += hi - lo;  // (the level above's entries; level 0: none, hi = lo = p_lo)
    lo = __builtin_amdgcn_readfirstlane(cp->lo[k]);
    hi = __builtin_amdgcn_readfirstlane(cp->hi[k]);
    ns = (hi - lo + 63) >> 6;
    if (ns == 0) k = levels;
  }
  // the cursor at slot g0 (p_lo: the run's first parent)
  __device__ __forceinline__ void start(const ChainChunk* cp, uint32_t levels, uint32_t g0, uint32_t p_lo) {
    k = 0;
    kb = 0;
    mb = 0;
    lo = hi = p_lo;
    enter(cp, levels);
    while (k < levels && g0 >= kb + ns) {
      kb += ns;
      ++k;
      enter(cp, levels);
    }
  }
  // the cursor at slot g (g = the previous slot + 1)
  __device__ __forceinline__ void step(const ChainChunk* cp, uint32_t levels, uint32_t g) {
    if (k < levels && g >= kb + ns) {
      kb += ns;
      ++k;
      enter(cp, levels);
    }
  }
};

// Issues the batch of slots g0 .. g0 + kMetaSlots - 1: the nodes' entries,
// contiguous per chunk in level order (k_chain_meta), 2 B per lane -- one
// 128-B line per slot -- into q (unconsumed, so nothing waits here).
// (Before round 5: each node's parent id and flag dword, two scattered
// lines per slot: ~1 KB of line-granular reads per wave.)
__device__ __forceinline__ void chain_meta_issue(const PullArgs& a, const ChainChunk* cp, uint32_t levels,
                                                 uint32_t p_lo, uint32_t g0, uint32_t lane, uint32_t moff,
                                                 uint32_t (&q)[kMetaSlots]) {
  MetaCursor m;
  m.start(cp, levels, g0, p_lo);
#pragma unroll
  for (uint32_t i = 0; i < kMetaSlots; ++i) {
    if (i) m.step(cp, levels, g0 + i);
    if (m.k >= levels) break;  // (past the chunk's last level: no loads)
    const uint32_t y = m.lo + (g0 + i - m.kb) * 64 + lane;
    const uint32_t yi = moff + (y < m.hi ? m.mb + (y - m.lo) : 0u);  // (clamped: the chunk's first entry)
    q[i] = a.chain_meta[yi];
  }
}

// Packs the issued batch (the first use of q: the loads' wait).
__device__ __forceinline__ void chain_meta_pack(const ChainChunk* cp, uint32_t levels, uint32_t p_lo, uint32_t g0,
                                                uint32_t lane, const uint32_t (&q)[kMetaSlots], ChainMeta& M) {
  M.g0 = g0;
  MetaCursor m;
  m.start(cp, levels, g0, p_lo);
#pragma unroll
  for (uint32_t i = 0; i < kMetaSlots; ++i) {
    if (i) m.step(cp, levels, g0 + i);
    if (m.k >= levels) break;  // (the slots past it are never picked)
    const uint32_t y = m.lo + (g0 + i - m.kb) * 64 + lane;
    // (the direct path's level-0 entries are kMetaNone already: k_chain_meta)
    const uint32_t e = y < m.hi ? (q[i] & 0xFFFFu) : kMetaNone;
    if (i & 1)
      M.w[i / 2] |= e << 16;
    else
      M.w[i / 2] = e;
  }
  // every batch load has landed (slots past the chunk's last level are never
  // consumed): without this the waitcnt pass keeps them pending across the
  // level loop and drains the row stores at its head
  __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
}

// The lane's entry of batch slot i (wave-uniform i < kMetaSlots): a select
// chain over the registers (no dynamic register index).
__device__ __forceinline__ uint32_t chain_meta_pick(const ChainMeta& M, uint32_t i) {
  uint32_t w = M.w[0];
#pragma unroll
  for (uint32_t r = 1; r < kMetaSlots / 2; ++r) {
    uint32_t t = M.w[r];
    asm volatile("" : "+v"(t));  // (a register value: keeps the chain from becoming an indexed scratch load)
    w = (i >> 1) == r ? t : w;
  }
  return (i & 1) ? w >> 16 : w & 0xFFFFu;
}

// One group of 64 nodes of level k (entry e per lane; j = the lane's index
// in the sub-run, y its node): the node's stage offset into ctab (kZero:
// zeros) and its own level-table entry into tab; generation stamped and nodes
// counted by the slice-0 wave.  carry: the parent index of the group's last
// node, for the next group's first (a parent counts once, at its first
// child).  pw: parent-row words read per counted parent (level 0: the
// parents' rows came from HBM; deeper levels: none, they are stage rows).
template <uint32_t kZero>
__device__ __forceinline__ void chain_group(const PullArgs& a, const ChainStep& C, uint32_t e, const uint8_t* up_tab,
                                            uint32_t y, uint32_t j, uint32_t* ctab, uint8_t* tab, uint32_t cur,
                                            uint32_t lane, uint32_t pw, uint32_t& carry, WaveCtr& c) {
  const bool in = e != kMetaNone;
  const uint32_t rel = e & (kMetaLive - 1);
  const uint8_t src = in ? up_tab[rel] : kChainNone;  // the parent's stage slot
  const bool up = in && ((a.all_current & 1u) || src != kChainNone);
  const bool ok = up && (e & kMetaLive);
  if (in) {
    ctab[j] = (ok && src < kChainZero) ? static_cast<uint32_t>(src) * C.S : kZero;
    tab[j] = ok ? (src < kChainZero ? src : kChainZero) : kChainNone;
  }
  if (ok && C.slice0) a.gen[y] = static_cast<uint8_t>(cur);
  const uint32_t mine = in ? rel : kNoneNode;
  uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(mine), 1, 64));
  if (lane == 0) prev = carry;
  carry = __builtin_amdgcn_readlane(mine, 63);
  // nodes and parents counted once per run (slice 0); words per slice
  const bool first = up && rel != prev;
  ctr_nodes(c, in && C.slice0, ok && C.slice0, first && C.slice0, C.S, pw);
  if (!C.slice0) {
    c.sw += static_cast<uint64_t>(__popcll(__ballot(ok))) * C.S;
    c.pwords += static_cast<uint64_t>(__popcll(__ballot(first))) * pw;
  }
}

// The partial slots of round r0 + k of a chain launch (a switch: no dynamic
// index into the kernel arguments).
__device__ __forceinline__ uint64_t* chain_slots(const PullArgs& a, uint32_t i) {
  switch (i) {
    case 0: return a.partials_r[0];
    case 1: return a.partials_r[1];
    case 2: return a.partials_r[2];
    case 3: return a.partials_r[3];
    case 4: return a.partials_r[4];
    default: return a.partials_r[5];
  }
}

__device__ __forceinline__ void chain_flush(WaveCtr& c, uint64_t* partials, uint64_t slot, uint32_t lane) {
  ctr_fold(c);
  const uint64_t v7[7] = {c.dsum, c.sw, c.kids, c.reached, c.parents, c.pwords, 0ull};
  if (partials && lane < kNumCtr) {
    const uint64_t v = pull_ctr_pick(v7, lane);
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(partials + slot * kNumCtr + lane),
                     static_cast<unsigned long long>(v));
  }
  c = WaveCtr{};
}

__global__ __launch_bounds__(kBlock) void k_chain_parents(ChainChunk* __restrict__ chunks, uint32_t n,
                                                          const uint32_t* __restrict__ node_parent) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  ChainChunk& c = chunks[i];
  c.p_lo = node_parent[c.node_begin];
  c.p_hi = node_parent[c.node_end - 1];
}

// The descendant ranges of every chain chunk: in BFS order the children of
// the level-(d + k) nodes [x0, x1) are the level-(d + k + 1) nodes
// first[k + 1] + [row_ptr[x0], row_ptr[x1]) - row_ptr[first[k]].  A range
// wider than `cap` (the LDS level tables) flags the plan as unusable.
__global__ __launch_bounds__(kBlock) void k_chain_ranges(ChainChunk* __restrict__ chunks, uint32_t n,
                                                         const uint32_t* __restrict__ row_ptr, uint32_t cap,
                                                         uint32_t* __restrict__ overflow) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  ChainChunk& c = chunks[i];
  uint32_t x0 = c.node_begin, x1 = c.node_end;
  bool over = false;
  c.lo[0] = x0;
  c.hi[0] = x1;
  for (uint32_t k = 1; k < c.levels && k < kChainLevels; ++k) {
    const uint32_t base = row_ptr[c.first[k - 1]];
    const uint32_t y0 = c.first[k] + (row_ptr[x0] - base), y1 = c.first[k] + (row_ptr[x1] - base);
    c.lo[k] = y0;
    c.hi[k] = y1;
    over |= y1 - y0 > cap;
    x0 = y0;
    x1 = y1;
  }
  if (over) atomicOr(overflow, 1u);
}

// Level 0 of a chain chunk whose parent span is wider than the stage (the
// run's parents are consecutive ids, but childless ones between them count
// in the span): the run resolves its parents as k_pull does and streams their
// rows from HBM into its own rows and the stage at its own slots (run nodes *
// S <= kStage, host plan); the run's level table holds each reached node's
// own slot.  (Eager seen, PS_F_NO_LAZY_SEEN: an unreached node's slot holds
// its own row, zeros, so every node keeps its slot.)  src: kChainPar row
// addresses (the ctab LDS, dead until level 1).
template <bool kRecord, bool kNT, bool kSlices>
__device__ __forceinline__ void chain_level0_direct(const PullArgs& a, const ChainStep& C, const ChainChunk* cp,
                                                 uint32_t p_lo, uint32_t p_hi, uint64_t* src, uint8_t* genl,
                                                 uint64_t* stage, uint8_t* tab0, uint32_t lane, uint32_t cur,
                                                 uint32_t round, uint64_t slot, uint64_t* partials,
                                                 uint64_t& words_out) {
  constexpr uint32_t kStage = kChainWords;
  const uint32_t node_begin = cp->node_begin, n0 = cp->node_end - node_begin;
  PullTopic P;
  P.W = C.W;
  P.nbase = C.nbase;
  P.base = C.base;
  P.root = cp->root;
  WaveCtr c;
  if constexpr (!kSlices) {
    pull_resolve(a, P, node_begin, n0, p_lo, p_hi, src, genl, lane, cur, c, kNoneNode, kChainPar);
    pull_stream<kRecord, kNT, true>(a, P, node_begin, n0, src, lane, round, c, stage);
  } else {
    // (pull_resolve stamps generations and counts whole rows: slice 0 keeps
    // its node counts, every slice its own words)
    PullCtr pc;
    pull_resolve(a, P, node_begin, n0, p_lo, p_hi, src, genl, lane, cur, pc, kNoneNode, kChainPar);
    const uint32_t nodes = __reduce_add_sync(~0ull, pc.kids), hit = __reduce_add_sync(~0ull, pc.reached);
    const uint32_t par = __reduce_add_sync(~0ull, pc.parents);
    if (C.slice0) {
      c.kids += __builtin_amdgcn_readfirstlane(nodes);
      c.reached += __builtin_amdgcn_readfirstlane(hit);
      c.parents += __builtin_amdgcn_readfirstlane(par);
    }
    c.sw += static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(hit)) * C.S;
    c.pwords += static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(par)) * C.S;
    chain_stream<kRecord, kNT, true, kStage>(a, C, node_begin, n0, nullptr, src, stage, 0u, lane, round, c);
  }
  for (uint32_t j = lane; j < n0; j += 64)
    tab0[j] = (src[j] != 0 || (a.all_current & 1u)) ? static_cast<uint8_t>(j) : kChainNone;
  words_out += c.sw;
  chain_flush(c, partials, slot, lane);
}

// kSlices: the launch's chunks of rows wider than the stage (column slices,
// a separate launch: the whole-row path keeps its registers).  kInNT: every
// level but the launch's last stores non-temporally (the default;
// ps_plan_opts.chain_nt = 0: plain stores, A/B); kNT: the last level too.
//
// One round trip before the first store: a run's parents are consecutive
// ids, so their rows (slices) are one block, copied into the stage by
// LDS-DMA beside the metadata batch (the run and its descendants) and the
// parents' generation bytes.  In a single-start window a reached node's row
// is its parent's row, so level 0 is written from the stage like every level
// below it: the parents' table (level -1) holds each reached parent's stage
// slot.  (The previous form read the topic table, then the run's metadata,
// then the parent rows: three dependent round trips per wave, 15 % of a
// bulk-launch wave's life, profiles/r04/chain_prof_*.)
template <bool kRecord, bool kNT, bool kSlices, bool kInNT = true, uint32_t kSimdWaves = 0>
__global__ __launch_bounds__(64) void k_pull_chain(PullArgs a, const ChainChunk* __restrict__ chunks,
                                                   uint32_t n_chunks, uint32_t round) {
  // kSimdWaves (3): a register the kernel never uses, declared clobbered,
  // sizes its VGPR allocation so that exactly that many waves fit per SIMD --
  // a residency cap spread evenly over the CU's 4 SIMDs (an LDS cap leaves
  // the placement to the dispatcher: 12 waves per CU 0.920 ms/step on cfg3,
  // 3 per SIMD 0.90, profiles/r04/ab_chain_waves.txt)
  if constexpr (kSimdWaves == 3) asm volatile("" ::: "v140");
  constexpr uint32_t kStage = kChainWords, kCap = kChainCap;
  __shared__ __attribute__((aligned(16))) uint64_t stage[kStage + 2];  // the parents' rows (slices); + the zero pair
  __shared__ __attribute__((aligned(16))) uint32_t ctab[kChainKids];   // a sub-run's stage offsets
  static_assert(kChainKids * 4 >= kChainPar * 8, "ctab holds the direct level 0's row addresses");
  __shared__ uint32_t gen_lds[kChainPar / 4 + 2];                      // the parents' generation bytes
  __shared__ uint8_t tabs[2][kCap];  // level tables: this level's and the one above (level -1: the parents)
  const uint32_t lane = threadIdx.x;
  const uint32_t cur = a.gen_cur & 0xFF;
  const uint32_t ci = blockIdx.x;
  if (ci >= n_chunks) return;
  // debug profile (PSAMD_CHAIN_PROFILE): the wave's start, end and words
  const uint64_t t_start = a.prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
  uint64_t words_out = 0;
  const ChainChunk* const cp = chunks + ci;
  // (levels and r0 through their dword: a sub-dword field read becomes a
  // vector load, one more round trip before the first store)
  static_assert(offsetof(ChainChunk, levels) == 40 && offsetof(ChainChunk, r0) == 41, "ChainChunk layout");
  const uint32_t lr = reinterpret_cast<const uint32_t*>(cp)[10];
  const uint32_t p_lo = cp->p_lo, p_hi = cp->p_hi, levels = lr & 0xFFu, r0 = (lr >> 8) & 0xFFu;
  ChainStep C;
  C.W = cp->W;
  C.w0 = kSlices ? cp->w0 : 0u;
  C.S = kSlices ? cp->S : C.W;
  C.nbase = cp->nbase;
  C.base = (static_cast<uint64_t>(cp->row0_hi) << 32 | cp->row0_lo) - static_cast<uint64_t>(C.nbase) * C.W;
  C.slice0 = C.w0 == 0;
  const uint64_t slot = blockIdx.x % a.slot_mod;
  // the parents [p_lo, p_hi]: their rows (slices) and generation bytes.  The
  // span holds every parent id between the run's first and last, childless
  // ones too, so it may exceed the run (the host sizes runs, not spans): a
  // span wider than the stage takes the direct path (level 0 from HBM, after
  // the metadata: one round trip more)
  const uint32_t n_par = p_hi - p_lo + 1;
  const bool direct = n_par > kChainPar || n_par * C.S > kStage;
  const uint32_t words = n_par * C.S;
  const uint64_t* prow = (p_lo == cp->root ? a.a_cur : a.seen) + C.base + static_cast<uint64_t>(p_lo) * C.W + C.w0;
  const uint32_t g0 = p_lo & ~3u;
  const uint32_t n_gd = (((p_hi + 4u) & ~3u) - g0) >> 2;  // the parents' generation dwords (<= kChainPar / 4 + 1)
  // the previous node's parent: a parent whose children straddle two runs counts once
  const uint32_t pm = cp->node_begin > C.nbase ? a.node_parent[cp->node_begin - 1] : kNoneNode;
  ChainMeta M;
  const uint32_t moff = cp->first[kChainLevels];  // (device copy: the chunk's first chain_meta entry)
  {
    uint32_t mq[kMetaSlots];
    chain_meta_issue(a, cp, levels, p_lo, 0u, lane, moff, mq);
    if (!direct) {
      if (lane < n_gd) PSAMD_DMA(reinterpret_cast<const uint32_t*>(a.gen + g0) + lane, gen_lds, 4);
      if (!(C.W & 1u)) {
        // 16-B units (even rows and slices start 16-B aligned), 1 KB per instruction
        const uint32_t units = words >> 1;
        const float rs = 1.0f / static_cast<float>(C.S);
        for (uint32_t u0 = 0; u0 < units; u0 += 64) {
          const uint32_t u = min(u0 + lane, units - 1);  // (lanes past the end repeat the last unit)
          int32_t kk, r;
          chain_split(2 * u, rs, C.S, kk, r);  // (word 2u: S is even, a unit never straddles two rows)
          PSAMD_DMA(prow + static_cast<uint64_t>(kk) * C.W + r, stage + 2 * u0, 16);
        }
      } else {
        // odd rows (whole rows only: slices are even): contiguous, dwords
        const uint32_t* pw32 = reinterpret_cast<const uint32_t*>(prow);
        for (uint32_t d0 = 0; d0 < 2 * words; d0 += 64)
          PSAMD_DMA(pw32 + min(d0 + lane, 2 * words - 1), reinterpret_cast<uint32_t*>(stage) + d0, 4);
      }
    }
    chain_meta_pack(cp, levels, p_lo, 0u, lane, mq, M);  // (waits for every load above)
  }
  if (lane < 2) stage[kStage + lane] = 0;
  uint32_t g = 0;   // the global metadata slot of the next node group
  uint32_t k0 = 0;  // the first level of the loop below
  if (!direct) {
    // the parents' table: a reached parent's stage slot (eager seen,
    // PS_F_NO_LAZY_SEEN: every generation counts as current)
    const uint8_t* genl = reinterpret_cast<const uint8_t*>(gen_lds);
    for (uint32_t i = lane; i < n_par; i += 64)
      tabs[1][i] = (genl[p_lo + i - g0] == cur || (a.all_current & 1u)) ? static_cast<uint8_t>(i) : kChainNone;
  } else {
    chain_level0_direct<kRecord, kInNT, kSlices>(a, C, cp, p_lo, p_hi, reinterpret_cast<uint64_t*>(ctab),
                                                 reinterpret_cast<uint8_t*>(gen_lds), stage, tabs[0], lane, cur,
                                                 round + r0, slot, chain_slots(a, r0), words_out);
    g = (cp->node_end - cp->node_begin + 63) >> 6;  // (the batch's level-0 slots)
    k0 = 1;
    asm volatile("" ::: "memory");  // (level 0's sources become ctab)
  }
  // levels k0 .. levels - 1, sub-run by sub-run (<= kChainKids nodes): every
  // node's parent and flag come from the preloaded batch and every source
  // row from the stage, so no level waits for the stores above it; a batch
  // is reloaded only when a chunk's levels hold more than kMetaSlots slots (a
  // wait, rare: runs are sized for less)
  for (uint32_t k = k0; k < levels; ++k) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(cp->lo[k]), hi = __builtin_amdgcn_readfirstlane(cp->hi[k]);
    const uint8_t* const up_tab = tabs[(k - 1) & 1];
    uint32_t carry = k == 0 && pm == p_lo ? 0u : kNoneNode;
    WaveCtr c;
    for (uint32_t y0 = lo; y0 < hi; y0 += kChainKids) {
      const uint32_t nk = min(kChainKids, hi - y0);
      const uint32_t ng = (nk + 63) >> 6;
      if (g + ng > M.g0 + kMetaSlots) {
        uint32_t mq[kMetaSlots];
        chain_meta_issue(a, cp, levels, p_lo, g, lane, moff, mq);
        chain_meta_pack(cp, levels, p_lo, g, lane, mq, M);
      }
      uint8_t* const tab = tabs[k & 1] + (y0 - lo);
#pragma unroll
      for (uint32_t s = 0; s < kChainKids / 64; ++s) {
        if (s >= ng) break;
        chain_group<kStage>(a, C, chain_meta_pick(M, g + s - M.g0), up_tab, y0 + s * 64 + lane, s * 64 + lane, ctab,
                            tab, cur, lane, k == 0 ? C.S : 0u, carry, c);
      }
      g += ng;
      if constexpr (!kSlices) {
        uint64_t* out = a.seen + C.base + static_cast<uint64_t>(y0) * C.W;
        if (k + 1 < levels)  // (only the launch's last level may be re-read soon)
          stage_stream<kRecord, kInNT, kStage>(a, out, nk, C.W, ctab, stage, lane, round + r0 + k, c);
        else
          stage_stream<kRecord, kNT, kStage>(a, out, nk, C.W, ctab, stage, lane, round + r0 + k, c);
      } else {
        chain_stream<kRecord, kInNT, false, kStage>(a, C, y0, nk, ctab, nullptr, stage, kNoneNode, lane,
                                                    round + r0 + k, c);
      }
      ctr_fold(c);
    }
    words_out += c.sw;
    chain_flush(c, chain_slots(a, r0 + k), slot, lane);
    asm volatile("" ::: "memory");
  }
  if (a.prof) {
    // (HW_ID: wave, SIMD, CU, SE bits; XCC_ID[3:0], hwreg 20 on gfx950)
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    // (bit 40: level 0 took the direct path)
    const uint64_t v = lane == 0   ? t_start
                       : lane == 1 ? t_end
                       : lane == 2 ? words_out
                                   : (static_cast<uint64_t>(direct) << 40 | static_cast<uint64_t>(xcc) << 32 | hw);
    if (lane < kChainProf) a.prof[static_cast<uint64_t>(ci) * kChainProf + lane] = v;
  }
}

}  // namespace

namespace {
// Dynamic LDS that caps a launch at `waves` resident
// workgroups per CU (160 KB of LDS per CU, allocated in 512-B granules): the
// static LDS plus the pad stays above 160 KB / (waves + 1).  0: no cap.
template <class K>
size_t lds_cap_pad(K kernel, uint32_t waves) {
  if (waves == 0) return 0;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kernel)) != hipSuccess) return 0;
  const size_t per = (160u * 1024u) / waves - 512u;
  return per > fa.sharedSizeBytes ? per - fa.sharedSizeBytes : 0;
}
}  // namespace

hipError_t launch_pull(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks,
                       uint32_t grid, uint32_t round, bool record, bool nt, bool cap, hipStream_t s) {
  if (n_chunks == 0 || grid == 0) return hipSuccess;
  // cap: the large (nt) rounds run at most 5 blocks per CU -- 10 KB of LDS
  // left unused per block caps residency (8 blocks: 6 % slower on cfg3's big
  // rounds on one rank); small rounds keep full residency, they need the
  // waves in flight
  const size_t kBigRoundLdsPad = cap ? 10240 : 0;
  if (record)  // parity runs: one variant
    hipLaunchKernelGGL((k_pull<true, false>), dim3(grid), dim3(kBlock), 0, s, a, chunks, n_chunks, round);
  else if (nt)
    hipLaunchKernelGGL((k_pull<false, true>), dim3(grid), dim3(kBlock), kBigRoundLdsPad, s, a, chunks, n_chunks,
                       round);
  else
    hipLaunchKernelGGL((k_pull<false, false>), dim3(grid), dim3(kBlock), 0, s, a, chunks, n_chunks, round);
  return hipGetLastError();
}

hipError_t launch_pull_pair(const PullArgs& a, const PullChunk* chunks, uint32_t n_chunks, uint32_t grid,
                            uint32_t round, bool record, bool nt2, hipStream_t s) {
  if (n_chunks == 0 || grid == 0) return hipSuccess;
  grid = grid < n_chunks ? grid : n_chunks;
  if (record)
    hipLaunchKernelGGL((k_pull_pair<true, false>), dim3(grid), dim3(64), 0, s, a, chunks, n_chunks, round);
  else if (nt2)
    hipLaunchKernelGGL((k_pull_pair<false, true>), dim3(grid), dim3(64), 0, s, a, chunks, n_chunks, round);
  else
    hipLaunchKernelGGL((k_pull_pair<false, false>), dim3(grid), dim3(64), 0, s, a, chunks, n_chunks, round);
  return hipGetLastError();
}

hipError_t launch_pair_kids(PullChunk* chunks, uint32_t n, const uint32_t* row_ptr, const uint32_t* col,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_kids, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chunks, n, row_ptr, col);
  return hipGetLastError();
}

hipError_t launch_pack(const ShipEntry* ship, const PackSeg* segs, uint32_t n_segs, uint64_t total_units,
                       const GhostSeg* gsegs, const uint64_t* seen, uint64_t* send, hipStream_t s) {
  if (total_units == 0 || n_segs == 0) return hipSuccess;
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(4096, (total_units + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_pack, dim3(grid), dim3(kBlock), 0, s, ship, segs, n_segs, total_units, gsegs, seen, send);
  return hipGetLastError();
}

hipError_t launch_chunk_parents(PullChunk* chunks, uint32_t n, const uint32_t* node_parent, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_chunk_parents, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chunks, n, node_parent);
  return hipGetLastError();
}


hipError_t launch_chain_parents(ChainChunk* chunks, uint32_t n, const uint32_t* node_parent, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_chain_parents, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chunks, n, node_parent);
  return hipGetLastError();
}

namespace {
// per chunk: its nodes over the chain's levels (the ranges k_chain_ranges set)
__global__ __launch_bounds__(kBlock) void k_chain_meta_count(const ChainChunk* __restrict__ chunks, uint32_t n,
                                                             uint32_t* __restrict__ counts) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i > n) return;
  uint32_t c = 0;
  if (i < n) {
    const ChainChunk& ch = chunks[i];
    const uint32_t levels = ch.levels;
    for (uint32_t k = 0; k < levels && k < kChainLevels; ++k) c += ch.hi[k] - ch.lo[k];
  }
  counts[i] = c;  // (counts[n] = 0: the scan's total lands at offs[n])
}

// one wave per chunk: entry = parent index relative to the level above (level
// 0: to the run's first parent) | live bit, as chain_meta_pack packed them
// from node_parent / node_flags in the kernel; kMetaNone for level 0 of a run
// that takes the direct path (its entries are never picked)
__global__ __launch_bounds__(kBlock) void k_chain_meta_fill(ChainChunk* __restrict__ chunks, uint32_t n,
                                                            const uint32_t* __restrict__ offs,
                                                            const uint32_t* __restrict__ node_parent,
                                                            const uint8_t* __restrict__ node_flags,
                                                            uint32_t* __restrict__ meta) {
  const uint32_t ci = (blockIdx.x * kBlock + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (ci >= n) return;
  ChainChunk& ch = chunks[ci];
  const uint32_t off = offs[ci];
  const uint32_t levels = ch.levels, p_lo = ch.p_lo, p_hi = ch.p_hi, S = ch.S;
  const uint32_t n_par = p_hi - p_lo + 1;
  const bool direct = n_par > kChainPar || n_par * S > kChainWords;
  uint32_t base = 0, plo = p_lo;
  for (uint32_t k = 0; k < levels && k < kChainLevels; ++k) {
    const uint32_t lo = ch.lo[k], hi = ch.hi[k];
    for (uint32_t y = lo + lane; y < hi; y += 64) {
      uint32_t e = kMetaNone;
      if (k > 0 || !direct)
        e = ((node_parent[y] - plo) & (kMetaLive - 1)) | ((node_flags[y] & kNodeLive) ? kMetaLive : 0u);
      meta[off + base + (y - lo)] = e;
    }
    base += hi - lo;
    plo = lo;
  }
  if (lane == 0) ch.first[kChainLevels] = off;
}
}  // namespace

size_t chain_meta_scan_bytes(uint32_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, static_cast<const uint32_t*>(nullptr),
                                         static_cast<uint32_t*>(nullptr), n + 1);
  return b;
}

hipError_t launch_chain_meta(ChainChunk* chunks, uint32_t n, const uint32_t* node_parent, const uint8_t* node_flags,
                             uint32_t* counts, void* scan_temp, size_t scan_bytes, uint32_t* meta, bool fill,
                             hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint32_t* offs = counts + n + 1;
  if (!fill) {
    hipLaunchKernelGGL(k_chain_meta_count, dim3((n + kBlock) / kBlock), dim3(kBlock), 0, s, chunks, n, counts);
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(scan_temp, scan_bytes, counts, offs, n + 1, s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_chain_meta_fill, dim3((static_cast<uint64_t>(n) * 64 + kBlock - 1) / kBlock), dim3(kBlock),
                     0, s, chunks, n, offs, node_parent, node_flags, meta);
  return hipGetLastError();
}

hipError_t launch_chain_ranges(ChainChunk* chunks, uint32_t n, const uint32_t* row_ptr, uint32_t cap,
                               uint32_t* overflow, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_chain_ranges, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chunks, n, row_ptr, cap,
                     overflow);
  return hipGetLastError();
}


hipError_t launch_pull_chain(const PullArgs& a, const ChainChunk* chunks, uint32_t n_chunks, uint32_t round,
                             bool record, bool nt, bool slices, bool inner_nt, uint32_t waves_per_cu,
                             hipStream_t s) {
  if (n_chunks == 0) return hipSuccess;
  // (every variant has the same static LDS: one pad for all)
  static const size_t pads[17] = {
      0,  lds_cap_pad(k_pull_chain<false, true, false>, 1), lds_cap_pad(k_pull_chain<false, true, false>, 2),
      lds_cap_pad(k_pull_chain<false, true, false>, 3),  lds_cap_pad(k_pull_chain<false, true, false>, 4),
      lds_cap_pad(k_pull_chain<false, true, false>, 5),  lds_cap_pad(k_pull_chain<false, true, false>, 6),
      lds_cap_pad(k_pull_chain<false, true, false>, 7),  lds_cap_pad(k_pull_chain<false, true, false>, 8),
      lds_cap_pad(k_pull_chain<false, true, false>, 9),  lds_cap_pad(k_pull_chain<false, true, false>, 10),
      lds_cap_pad(k_pull_chain<false, true, false>, 11), lds_cap_pad(k_pull_chain<false, true, false>, 12),
      lds_cap_pad(k_pull_chain<false, true, false>, 13), lds_cap_pad(k_pull_chain<false, true, false>, 14),
      lds_cap_pad(k_pull_chain<false, true, false>, 15), lds_cap_pad(k_pull_chain<false, true, false>, 16)};
  // 12 per CU: 3 per SIMD through the register allocation (the production
  // variants); other caps through an LDS pad
  const uint32_t simd = waves_per_cu == 12 ? 3u : 0u;
  const size_t pad = simd ? 0 : pads[std::min<uint32_t>(waves_per_cu, 16)];
  const dim3 g(n_chunks), b(64);
#define PSAMD_CHAIN(...) hipLaunchKernelGGL((k_pull_chain<__VA_ARGS__>), g, b, pad, s, a, chunks, n_chunks, round)
  if (slices) {
    if (record)
      PSAMD_CHAIN(true, false, true);
    else if (simd == 3)
      PSAMD_CHAIN(false, true, true, true, 3);
    else
      PSAMD_CHAIN(false, true, true);
  } else if (record) {
    PSAMD_CHAIN(true, false, false);
  } else if (!inner_nt) {  // (A/B: plain stores for level 0 and the inner levels)
    if (nt)
      PSAMD_CHAIN(false, true, false, false);
    else
      PSAMD_CHAIN(false, false, false, false);
  } else if (simd == 3) {
    if (nt)
      PSAMD_CHAIN(false, true, false, true, 3);
    else
      PSAMD_CHAIN(false, false, false, true, 3);
  } else if (nt) {
    PSAMD_CHAIN(false, true, false);
  } else {
    PSAMD_CHAIN(false, false, false);
  }
#undef PSAMD_CHAIN
  return hipGetLastError();
}

}  // namespace psamd
