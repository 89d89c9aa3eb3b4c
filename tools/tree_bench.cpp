// tree_bench.cpp -- host-only timing of the restated tree maintenance
// (tree.cpp) on a churn plan dumped by tools/tree_bench.py: the cfg5 join /
// leave cost without a GPU.
//   g++ -O3 -std=c++17 -Iinclude -Igo-libp2p-pubsub_amd/csrc tools/tree_bench.cpp
//       go-libp2p-pubsub_amd/csrc/tree.cpp -o /tmp/tree_bench && /tmp/tree_bench plan.bin
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "tree.hpp"

using namespace psamd;

static std::vector<uint32_t> read_vec(FILE* f) {
  uint32_t n = 0;
  if (fread(&n, 4, 1, f) != 1) return {};
  std::vector<uint32_t> v(n);
  if (n && fread(v.data(), 4, n, f) != n) return {};
  return v;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint32_t hdr[5];
  if (fread(hdr, 4, 5, f) != 5) return 2;
  const uint32_t n = hdr[0], root = hdr[1], w = hdr[2], mw = hdr[3], batches = hdr[4];
  std::vector<uint32_t> order = read_vec(f);
  std::vector<std::vector<uint32_t>> leave(batches), join(batches);
  for (uint32_t b = 0; b < batches; ++b) {
    leave[b] = read_vec(f);
    join[b] = read_vec(f);
  }
  fclose(f);
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  SubscriptionTree T(n, root, w, mw, 12345);
  auto t0 = clk::now();
  for (uint32_t p : order) T.subscribe(p);
  std::vector<uint32_t> touched;
  T.take_touched(touched);
  std::printf("initial %zu joins %.1f ms\n", order.size(), ms(t0, clk::now()));
  double tl = 0, tj = 0, tp = 0;
  for (uint32_t b = 0; b < batches; ++b) {
    auto a = clk::now();
    constexpr size_t kAhead0 = 16, kAhead1 = 8;
    const auto& L = leave[b];
    for (size_t i = 0; i < std::min(L.size(), kAhead0); ++i) T.prefetch_leave(L[i], 0);
    for (size_t i = 0; i < std::min(L.size(), kAhead1); ++i) T.prefetch_leave(L[i], 1);
    for (size_t i = 0; i < L.size(); ++i) {
      if (i + kAhead0 < L.size()) T.prefetch_leave(L[i + kAhead0], 0);
      if (i + kAhead1 < L.size()) T.prefetch_leave(L[i + kAhead1], 1);
      T.close_client(L[i]);
    }
    auto c = clk::now();
    // (as ps_topic_join: each joiner's own line fetched a few joins ahead)
    const auto& J = join[b];
    for (size_t i = 0; i < std::min(J.size(), size_t(8)); ++i) T.prefetch_join(J[i]);
    for (size_t i = 0; i < J.size(); ++i) {
      if (i + 8 < J.size()) T.prefetch_join(J[i + 8]);
      T.subscribe(J[i]);
    }
    const auto d0 = clk::now();
    const size_t pend = T.parted_parents();
    // the engine answers reach (and cut-for-good) from the GPU node space;
    // here from a BFS and upward walks, outside the timed part
    std::vector<uint32_t> par;
    T.attached_parents(par);
    double tq = 0;
    SubscriptionTree::ReachQuery q = [&](const std::vector<uint32_t>& peers, std::vector<uint8_t>& out) {
      const auto q0 = clk::now();
      for (size_t i = 0; i < peers.size(); ++i) {
        const uint32_t p = peers[i];
        out[i] = p == root || par[p] != kNone;
        for (uint32_t x = p; !out[i] && x != root;) {
          const uint32_t up = T.upstream_code(x);
          if (up >= n) {
            out[i] = up == SubscriptionTree::kOrphanUp ? 2 : 0;
            break;
          }
          x = up;
        }
      }
      tq += ms(q0, clk::now());
      return 0;
    };
    const auto d = clk::now();
    T.after_message(&q);
    if (b == 0 || b + 1 == batches) std::printf("batch %u: %zu parted parents before the pass, %zu after\n", b, pend, T.parted_parents());
    T.take_touched(touched);
    auto e = clk::now();
    tl += ms(a, c);
    tj += ms(c, d0);
    tp += ms(d, e) - tq;
  }
  std::printf("per batch: leave %.3f ms  join %.3f ms  prune (reach given) %.3f ms  (%u batches, %zu/%zu ops)\n",
              tl / batches, tj / batches, tp / batches, batches, leave[0].size(), join[0].size());
  std::vector<uint32_t> par;
  T.attached_parents(par);
  uint64_t h = 1469598103934665603ull, att = 0;
  for (uint32_t p = 0; p < n; ++p) {
    h = (h ^ par[p]) * 1099511628211ull;
    h = (h ^ static_cast<uint32_t>(T.state(p))) * 1099511628211ull;
    att += par[p] != kNone;
  }
  std::printf("attached %llu  digest %016llx\n", static_cast<unsigned long long>(att), static_cast<unsigned long long>(h));
  return 0;
}
