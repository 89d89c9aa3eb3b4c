// tree_bench.cpp -- host cost of cfg5's churn on the subscription tree
// (csrc/tree.cpp) without a GPU: 1M peers, W=2/MaxW=5, 90 % subscribed in
// peer order through the join protocol, then batches of 1 % graceful leaves
// (Part + repair) and 1 % joins, as bench.py's cfg5 step drives them
// (engine-level bookkeeping around the tree -- touched lists, the GPU
// delta upload -- not included).
//   g++ -O2 -std=c++17 -I include -I go-libp2p-pubsub_amd/csrc \
//       tools/probe/tree_bench.cpp go-libp2p-pubsub_amd/csrc/tree.cpp -o /tmp/tree_bench
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <random>
#include <vector>

#include "tree.hpp"

using namespace psamd;
using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? static_cast<uint32_t>(std::atoi(argv[1])) : 1000000u;
  const int batches = argc > 2 ? std::atoi(argv[2]) : 20;
  SubscriptionTree T(n, 0, 2, 5, 12345);
  std::mt19937_64 rng(7);
  std::vector<uint8_t> member(n, 0);
  auto t0 = clk::now();
  for (uint32_t p = 1; p < n; ++p)
    if ((rng() % 10) != 0) {
      if (T.subscribe(p) == 0) member[p] = 1;
    }
  std::vector<uint32_t> touched;
  T.take_touched(touched);
  auto t1 = clk::now();
  std::printf("initial joins: %.1f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
  double tl = 0, tj = 0, tm = 0;
  for (int b = 0; b < batches; ++b) {
    std::vector<uint32_t> ins, outs;
    for (uint32_t p = 1; p < n; ++p) (member[p] ? ins : outs).push_back(p);
    std::shuffle(ins.begin(), ins.end(), rng);
    std::shuffle(outs.begin(), outs.end(), rng);
    const size_t k = n / 100;
    std::vector<uint32_t> leave(ins.begin(), ins.begin() + std::min(k, ins.size()));
    std::vector<uint32_t> join(outs.begin(), outs.begin() + std::min(k, outs.size()));
    std::sort(leave.begin(), leave.end());
    std::sort(join.begin(), join.end());
    auto a = clk::now();
    for (uint32_t p : leave) {
      T.close_client(p);
      member[p] = 0;
    }
    auto bb = clk::now();
    const bool pf = std::getenv("TB_PREFETCH") != nullptr;
    for (size_t i = 0; i < join.size(); ++i) {
      if (pf && i + 8 < join.size()) T.prefetch_join(join[i + 8]);
      if (T.subscribe(join[i]) == 0) member[join[i]] = 1;
    }
    auto c = clk::now();
    T.after_message(nullptr);
    T.take_touched(touched);
    auto d = clk::now();
    tl += std::chrono::duration<double, std::milli>(bb - a).count();
    tj += std::chrono::duration<double, std::milli>(c - bb).count();
    tm += std::chrono::duration<double, std::milli>(d - c).count();
  }
  std::printf("per batch: leaves %.3f ms, joins %.3f ms, after_message (host reach walk) %.3f ms\n", tl / batches,
              tj / batches, tm / batches);
  return 0;
}
