// Host merge of the zero-copy exchange (pe_merge.h merge_rank_lists, what the exchange thread runs
// per group) on synthetic windows: G groups x W rank lists of K ascending keys each, scores drawn so
// every rank contributes to the merged top K + 1.  Checks every merged list against a sort of the
// union, then times the merge per group and per window.
//   g++ -O3 -std=c++17 -march=x86-64-v3 -I../training-operator_amd/csrc bench_merge.cc -o bench_merge
//   ./bench_merge [W ...]       (default 2 4 8 16)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "pe_merge.h"

int main(int argc, char** argv) {
  const int G = 112, K = 256, reps = argc > 1 && std::atoi(argv[1]) < 0 ? -std::atoi(argv[1]) : 200;
  std::vector<int> worlds;
  for (int i = 1; i < argc; ++i)
    if (std::atoi(argv[i]) > 0) worlds.push_back(std::atoi(argv[i]));
  if (worlds.empty()) worlds = {2, 4, 8, 16};
  std::mt19937_64 rng(42);
  int bad = 0;
  for (int W : worlds) {
    // lists[w][r]: K keys ascending, node ids of rank r's contiguous shard (1M nodes / W)
    std::vector<std::vector<uint64_t>> lists((size_t)G * W);
    std::vector<uint64_t> limits((size_t)G * W);
    const uint64_t shard = (1u << 20) / W;
    for (int g = 0; g < G; ++g)
      for (int r = 0; r < W; ++r) {
        auto& l = lists[(size_t)g * W + r];
        std::vector<uint64_t> ks;
        for (int i = 0; i < K + 1; ++i) {
          const uint64_t score = (1000000 + (rng() % 5000000)) ;
          ks.push_back(score << 24 | (r * shard + rng() % shard));
        }
        std::sort(ks.begin(), ks.end());
        ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
        limits[(size_t)g * W + r] = ks[K];
        l.assign(ks.begin(), ks.begin() + K);
      }
    std::vector<uint64_t> dst((size_t)K + 16);
    // correctness: full lists, then (pass 1) short lists of random lengths and random limits
    for (int pass = 0; pass < 2; ++pass)
    for (int g = 0; g < G; ++g) {
      const uint64_t* lp[pe::MERGE_MAX_WORLD];
      int ns[pe::MERGE_MAX_WORLD];
      uint64_t L = ~0ull;
      std::vector<uint64_t> all;
      for (int r = 0; r < W; ++r) {
        lp[r] = lists[(size_t)g * W + r].data();
        ns[r] = pass == 0 ? K : (int)(rng() % (K + 1));
        L = std::min<uint64_t>(L, pass == 0 || ns[r] == K ? limits[(size_t)g * W + r] : (rng() % 4 ? ~0ull : lp[r][rng() % K]));
      }
      for (int r = 0; r < W; ++r)
        for (int i = 0; i < ns[r]; ++i)
          if (lp[r][i] < L) all.push_back(lp[r][i]);
      std::sort(all.begin(), all.end());
      uint64_t lim;
      const int m = pe::merge_rank_lists(lp, ns, W, L, K, dst.data(), &lim);
      const int want = std::min((int)all.size(), K);
      if (m != want || !std::equal(dst.begin(), dst.begin() + m, all.begin()) ||
          lim != ((int)all.size() > K ? all[K] : L))
        ++bad;
    }
    // timing: every group of the window, reps windows
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t sink = 0;
    for (int rep = 0; rep < reps; ++rep)
      for (int g = 0; g < G; ++g) {
        const uint64_t* lp[pe::MERGE_MAX_WORLD];
        int ns[pe::MERGE_MAX_WORLD];
        uint64_t L = ~0ull;
        for (int r = 0; r < W; ++r) {
          lp[r] = lists[(size_t)g * W + r].data();
          ns[r] = K;
          L = std::min(L, limits[(size_t)g * W + r]);
        }
        uint64_t lim;
        sink += (uint64_t)pe::merge_rank_lists(lp, ns, W, L, K, dst.data(), &lim) + lim;
      }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::printf("W %2d  merge %.3f us/group  %.1f us/window (%d groups, K %d)%s\n", W, us / reps / G, us / reps, G, K,
                sink == 42 ? " " : "");
  }
  std::printf("%s: %d wrong merged lists\n", bad ? "FAIL" : "ok", bad);
  return bad ? 1 : 0;
}
