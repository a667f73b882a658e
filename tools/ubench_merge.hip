// Merge-kernel microbenchmark: 64 groups x 977 wave lists (the 1M-node window), synthetic lists
// with a controlled number T of candidates below the min bound G.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Itraining-operator_amd/csrc tools/ubench_merge.hip -o tools/ubench_merge
#include "pe_kernels.hip"
#include <stdio.h>
#include <vector>
#include <random>
#include <algorithm>

int main() {
  const int G = 64, nw = 977, K = 64;
  const int64_t Ns = 1000000, stride = 1000192;
  std::vector<int64_t> res((size_t)4 * stride, 1000);
  std::vector<uint32_t> lab(stride, 0);
  int64_t* d_res; uint32_t* d_lab; uint64_t *d_cand, *d_bound; int32_t* d_cnt; uint8_t* d_out;
  hipMalloc(&d_res, res.size() * 8); hipMalloc(&d_lab, lab.size() * 4);
  hipMemcpy(d_res, res.data(), res.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(d_lab, lab.data(), lab.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&d_cand, (size_t)G * nw * 64 * 8); hipMalloc(&d_bound, (size_t)G * nw * 8); hipMalloc(&d_cnt, (size_t)G * nw * 4);
  hipMalloc(&d_out, (size_t)G * pe::cand_group_bytes(K));
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  std::mt19937_64 rng(7);
  for (int per : {0, 1, 4, 16}) {        // lane minima below G per wave list (T = per * 977)
    for (int cnt_each : {8, 24}) {
      std::vector<uint64_t> cand((size_t)G * nw * 64), bound((size_t)G * nw);
      std::vector<int32_t> cnt((size_t)G * nw);
      for (int g = 0; g < G; ++g)
        for (int w = 0; w < nw; ++w) {
          const size_t slot = (size_t)g * nw + w;
          const uint64_t Gk = 1ull << 40;
          cnt[slot] = cnt_each;
          for (int i = 0; i < cnt_each; ++i) {
            const uint64_t score = i < per ? (rng() % (1ull << 15)) : (1ull << 16) + (rng() % (1ull << 15));
            cand[slot * 64 + i] = (score << 24) | (uint64_t)((w * 1024 + i) % Ns);
          }
          bound[slot] = ((w == 0 ? (1ull << 16) : (1ull << 17)) << 24);
          (void)Gk;
        }
      hipMemcpy(d_cand, cand.data(), cand.size() * 8, hipMemcpyHostToDevice);
      hipMemcpy(d_bound, bound.data(), bound.size() * 8, hipMemcpyHostToDevice);
      hipMemcpy(d_cnt, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice);
      float best = 1e9f;
      for (int r = 0; r < 10; ++r) {
        hipEventRecord(a, 0);
        pe::launch_merge(0, d_cand, d_cnt, d_bound, nw, K, d_out, G);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms);
      }
      printf("T/list=%2d cnt=%2d  T=%6d  merge %.1f us\n", per, cnt_each, per * nw, best * 1e3);
    }
  }
  return 0;
}
