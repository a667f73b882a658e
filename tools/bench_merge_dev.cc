// The device shard merge of the copying exchange (RCCL all-gather, then pe::launch_merge_shards /
// launch_merge_ranked over the gathered window) in isolation on one GPU -- the rank merge both with
// system-scope loads (as the host exchange's pinned lists are read) and with plain loads (as the
// all-gather's device buffer is read).  G groups x W rank lists of K ascending keys each, laid out as the all-gather leaves them (rank r's window blob at r * G * gb).
// Checks every merged list against a sort of the union, then times one launch per window with HIP
// events (the kernel alone: nothing else on the GPU, unlike the 8-contexts-on-one-card study).
//   hipcc -O3 -std=c++17 -I../training-operator_amd/csrc bench_merge_dev.cc -L.. -lplacement -o bench_merge_dev
//   ./bench_merge_dev [W ...]     (default 2 4 8 16)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pe_kernels.h"

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

int main(int argc, char** argv) {
  const int G = 112, K = 256, reps = 200;
  std::vector<int> worlds;
  for (int i = 1; i < argc; ++i) worlds.push_back(std::atoi(argv[i]));
  if (worlds.empty()) worlds = {2, 4, 8, 16};
  const size_t gb = pe::cand_group_bytes(K);
  std::mt19937_64 rng(7);
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad_all = 0;
  for (int W : worlds) {
    // host image of the gathered window, and the expected merged lists
    std::vector<uint8_t> gath((size_t)W * G * gb, 0);
    std::vector<std::vector<uint64_t>> want((size_t)G);
    std::vector<uint64_t> want_lim((size_t)G);
    const uint64_t shard = (1u << 20) / W;
    for (int g = 0; g < G; ++g) {
      std::vector<uint64_t> all;
      uint64_t L = pe::NO_KEY;
      for (int r = 0; r < W; ++r) {
        std::vector<uint64_t> ks;
        const int n = g % 7 == 3 ? (int)(rng() % (K + 1)) : K;   // some short lists (a shard ran out)
        for (int i = 0; i < K + 1; ++i) ks.push_back((1000000 + rng() % 5000000) << 24 | (r * shard + rng() % shard));
        std::sort(ks.begin(), ks.end());
        ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
        const uint64_t lim = n == K ? ks[K] : pe::NO_KEY;
        uint8_t* blob = gath.data() + ((size_t)r * G + g) * gb;
        pe::CandHdr h{n, 0, lim};
        std::memcpy(blob, &h, sizeof h);
        std::memcpy(blob + sizeof h, ks.data(), (size_t)n * 8);
        L = std::min(L, lim);
        all.insert(all.end(), ks.begin(), ks.begin() + n);
      }
      std::sort(all.begin(), all.end());
      std::vector<uint64_t> below;
      for (uint64_t k : all)
        if (k < L) below.push_back(k);
      want[g].assign(below.begin(), below.begin() + std::min<size_t>(below.size(), K));
      want_lim[g] = below.size() > (size_t)K ? below[K] : L;
    }
    uint8_t *dg = nullptr, *dout = nullptr;
    CK(hipMalloc(&dg, gath.size()));
    CK(hipMalloc(&dout, (size_t)G * gb));
    CK(hipMemcpy(dg, gath.data(), gath.size(), hipMemcpyHostToDevice));
    struct Kind {
      const char* name;
      hipError_t (*fn)(hipStream_t, const uint8_t*, int, int, int, uint8_t*, uint32_t, int64_t, const uint64_t*, bool);
      bool sys;
    } kinds[] = {{"merge_shards", &pe::launch_merge_shards, true},
                 {"ranked/sys", &pe::launch_merge_ranked, true},
                 {"ranked/plain", &pe::launch_merge_ranked, false}};
    for (const Kind& kd : kinds) {
      CK(hipMemset(dout, 0xff, (size_t)G * gb));
      const hipError_t le = kd.fn(s, dg, W, G, K, dout, 0, 0, nullptr, kd.sys);
      if (le != hipSuccess) {
        std::printf("W %2d  %-13s not launchable (%s)\n", W, kd.name, hipGetErrorString(le));
        continue;
      }
      CK(hipStreamSynchronize(s));
      std::vector<uint8_t> out((size_t)G * gb);
      CK(hipMemcpy(out.data(), dout, out.size(), hipMemcpyDeviceToHost));
      int bad = 0;
      for (int g = 0; g < G; ++g) {
        pe::CandHdr h;
        std::memcpy(&h, out.data() + (size_t)g * gb, sizeof h);
        const uint64_t* k = reinterpret_cast<const uint64_t*>(out.data() + (size_t)g * gb + sizeof h);
        if (h.n != (int)want[g].size() || h.limit != want_lim[g] || !std::equal(k, k + h.n, want[g].begin())) ++bad;
      }
      for (int i = 0; i < 10; ++i) CK(kd.fn(s, dg, W, G, K, dout, 0, 0, nullptr, kd.sys));
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) CK(kd.fn(s, dg, W, G, K, dout, 0, 0, nullptr, kd.sys));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("W %2d  %-13s %7.1f us/window (%d groups, K %d)  %d wrong\n", W, kd.name, 1000.0 * ms / reps, G, K,
                  bad);
      bad_all += bad;
    }
    CK(hipFree(dg));
    CK(hipFree(dout));
  }
  std::printf("%s: %d wrong merged lists\n", bad_all ? "FAIL" : "ok", bad_all);
  return bad_all ? 1 : 0;
}
