// Host resolver replay: runs pe::Resolver over a window dump recorded on the GPU box
// (PE_DUMP_WINDOWS=<file> python bench.py ...: every resolve call with its groups, candidate blob
// and dirty seeds, sequential or pipelined) and times it on this CPU: the exact host work of the run.
//   g++ -O3 -march=x86-64-v3 -std=c++17 -Itraining-operator_amd/csrc -Iinclude tools/replay_resolver.cc \
//       training-operator_amd/csrc/pe_resolver.cpp -o tools/replay_resolver && tools/replay_resolver dump.bin [reps]
#include <time.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pe_resolver.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s dump.bin [reps]\n", argv[0]);
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  const int warm = std::getenv("REPLAY_WARM") ? std::atoi(std::getenv("REPLAY_WARM")) : 0;
  int64_t hdr[3];
  if (std::fread(hdr, 8, 3, f) != 3) return 2;
  const int64_t J = hdr[0], G = hdr[1];
  const int K = (int)hdr[2];
  std::vector<int32_t> jgo(J + 1), pri(J), cnt(G);
  std::vector<int64_t> req(G * 4);
  std::vector<uint32_t> need(G);
  size_t ok = std::fread(jgo.data(), 4, J + 1, f) + std::fread(pri.data(), 4, J, f) + std::fread(cnt.data(), 4, G, f) +
              std::fread(req.data(), 8, G * 4, f) + std::fread(need.data(), 4, G, f);
  if (ok != (size_t)(J + 1 + J + G + G * 4 + G)) return 2;
  int64_t N = 0;
  if (std::fread(&N, 8, 1, f) != 1) return 2;
  std::vector<pe::NodeState> mirror0(N);
  if (std::fread(mirror0.data(), sizeof(pe::NodeState), N, f) != (size_t)N) return 2;
  struct Win {
    std::vector<int32_t> groups;
    std::vector<uint8_t> blob;
    std::vector<pe::Update> seed;
  };
  std::vector<Win> wins;
  const size_t gb = 16 + (size_t)K * 8;   // key-only lists
  for (;;) {
    int32_t wg;
    if (std::fread(&wg, 4, 1, f) != 1) break;
    Win w;
    w.groups.resize(wg);
    w.blob.resize(wg * gb);
    int32_t ns = 0;
    if (std::fread(w.groups.data(), 4, wg, f) != (size_t)wg || std::fread(w.blob.data(), 1, w.blob.size(), f) != w.blob.size() ||
        std::fread(&ns, 4, 1, f) != 1)
      return 2;
    w.seed.resize(ns);
    if (ns && std::fread(w.seed.data(), sizeof(pe::Update), ns, f) != (size_t)ns) return 2;
    wins.push_back(std::move(w));
  }
  std::fclose(f);
  std::printf("jobs %lld groups %lld K %d windows %zu\n", (long long)J, (long long)G, K, wins.size());
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    pe::Resolver R(J, jgo.data(), pri.data(), cnt.data(), req.data(), need.data());
    std::vector<pe::NodeState, pe::HugeAlloc<pe::NodeState>> mirror(mirror0.begin(), mirror0.end());   // (as the engine's)
    R.set_mirror(pe::Mirror{mirror.data(), N});
    std::vector<pe::GroupCands> cands;
    std::vector<pe::Update> upd;
    double t_resolve = 0, t_cpu = 0;
    auto cpu_ms = [] {   // this thread's CPU time (excludes time the host took the vCPU away, where accounted)
      timespec ts;
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
      return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
    };
    size_t wi = 0;
    for (; wi < wins.size(); ++wi) {       // the resolve calls of the run, in order
      const Win& w = wins[wi];
      pe::parse_window_keys(w.blob.data(), 1, (int)w.groups.size(), K, cands);
      if (warm) {   // REPLAY_WARM=n (experiment): the first n list entries' mirror lines cached before the resolve
        volatile int64_t sink = 0;
        for (const pe::GroupCands& gc : cands)
          for (size_t i = 0; i < std::min<size_t>((size_t)warm, gc.size()); ++i) sink += mirror[gc.key(i) & 0xFFFFFF].res[0];
        for (size_t i = 0; i < w.blob.size(); i += 64) sink += w.blob[i];
      }
      upd.clear();
      const auto a = std::chrono::steady_clock::now();
      const double c0 = cpu_ms();
      R.resolve(w.groups, cands, upd, w.seed.empty() ? nullptr : &w.seed);
      t_cpu += cpu_ms() - c0;
      for (const pe::Update& u : upd)
        for (int d = 0; d < 4; ++d) mirror[u.gid].res[d] = u.res[d];
      t_resolve += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    }
    if (!R.done() && r == 0) std::printf("(partial dump: the batch is not decided after %zu windows)\n", wi);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    best = ms < best ? ms : best;
    uint64_t h = 1469598103934665603ull;   // FNV-1a over the placements and job states (A/B exactness)
    for (int32_t v : R.pod_node()) h = (h ^ (uint32_t)v) * 1099511628211ull;
    for (int32_t v : R.job_status()) h = (h ^ (uint32_t)v) * 1099511628211ull;
    std::printf("rep %d: %.3f ms total, %.3f ms in resolve, %.3f ms cpu, %zu windows, %lld pods placed, %lld rescans, result %016llx\n",
                r, ms, t_resolve, t_cpu, wi, (long long)R.pods_placed(), (long long)R.rescans(), (unsigned long long)h);
  }
  std::printf("best %.3f ms\n", best);
  return 0;
}
