// CPU emulation of the engine's pipelined greedy (depth 1) that writes the same window dump as
// PE_DUMP_WINDOWS (tools/replay_resolver.cc reads it): host resolver work can then be replayed and
// A/B'd without a GPU.  The "device" here is a residual array updated like the apply kernel, and a
// window scan is the exact per-group top-(K+1) over all nodes (pe::key_of, OpenMP over groups):
// the same lists the walk kernel writes (n = min(K, fits), limit = the (K+1)-th key or none).
//   inputs from tools/emulate_dump.py;  g++ -O3 -march=native -fopenmp -std=c++17
//   -Itraining-operator_amd/csrc tools/emulate_dump.cc training-operator_amd/csrc/pe_resolver.cpp
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>

#include "pe_resolver.h"

static constexpr uint64_t kNoKey = ~0ull;

template <class T>
static bool rd(FILE* f, std::vector<T>& v, size_t n) {
  v.resize(n);
  return std::fread(v.data(), sizeof(T), n, f) == n;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s inputs.bin dump.bin [K] [window_groups] [window_pods]\n", argv[0]);
    return 2;
  }
  const int K = argc > 3 ? std::atoi(argv[3]) : 256;
  const int Wmax = argc > 4 ? std::atoi(argv[4]) : 128;
  const int64_t Pmax = argc > 5 ? std::atoll(argv[5]) : 1024;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int64_t hdr[2];
  if (std::fread(hdr, 8, 2, f) != 2) return 2;
  const int64_t N = hdr[0], J = hdr[1];
  std::vector<int64_t> res;   // [4][N]
  std::vector<uint32_t> lab;
  std::vector<int32_t> jgo, pri, cnt;
  if (!rd(f, res, 4 * N) || !rd(f, lab, N) || !rd(f, jgo, J + 1) || !rd(f, pri, J)) return 2;
  const int64_t G = jgo[J];
  std::vector<int64_t> req;
  std::vector<uint32_t> need;
  if (!rd(f, cnt, G) || !rd(f, req, 4 * G) || !rd(f, need, G)) return 2;
  std::fclose(f);

  std::vector<pe::NodeState> mirror(N);
  for (int64_t n = 0; n < N; ++n) {
    for (int d = 0; d < 4; ++d) mirror[n].res[d] = res[d * N + n];
    mirror[n].labels = lab[n];
  }
  std::vector<pe::NodeState> dev = mirror;   // the "device" residuals (updates applied like apply_kernel)
  FILE* out = std::fopen(argv[2], "wb");
  if (!out) return 2;
  const int64_t h3[3] = {J, G, (int64_t)K};
  std::fwrite(h3, 8, 3, out);
  std::fwrite(jgo.data(), 4, J + 1, out);
  std::fwrite(pri.data(), 4, J, out);
  std::fwrite(cnt.data(), 4, G, out);
  std::fwrite(req.data(), 8, 4 * G, out);
  std::fwrite(need.data(), 4, G, out);
  std::fwrite(&N, 8, 1, out);
  std::fwrite(mirror.data(), sizeof(pe::NodeState), N, out);

  pe::Resolver R(J, jgo.data(), pri.data(), cnt.data(), req.data(), need.data());
  R.set_mirror(pe::Mirror{mirror.data(), N});
  const size_t gb = 16 + (size_t)K * 8;
  auto scan = [&](const std::vector<int32_t>& groups, std::vector<uint8_t>& blob) {
    blob.assign(groups.size() * gb, 0);
#pragma omp parallel
    {
      std::vector<uint64_t> keys;
#pragma omp for schedule(dynamic, 1)
      for (size_t w = 0; w < groups.size(); ++w) {
        const int64_t* q = R.scan_req(groups[w]);
        const uint32_t nd = need[groups[w]];
        keys.clear();
        for (int64_t n = 0; n < N; ++n) {
          const uint64_t k = pe::key_of(dev[n].res, dev[n].labels, q, nd, (uint64_t)n);
          if (k != kNoKey) keys.push_back(k);
        }
        const size_t take = std::min(keys.size(), (size_t)K + 1);
        std::partial_sort(keys.begin(), keys.begin() + take, keys.end());
        const int32_t n = (int32_t)std::min(keys.size(), (size_t)K);
        const uint64_t limit = keys.size() > (size_t)K ? keys[K] : kNoKey;
        uint8_t* b = blob.data() + w * gb;
        std::memcpy(b, &n, 4);
        std::memcpy(b + 8, &limit, 8);
        std::memcpy(b + 16, keys.data(), (size_t)n * 8);
      }
    }
  };
  auto apply = [&](const std::vector<pe::Update>& u) {
    for (const pe::Update& x : u)
      for (int d = 0; d < 4; ++d) dev[x.gid].res[d] = x.res[d];
  };
  struct Flight {
    std::vector<int32_t> groups;
    pe::Cursor end;
    std::vector<uint8_t> blob;
    size_t ver = 0;
  };
  std::deque<Flight> fl;
  std::vector<std::vector<pe::Update>> hist;
  size_t n_app = 0;
  auto add_flight = [&](const pe::Cursor& from) -> Flight* {
    Flight fx;
    R.next_window_from(from, Wmax, Pmax, fx.groups, &fx.end);
    if (fx.groups.empty()) return nullptr;
    fx.ver = hist.size();
    fl.push_back(std::move(fx));
    return &fl.back();
  };
  auto restart = [&] {
    fl.clear();
    hist.clear();
    n_app = 0;
    if (Flight* fx = add_flight(R.cursor())) scan(fx->groups, fx->blob);
  };
  restart();
  std::vector<pe::GroupCands> cands;
  std::vector<pe::Update> seed, upd;
  int64_t windows = 0;
  while (!fl.empty()) {
    // the launch helper's part: apply the resolved windows' updates, scan the next window
    for (; n_app < hist.size(); ++n_app) apply(hist[n_app]);
    if (fl.size() < 2)
      if (Flight* fx = add_flight(fl.back().end)) scan(fx->groups, fx->blob);
    Flight& cur = fl.front();
    seed.clear();
    for (size_t k = cur.ver; k < hist.size(); ++k) seed.insert(seed.end(), hist[k].begin(), hist[k].end());
    // the dump record of this resolve call (PE_DUMP_WINDOWS layout)
    const int32_t wg = (int32_t)cur.groups.size(), ns = (int32_t)seed.size();
    std::fwrite(&wg, 4, 1, out);
    std::fwrite(cur.groups.data(), 4, (size_t)wg, out);
    std::fwrite(cur.blob.data(), 1, cur.blob.size(), out);
    std::fwrite(&ns, 4, 1, out);
    if (ns) std::fwrite(seed.data(), sizeof(pe::Update), (size_t)ns, out);
    pe::parse_window_keys(cur.blob.data(), 1, wg, K, cands);
    upd.clear();
    const bool consumed = R.resolve(cur.groups, cands, upd, seed.empty() ? nullptr : &seed);
    for (const pe::Update& u : upd)
      for (int d = 0; d < 4; ++d) mirror[u.gid].res[d] = u.res[d];
    ++windows;
    const bool landed = consumed && R.cursor() == cur.end && fl.size() > 1;
    if (landed && !R.done()) {
      hist.push_back(upd);
      fl.pop_front();
      continue;
    }
    for (; n_app < hist.size(); ++n_app) apply(hist[n_app]);
    apply(upd);
    if (R.done()) break;
    restart();
  }
  std::fclose(out);
  uint64_t h = 1469598103934665603ull;
  for (int32_t v : R.pod_node()) h = (h ^ (uint32_t)v) * 1099511628211ull;
  for (int32_t v : R.job_status()) h = (h ^ (uint32_t)v) * 1099511628211ull;
  std::printf("windows %lld pods placed %lld jobs placed %lld rescans %lld result %016llx\n", (long long)windows,
              (long long)R.pods_placed(), (long long)R.jobs_placed(), (long long)R.rescans(), (unsigned long long)h);
  return 0;
}
