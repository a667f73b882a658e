// CPU tests of pe::WindowFeed (pe_resolver.h): the per-group hand-over of a signalled walk window.
// Built and run by tests/test_feed_cpu.py (g++ against training-operator_amd/csrc/pe_resolver.cpp).
//   1. parsing follows the signals in group order (a later group signalled first waits);
//   2. wait() returns once another thread signals the group, and throws when idle() reports that
//      the producer is done without having signalled it;
//   3. a resolve fed group by group by a producer thread (random delays) places every pod exactly
//      as the same resolve over the fully parsed blob, with and without pipelined seeds.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>

#include "pe_resolver.h"

static int failed = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      ++failed;                                                    \
    }                                                              \
  } while (0)

static constexpr uint64_t kNoKey = ~0ull;

struct Blob {
  int K;
  std::vector<uint8_t> b;
  size_t gb() const { return 16 + (size_t)K * 8; }
  Blob(int groups, int k) : K(k), b((size_t)groups * (16 + (size_t)k * 8), 0) {}
  void set_group(int w, const std::vector<uint64_t>& keys, uint64_t limit) {
    uint8_t* g = b.data() + (size_t)w * gb();
    const int32_t n = (int32_t)keys.size();
    std::memcpy(g, &n, 4);
    std::memcpy(g + 8, &limit, 8);
    std::memcpy(g + 16, keys.data(), keys.size() * 8);
  }
  void signal(int w, uint32_t gen) {
    __atomic_store_n(reinterpret_cast<int32_t*>(b.data() + (size_t)w * gb() + 4), (int32_t)gen, __ATOMIC_RELEASE);
  }
};

static void test_order_and_wait() {
  Blob bl(5, 4);
  for (int w = 0; w < 5; ++w) bl.set_group(w, {(uint64_t)(10 + w), (uint64_t)(20 + w)}, 100 + w);
  std::vector<pe::GroupCands> cands;
  pe::WindowFeed f;
  f.reset(bl.b.data(), 5, 4, 7, &cands);
  f.advance();
  CHECK(f.parsed() == 0);
  bl.signal(0, 7);
  bl.signal(2, 7);
  f.advance();
  CHECK(f.parsed() == 1);                       // group 1 not there: group 2 waits
  CHECK(cands[0].n == 2 && cands[0].key(1) == 20 && cands[0].limit == 100);
  bl.signal(1, 6);                              // a stale generation is not a signal
  f.advance();
  CHECK(f.parsed() == 1);
  bl.signal(1, 7);
  f.advance();
  CHECK(f.parsed() == 3);
  CHECK(cands[2].key(0) == 12 && cands[2].limit == 102);
  std::thread prod([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    bl.signal(3, 7);
    bl.signal(4, 7);
  });
  f.wait(4);
  prod.join();
  CHECK(f.parsed() == 5);
  CHECK(cands[4].key(1) == 24 && cands[4].limit == 104);
  CHECK(f.spin_ms() > 1.0);
  // a group the producer never signals: wait() gives up when idle() says the producer is done
  Blob b2(2, 4);
  b2.set_group(0, {1}, kNoKey);
  b2.set_group(1, {2}, kNoKey);
  b2.signal(0, 9);
  pe::WindowFeed g;
  int calls = 0;
  g.idle = [](void* u) { return ++*static_cast<int*>(u) < 3; };
  g.idle_user = &calls;
  g.reset(b2.b.data(), 2, 4, 9, &cands);
  bool threw = false;
  try {
    g.wait(1);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw && calls == 3 && g.parsed() == 1);
  // a producer that stays busy and never signals (a stuck collective): with a deadline set, wait()
  // throws CollectiveTimeout once it has passed, and not before
  pe::WindowFeed h;
  h.idle = [](void*) { return true; };
  h.timeout_s = 0.05;
  h.reset(b2.b.data(), 2, 4, 9, &cands);
  const auto t0 = std::chrono::steady_clock::now();
  bool timed_out = false;
  try {
    h.wait(1);
  } catch (const pe::CollectiveTimeout&) {
    timed_out = true;
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  CHECK(timed_out && dt >= 0.05 && dt < 5.0 && h.parsed() == 1);
  std::printf("ok   order/wait/idle/deadline\n");
}

// exact candidate lists of a window: per group every fitting node's key, ascending, cut at K
static void build_lists(Blob& bl, const std::vector<int32_t>& groups, const std::vector<pe::NodeState>& st,
                        const std::vector<int64_t>& qeff, const std::vector<uint32_t>& need) {
  for (size_t w = 0; w < groups.size(); ++w) {
    const int32_t g = groups[w];
    std::vector<uint64_t> keys;
    for (size_t n = 0; n < st.size(); ++n) {
      const uint64_t k = pe::key_of(st[n].res, st[n].labels, &qeff[(size_t)g * 4], need[g], n);
      if (k != kNoKey) keys.push_back(k);
    }
    std::sort(keys.begin(), keys.end());
    uint64_t limit = kNoKey;
    if ((int)keys.size() > bl.K) {
      limit = keys[(size_t)bl.K];
      keys.resize((size_t)bl.K);
    }
    bl.set_group((int)w, keys, limit);
  }
}

static void test_fed_resolve(unsigned seed_base) {
  std::mt19937_64 rng(seed_base);
  const int N = 400, J = 150, K = 16;
  std::vector<pe::NodeState> st0((size_t)N);
  for (auto& s : st0) {
    s.res[0] = 2000 + (int64_t)(rng() % 30) * 1000;
    s.res[1] = (int64_t)(4 + rng() % 60) << 30;
    s.res[2] = (int64_t)(rng() % 3 == 0 ? 8 : 0);
    s.res[3] = (int64_t)(100 + rng() % 400) << 30;
    s.labels = (uint32_t)(rng() & 3) | (s.res[2] ? 1u : 0u);
  }
  std::vector<int32_t> jgo(J + 1), pri(J), cnt;
  std::vector<int64_t> req;
  std::vector<uint32_t> need;
  for (int j = 0; j < J; ++j) {
    jgo[j] = (int32_t)cnt.size();
    pri[j] = (int32_t)(rng() % 5);
    const int ng = 1 + (int)(rng() % 2);
    for (int g = 0; g < ng; ++g) {
      cnt.push_back(1 + (int32_t)(rng() % 6));
      req.push_back(500 * (int64_t)(1 + rng() % 8));
      req.push_back((int64_t)(1 + rng() % 16) << 30);
      req.push_back(rng() % 4 == 0 ? 2 : 0);
      req.push_back((int64_t)(rng() % 50) << 30);
      need.push_back(rng() % 3 == 0 ? 1u : 0u);
    }
  }
  jgo[J] = (int32_t)cnt.size();
  // two runs over the same window sequence (window = 12 groups, exact lists from the current
  // state): A parses each blob whole, B is fed group by group by a producer thread.  "pipelined":
  // every window also gets the previous window's updates as seeds (their states are current, so
  // the lists stay exact; this drives the seed scorer and the seed-set takeover)
  std::vector<int32_t> first_nodes;
  for (const bool pipelined : {false, true}) {
    std::vector<int32_t> res_nodes[2], res_status[2];
    for (int run = 0; run < 2; ++run) {
      pe::Resolver R(J, jgo.data(), pri.data(), cnt.data(), req.data(), need.data());
      std::vector<pe::NodeState> mirror = st0;
      R.set_mirror(pe::Mirror{mirror.data(), N});
      std::vector<int64_t> qeff((size_t)jgo[J] * 4);
      for (int32_t g = 0; g < jgo[J]; ++g)
        for (int d = 0; d < 4; ++d) qeff[(size_t)g * 4 + d] = R.scan_req(g)[d];
      std::vector<pe::Update> seed, upd;
      std::vector<pe::GroupCands> cands;
      uint32_t gen = 0;
      while (!R.done()) {
        std::vector<int32_t> groups;
        R.next_window(12, 1 << 20, groups);
        Blob bl((int)groups.size(), K);
        build_lists(bl, groups, mirror, qeff, need);
        upd.clear();
        ++gen;
        const std::vector<pe::Update>* sd = pipelined && !seed.empty() ? &seed : nullptr;
        if (run == 0) {
          for (int w = 0; w < (int)groups.size(); ++w) bl.signal(w, gen);
          pe::parse_window_keys(bl.b.data(), 1, (int)groups.size(), K, cands);
          R.resolve(groups, cands, upd, sd);
        } else {
          pe::WindowFeed f;
          std::atomic<bool> done{false};
          f.reset(bl.b.data(), (int)groups.size(), K, gen, &cands);
          std::thread prod([&] {
            std::mt19937 r2(gen * 7919u + seed_base);
            for (int w = 0; w < (int)groups.size(); ++w) {
              if (r2() % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(r2() % 200));
              bl.signal(w, gen);
            }
            done.store(true);
          });
          f.idle = [](void* u) { return !static_cast<std::atomic<bool>*>(u)->load(); };
          f.idle_user = &done;
          f.wait(0);
          R.resolve(groups, cands, upd, sd, &f);
          prod.join();
        }
        for (const pe::Update& u : upd)
          for (int d = 0; d < 4; ++d) mirror[u.gid].res[d] = u.res[d];
        seed = upd;
      }
      res_nodes[run] = R.pod_node();
      res_status[run] = R.job_status();
    }
    CHECK(res_nodes[0] == res_nodes[1]);
    CHECK(res_status[0] == res_status[1]);
    int placed = 0;
    for (int32_t s : res_status[0]) placed += s == 0;
    CHECK(placed > 0);
    if (!pipelined) first_nodes = res_nodes[0];
    else CHECK(first_nodes == res_nodes[0]);   // seeds never change a placement
  }
  std::printf("ok   fed resolve == parsed resolve (seed %u)\n", seed_base);
}

// SeedScorer start()/stop() back to back (advisor r2: a stale cancel read by the helper must not
// acknowledge the next window).  After stop() returns, the window's inputs are rewritten at once:
// a helper still inside the window would race with it (ThreadSanitizer) or see torn inputs.  The
// -DPE_SEED_TEST_YIELD build yields between the helper's state read and its action.
static void test_scorer_handshake() {
  std::mt19937 rng(7);
  pe::DirtySet seeds;
  for (int i = 0; i < 64; ++i) {
    pe::NodeState st{};
    for (int d = 0; d < pe::RD; ++d) st.res[d] = 1000 + (int64_t)(rng() % 1000);
    seeds.upsert(i * 3, st);
  }
  std::vector<int64_t> req(4 * 8, 1);
  std::vector<uint32_t> need(8, 0);
  // one CPU for this thread and the helper (it inherits the mask): every yield is a real switch
  cpu_set_t old_set, one;
  (void)pthread_getaffinity_np(pthread_self(), sizeof(old_set), &old_set);
  CPU_ZERO(&one);
  CPU_SET(sched_getcpu(), &one);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
  int cycles = 0;
  {
  pe::SeedScorer sc;
  for (int it = 0; it < 20000; ++it) {
    std::vector<int32_t> groups((size_t)(1 + rng() % 8));
    for (size_t i = 0; i < groups.size(); ++i) groups[i] = (int32_t)i;
    std::vector<pe::GroupCands> cands(groups.size());
    std::vector<uint64_t> keys(16);
    for (size_t i = 0; i < keys.size(); ++i) keys[i] = ((uint64_t)(i + 1) << 24) | (uint64_t)(1000 + i);
    for (auto& gc : cands) {
      gc.keys = keys.data();
      gc.keyed = true;
      gc.n = keys.size();
      gc.limit = kNoKey;
    }
    sc.start(&seeds, &groups, &cands, req.data(), need.data());
    if (rng() % 3 == 0) std::this_thread::yield();
    sc.stop();
    // the helper is idle now: clobber what it read
    for (auto& gc : cands) gc.keys = nullptr, gc.n = 0;
    std::fill(keys.begin(), keys.end(), 0);
    groups.assign(groups.size(), -1);
    ++cycles;
  }
  }
  (void)pthread_setaffinity_np(pthread_self(), sizeof(old_set), &old_set);
  CHECK(cycles == 20000);
  std::printf("ok   seed scorer start/stop handshake (%d cycles)\n", cycles);
}

int main() {
  test_scorer_handshake();
  test_order_and_wait();
  for (unsigned s = 1; s <= 6; ++s) test_fed_resolve(s);
  std::printf("%d failed checks\n", failed);
  return failed ? 1 : 0;
}
