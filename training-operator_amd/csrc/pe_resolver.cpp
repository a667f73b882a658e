// Host resolver of the windowed greedy placement (see pe_resolver.h for the exactness argument).
#include "pe_resolver.h"

#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <string>
#include <cstring>
#include <numeric>
#include <utility>
#include <cstdio>
#include <cstdlib>

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#ifdef PE_RES_PROF
#include <x86intrin.h>
#endif

namespace pe {
#ifdef PE_RES_PROF   // section cycle counts for tools/replay_resolver (-DPE_RES_PROF)
struct ResProf { long cgroups = 0, cskip = 0, cdirty = 0; unsigned long long p1 = 0, p2 = 0, p3 = 0, la = 0, ka = 0, st = 0, seed = 0, keys = 0, skip = 0, place = 0, fin = 0, other = 0; long skips = 0, pods = 0, groups = 0, dirty = 0, scored = 0, sready = 0, slocal = 0, sfull = 0;
  ~ResProf() { std::fprintf(stderr, "keys split: lookahead %.1fM keys_all %.1fM seed top %.1fM | place split: choose+fetch %.1fM m %.1fM upsert..key %.1fM\n", la / 1e6, ka / 1e6, st / 1e6, p1 / 1e6, p2 / 1e6, p3 / 1e6); std::fprintf(stderr, "cycles seed %.1fM keys %.1fM skip %.1fM place %.1fM fin %.1fM | skips %ld pods %ld | per group: dirty %.0f scored %.1f\n", seed / 1e6, keys / 1e6, skip / 1e6, place / 1e6, fin / 1e6, skips, pods, (double)dirty / groups, (double)scored / groups); std::fprintf(stderr, "seed tops: helper %ld local %ld full %ld\n", sready, slocal, sfull); std::fprintf(stderr, "window conflicts: %ld of %ld groups depend on an earlier group of their window (%ld via a skipped list entry, %ld via a chosen changed node)\n", cgroups, groups, cskip, cdirty); } };
static ResProf rp;
#define RP_T() __rdtsc()
#define RP_ADD(f, t) (rp.f += __rdtsc() - (t))
#else
#define RP_T() 0ull
#define RP_ADD(f, t) (void)(t)
#endif

static constexpr uint64_t kNoKey = ~0ull;
static constexpr uint32_t kNeedIsland = 0x80000000u;   // placement.h PE_NEED_ISLAND
#ifndef PE_LOOK_STATES
#define PE_LOOK_STATES 2
#endif
static constexpr size_t kLookStates = PE_LOOK_STATES, kLookLines = PE_LOOK_STATES + 2;   // groups ahead
static constexpr uint64_t kScoreMax = (1ull << 40) - 1;

uint64_t score_of(const int64_t left[RD]) {
  uint64_t a = (uint64_t)left[0];
  uint64_t b = (uint64_t)left[1] >> 20;
  uint64_t c = (uint64_t)left[2] >= (1ull << 20) ? kScoreMax : ((uint64_t)left[2] << 20);
  uint64_t d = (uint64_t)left[3] >> 24;
  a = std::min(a, kScoreMax);
  b = std::min(b, kScoreMax);
  c = std::min(c, kScoreMax);
  d = std::min(d, kScoreMax);
  return std::min(a + b + c + d, kScoreMax);
}

uint64_t key_of(const int64_t res[RD], uint32_t labels, const int64_t q[RD], uint32_t need, uint64_t gid) {
  if ((labels & need) != need) return kNoKey;
  int64_t left[RD];
  for (int d = 0; d < RD; ++d) {
    if (q[d] > res[d]) return kNoKey;
    left[d] = res[d] - q[d];
  }
  return (score_of(left) << 24) | gid;
}

// ------------------------------------------------------------------ DirtySet

void DirtySet::swap(DirtySet& o) noexcept {
  std::swap(gid, o.gid);
  std::swap(r0, o.r0);
  std::swap(r1, o.r1);
  std::swap(r2, o.r2);
  std::swap(r3, o.r3);
  std::swap(lab, o.lab);
  std::swap(kn, o.kn);
  std::swap(n_, o.n_);
  std::swap(cap_, o.cap_);
  std::swap(buf_, o.buf_);
  std::swap(slot_, o.slot_);
  std::swap(bits_, o.bits_);
}

void DirtySet::grow() {
  const size_t cap = std::max<size_t>(1024, 2 * cap_);
  // one allocation, 64-B aligned columns: five int64, K(n), labels
  const size_t col = (cap * 8 + 63) / 64 * 64, lcol = (cap * 4 + 63) / 64 * 64;
  uint8_t* b = static_cast<uint8_t*>(::operator new(6 * col + lcol, std::align_val_t(64)));
  int64_t* ng = reinterpret_cast<int64_t*>(b);
  int64_t* n0 = reinterpret_cast<int64_t*>(b + col);
  int64_t* n1 = reinterpret_cast<int64_t*>(b + 2 * col);
  int64_t* n2 = reinterpret_cast<int64_t*>(b + 3 * col);
  int64_t* n3 = reinterpret_cast<int64_t*>(b + 4 * col);
  uint64_t* nk = reinterpret_cast<uint64_t*>(b + 5 * col);
  uint32_t* nl = reinterpret_cast<uint32_t*>(b + 6 * col);
  if (n_) {
    std::memcpy(ng, gid, n_ * 8);
    std::memcpy(n0, r0, n_ * 8);
    std::memcpy(n1, r1, n_ * 8);
    std::memcpy(n2, r2, n_ * 8);
    std::memcpy(n3, r3, n_ * 8);
    std::memcpy(nk, kn, n_ * 8);
    std::memcpy(nl, lab, n_ * 4);
  }
  ::operator delete(buf_, std::align_val_t(64));
  buf_ = b;
  gid = ng;
  r0 = n0;
  r1 = n1;
  r2 = n2;
  r3 = n3;
  kn = nk;
  lab = nl;
  cap_ = cap;
}

int32_t DirtySet::upsert(int64_t g, const NodeState& st) {
  int32_t i = slot_.insert(g, (int32_t)n_);
  if (i == (int32_t)n_) {
    const size_t w = (size_t)g >> 6;
    if (w >= bits_.size()) bits_.resize(std::max(w + 1, 2 * bits_.size()), 0);
    bits_[w] |= 1ull << (g & 63);
    if (n_ == cap_) grow();
    gid[n_++] = g;
  }
  set(i, st);
  return i;
}

// Node-only key of the device scan (pe_kernels.hip node_prep): (S << 24) | gid with
// S = r0 + (r1 >> 20) + (r2 << 20) + (r3 >> 24), or ~0 where a term can saturate or a residual is
// negative (such nodes are always scored in full).
static uint64_t node_only_key(const NodeState& st, int64_t g) {
  const int64_t* r = st.res;
  if ((r[0] | r[1] | r[2] | r[3]) < 0 || (uint64_t)r[0] > kScoreMax || r[1] >= (1ll << 60) || r[2] >= (1ll << 20))
    return kNoKey;
  const uint64_t S = (uint64_t)r[0] + ((uint64_t)r[1] >> 20) + ((uint64_t)r[2] << 20) + ((uint64_t)r[3] >> 24);
  return S < kScoreMax ? (S << 24) | (uint64_t)g : kNoKey;
}

void DirtySet::set(int32_t i, const NodeState& st) {
  r0[i] = st.res[0];
  r1[i] = st.res[1];
  r2[i] = st.res[2];
  r3[i] = st.res[3];
  lab[i] = st.labels;
  kn[i] = node_only_key(st, gid[i]);
}

NodeState DirtySet::get(int32_t i) const {
  NodeState st;
  st.res[0] = r0[i];
  st.res[1] = r1[i];
  st.res[2] = r2[i];
  st.res[3] = r3[i];
  st.labels = lab[i];
  return st;
}

void DirtySet::clear() {
  slot_.clear(gid, gid + n_);
  for (size_t i = 0; i < n_; ++i) bits_[(size_t)gid[i] >> 6] = 0;
  n_ = 0;
}

// Branch-free Appendix-B key (same arithmetic as the device's node_key)
static inline uint64_t key_bf(int64_t x0, int64_t x1, int64_t x2, int64_t x3, uint32_t l, const int64_t q[RD],
                              uint32_t need, uint64_t g) {
  const bool fit = ((l & need) == need) & (q[0] <= x0) & (q[1] <= x1) & (q[2] <= x2) & (q[3] <= x3);
  const uint64_t a = (uint64_t)x0 - (uint64_t)q[0];
  const uint64_t b = ((uint64_t)x1 - (uint64_t)q[1]) >> 20;
  const uint64_t c = (uint64_t)x2 - (uint64_t)q[2];
  const uint64_t d = ((uint64_t)x3 - (uint64_t)q[3]) >> 24;
  const bool big = (a > kScoreMax) | (b > kScoreMax) | (c >= (1ull << 20)) | (d > kScoreMax);
  const uint64_t sum = a + b + (c << 20) + d;
  const uint64_t score = (big | (sum > kScoreMax)) ? kScoreMax : sum;
  return fit ? ((score << 24) | g) : kNoKey;
}

void DirtySet::keys(const int64_t q[RD], uint32_t need, uint64_t limit, std::vector<uint64_t>& out,
                    IdxVec& idx) const {   // limit: keys >= it may be left out
  const size_t n = n_;
  if (out.size() < n) out.resize(n);   // only the slots listed in idx are read
  idx.clear();
  // [lo, hi): the K(n) that can give a fitting key < limit (s(q) saturated: then nothing but the
  // always-scored nodes can fit)
  uint64_t sq = (uint64_t)q[0] + ((uint64_t)q[1] >> 20) + ((uint64_t)q[3] >> 24);
  sq = (uint64_t)q[0] > kScoreMax || (uint64_t)q[2] >= (1ull << 20) || sq >= kScoreMax ? kScoreMax
                                                                                      : sq + ((uint64_t)q[2] << 20);
  const uint64_t lo = sq >= kScoreMax ? kNoKey : sq << 24;
  const uint64_t q2 = sq + 2 >= (1ull << 40) ? kNoKey : (sq + 2) << 24;
  const uint64_t hi = limit == kNoKey || limit >= kNoKey - q2 ? kNoKey : limit + q2;
  const uint64_t span = hi > lo ? hi - lo : 0;
  // the range test k - lo < span (unsigned) or k == ~0, four nodes per AVX2 step (signed compare
  // of sign-flipped values); the few hits are scored below
  const uint64_t* kp = kn;
  const __m256i flip = _mm256_set1_epi64x(INT64_MIN), vlo = _mm256_set1_epi64x((int64_t)lo),
                vspan = _mm256_set1_epi64x((int64_t)(span ^ (1ull << 63))), ones = _mm256_set1_epi64x(-1);
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const __m256i k = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(kp + i));
    const __m256i d = _mm256_xor_si256(_mm256_sub_epi64(k, vlo), flip);
    const __m256i hit = _mm256_or_si256(_mm256_cmpgt_epi64(vspan, d), _mm256_cmpeq_epi64(k, ones));
    for (int m = _mm256_movemask_pd(_mm256_castsi256_pd(hit)); m; m &= m - 1)
      idx.push_back((int32_t)(i + __builtin_ctz(m)));
  }
  for (; i < n; ++i)
    if (kp[i] - lo < span || kp[i] == kNoKey) idx.push_back((int32_t)i);
  for (int32_t j : idx) out[j] = key_bf(r0[j], r1[j], r2[j], r3[j], lab[j], q, need, (uint64_t)gid[j]);
}

// keys_all, 8 dirty nodes per AVX-512 step: the K(n) range test, the Appendix-B fit and key (the
// arithmetic of key_bf), the fitting slots compressed into idx and the running minimum.  Only the
// fitting slots' keys are stored: callers read out[] at the slots listed in idx.
__attribute__((target("avx512f,avx512dq,avx512vl,avx512bw"))) static uint64_t keys_avx512(
    size_t n, const uint64_t* kn, const int64_t* x0p, const int64_t* x1p, const int64_t* x2p, const int64_t* x3p,
    const uint32_t* lab, const int64_t* gid, const int64_t q[RD], uint32_t need, uint64_t lo, uint64_t span,
    uint64_t* out, int32_t* idx, size_t* n_idx) {
  const __m512i ones = _mm512_set1_epi64(-1), vlo = _mm512_set1_epi64((int64_t)lo),
                vspan = _mm512_set1_epi64((int64_t)span), vneed = _mm512_set1_epi64(need),
                q0 = _mm512_set1_epi64(q[0]), q1 = _mm512_set1_epi64(q[1]), q2 = _mm512_set1_epi64(q[2]),
                q3 = _mm512_set1_epi64(q[3]), smax = _mm512_set1_epi64((int64_t)kScoreMax),
                c20 = _mm512_set1_epi64(1ll << 20);
  const __m256i lane = _mm256_set_epi32(7, 6, 5, 4, 3, 2, 1, 0);
  __m512i vmin = ones;
  size_t ni = 0;
  for (size_t i = 0; i < n; i += 8) {
    const __mmask8 m = n - i >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << (n - i)) - 1);
    const __m512i k = _mm512_maskz_loadu_epi64(m, kn + i);
    __mmask8 fit = m & (_mm512_cmplt_epu64_mask(_mm512_sub_epi64(k, vlo), vspan) | _mm512_cmpeq_epi64_mask(k, ones));
    // (out is read at the slots listed in idx only.  Measured in the box replay, round 6: scoring every
    // group without this skip, +20 %; a range pass compacting the hits, then the hits through
    // gathers, +15 % -- ~9.6 of ~235 dirty nodes pass the range test per group)
    if (!fit) continue;
    const __m512i x0 = _mm512_maskz_loadu_epi64(m, x0p + i), x1 = _mm512_maskz_loadu_epi64(m, x1p + i),
                  x2 = _mm512_maskz_loadu_epi64(m, x2p + i), x3 = _mm512_maskz_loadu_epi64(m, x3p + i);
    const __m512i l = _mm512_cvtepu32_epi64(_mm256_maskz_loadu_epi32(m, lab + i));
    fit &= _mm512_cmpeq_epi64_mask(_mm512_and_si512(l, vneed), vneed) & _mm512_cmple_epi64_mask(q0, x0) &
           _mm512_cmple_epi64_mask(q1, x1) & _mm512_cmple_epi64_mask(q2, x2) & _mm512_cmple_epi64_mask(q3, x3);
    const __m512i a = _mm512_sub_epi64(x0, q0), b = _mm512_srli_epi64(_mm512_sub_epi64(x1, q1), 20),
                  c = _mm512_sub_epi64(x2, q2), d = _mm512_srli_epi64(_mm512_sub_epi64(x3, q3), 24);
    const __m512i sum = _mm512_add_epi64(_mm512_add_epi64(a, b), _mm512_add_epi64(_mm512_slli_epi64(c, 20), d));
    const __mmask8 big = _mm512_cmpgt_epu64_mask(a, smax) | _mm512_cmpgt_epu64_mask(b, smax) |
                         _mm512_cmpge_epu64_mask(c, c20) | _mm512_cmpgt_epu64_mask(d, smax) |
                         _mm512_cmpgt_epu64_mask(sum, smax);
    const __m512i score = _mm512_mask_mov_epi64(sum, big, smax);
    const __m512i key = _mm512_mask_mov_epi64(
        ones, fit, _mm512_or_si512(_mm512_slli_epi64(score, 24), _mm512_maskz_loadu_epi64(m, gid + i)));
    _mm512_mask_storeu_epi64(out + i, fit, key);
    vmin = _mm512_min_epu64(vmin, key);
    _mm256_mask_compressstoreu_epi32(idx + ni, fit, _mm256_add_epi32(lane, _mm256_set1_epi32((int32_t)i)));
    ni += (size_t)__builtin_popcount(fit);
  }
  *n_idx = ni;
  return (uint64_t)_mm512_reduce_min_epu64(vmin);
}

uint64_t DirtySet::keys_all(const int64_t q[RD], uint32_t need, uint64_t limit, std::vector<uint64_t>& out,
                            IdxVec& idx) const {
  // PE_NO_AVX512=1 forces the AVX2 path (tests cover both)
  static const bool avx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
                             __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512bw") &&
                             !std::getenv("PE_NO_AVX512");
  const size_t n = n_;
  if (out.size() < n) out.resize(n);
  if (!avx512) {
    keys(q, need, limit, out, idx);
    uint64_t mk = kNoKey;
    IdxVec fit;
    for (int32_t j : idx)
      if (out[j] != kNoKey) fit.push_back(j);
    std::vector<uint8_t> seen(n, 0);
    for (int32_t j : idx) seen[j] = 1;
    for (size_t j = 0; j < n; ++j)
      if (!seen[j]) out[j] = kNoKey;
    for (int32_t j : fit) mk = std::min(mk, out[j]);
    idx.swap(fit);
    return mk;
  }
  uint64_t sq = (uint64_t)q[0] + ((uint64_t)q[1] >> 20) + ((uint64_t)q[3] >> 24);
  sq = (uint64_t)q[0] > kScoreMax || (uint64_t)q[2] >= (1ull << 20) || sq >= kScoreMax ? kScoreMax
                                                                                      : sq + ((uint64_t)q[2] << 20);
  const uint64_t lo = sq >= kScoreMax ? kNoKey : sq << 24;
  const uint64_t q2 = sq + 2 >= (1ull << 40) ? kNoKey : (sq + 2) << 24;
  const uint64_t hi = limit == kNoKey || limit >= kNoKey - q2 ? kNoKey : limit + q2;
  const uint64_t span = hi > lo ? hi - lo : 0;
  if (idx.size() < n + 16) idx.resize(n + 16);
  size_t ni = 0;
  const uint64_t mk = keys_avx512(n, kn, r0, r1, r2, r3, lab, gid, q, need, lo, span, out.data(), idx.data(), &ni);
  idx.resize(ni);
  return mk;
}

uint64_t DirtySet::key_at(int32_t i, const int64_t q[RD], uint32_t need) const {
  return key_bf(r0[i], r1[i], r2[i], r3[i], lab[i], q, need, (uint64_t)gid[i]);
}

void merge_shards(const std::vector<const GroupCands*>& parts, GroupCands& out) {
  out.own.clear();
  out.limit = kNoKey;
  for (const GroupCands* p : parts) out.limit = std::min(out.limit, p->limit);
  for (const GroupCands* p : parts)
    for (size_t i = 0; i < p->n; ++i)
      if (p->data[i].key < out.limit) out.own.push_back(p->data[i]);
  std::sort(out.own.begin(), out.own.end(), [](const Cand& a, const Cand& b) { return a.key < b.key; });
  out.data = out.own.data();
  out.keys = nullptr;
  out.keyed = false;
  out.n = out.own.size();
}

static std::string list_where(int w, int r) {
  return "corrupt candidate list (group " + std::to_string(w) + ", shard " + std::to_string(r) + "): ";
}

// A header count the slot cannot hold: n < 0 (other than the exchange's timeout marker, handled by
// the caller) or n > K would read outside the group's slot.
static size_t checked_count(int32_t n, int K, int w, int r) {
  if (n < 0 || n > K)
    throw CorruptList(list_where(w, r) + "header count " + std::to_string(n) + " outside [0, " + std::to_string(K) + "]");
  return (size_t)n;
}

void parse_window(const uint8_t* blob, int n_shards, int n_groups, int K, std::vector<GroupCands>& cands,
                  bool copy_blob, int64_t n_nodes) {
  const size_t gb = 16 + (size_t)K * 48;
  const size_t shard_bytes = (size_t)n_groups * gb;
  // validate every header and record before anything is used (no partial window)
  for (int r = 0; r < n_shards; ++r)
    for (int w = 0; w < n_groups; ++w) {
      const uint8_t* base = blob + (size_t)r * shard_bytes + (size_t)w * gb;
      int32_t n;
      std::memcpy(&n, base, 4);
      const size_t m = checked_count(n, K, w, r);
      const Cand* c = reinterpret_cast<const Cand*>(base + 16);
      for (size_t i = 0; i < m; ++i) {
        const uint64_t k = c[i].key;
        if ((int64_t)(k & 0xFFFFFFull) >= n_nodes)
          throw CorruptList(list_where(w, r) + "node id " + std::to_string(k & 0xFFFFFFull) + " outside the " +
                            std::to_string(n_nodes) + "-node inventory");
        if (i > 0 && k <= c[i - 1].key) throw CorruptList(list_where(w, r) + "keys not ascending at entry " + std::to_string(i));
      }
    }
  cands.resize((size_t)n_groups);
  std::vector<GroupCands> parts((size_t)n_shards);
  std::vector<const GroupCands*> pp((size_t)n_shards);
  for (int w = 0; w < n_groups; ++w) {
    for (int r = 0; r < n_shards; ++r) {
      const uint8_t* base = blob + (size_t)r * shard_bytes + (size_t)w * gb;
      int32_t n;
      uint64_t limit;
      std::memcpy(&n, base, 4);
      std::memcpy(&limit, base + 8, 8);
      GroupCands& gc = n_shards == 1 ? cands[w] : parts[r];
      gc.limit = limit;
      gc.n = (size_t)n;   // (validated above)
      gc.data = reinterpret_cast<const Cand*>(base + 16);   // 16-B aligned records in the blob
      gc.keys = nullptr;
      gc.keyed = false;
      if (copy_blob && n_shards == 1) {
        gc.own.assign(gc.data, gc.data + gc.n);
        gc.data = gc.own.data();
      }
      pp[r] = &parts[r];
    }
    if (n_shards > 1) merge_shards(pp, cands[w]);
  }
}

// One group of a one-shard key blob: the list points into the blob.
static void parse_group_keys(const uint8_t* base, int K, size_t w, GroupCands& gc) {
  int32_t n;
  uint64_t limit;
  std::memcpy(&n, base, 4);
  std::memcpy(&limit, base + 8, 8);
  if (n == -1)   // (the zero-copy exchange wait timed out on a peer's list: pe_kernels.h CAND_TIMEOUT)
    throw ExchangeError("host exchange: a rank's candidate lists never arrived (peer stalled or failed; rank " +
                        std::to_string((limit >> 32) & 0x7fffffffu) + "'s slot still held generation " +
                        std::to_string((uint32_t)limit) + ")");
  if (n == -2)   // (a merge found a shard list whose header count was outside [0, K]: CAND_CORRUPT)
    throw CorruptList(list_where((int)w, -1) + "a shard's header count was outside [0, " + std::to_string(K) +
                      "] (merged group marked corrupt)");
  gc.keyed = true;
  gc.data = nullptr;
  gc.merged.clear();
  gc.part.clear();
  gc.part_n.clear();
  gc.limit = limit;
  gc.keys = reinterpret_cast<const uint64_t*>(base + 16);
  gc.n = checked_count(n, K, (int)w, 0);
  for (int l = 0; l < 4; ++l) __builtin_prefetch(gc.keys + 8 * l);   // list heads, fresh from the device
}

void WindowFeed::reset(const uint8_t* blob, int n_groups, int K, uint32_t gen, std::vector<GroupCands>* cands) {
  blob_ = blob;
  n_ = (size_t)std::max(n_groups, 0);
  gb_ = 16 + (size_t)K * 8;
  K_ = K;
  gen_ = gen;
  cands_ = cands;
  cands->resize(n_);
  parsed_.store(0, std::memory_order_relaxed);
  spin_ms_ = 0;
}

bool WindowFeed::signalled(size_t w) const {
  const int32_t* f = reinterpret_cast<const int32_t*>(blob_ + w * gb_ + 4);
  return (uint32_t)__atomic_load_n(f, __ATOMIC_ACQUIRE) == gen_;
}

void WindowFeed::advance() {
  size_t p = parsed_.load(std::memory_order_relaxed);
  const size_t p0 = p;
  while (p < n_ && signalled(p)) {
    parse_group_keys(blob_ + p * gb_, K_, p, (*cands_)[p]);
    ++p;
  }
  if (p != p0) parsed_.store(p, std::memory_order_release);
}

void WindowFeed::wait(size_t w) {
  if (w >= n_) return;
  advance();
  if (w < parsed_.load(std::memory_order_relaxed)) return;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 1;; ++spin) {
    _mm_pause();
    if (signalled(parsed_.load(std::memory_order_relaxed))) {
      advance();
      if (w < parsed_.load(std::memory_order_relaxed)) break;
    }
    if ((spin & 4095) == 0) {
      if (idle && !idle(idle_user)) {
        advance();   // the device is idle: every group it will ever signal is visible now
        if (w < parsed_.load(std::memory_order_relaxed)) break;
        throw std::runtime_error("walk window: group " + std::to_string(w) + " was never signalled");
      }
      if (timeout_s > 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
        if (on_timeout) on_timeout(timeout_user);
        throw CollectiveTimeout("RCCL window: group " + std::to_string(w) + " not merged within " +
                                std::to_string(timeout_s) +
                                " s -- its all-gather is stuck (a peer stalled or was lost; PE_RCCL_TIMEOUT_S)");
      }
    }
  }
  spin_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void parse_window_keys(const uint8_t* blob, int n_shards, int n_groups, int K, std::vector<GroupCands>& cands) {
  const size_t gb = 16 + (size_t)K * 8;
  const size_t shard_bytes = (size_t)n_groups * gb;
  cands.resize((size_t)n_groups);
  for (int w = 0; w < n_groups; ++w) {
    GroupCands& gc = cands[w];
    gc.keyed = true;
    gc.data = nullptr;
    gc.merged.clear();
    gc.part.clear();
    gc.part_n.clear();
    gc.limit = kNoKey;
    for (int r = 0; r < n_shards; ++r) {
      const uint8_t* base = blob + (size_t)r * shard_bytes + (size_t)w * gb;
      int32_t n;
      uint64_t limit;
      std::memcpy(&n, base, 4);
      std::memcpy(&limit, base + 8, 8);
      gc.limit = std::min(gc.limit, limit);
      gc.part.push_back(reinterpret_cast<const uint64_t*>(base + 16));
      gc.part_n.push_back(checked_count(n, K, w, r));
    }
    if (n_shards == 1) {
      gc.keys = gc.part[0];
      gc.n = gc.part_n[0];
      for (int l = 0; l < 4; ++l) __builtin_prefetch(gc.keys + 8 * l);   // list heads, fresh from the device
      continue;
    }
    // global list = every shard's keys below the smallest shard limit
    gc.keys = nullptr;
    gc.n = 0;
    for (int r = 0; r < n_shards; ++r) {
      gc.part_n[r] = (size_t)(std::lower_bound(gc.part[r], gc.part[r] + gc.part_n[r], gc.limit) - gc.part[r]);
      gc.n += gc.part_n[r];
    }
    gc.head.assign((size_t)n_shards, 0);
  }
}

// ------------------------------------------------------------------ SeedScorer

// CPUs sharing cpu's last-level cache (sysfs cache/index3/shared_cpu_list, e.g. "0-7,128-135").
bool l3_cpus(int cpu, cpu_set_t* set) {
  if (cpu < 0) return false;
  char path[96];
  std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char buf[512] = {0};
  const bool ok = std::fgets(buf, sizeof(buf), f) != nullptr;
  std::fclose(f);
  if (!ok) return false;
  CPU_ZERO(set);
  int n = 0;
  for (char* p = buf; *p && *p != '\n';) {
    char* e;
    const long a = std::strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    if (*e == '-') b = std::strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c, ++n) CPU_SET((int)c, set);
    p = *e == ',' ? e + 1 : e;
  }
  return n > 0;
}

int l3_pick(const cpu_set_t& allowed, int k) {
  std::vector<int> first;   // first allowed CPU of each L3 domain
  cpu_set_t seen;
  CPU_ZERO(&seen);
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &allowed) || CPU_ISSET(c, &seen)) continue;
    cpu_set_t dom;
    if (!l3_cpus(c, &dom)) return -1;
    CPU_OR(&seen, &seen, &dom);
    first.push_back(c);
  }
  if (first.empty() || k < 0) return -1;
  return first[(size_t)k % first.size()];
}

void SeedScorer::compute(const DirtySet& seeds, const GroupCands& gc, const int64_t q[RD], uint32_t need,
                         SeedTop& top, std::vector<uint64_t>& out, IdxVec& idx) {
  size_t h = 0;   // (plain key arrays only: a lazily merged shard list is the resolver's to read)
  if (gc.keys)
    while (h < gc.size() && seeds.contains((int64_t)(gc.keys[h] & 0xFFFFFFull))) ++h;
  top.head = h;
  seeds.keys_all(q, need, gc.limit, out, idx);
  int n = 0;
  bool trunc = false;
  for (int32_t i : idx) {   // insertion into the ascending top (few fit below the limit)
    const uint64_t k = out[(size_t)i];
    if (k >= gc.limit) continue;
    if (n == SeedTop::kTop) {
      trunc = true;
      if (k >= top.key[n - 1]) continue;
      --n;
    }
    int j = n++;
    for (; j > 0 && top.key[j - 1] > k; --j) top.key[j] = top.key[j - 1];
    top.key[j] = k;
  }
  top.n = n;
  top.truncated = trunc;
}

SeedScorer::~SeedScorer() {
  if (!th_) return;
  stop();
  state_.store(3, std::memory_order_seq_cst);
  {
    std::lock_guard<std::mutex> lk(park_mu_);
    park_cv_.notify_one();
  }
  th_->join();
}

void SeedScorer::pin(const cpu_set_t& set) {
  pin_set_ = set;
  have_pin_ = true;
  if (th_) (void)pthread_setaffinity_np(th_->native_handle(), sizeof(set), &set);
}

void SeedScorer::start(const DirtySet* seeds, const std::vector<int32_t>* groups,
                       const std::vector<GroupCands>* cands, const int64_t* scan_req, const uint32_t* need,
                       const WindowFeed* feed, const NodeState* mirror, int64_t mirror_n) {
  seeds_ = seeds;
  mirror_ = mirror;
  mirror_n_ = mirror ? mirror_n : 0;
  groups_ = groups;
  cands_ = cands;
  feed_ = feed;
  req_ = scan_req;
  need_ = need;
  if (cap_ < groups->size()) {
    cap_ = std::max<size_t>(groups->size(), 2 * cap_);
    slots_.reset(new TopSlot[cap_]);
    gen_ = 0;
  }
  if (++gen_ == 0) {   // generation wrap-around: clear the flags
    for (size_t i = 0; i < cap_; ++i) slots_[i].gen.store(0, std::memory_order_relaxed);
    gen_ = 1;
  }
  main_wi_.store(0, std::memory_order_relaxed);
  if (!th_) {
    th_.reset(new std::thread([this] { loop(); }));
    // The resolver and the helper exchange a few cache lines per group (flags, tops): keep the
    // helper on the CPUs that share the resolver thread's L3 (one CCD), not across the machine.
#ifndef PE_SEED_TEST_YIELD   // (the handshake test keeps both threads on one CPU)
    cpu_set_t set;
    if (have_pin_) (void)pthread_setaffinity_np(th_->native_handle(), sizeof(pin_set_), &pin_set_);
    else if (l3_cpus(sched_getcpu(), &set)) (void)pthread_setaffinity_np(th_->native_handle(), sizeof(set), &set);
#endif
  }
  // seq_cst with the helper's parked_ store and predicate load: either it sees 1 before sleeping
  // or this sees parked_ and wakes it (no lost wake-up)
  state_.store(1, std::memory_order_seq_cst);
  if (parked_.load(std::memory_order_seq_cst)) {   // the helper sleeps (long idle): wake it
    std::lock_guard<std::mutex> lk(park_mu_);
    park_cv_.notify_one();
  }
}

// Handshake (no separate busy flag): stop() moves 1 -> 2 and waits for 0; only the helper moves
// 2 -> 0, with a CAS, once it has left the window (or never entered it).  A stale read of 2 by the
// helper cannot acknowledge a later window: the CAS fails on the 1 that start() stored.
void SeedScorer::stop() {
  if (!th_) return;
  int posted = 1;
  if (!state_.compare_exchange_strong(posted, 2, std::memory_order_acq_rel)) return;   // nothing posted
  for (int spin = 0; state_.load(std::memory_order_acquire) != 0; ++spin)   // at most one group's work
    if (spin < 4096) _mm_pause();
    else std::this_thread::yield();   // the helper is not running (oversubscribed host)
}

void SeedScorer::loop() {
  int idle = 0;
  for (;;) {
    const int st = state_.load(std::memory_order_acquire);
#ifdef PE_SEED_TEST_YIELD   // tests/cpp/test_feed.cc: widen the gap between reading the state and acting on it
    std::this_thread::yield();
#endif
    if (st == 3) return;
    if (st == 2) {   // cancel seen (window done or never started): acknowledge
      int c = 2;
      state_.compare_exchange_strong(c, 0, std::memory_order_acq_rel);
      continue;
    }
    if (st != 1) {
      if (++idle < 4096) _mm_pause();
      else if (idle < kParkAfter) std::this_thread::yield();   // idle: let others run
      else {   // long idle (e.g. a pe_resolver between ABI calls): sleep until start() or exit
        std::unique_lock<std::mutex> lk(park_mu_);
        parked_.store(true, std::memory_order_seq_cst);
        park_cv_.wait_for(lk, std::chrono::milliseconds(20),
                          [this] { return state_.load(std::memory_order_seq_cst) != 0; });
        parked_.store(false, std::memory_order_relaxed);
      }
      continue;
    }
    idle = 0;
    const size_t W = groups_->size();
    const uint32_t gen = gen_;
    for (size_t wi = 0; wi < W; ++wi) {
      if (state_.load(std::memory_order_acquire) != 1) break;   // cancelled: the resolver moved on
      wi = std::max(wi, main_wi_.load(std::memory_order_relaxed) + 1);   // leapfrog a resolver ahead
      if (wi >= W) break;
      if (feed_ && wi >= feed_->parsed()) {   // its list has not arrived yet: wait (or be overtaken)
        bool go = true;
        for (int spin = 0; wi >= feed_->parsed(); ++spin) {
          if (state_.load(std::memory_order_acquire) != 1) {
            go = false;
            break;
          }
          if (spin < 4096) _mm_pause();
          else std::this_thread::yield();
          wi = std::max(wi, main_wi_.load(std::memory_order_relaxed) + 1);
          if (wi >= W) {
            go = false;
            break;
          }
        }
        if (!go) break;
      }
#ifdef PE_SEED_TEST_YIELD
      std::this_thread::yield();
#endif
      const int32_t g = (*groups_)[wi];
      try {
        compute(*seeds_, (*cands_)[wi], req_ + (int64_t)g * RD, need_[g], slots_[wi].top, out_, idx_);
      } catch (...) {   // (bad_alloc) the resolver scores the remaining groups itself
        break;
      }
      slots_[wi].gen.store(gen, std::memory_order_release);
      if (mirror_) {   // the first non-seed entries' states, read here (see mirror_)
        const GroupCands& gc = (*cands_)[wi];
        if (gc.keys) {
          int64_t sink = 0;
          for (size_t i = slots_[wi].top.head, e = std::min(gc.size(), i + (size_t)kWarmStates); i < e; ++i) {
            const uint64_t id = gc.keys[i] & 0xFFFFFFull;
            if (id < (uint64_t)mirror_n_) sink += mirror_[id].res[0];   // (an id outside: the resolver raises on it)
          }
          warm_sink_ += sink;
        }
      }
    }
    // done with the window: wait for stop() (state 2, acknowledged at the top of the loop)
    for (int spin = 0; state_.load(std::memory_order_acquire) == 1; ++spin)
      if (spin < 4096) _mm_pause();
      else std::this_thread::yield();
  }
}

Resolver::Resolver(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority, const int32_t* group_count,
                   const int64_t* group_req, const uint32_t* group_need) {
  reset(n_jobs, job_group_off, priority, group_count, group_req, group_need);
}

void Resolver::reset(int64_t n_jobs, const int32_t* job_group_off, const int32_t* priority, const int32_t* group_count,
                     const int64_t* group_req, const uint32_t* group_need) {
  J_ = n_jobs;
  jgo_ = job_group_off;
  cnt_ = group_count;
  req_ = group_req;
  need_ = group_need;
  oi_ = 0;
  g_ = 0;
  p_ = 0;
  dirty_.clear();
  seeds_.clear();
  prev_.clear();
  prev_ok_ = false;
  std::fill(any_.begin(), any_.end(), 0ull);   // (cleared per window; a call that threw may have left bits)
  if (!changed_.empty()) {
    changed_slot_.clear(changed_gid_.begin(), changed_gid_.end());
    changed_.clear();
    changed_gid_.clear();
  }
  jobs_placed_ = jobs_failed_ = pods_placed_ = rescans_ = 0;
  // job order: priority desc, index asc.  Priorities within a range of a few times J (the usual
  // case: a handful of PriorityClass values) take one counting pass; a stable merge sort of 10k jobs
  // was ~0.3 ms of every batch's set-up on the box.
  order_.resize((size_t)J_);
  int32_t plo = INT32_MAX, phi = INT32_MIN;
  for (int64_t j = 0; j < J_; ++j) {
    plo = std::min(plo, priority[j]);
    phi = std::max(phi, priority[j]);
  }
  const uint64_t prange = J_ > 0 ? (uint64_t)((int64_t)phi - (int64_t)plo) + 1 : 0;
  if (J_ > 0 && prange <= (uint64_t)std::max<int64_t>(65536, 4 * J_)) {
    std::vector<int64_t> at(prange + 1, 0);   // bucket b = phi - priority: highest priority first
    for (int64_t j = 0; j < J_; ++j) ++at[(size_t)(phi - priority[j]) + 1];
    for (size_t b = 1; b <= prange; ++b) at[b] += at[b - 1];
    for (int64_t j = 0; j < J_; ++j) order_[(size_t)at[(size_t)(phi - priority[j])]++] = j;
  } else {
    std::iota(order_.begin(), order_.end(), 0);
    std::stable_sort(order_.begin(), order_.end(), [&](int64_t a, int64_t b) { return priority[a] > priority[b]; });
  }
  const int64_t G = J_ > 0 ? jgo_[J_] : 0;
  pod_off_.assign((size_t)G + 1, 0);
  for (int64_t g = 0; g < G; ++g) pod_off_[g + 1] = pod_off_[g] + std::max<int32_t>(cnt_[g], 0);
  pod_node_.assign((size_t)pod_off_[G], -1);
  job_status_.assign((size_t)J_, 0);
  qeff_.assign(req_, req_ + (size_t)G * RD);
  unit_.assign((size_t)G, 0);
  for (int64_t g = 0; g < G; ++g)
    if (need_[g] & kNeedIsland) {
      unit_[g] = 1;
      for (int d = 0; d < RD; ++d)
        if (__builtin_mul_overflow(req_[g * RD + d], (int64_t)std::max<int32_t>(cnt_[g], 0), &qeff_[g * RD + d])) {
          unit_[g] = 2;   // fits nowhere; the scan request saturates
          qeff_[g * RD + d] = INT64_MAX;
        }
    }
  if (!done()) g_ = jgo_[order_[0]];
  advance_group();
}

// Move the cursor to the next pod that needs placing, finishing jobs whose groups are all placed.
void Resolver::advance_group() {
  while (!done()) {
    const int64_t j = order_[oi_];
    if (g_ >= jgo_[j + 1]) {
      finish_job(true);
      continue;
    }
    if (p_ >= cnt_[g_]) {
      ++g_;
      p_ = 0;
      continue;
    }
    break;
  }
}

// A node the current job placed pods on: in the window's dirty set if this window changed it,
// else its state as of the end of the window that last changed it (mirror, or changed_).
NodeState Resolver::current_state(int64_t gid) const {
  const int32_t i = dirty_.find(gid);
  if (i >= 0) return dirty_.get(i);
  if (mirror_.nodes) return mirror_.nodes[gid];
  const int32_t c = changed_slot_.find(gid);
  if (c < 0) throw std::logic_error("resolver: rollback of a node with no known state");
  return changed_[(size_t)c];
}

void Resolver::finish_job(bool ok) {
  const int64_t j = order_[oi_];
  if (ok) {
    job_status_[j] = 0;
    ++jobs_placed_;
  } else {
    // all-or-nothing: give back every pod this job placed, the restored nodes become dirty
    for (int32_t g = jgo_[j]; g < jgo_[j + 1]; ++g) {
      const int64_t* q = req_ + (int64_t)g * RD;
      for (int32_t p = 0; p < cnt_[g]; ++p) {
        int32_t& slot = pod_node_[pod_off_[g] + p];
        if (slot < 0) continue;
        NodeState st = current_state(slot);
        for (int d = 0; d < RD; ++d) st.res[d] += q[d];
        dirty_.upsert(slot, st);
        any_set(slot);
        slot = -1;
        --pods_placed_;
      }
    }
    job_status_[j] = 1;
    ++jobs_failed_;
  }
  // the states recorded for rollbacks so far belong to this job's windows: a later job rolls back
  // only nodes it placed on, whose states are recorded after it started (bounded memory)
  if (!changed_.empty()) {
    changed_slot_.clear(changed_gid_.begin(), changed_gid_.end());
    changed_.clear();
    changed_gid_.clear();
  }
  ++oi_;
  p_ = 0;
  if (!done()) g_ = jgo_[order_[oi_]];
}

void Resolver::next_window(int max_groups, int64_t max_pods, std::vector<int32_t>& groups) {
  Cursor end;
  next_window_from(cursor(), max_groups, max_pods, groups, &end);
}

void Resolver::next_window_from(const Cursor& from, int max_groups, int64_t max_pods, std::vector<int32_t>& groups,
                                Cursor* end) const {
  groups.clear();
  *end = from;
  if (from.oi >= (int64_t)order_.size()) return;
  int64_t pods = 0;
  int64_t oi = from.oi;
  int32_t g = from.g;
  int32_t p = from.p;
  while (oi < (int64_t)order_.size() && (int)groups.size() < max_groups) {
    const int64_t j = order_[oi];
    if (g >= jgo_[j + 1]) {
      ++oi;
      if (oi < (int64_t)order_.size()) g = jgo_[order_[oi]];
      p = 0;
      continue;
    }
    if (cnt_[g] > p) {
      if (!groups.empty() && pods + (cnt_[g] - p) > max_pods) break;
      groups.push_back(g);
      pods += cnt_[g] - p;
    }
    ++g;
    p = 0;
  }
  // normalise the end like advance_group() would: skip empty groups and finished jobs
  while (oi < (int64_t)order_.size()) {
    const int64_t j = order_[oi];
    if (g >= jgo_[j + 1]) {
      ++oi;
      if (oi < (int64_t)order_.size()) g = jgo_[order_[oi]];
      p = 0;
      continue;
    }
    if (p >= cnt_[g]) {
      ++g;
      p = 0;
      continue;
    }
    break;
  }
  *end = Cursor{oi, g, p};
}

// The dirty set holds exactly these updates, in order (it produced them).
static bool same_updates(const DirtySet& d, const std::vector<Update>& u) {
  if (d.size() != u.size()) return false;
  for (size_t i = 0; i < u.size(); ++i)
    if (d.gid[i] != u[i].gid || d.r0[i] != u[i].res[0] || d.r1[i] != u[i].res[1] || d.r2[i] != u[i].res[2] ||
        d.r3[i] != u[i].res[3] || d.lab[i] != u[i].labels)
      return false;
  return true;
}

bool Resolver::resolve(const std::vector<int32_t>& groups, const std::vector<GroupCands>& cands,
                       std::vector<Update>& updates, const std::vector<Update>* seed, WindowFeed* feed) {
  bool consumed = true;
  unsigned long long t_ = RP_T();
  // Pipelined windows: the seeds (dirty for the whole window, their state known) are kept apart
  // from the window's own changes (dirty_); the helper thread scores them for every group ahead of
  // this thread.  A seed this window changes moves to dirty_ and is scored here from then on.
  const bool useS = seed && !seed->empty();
  struct ScorerStop {   // the helper never outlives this call (it reads groups / cands / seeds_)
    SeedScorer& s;
    ~ScorerStop() { s.stop(); }
  } scorer_stop{scorer_};
  if (useS) {
    if (prev_ok_ && same_updates(prev_, *seed)) {
      std::swap(seeds_, prev_);   // the previous window's changes, as this window's seeds
    } else {
      seeds_.clear();
      for (const Update& u : *seed) {
        NodeState st;
        for (int d = 0; d < RD; ++d) st.res[d] = u.res[d];
        st.labels = u.labels;
        seeds_.upsert(u.gid, st);
      }
    }
    scorer_.start(&seeds_, &groups, &cands, qeff_.data(), need_, feed, mirror_.nodes, mirror_.n);
    for (size_t i = 0; i < seeds_.size(); ++i) any_set(seeds_.gid[i]);
  }
  if (feed) feed->advance();
  auto have = [&](size_t w) { return !feed || w < feed->parsed(); };   // list of group w is there
  auto is_dirty = [&](int64_t gid) { return any_has(gid); };   // dirty_.contains || (useS && seeds_.contains)
  RP_ADD(seed, t_);
  for (int32_t g : groups) {   // the window's group records (scattered over the batch arrays)
    __builtin_prefetch(req_ + (int64_t)g * RD);
    __builtin_prefetch(&cnt_[g]);
    __builtin_prefetch(&need_[g]);
    __builtin_prefetch(&pod_off_[g]);
  }
  head_.assign(groups.size(), 0);
  for (size_t w = 0; w < std::min<size_t>(kLookStates, groups.size()); ++w)   // the first groups' list heads
    if (have(w) && cands[w].keyed)
      for (size_t i = 0; i < std::min<size_t>(4, cands[w].size()); ++i)
        __builtin_prefetch(&mirror_.nodes[cands[w].key(i) & 0xFFFFFFull]);
  size_t wi = 0;
  std::vector<uint64_t>& dk = dk_;  // keys of the dirty nodes for the current group
  IdxVec& dki = dki_;  // the slots among them that can hold a key
  auto argmin = [&dk, &dki]() -> int32_t {
    int32_t b = -1;
    uint64_t bk = kNoKey;
    for (int32_t i : dki)
      if (dk[i] < bk) {
        bk = dk[i];
        b = i;
      }
    return b;
  };
  while (!done() && wi < groups.size()) {
    while (wi < groups.size() && groups[wi] != g_) ++wi;  // groups of failed jobs are skipped
    if (wi == groups.size()) break;
    if (feed) {
      feed->advance();
      if (wi >= feed->parsed()) feed->wait(wi);
    }
    const GroupCands& gc = cands[wi];
    const int64_t* q = scan_req(g_);   // an island group is one unit of count x request
    const uint32_t need = need_[g_];
    const uint8_t unit = unit_[g_];
    t_ = RP_T();
    // Look ahead: the list lines of the group kLookLines ahead on their way; the first clean entries
    // of the group kLookStates ahead found (the dirty entries before them skipped for good -- the
    // dirty set only grows during a resolve; the seed helper reads their mirror states).
    if (wi + kLookLines < groups.size() && have(wi + kLookLines) && cands[wi + kLookLines].keys)
      for (int l = 0; l < 2; ++l) __builtin_prefetch(cands[wi + kLookLines].keys + 8 * l);
    if (wi + kLookStates < groups.size() && have(wi + kLookStates) && cands[wi + kLookStates].keyed) {
      const size_t wn = wi + kLookStates;
      const GroupCands& gn = cands[wn];
      size_t p = useS && scorer_.ready(wn) ? scorer_.top(wn).head : 0;   // (the helper skipped the seeds)
      while (p < gn.size() && is_dirty((int64_t)(gn.key(p) & 0xFFFFFFull))) ++p;
      head_[wn] = p;
      // (its first clean entries' mirror states are read by the seed helper: SeedScorer::mirror_.
      // Prefetching them here as well was ~1.5 % slower in the box replay, profiles/r17_resolver_ab.txt)
    }
    RP_ADD(la, t_);
    unsigned long long t2_ = RP_T();
    dirty_.keys_all(q, need, gc.limit, dk, dki);   // dirty keys >= limit never decide (list head or rescan)
    int32_t best = argmin();
    RP_ADD(ka, t2_);
    t2_ = RP_T();
    // the seeds' keys: the helper's top (or computed here when it is not ready yet)
    SeedTop local;
    const SeedTop* top = nullptr;
    if (useS) {
      scorer_.at(wi);
      if (scorer_.ready(wi)) {
        top = &scorer_.top(wi);
#ifdef PE_RES_PROF
        rp.sready++;
#endif
      } else {
#ifdef PE_RES_PROF
        rp.slocal++;
#endif
        SeedScorer::compute(seeds_, gc, q, need, local, sk_out_, sk_idx_);
        top = &local;
      }
    }
    size_t sp = 0;        // next candidate of the seed top
    bool sfull = false;   // the top ran out (truncated): every seed key below the limit in sfull_
    auto seed_key = [&]() -> uint64_t {   // smallest key of a seed this window has not changed
      if (!useS) return kNoKey;
      for (;;) {
        const uint64_t* ks = sfull ? sfull_.data() : top->key;
        const size_t n = sfull ? sfull_.size() : (size_t)top->n;
        while (sp < n && dirty_.contains((int64_t)(ks[sp] & 0xFFFFFFull))) ++sp;
        if (sp < n) return ks[sp];
        if (sfull || !top->truncated) return kNoKey;
        seeds_.keys_all(q, need, gc.limit, sk_out_, sk_idx_);
        sfull_.clear();
        for (int32_t i : sk_idx_)
          if (sk_out_[(size_t)i] < gc.limit) sfull_.push_back(sk_out_[(size_t)i]);
        std::sort(sfull_.begin(), sfull_.end());
#ifdef PE_RES_PROF
        rp.sfull++;
#endif
        sfull = true;
        sp = 0;
      }
    };
    RP_ADD(st, t2_);
    RP_ADD(keys, t_);
#ifdef PE_RES_PROF
    rp.groups++;
    rp.dirty += (long)dirty_.size();
    rp.scored += (long)dki.size();
#endif
    size_t ptr = useS ? std::max(top->head, head_[wi]) : head_[wi];
    size_t pf = ptr;   // clean entries up to pf have been prefetched
    bool failed = false;
#ifdef PE_RES_PROF
    // does this group's answer depend on an earlier group of the window (a node changed in this
    // window: skipped at its list head, or chosen from the dirty set)?  Then resolving the group
    // apart from its predecessors (speculatively, on another thread) would have to be redone.
    bool conflict = false;
    for (size_t i = 0; i < ptr && i < gc.size(); ++i)
      if (dirty_.contains((int64_t)(gc.key(i) & 0xFFFFFFull))) { conflict = true; rp.cskip++; break; }
#endif
    if (unit == 2) failed = true;   // an island group whose summed request overflows fits nowhere
    while (!failed && p_ < cnt_[g_]) {
      t_ = RP_T();
      while (ptr < gc.size() && is_dirty((int64_t)(gc.key(ptr) & 0xFFFFFFull))) {
#ifdef PE_RES_PROF
        rp.skips++;
        if (!conflict && dirty_.contains((int64_t)(gc.key(ptr) & 0xFFFFFFull))) conflict = true, rp.cskip++;
#endif
        ++ptr;
      }
      RP_ADD(skip, t_);
      t_ = RP_T();
      const uint64_t kc = ptr < gc.size() ? gc.key(ptr) : kNoKey;
      const uint64_t kdT = best >= 0 ? dk[best] : kNoKey;
      const uint64_t kdS = seed_key();
      const uint64_t kd = std::min(kdT, kdS);
      if (ptr == gc.size() && gc.limit != kNoKey && kd >= gc.limit) {
        consumed = false;  // clean nodes beyond the limit could win: rescan from this pod
        break;
      }
      const uint64_t bkey = std::min(kc, kd);
      if (bkey == kNoKey) {
        failed = true;
        break;
      }
      const int64_t gid = (int64_t)(bkey & 0xFFFFFFull);
      NodeState st;
      int32_t slot;
      if (bkey == kdT) {
        slot = best;
        st = dirty_.get(slot);
#ifdef PE_RES_PROF
        if (!conflict) conflict = true, rp.cdirty++;   // (every dirty entry is this window's change)
#endif
      } else if (bkey == kdS) {   // an unchanged seed: its window-start state is current
        st = seeds_.get(seeds_.find(gid));
        slot = -1;
      } else {
        if (gc.keyed) {   // clean: the mirror holds the snapshot state
          if (__builtin_expect(gid >= mirror_.n, 0))   // (a device-written id: checked where it is used)
            throw CorruptList(list_where((int)wi, -1) + "node id " + std::to_string(gid) + " outside the " +
                              std::to_string(mirror_.n) + "-node inventory");
          st = mirror_.nodes[gid];
          // keep the next two clean entries' states on their way
#ifndef PE_PLACE_PREFETCH
#define PE_PLACE_PREFETCH 2
#endif
#ifndef PE_NO_PLACE_PREFETCH   // (A/B: without it the box replay took 10.6-11.1 instead of 8.2-8.5 ms)
          for (int c = 0; pf < gc.size() && c < PE_PLACE_PREFETCH; ++pf)
            if (pf > ptr && !is_dirty((int64_t)(gc.key(pf) & 0xFFFFFFull))) {
              __builtin_prefetch(&mirror_.nodes[gc.key(pf) & 0xFFFFFFull]);
              ++c;
            }
#endif
        } else {
          const Cand& c = gc.data[ptr];
          for (int d = 0; d < RD; ++d) st.res[d] = c.res[d];
          st.labels = c.labels;
        }
        slot = -1;
      }
      RP_ADD(p1, t_);
      unsigned long long t3_ = RP_T();
      // The chosen node's key only falls while it still fits (its leftovers shrink), so it stays
      // the minimum for every following pod of the group that still fits on it: place them all
      // at once, m = min(pods left, min over q_d > 0 of res_d / q_d).
      int64_t m = cnt_[g_] - p_;
      if (unit) {             // the whole island group on this node (it fits count x request)
        for (int d = 0; d < RD; ++d) st.res[d] -= q[d];
      } else if (m > 1) {   // (the chosen node fits one pod; divide only when the rest may not fit)
        bool all = true;
        for (int d = 0; d < RD; ++d) {
          int64_t need_d;
          all &= q[d] == 0 || (!__builtin_mul_overflow(q[d], m, &need_d) && need_d <= st.res[d]);
        }
        if (!all)
          for (int d = 0; d < RD; ++d)
            if (q[d] > 0) m = std::min<int64_t>(m, st.res[d] / q[d]);
      }
      if (!unit)
        for (int d = 0; d < RD; ++d) st.res[d] -= m * q[d];
      RP_ADD(p2, t3_);
      t3_ = RP_T();
      if (slot < 0) {
        slot = dirty_.upsert(gid, st);
        any_set(gid);
        if (dk.size() <= (size_t)slot) dk.resize((size_t)slot + 1);
        dki.push_back(slot);
      } else {
        dirty_.set(slot, st);
      }
      std::fill_n(pod_node_.begin() + pod_off_[g_] + p_, m, (int32_t)gid);
      p_ += (int32_t)m;
      pods_placed_ += m;
      // still fitting only if the group ran out of pods first; then it stays the minimum
      dk[slot] = dirty_.key_at(slot, q, need);
      if (dk[slot] != kNoKey) best = slot;
      else if (best == slot) best = argmin();
      RP_ADD(p3, t3_);
      RP_ADD(place, t_);
#ifdef PE_RES_PROF
      rp.pods++;
#endif
    }
#ifdef PE_RES_PROF
    rp.cgroups += conflict;
#endif
    if (!consumed) break;
    if (failed) {
      finish_job(false);
      advance_group();
    } else {
      ++g_;
      p_ = 0;
      advance_group();
    }
    ++wi;
  }
  t_ = RP_T();
  for (size_t i = 0; i < dirty_.size(); ++i) {   // (every entry: the seeds live apart, in seeds_)
    Update u;
    u.gid = dirty_.gid[i];
    const NodeState st = dirty_.get((int32_t)i);
    for (int d = 0; d < RD; ++d) u.res[d] = st.res[d];
    u.labels = st.labels;
    updates.push_back(u);
    if (!mirror_.nodes) {   // (record-form lists: the resolver keeps the states it gave for rollbacks)
      const int32_t c = changed_slot_.insert(u.gid, (int32_t)changed_.size());
      if (c == (int32_t)changed_.size()) {
        changed_.push_back(st);
        changed_gid_.push_back(u.gid);
      } else {
        changed_[(size_t)c] = st;
      }
    }
  }
  for (size_t i = 0; i < dirty_.size(); ++i) any_[(size_t)dirty_.gid[i] >> 6] = 0;   // (whole words: every bit set is listed)
  if (useS)
    for (size_t i = 0; i < seeds_.size(); ++i) any_[(size_t)seeds_.gid[i] >> 6] = 0;
  prev_.clear();               // (last window's changes, or the seeds taken over from them)
  std::swap(prev_, dirty_);    // kept: the next window's seeds if it is pipelined on this one
  prev_ok_ = true;
  RP_ADD(fin, t_);
  if (!consumed) ++rescans_;
  return consumed;
}

}  // namespace pe
