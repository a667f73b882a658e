// Host merge of per-rank candidate lists (the zero-copy shared-memory exchange, pe_engine.cpp): the
// rule of merge_shards_kernel on the host -- the keys below the smallest rank limit L, the Kc + 1
// smallest of them; the merged list holds the first Kc, its limit is the (Kc+1)-th key, else L.
// Pure host code (no HIP), so tools/bench_merge.cc times exactly what the exchange thread runs.
#pragma once
#include <immintrin.h>
#include <stdint.h>

#include <algorithm>

namespace pe {

constexpr int MERGE_MAX_WORLD = 32;   // (HX_ZC_MAX_WORLD)
constexpr int MERGE_MAX_LIST = 2048;  // keys per rank list the merge buffers hold (MG_CAP / world >= this)

// Two ascending u64 lists (unique keys) merged: the first `want` keys of their union into out (which
// holds want rounded up to 8, + 8).  AVX-512 bitonic merge, 8 keys per step (the scalar merge is a
// chain of dependent loads and compares, ~7 cycles per key).
#define PE_AVX512 __attribute__((target("avx512f")))
PE_AVX512 static inline __m512i bitonic8(__m512i v) {   // a bitonic 8-vector, sorted ascending
  const __m512i p4 = _mm512_set_epi64(3, 2, 1, 0, 7, 6, 5, 4), p2 = _mm512_set_epi64(5, 4, 7, 6, 1, 0, 3, 2),
                p1 = _mm512_set_epi64(6, 7, 4, 5, 2, 3, 0, 1);
  __m512i q = _mm512_permutexvar_epi64(p4, v);
  v = _mm512_mask_blend_epi64(0xF0, _mm512_min_epu64(v, q), _mm512_max_epu64(v, q));
  q = _mm512_permutexvar_epi64(p2, v);
  v = _mm512_mask_blend_epi64(0xCC, _mm512_min_epu64(v, q), _mm512_max_epu64(v, q));
  q = _mm512_permutexvar_epi64(p1, v);
  return _mm512_mask_blend_epi64(0xAA, _mm512_min_epu64(v, q), _mm512_max_epu64(v, q));
}
PE_AVX512 static inline void merge16(__m512i& lo, __m512i& hi, __m512i a, __m512i b) {   // a, b sorted
  const __m512i rev = _mm512_set_epi64(0, 1, 2, 3, 4, 5, 6, 7);
  const __m512i rb = _mm512_permutexvar_epi64(rev, b);
  lo = bitonic8(_mm512_min_epu64(a, rb));
  hi = bitonic8(_mm512_max_epu64(a, rb));
}
PE_AVX512 static inline __m512i load8pad(const uint64_t* p, int i, int n) {   // p[i .. i+8), ~0 past n
  const int k = std::max(0, std::min(8, n - i));
  return _mm512_mask_loadu_epi64(_mm512_set1_epi64(-1), (__mmask8)((1u << k) - 1u), p + i);
}
PE_AVX512 static inline int merge2_avx512(const uint64_t* a, int na, const uint64_t* b, int nb, int want, uint64_t* out) {
  __m512i lo, hi;
  merge16(lo, hi, load8pad(a, 0, na), load8pad(b, 0, nb));
  int ia = 8, ib = 8, m = 8;
  _mm512_storeu_si512(out, lo);
  // branch-free steps: the next 8 keys come from the list whose next key is smaller (a random choice
  // per step -- as a branch it mispredicted half the time, ~3x the step's own cost)
  while (m < want) {
    const uint64_t xa = ia < na ? a[ia] : ~0ull, xb = ib < nb ? b[ib] : ~0ull;
    if ((xa & xb) == ~0ull) {   // (both exhausted: ~0 is never a key)
      _mm512_storeu_si512(out + m, hi);
      m += 8;
      break;
    }
    const bool ta = xa < xb;
    const uint64_t* p = ta ? a + ia : b + ib;
    const int n = ta ? na - ia : nb - ib;
    ia += ta ? 8 : 0;
    ib += ta ? 0 : 8;
    merge16(lo, hi, hi, load8pad(p, 0, n));
    _mm512_storeu_si512(out + m, lo);
    m += 8;
  }
  return std::min(m, want);
}
static const bool kHaveAvx512 = __builtin_cpu_supports("avx512f");

// Up to MERGE_MAX_WORLD / 2 independent two-list merges advanced in lockstep, one 8-key step of each
// in turn: a single bitonic merge is a chain of dependent steps (~20 cycles of latency each, the core
// otherwise idle), so the merges of one tree level overlap in the out-of-order window instead.
struct MergeStream {
  const uint64_t *a, *b;
  int na, nb, ia, ib, m, want;
  uint64_t* out;
  __m512i hi;
};
PE_AVX512 static inline void merge_streams_avx512(MergeStream* st, int ns) {
  for (int i = 0; i < ns; ++i) {
    MergeStream& x = st[i];
    if (x.want <= 0) {
      x.m = 0;
      continue;
    }
    __m512i lo;
    merge16(lo, x.hi, load8pad(x.a, 0, x.na), load8pad(x.b, 0, x.nb));
    _mm512_storeu_si512(x.out, lo);
    x.ia = x.ib = x.m = 8;
  }
  for (bool more = true; more;) {
    more = false;
    for (int i = 0; i < ns; ++i) {
      MergeStream& x = st[i];
      if (x.m >= x.want) continue;
      const uint64_t xa = x.ia < x.na ? x.a[x.ia] : ~0ull, xb = x.ib < x.nb ? x.b[x.ib] : ~0ull;
      if ((xa & xb) == ~0ull) {   // both exhausted
        _mm512_storeu_si512(x.out + x.m, x.hi);
        x.m += 8;
        x.want = std::min(x.want, x.m);
        continue;
      }
      const bool ta = xa < xb;
      const uint64_t* p = ta ? x.a + x.ia : x.b + x.ib;
      const int n = ta ? x.na - x.ia : x.nb - x.ib;
      x.ia += ta ? 8 : 0;
      x.ib += ta ? 0 : 8;
      __m512i lo;
      merge16(lo, x.hi, x.hi, load8pad(p, 0, n));
      _mm512_storeu_si512(x.out + x.m, lo);
      x.m += 8;
      more |= x.m < x.want;
    }
  }
  for (int i = 0; i < ns; ++i) st[i].m = std::min(st[i].m, st[i].want);
}

// The tree merge's level buffers, one set per thread (528 KiB)
using MergeTreeBuf = uint64_t[2][MERGE_MAX_WORLD / 2][MERGE_MAX_LIST + 16];
static inline MergeTreeBuf& merge_tree_buf() {
  alignas(64) static thread_local MergeTreeBuf buf;
  return buf;
}

// A merge thread's first-touch page faults on its buffers, taken before its first window (posted to
// each merge thread as it starts) instead of inside it
static inline void merge_warm() {
  MergeTreeBuf& b = merge_tree_buf();
  volatile uint64_t* p = &b[0][0][0];
  for (size_t i = 0; i < sizeof(MergeTreeBuf) / sizeof(uint64_t); i += 512) p[i] = 0;   // one store per 4 KiB page
}

// The balanced tree of merge_rank_lists: each level's merges in lockstep; level l reads cur[], writes
// into buf[l & 1].  Returns the merged count (<= Kc + 1) and its keys in *out (thread-local storage).
PE_AVX512 static inline int merge_tree_avx512(const uint64_t* const* lists, const int* ns, int W, int Kc,
                                              const uint64_t** out) {
  MergeTreeBuf& buf = merge_tree_buf();
  const uint64_t* cur[MERGE_MAX_WORLD];
  int cn[MERGE_MAX_WORLD];
  int n = W;
  for (int r = 0; r < W; ++r) {
    cur[r] = lists[r];
    cn[r] = std::min(ns[r], Kc + 1);
  }
  for (int level = 0; n > 1; ++level) {
    MergeStream st[MERGE_MAX_WORLD / 2];
    const int pairs = n / 2;
    for (int i = 0; i < pairs; ++i)
      st[i] = MergeStream{cur[2 * i], cur[2 * i + 1], cn[2 * i], cn[2 * i + 1], 0, 0, 0,
                          std::min(Kc + 1, cn[2 * i] + cn[2 * i + 1]), buf[level & 1][i], _mm512_setzero_si512()};
    merge_streams_avx512(st, pairs);
    for (int i = 0; i < pairs; ++i) {
      cur[i] = st[i].out;
      cn[i] = st[i].m;
    }
    if (n & 1) {   // the odd list out moves up a level as it is
      cur[pairs] = cur[n - 1];
      cn[pairs] = cn[n - 1];
    }
    n = pairs + (n & 1);
  }
  *out = cur[0];
  return cn[0];
}

// Index of the first key >= X in the ascending p[from, n) (n if none): 8 keys per compare, so only the
// lines up to the answer are read (a binary search touched lines all over a cold 2 KB list).
PE_AVX512 static inline int first_at_least(const uint64_t* p, int from, int n, uint64_t X) {
  const __m512i x = _mm512_set1_epi64((long long)X);
  for (int i = from; i < n; i += 8) {
    const int k = std::min(8, n - i);
    const __m512i v = _mm512_mask_loadu_epi64(_mm512_set1_epi64(-1), (__mmask8)((1u << k) - 1u), p + i);
    const unsigned below = (unsigned)_mm512_cmplt_epu64_mask(v, x);   // a prefix of the 8 (ascending keys)
    if (below != 0xFFu) return i + __builtin_popcount(below);
  }
  return n;
}

// lists[r][0 .. ns[r]) ascending (ns already within the list slots), L = the smallest rank limit.
// Writes the first min(#keys below L, Kc) merged keys into dst and returns their count; *lim = the
// (Kc+1)-th key below L if there is one, else L.  ns is cut in place.
// Three rank lists or more (AVX-512): every list is cut at U, the largest of the lists' c-th keys below
// L (c = ceil((Kc+1) / W)) -- at least Kc + 1 keys lie at or below U, so the Kc + 1 smallest are all
// among the cut lists (~1.3 (Kc+1) keys in all at 8 ranks, instead of 8 x Kc) -- and the cut lists are
// merged as a balanced tree whose levels run lockstep (merge_streams).  The cuts scan each list from
// its head, so a cold list is read only as far as it is used.
static inline int merge_rank_lists(const uint64_t* const* lists, int* ns, int W, uint64_t L, int Kc, uint64_t* dst,
                                   uint64_t* lim) {
  *lim = L;
  if (kHaveAvx512 && W >= 3 && Kc + 1 <= MERGE_MAX_LIST && W <= MERGE_MAX_WORLD) {
    const int c = (Kc + 1 + W - 1) / W;
    int have = 0;
    uint64_t U = 0;
    int head[MERGE_MAX_WORLD];
    for (int r = 0; r < W; ++r) {
      head[r] = first_at_least(lists[r], 0, std::min(ns[r], c), L);   // (<= c keys below L)
      have += head[r];
      if (head[r] > 0) U = std::max(U, lists[r][head[r] - 1]);
    }
    for (int r = 0; r < W; ++r)   // at or below U (< L), else every key below L
      ns[r] = have >= Kc + 1 ? first_at_least(lists[r], head[r], ns[r], U + 1) : first_at_least(lists[r], head[r], ns[r], L);
    const uint64_t* res = nullptr;
    const int m = merge_tree_avx512(lists, ns, W, Kc, &res);
    std::copy(res, res + std::min(m, Kc), dst);
    if (m > Kc) *lim = res[Kc];
    return std::min(m, Kc);
  }
  for (int r = 0; r < W; ++r)   // keys below L only (ascending lists: cut each at L)
    ns[r] = (int)(std::lower_bound(lists[r], lists[r] + ns[r], L) - lists[r]);
  int m = 0;
  if (W == 1) {
    m = std::min(ns[0], Kc + 1);
    std::copy(lists[0], lists[0] + std::min(m, Kc), dst);
    if (m > Kc) *lim = lists[0][Kc];
    return std::min(m, Kc);
  }
  if (kHaveAvx512 && Kc + 1 <= MERGE_MAX_LIST) {   // two ranks: one bitonic merge
    alignas(64) uint64_t tmp[MERGE_MAX_LIST + 16];
    const int want = std::min(Kc + 1, ns[0] + ns[1]);
    m = want > 0 ? merge2_avx512(lists[0], ns[0], lists[1], ns[1], want, tmp) : 0;
    std::copy(tmp, tmp + std::min(m, Kc), dst);
    if (m > Kc) *lim = tmp[Kc];
    return std::min(m, Kc);
  }
  int hd[MERGE_MAX_WORLD] = {0};
  for (;;) {   // (no AVX-512) scalar k-way merge
    int br = -1;
    uint64_t bk = ~0ull;
    for (int r = 0; r < W; ++r)
      if (hd[r] < ns[r] && lists[r][hd[r]] < bk) {
        bk = lists[r][hd[r]];
        br = r;
      }
    if (br < 0) break;
    ++hd[br];
    if (m == Kc) {
      *lim = bk;
      return m;
    }
    dst[m++] = bk;
  }
  return m;
}

// Bytes of a rank list's slot (16-B header + keys) the merge of W ranks usually reads: the head up to
// ~2c keys (the exchange thread prefetches this much of the groups ahead, not the whole slot).
static inline size_t merge_read_bytes(int W, int Kc, size_t slot_bytes) {
  const size_t c = (size_t)(Kc + 1 + W - 1) / (size_t)W;
  return std::min(slot_bytes, W >= 3 ? 16 + 8 * (3 * c + 8) : slot_bytes);
}

}  // namespace pe
