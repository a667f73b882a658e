/*
 * oracle.c -- CPU restatement of the gang-placement hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline -- never as the product path.
 * The product is include/placement.h -> training-operator_amd/csrc (HIP, gfx950).
 *
 * What this restates (reference = /root/reference, Go, uncompilable here: no Go toolchain):
 *
 *  orc_pg_min_resources, mode ORC_V1:
 *      pkg/controller.v1/common/util.go:108-145 CalcPGMinResources (per-pod loop, break at
 *      podCnt >= minMember, every container's effective request, init containers ignored)
 *      pkg/controller.v1/common/util.go:79-104 AddResourceList (Requests, or Limits only when
 *      the Requests map is nil -- that choice is made by the flattener and arrives here as the
 *      container's presence bits).  Go's per-pod loop equals k_t * podvec_t because the pods of
 *      one replica type are identical; arithmetic is exact int64, overflow is FLAGGED (Go
 *      switches resource.Quantity to inf.Dec, we refuse to wrap).
 *  orc_pg_min_resources, mode ORC_V2:
 *      pkg/runtime.v2/runtime.go:115-145 NewInfo -> kueue v0.6.3 limitrange.TotalRequests
 *      (requests only; sidecars = init containers with restartPolicy Always;
 *       total = max(sum(sidecars) + sum(containers), max_i(init_i + sidecars before i)) + overhead)
 *      pkg/runtime.v2/framework/plugins/coscheduling/coscheduling.go:103-118 Build
 *      (MinMember = sum Replicas with Go int32 wrap-around, MinResources = sum Replicas*PodRequests;
 *       keys present even when Replicas == 0).
 *  orc_fit_mask / orc_place_greedy:
 *      NO reference implementation exists (placement is done by external schedulers, SURVEY.md
 *      sec. 0.2).  The rule is build-defined in SURVEY.md Appendix B and restated here:
 *      fit  = ((labels & need) == need) && for all d: req[d] <= res[d]  (signed int64)
 *      score= min(a+b+c+d, 2^40-1), a = left_cpu, b = left_mem>>20, c = left_gpu<<20,
 *             d = left_eph>>24, each term saturated at 2^40-1
 *      key  = fit ? (score << 24) | node : UINT64_MAX     (argmin => ties to lowest node id)
 *      greedy: jobs by (priority desc, index asc); groups in given order; one argmin per pod;
 *              a pod with no fitting node fails the job -> roll back all its pods.
 *              Island groups (need bit 31, Appendix B extension for BASELINE config 4): the
 *              group's pods as one unit, argmin over the key of count x request, all on that
 *              node (node label bit 31 = the node has an xGMI island).
 *      => the greedy/fit oracle is "parity unpinned" against the reference (nothing to pin to);
 *         the aggregation oracle is pinned by the reference's own test known answers
 *         (tests/golden/ fixtures, tests/test_oracle_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_D 4
#define ORC_V1 1
#define ORC_V2 2
#define SCORE_MAX ((uint64_t)0xFFFFFFFFFFull) /* 2^40 - 1 */
#define ORC_NEED_ISLAND 0x80000000u /* island group: pods co-located as one unit (placement.h) */

/* ------------------------------------------------------------------ aggregation */

static int add_ovf(int64_t a, int64_t b, int64_t* r) { return __builtin_add_overflow(a, b, r); }
static int mul_ovf(int64_t a, int64_t b, int64_t* r) { return __builtin_mul_overflow(a, b, r); }

/* container flags: bits 0-3 presence of dims, bits 4-5 kind (the four engine dimensions), or, for a
 * per-call key table (pe_pg_min_resources_keys), bits 0-15 presence of keys, bits 16-17 kind */
#define K_CONTAINER 0
#define K_INIT 1
#define K_SIDECAR 2
#define K_OVERHEAD 3
#define ORC_MAX_KEYS 16

/* (the helpers below are inlined into each entry point with its nd / fb constant, so the fixed
 * four-key call is the tight loop of the round-5 oracle, not a generic 16-key one) */
#define ORC_INLINE static inline __attribute__((always_inline))

/* flag word of container c: u8 (fixed dims) or u32 (key table) */
ORC_INLINE uint32_t flag_at(const void* fl, int fb, int32_t c) {
  return fb == 1 ? ((const uint8_t*)fl)[c] : ((const uint32_t*)fl)[c];
}

/* v1 pod vector: sum of regular containers (util.go:133-140; init containers ignored). */
ORC_INLINE int v1_pod(int32_t c0, int32_t c1, int nd, int ks, const int64_t* req, const void* fl, int fb,
                      int64_t out[ORC_MAX_KEYS], uint32_t* present) {
  int ovf = 0;
  for (int d = 0; d < nd; ++d) out[d] = 0;
  *present = 0;
  for (int32_t c = c0; c < c1; ++c) {
    const uint32_t f = flag_at(fl, fb, c);
    if (((f >> ks) & 3) != K_CONTAINER) continue;
    for (int d = 0; d < nd; ++d)
      if (f & (1u << d)) {
        ovf |= add_ovf(out[d], req[(int64_t)c * nd + d], &out[d]);
        *present |= 1u << d;
      }
  }
  return ovf;
}

/* v2 pod vector: kueue v0.6.3 limitrange.TotalRequests restated (runtime.go:134). */
ORC_INLINE int v2_pod(int32_t c0, int32_t c1, int nd, int ks, const int64_t* req, const void* fl, int fb,
                      int64_t out[ORC_MAX_KEYS], uint32_t* present) {
  int ovf = 0;
  int64_t side[ORC_MAX_KEYS], initmax[ORC_MAX_KEYS], main_[ORC_MAX_KEYS], over[ORC_MAX_KEYS];
  for (int d = 0; d < nd; ++d) side[d] = initmax[d] = main_[d] = over[d] = 0;
  *present = 0;
  for (int32_t c = c0; c < c1; ++c) {
    const uint32_t f = flag_at(fl, fb, c);
    const int kind = (f >> ks) & 3;
    for (int d = 0; d < nd; ++d) {
      if (!(f & (1u << d))) continue;
      const int64_t v = req[(int64_t)c * nd + d];
      *present |= 1u << d;
      if (kind == K_SIDECAR) ovf |= add_ovf(side[d], v, &side[d]);
      else if (kind == K_CONTAINER) ovf |= add_ovf(main_[d], v, &main_[d]);
      else if (kind == K_OVERHEAD) ovf |= add_ovf(over[d], v, &over[d]);
      else {
        int64_t u;
        ovf |= add_ovf(side[d], v, &u); /* init_i + sidecars declared before i */
        if (u > initmax[d]) initmax[d] = u;
      }
    }
  }
  for (int d = 0; d < nd; ++d) {
    int64_t t;
    ovf |= add_ovf(side[d], main_[d], &t);
    if (initmax[d] > t) t = initmax[d];
    ovf |= add_ovf(t, over[d], &out[d]);
  }
  return ovf;
}

/* nd values per container / job, flags of fb bytes with the kind at bit ks; presence out as u8 or u16 */
ORC_INLINE int pg_min_resources_nd(int32_t mode, int64_t n_jobs, int nd, int fb, const int32_t* job_group_off,
                               const int32_t* min_member, const int32_t* group_replicas,
                               const int32_t* group_cont_off, const int64_t* cont_req, const void* cont_flags,
                               int64_t* out_res, void* out_present, int32_t* out_members, uint8_t* out_overflow) {
  if (mode != ORC_V1 && mode != ORC_V2) return -1;
  const int ks = fb == 1 ? 4 : 16;
  for (int64_t j = 0; j < n_jobs; ++j) {
    int64_t acc[ORC_MAX_KEYS];
    for (int d = 0; d < nd; ++d) acc[d] = 0;
    uint32_t pres = 0;
    uint8_t ovf = 0;
    int32_t pod_cnt = 0;
    uint32_t members = 0; /* Go int32 arithmetic wraps */
    for (int32_t g = job_group_off[j]; g < job_group_off[j + 1]; ++g) {
      int64_t pod[ORC_MAX_KEYS];
      uint32_t pp;
      int64_t k;
      const int32_t r = group_replicas[g];
      if (mode == ORC_V1) {
        if (r <= 0) continue; /* Replicas == nil (util.go:129) or loop never entered */
        int64_t room = (int64_t)min_member[j] - pod_cnt;
        if (room <= 0) continue;
        k = r < room ? r : room;
        pod_cnt += (int32_t)k;
        ovf |= v1_pod(group_cont_off[g], group_cont_off[g + 1], nd, ks, cont_req, cont_flags, fb, pod, &pp);
      } else {
        members += (uint32_t)r;
        k = r;
        ovf |= v2_pod(group_cont_off[g], group_cont_off[g + 1], nd, ks, cont_req, cont_flags, fb, pod, &pp);
      }
      for (int d = 0; d < nd; ++d)
        if (pp & (1u << d)) {
          int64_t t;
          ovf |= mul_ovf(pod[d], k, &t);
          ovf |= add_ovf(acc[d], t, &acc[d]);
        }
      pres |= pp;
    }
    /* an overflowed job has no int64 answer (Go holds it in inf.Dec): values are defined as 0 */
    for (int d = 0; d < nd; ++d) out_res[j * nd + d] = ovf ? 0 : acc[d];
    if (fb == 1) ((uint8_t*)out_present)[j] = (uint8_t)pres;
    else ((uint16_t*)out_present)[j] = (uint16_t)pres;
    out_members[j] = mode == ORC_V1 ? pod_cnt : (int32_t)members;
    out_overflow[j] = ovf ? 1 : 0;
  }
  return 0;
}

int orc_pg_min_resources(int32_t mode, int64_t n_jobs, const int32_t* job_group_off,
                         const int32_t* min_member, const int32_t* group_replicas,
                         const int32_t* group_cont_off, const int64_t* cont_req,
                         const uint8_t* cont_flags, int64_t* out_res, uint8_t* out_present,
                         int32_t* out_members, uint8_t* out_overflow) {
  return pg_min_resources_nd(mode, n_jobs, ORC_D, 1, job_group_off, min_member, group_replicas, group_cont_off,
                             cont_req, cont_flags, out_res, out_present, out_members, out_overflow);
}

/* Key-table form (placement.h pe_pg_min_resources_keys): n_keys <= 16 keys of the caller's choosing,
 * each an exact int64 at the caller's per-key decimal scale; the same rule per key (util.go:80-103 and
 * coscheduling.go:112-116 sum any ResourceName). */
int orc_pg_min_resources_keys(int32_t mode, int64_t n_jobs, int32_t n_keys, const int32_t* job_group_off,
                              const int32_t* min_member, const int32_t* group_replicas,
                              const int32_t* group_cont_off, const int64_t* cont_req,
                              const uint32_t* cont_flags, int64_t* out_res, uint16_t* out_present,
                              int32_t* out_members, uint8_t* out_overflow) {
  if (n_keys < 1 || n_keys > ORC_MAX_KEYS) return -1;
  return pg_min_resources_nd(mode, n_jobs, n_keys, 4, job_group_off, min_member, group_replicas, group_cont_off,
                             cont_req, cont_flags, out_res, out_present, out_members, out_overflow);
}

/* ------------------------------------------------------------------ fit / score */

static inline int fits(const int64_t* res, int64_t N, int64_t n, uint32_t labels, const int64_t* q,
                       uint32_t need) {
  if ((labels & need) != need) return 0;
  for (int d = 0; d < ORC_D; ++d)
    if (q[d] > res[(int64_t)d * N + n]) return 0;
  return 1;
}

uint64_t orc_score(const int64_t left[ORC_D]) {
  uint64_t a = (uint64_t)left[0];
  uint64_t b = (uint64_t)left[1] >> 20;
  uint64_t c = (uint64_t)left[2] >= (1ull << 20) ? SCORE_MAX : ((uint64_t)left[2] << 20);
  uint64_t d = (uint64_t)left[3] >> 24;
  if (a > SCORE_MAX) a = SCORE_MAX;
  if (b > SCORE_MAX) b = SCORE_MAX;
  if (c > SCORE_MAX) c = SCORE_MAX;
  if (d > SCORE_MAX) d = SCORE_MAX;
  uint64_t s = a + b + c + d;
  return s > SCORE_MAX ? SCORE_MAX : s;
}

static inline uint64_t node_key(const int64_t* res, int64_t N, int64_t n, uint64_t gid, uint32_t labels,
                                const int64_t* q, uint32_t need) {
  if (!fits(res, N, n, labels, q, need)) return UINT64_MAX;
  int64_t left[ORC_D];
  for (int d = 0; d < ORC_D; ++d) left[d] = res[(int64_t)d * N + n] - q[d];
  return (orc_score(left) << 24) | gid;
}

/* Key of one node given its residual vector (used by tests to re-derive candidates). */
uint64_t orc_key(const int64_t res[ORC_D], uint32_t labels, const int64_t q[ORC_D], uint32_t need,
                 uint64_t gid) {
  return node_key(res, 1, 0, gid, labels, q, need);
}

/* J x N feasibility bitmask, row-major [J][ceil(N/64)] u64, bit n%64 of word n/64 = fit(j, n). */
int orc_fit_mask(int64_t N, const int64_t* res, const uint32_t* labels, int64_t J, const int64_t* req,
                 const uint32_t* need, uint64_t* mask, int64_t* counts, int nthreads) {
  const int64_t W = (N + 63) / 64;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t j = 0; j < J; ++j) {
    const int64_t* q = req + j * ORC_D;
    int64_t cnt = 0;
    for (int64_t w = 0; w < W; ++w) {
      uint64_t word = 0;
      const int64_t n0 = w * 64, n1 = n0 + 64 < N ? n0 + 64 : N;
      for (int64_t n = n0; n < n1; ++n) word |= (uint64_t)fits(res, N, n, labels[n], q, need[j]) << (n - n0);
      if (mask) mask[j * W + w] = word;
      cnt += __builtin_popcountll(word);
    }
    counts[j] = cnt;
  }
  return 0;
}

/* Argmin key over all nodes for one pod request (node-range parallel). */
static uint64_t argmin_key(int64_t N, const int64_t* res, const uint32_t* labels, const int64_t* q,
                           uint32_t need, int64_t id_base) {
  uint64_t best = UINT64_MAX;
#ifdef _OPENMP
#pragma omp parallel for reduction(min : best) schedule(static) if (N > 65536)
#endif
  for (int64_t n = 0; n < N; ++n) {
    uint64_t k = node_key(res, N, n, (uint64_t)(id_base + n), labels[n], q, need);
    if (k < best) best = k;
  }
  return best;
}

/* Sequential greedy best-fit gang placement (Appendix B).  res is [4][N] and is updated in place.
 * out_pod_node is indexed by (group-in-input-order) pod slots; -1 = not placed.
 * out_job_status: 0 placed, 1 unschedulable.  Returns number of jobs placed. */
int64_t orc_place_greedy(int64_t N, int64_t* res, const uint32_t* labels, int64_t J,
                         const int32_t* job_group_off, const int32_t* priority, const int32_t* group_count,
                         const int64_t* group_req, const uint32_t* group_need, int32_t* out_pod_node,
                         int32_t* out_job_status, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  const int64_t G = job_group_off[J];
  int64_t* pod_off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(G + 1));
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(J > 0 ? J : 1));
  pod_off[0] = 0;
  for (int64_t g = 0; g < G; ++g) pod_off[g + 1] = pod_off[g] + (group_count[g] > 0 ? group_count[g] : 0);
  for (int64_t i = 0; i < pod_off[G]; ++i) out_pod_node[i] = -1;
  /* stable order: priority desc, index asc (insertion into a merge-sort would do; J small enough
   * for a counting approach is not guaranteed, so use a simple stable merge sort) */
  for (int64_t j = 0; j < J; ++j) order[j] = j;
  {
    int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(J > 0 ? J : 1));
    for (int64_t width = 1; width < J; width *= 2) {
      for (int64_t lo = 0; lo < J; lo += 2 * width) {
        int64_t mid = lo + width < J ? lo + width : J, hi = lo + 2 * width < J ? lo + 2 * width : J;
        int64_t a = lo, b = mid, o = lo;
        while (a < mid && b < hi) tmp[o++] = (priority[order[b]] > priority[order[a]]) ? order[b++] : order[a++];
        while (a < mid) tmp[o++] = order[a++];
        while (b < hi) tmp[o++] = order[b++];
      }
      memcpy(order, tmp, sizeof(int64_t) * (size_t)J);
    }
    free(tmp);
  }
  int64_t placed = 0;
  for (int64_t oi = 0; oi < J; ++oi) {
    const int64_t j = order[oi];
    int ok = 1;
    for (int32_t g = job_group_off[j]; g < job_group_off[j + 1] && ok; ++g) {
      const int64_t* q = group_req + (int64_t)g * ORC_D;
      if (group_need[g] & ORC_NEED_ISLAND) {
        /* island group (placement.h PE_NEED_ISLAND): all group_count pods as one unit on the node
         * with the smallest key for count x request; a sum that overflows fits nowhere */
        int64_t qe[ORC_D];
        int ovf = 0;
        for (int d = 0; d < ORC_D; ++d) ovf |= mul_ovf(q[d], (int64_t)(group_count[g] > 0 ? group_count[g] : 0), &qe[d]);
        if (group_count[g] <= 0) continue;
        uint64_t k = ovf ? UINT64_MAX : argmin_key(N, res, labels, qe, group_need[g], 0);
        if (k == UINT64_MAX) { ok = 0; break; }
        int64_t n = (int64_t)(k & 0xFFFFFFull);
        for (int d = 0; d < ORC_D; ++d) res[(int64_t)d * N + n] -= qe[d];
        for (int32_t p = 0; p < group_count[g]; ++p) out_pod_node[pod_off[g] + p] = (int32_t)n;
        continue;
      }
      for (int32_t p = 0; p < group_count[g]; ++p) {
        uint64_t k = argmin_key(N, res, labels, q, group_need[g], 0);
        if (k == UINT64_MAX) { ok = 0; break; }
        int64_t n = (int64_t)(k & 0xFFFFFFull);
        for (int d = 0; d < ORC_D; ++d) res[(int64_t)d * N + n] -= q[d];
        out_pod_node[pod_off[g] + p] = (int32_t)n;
      }
    }
    if (!ok) { /* all-or-nothing rollback */
      for (int32_t g = job_group_off[j]; g < job_group_off[j + 1]; ++g) {
        const int64_t* q = group_req + (int64_t)g * ORC_D;
        for (int32_t p = 0; p < group_count[g]; ++p) {
          int32_t n = out_pod_node[pod_off[g] + p];
          if (n < 0) continue;
          for (int d = 0; d < ORC_D; ++d) res[(int64_t)d * N + n] += q[d];
          out_pod_node[pod_off[g] + p] = -1;
        }
      }
      out_job_status[j] = 1;
    } else {
      out_job_status[j] = 0;
      ++placed;
    }
  }
  free(pod_off);
  free(order);
  return placed;
}

/* One greedy scan window restated on the CPU (the windowed protocol's device half, SURVEY.md sec. 7
 * step 7): for each of the n_groups requests, the K smallest keys over all N nodes and the limit
 * (the (K+1)-th smallest key, UINT64_MAX when at most K nodes fit), written in the pe_resolver_*
 * blob layout of include/placement.h (16-B header {i32 n, i32 flags, u64 limit} + K 48-B records
 * {u64 key, i64 res[4], u64 labels}).  Used by bench.py's same-algorithm CPU greedy baseline and by
 * tests; groups run in parallel, each a bounded max-heap pass over the nodes. */
static void heap_sift_down(uint64_t* h, int n, int i) {
  for (;;) {
    int l = 2 * i + 1, r = l + 1, m = i;
    if (l < n && h[l] > h[m]) m = l;
    if (r < n && h[r] > h[m]) m = r;
    if (m == i) return;
    uint64_t t = h[i];
    h[i] = h[m];
    h[m] = t;
    i = m;
  }
}

static int cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

int orc_window_cands(int64_t N, const int64_t* res, const uint32_t* labels, int32_t n_groups,
                     const int64_t* group_req, const uint32_t* group_need, int32_t K, uint8_t* blob,
                     int nthreads) {
  if (K < 1) return -1;
  const size_t gbytes = 16 + (size_t)K * 48;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int32_t g = 0; g < n_groups; ++g) {
    const int64_t* q = group_req + (int64_t)g * ORC_D;
    const int cap = K + 1;
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)cap);
    int n = 0;
    for (int64_t i = 0; i < N; ++i) {
      const uint64_t k = node_key(res, N, i, (uint64_t)i, labels[i], q, group_need[g]);
      if (k == UINT64_MAX) continue;
      if (n < cap) {
        h[n++] = k;
        if (n == cap)
          for (int s = cap / 2 - 1; s >= 0; --s) heap_sift_down(h, cap, s);
      } else if (k < h[0]) {
        h[0] = k;
        heap_sift_down(h, cap, 0);
      }
    }
    qsort(h, (size_t)n, sizeof(uint64_t), cmp_u64);
    uint8_t* out = blob + (size_t)g * gbytes;
    memset(out, 0, gbytes);
    const int32_t listed = n > K ? K : n;
    const uint64_t limit = n > K ? h[K] : UINT64_MAX;
    memcpy(out, &listed, 4);
    memcpy(out + 8, &limit, 8);
    for (int32_t i = 0; i < listed; ++i) {
      uint8_t* rec = out + 16 + (size_t)i * 48;
      const int64_t node = (int64_t)(h[i] & 0xFFFFFFull);
      uint64_t lab = labels[node];
      memcpy(rec, &h[i], 8);
      for (int d = 0; d < ORC_D; ++d) memcpy(rec + 8 + 8 * d, &res[(int64_t)d * N + node], 8);
      memcpy(rec + 40, &lab, 8);
    }
    free(h);
  }
  return 0;
}

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
