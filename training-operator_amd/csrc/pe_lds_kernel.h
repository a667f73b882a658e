// The LDS digit-plane fit kernel (pe_kernels.h LdsSpec), templated on the block size W and on the
// batch's field shape: N4 fields of four digit levels, then N3 of three, N2 of two and N1 of one (the
// host orders the fields that way).  With the shape fixed at compile time a job's body is
// straight-line code -- every plane read issued first, one AND-OR per level, no branches -- so the
// scheduler can overlap consecutive jobs of the 16-job batch.  Included by pe_lds_w{1,2,4}.hip, one W
// each.  Four-level fields exist for W >= 2 only: they let a 4096-node block (one ds_read_b64 per
// plane, 256 B/clk of LDS, twice the b32 rate) hold fields that need ~130 planes each at three levels.
#pragma once
#include "pe_kernels.h"
#include "pe_wave.h"

namespace pe {

template <int W> struct LdVec;
template <> struct LdVec<1> { typedef uint32_t T; };
template <> struct LdVec<2> { typedef uint32_t T __attribute__((ext_vector_type(2))); };
template <> struct LdVec<4> { typedef uint32_t T __attribute__((ext_vector_type(4))); };

template <int W>
__device__ __forceinline__ uint32_t popc_vec(typename LdVec<W>::T v) {
  if constexpr (W == 1) return __popc(v);
  else if constexpr (W == 2) return __popc(v.x) + __popc(v.y);
  else return __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
}

// A slice as W separate u32 words and back: the AND / AND-OR combines run on plain u32 values, which
// the compiler folds into three-input v_bitop3_b32 (on the vector type it emitted one v_and / v_or per
// word and input: 61 VALU per job at W = 2 instead of ~40).
template <int W>
__device__ __forceinline__ void slice_split(typename LdVec<W>::T v, uint32_t (&o)[W]) {
  if constexpr (W == 1) o[0] = v;
  else {
#pragma unroll
    for (int i = 0; i < W; ++i) o[i] = v[i];
  }
}
template <int W>
__device__ __forceinline__ typename LdVec<W>::T slice_join(const uint32_t (&o)[W]) {
  typename LdVec<W>::T v;
  if constexpr (W == 1) v = o[0];
  else {
#pragma unroll
    for (int i = 0; i < W; ++i) v[i] = o[i];
  }
  return v;
}

// Plane p's slice of lane `lane` (W u32 words: nodes 32 W lane .. +32 W - 1 of the block).
template <int W>
__device__ __forceinline__ typename LdVec<W>::T plane_rd(const uint32_t* lds, uint32_t p, int lane) {
  return *reinterpret_cast<const typename LdVec<W>::T*>(lds + p * (64u * W) + (uint32_t)lane * W);
}

// One workgroup = node block blk (S = 2048 W nodes) x job phase r.
//  1. zero the digit planes; scatter one equality bit per (node, field, level) into the plane of its
//     digit -- work items are (field, level, u32 word column), so no two threads write one word;
//  2. suffix OR per (field, level): GE(v) = E(v) | GE(v + 1), turning equality into threshold planes;
//     need planes by wave ballots (label test AND the folded dimensions AND, per crossed single-level
//     field, the plane's threshold of it);
//  3. waves stream jobs r + R (w + 16 t): per job the need plane AND, per field, the last level's
//     plane, then GE_k(c + 1) | (GE_k(c) & acc) per higher level; the slice is stored, its popcount
//     joins a 16-job batch that one column sum (reduce16x64) turns into 16 per-job counts, added by ONE
//     atomic instruction into 16 CONSECUTIVE u32 count slots (the wave's t-major run, like its codes:
//     one 64-B request per batch instead of 16 scattered 8-B atomics -- at W = 1 those were ~12 % of
//     the kernel's HBM traffic); lds_counts_kernel maps the slots back to jobs.  Past the wave's last
//     job the batch's slices are not stored (uniform branch).
template <int W, int N4, int N3, int N2, int N1>
__global__ __launch_bounds__(LD_THREADS) void fit_mask_lds_kernel(const LdsSpec* __restrict__ spp,
                                                                  const uint32_t* __restrict__ ranks, int64_t npad,
                                                                  const uint32_t* __restrict__ aux, int64_t nblk,
                                                                  const uint2* __restrict__ codes, int64_t J,
                                                                  int64_t R, int64_t Tpad, int64_t pitch_bytes,
                                                                  uint8_t* __restrict__ mask,
                                                                  uint32_t* __restrict__ slots,
                                                                  uint32_t* __restrict__ units) {
  typedef typename LdVec<W>::T V;
  constexpr int S = 2048 * W;                 // nodes per block
  constexpr int WPP = S / 32;                 // u32 words per plane
  extern __shared__ uint32_t lds[];
  const LdsSpec& sp = *spp;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t blk = blockIdx.x % nblk, r = blockIdx.x / nblk;
  const int64_t n0 = blk * S;

  // 1. equality bits
  const int ndig = sp.need_pbase * WPP;       // digit planes occupy planes [0, need_pbase)
  for (int i = tid; i < ndig; i += LD_THREADS) lds[i] = 0u;
  __syncthreads();
  int cols = 0;                               // (field, level, word column) items
  for (int f = 0; f < sp.nf; ++f) cols += sp.L[f] * WPP;
  for (int c = tid; c < cols; c += LD_THREADS) {
    int f = 0, rest = c;
    while (rest >= sp.L[f] * WPP) rest -= sp.L[f++] * WPP;
    const int k = rest / WPP, w = rest % WPP;
    const uint32_t* rk = ranks + f * npad + n0 + 32 * w;
    const uint32_t dv = sp.div[f][k], md = sp.mod[f][k];
    const int vlo = sp.vlo[f][k], nv = sp.nv[f][k];
    uint32_t* const base = lds + sp.pbase[f][k] * WPP + w;
    for (int b = 0; b < 32; ++b) {
      uint32_t d = rk[b] / dv;
      if (md) d %= md;
      const int v = (int)d - vlo;
      if (v >= 0 && v < nv) base[v * WPP] |= 1u << b;
    }
  }
  __syncthreads();
  // 2. threshold planes, one (field, level, word) column per thread; need planes by ballots
  for (int c = tid; c < cols; c += LD_THREADS) {
    int f = 0, rest = c;
    while (rest >= sp.L[f] * WPP) rest -= sp.L[f++] * WPP;
    const int k = rest / WPP, w = rest % WPP;
    uint32_t* const base = lds + sp.pbase[f][k] * WPP + w;
    uint32_t acc = 0u;
    for (int v = sp.nv[f][k] - 1; v >= 0; --v) {
      acc |= base[v * WPP];
      base[v * WPP] = acc;
    }
  }
  for (int g = wave; g < S / 64; g += LD_THREADS / 64) {
    const int64_t n = n0 + 64 * g + lane;
    const bool ok = aux[n] != 0u;
    const uint32_t lab = aux[npad + n];
    uint32_t xr[LD_MAXF];                     // the crossed fields' ranks of this node
#pragma unroll
    for (int x = 0; x < LD_MAXF; ++x) xr[x] = x < sp.nx ? ranks[(sp.nf + x) * npad + n] : 0u;
    for (int i = 0; i < sp.nneed; ++i) {
      const bool li = ok && (lab & sp.needs[i]) == sp.needs[i];
      uint32_t dig[LD_MAXF] = {0u, 0u, 0u, 0u};   // plane (i, c)'s value index per crossed field
      for (int c = 0; c < sp.xprod; ++c) {
        bool pass = li;
#pragma unroll
        for (int x = 0; x < LD_MAXF; ++x) pass = pass && (x >= sp.nx || xr[x] > dig[x]);
        const uint64_t b = __ballot(pass);
        if (lane == 0) *reinterpret_cast<uint64_t*>(lds + (sp.need_pbase + i * sp.xprod + c) * WPP + 2 * g) = b;
        bool carry = true;                    // next c: the crossed values count up, field 0 fastest
#pragma unroll
        for (int x = 0; x < LD_MAXF; ++x)
          if (carry && x < sp.nx) {
            carry = ++dig[x] == (uint32_t)sp.m[sp.nf + x];
            if (carry) dig[x] = 0u;
          }
      }
    }
  }
  __syncthreads();

  // 3. the jobs: run (r', w') = jobs r' + R (w' + 16 t), t < T(r', w'), in 16-job batches.  A run's codes
  //    are contiguous (t-major, padded to 16 jobs): a batch is 512 B, one 8-B load per lane issued a
  //    batch ahead; lane 4K + i holds dwords 2i, 2i + 1 of batch job K (v_readlane).  units != nullptr:
  //    the block's R x 16 waves take (run, batch) units batch-major from the block's counter (the odd
  //    XCDs write slower -- pe_kernels.hip fit_mask_planes_rows_kernel), so a fast wave takes over a slow
  //    one's batches; else wave (r, wave) streams its own run.  Either way a batch lands in its run's rows
  //    and count slots.
  //    (Round-3 A/B, profiles/r10_lds_ab.txt: scalar loads of the codes instead of the readlanes were
  //    35 % slower -- they share lgkmcnt with the LDS reads -- and sorting the batch by digits so that
  //    consecutive jobs reuse plane pairs kept in VGPRs saved 3.6 % on the adversarial batch but cost
  //    7-8 % elsewhere: the sorted jobs' rows scatter the mask stores, which this job interleave keeps
  //    in one sweeping window.)
  const int64_t step = 16 * R;
  auto runT = [&](int64_t q) -> int64_t {     // jobs of run q = r' * 16 + w'
    const int64_t j0q = q / 16 + R * (q % 16);
    return j0q < J ? (J - j0q + step - 1) / step : 0;
  };
  const int64_t nq = R * 16;                  // runs
  const int64_t nbt = (runT(0) + 15) / 16;    // batches of the longest run
  const int64_t Ulast = units ? nq * nbt : (runT(r * 16 + wave) + 15) / 16;
  uint8_t* const col0 = mask + blk * (S / 8);       // this block's column of row 0 (wave-uniform)
  const uint32_t lane_off = (uint32_t)lane * (4 * W);
  uint32_t sigma;
  {
    uint32_t probe[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) probe[k] = lane == 0 ? (uint32_t)k : 0u;
    sigma = reduce16x64(probe, lane);
  }
  auto run_of = [&](int64_t u) -> int64_t { return units ? u % nq : r * 16 + wave; };
  auto batch_of = [&](int64_t u) -> int64_t { return units ? u / nq : u; };
  int64_t st = 0;
  auto grab = [&]() -> int64_t {
    if (!units) return st++;
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(units + blk, 1u);
    return (int64_t)v;                        // (lane 0's; read out where used)
  };
  auto codes_of = [&](int64_t u) -> uint2 {   // the unit's batch codes (index clamped into the padded run)
    const int64_t q = u < Ulast ? run_of(u) : 0, t0 = u < Ulast ? 16 * batch_of(u) : 0;
    return codes[q * Tpad * (LD_CODE / 4) + min<int64_t>(t0, Tpad - 16) * (LD_CODE / 4) + lane];
  };
  int64_t u0 = __builtin_amdgcn_readfirstlane((int)grab());
  int64_t u1v = grab();
  uint2 cv = codes_of(u0);
  // (wait for the first batch's codes here, once: left pending into the loop, the header would merge
  // that pending load with the latch's state and wait vmcnt(0) -- every store drained -- per batch)
  asm volatile("" : : "v"(cv.x), "v"(cv.y));
  while (u0 < Ulast) {
    const int64_t u1 = __builtin_amdgcn_readfirstlane((int)u1v);
    const int64_t u2v = grab();               // two ahead, in flight during this batch
    const int64_t q = run_of(u0), t0 = 16 * batch_of(u0), T = runT(q);
    const int64_t j0 = q / 16 + R * (q % 16);
    uint32_t* const sl = slots + q * Tpad;
    // (a 32-bit wave-uniform count: the per-job `K < n` tests of the store sizes stay scalar compares;
    // as a 64-bit value they were 15 v_cmp_gt_u64 per batch)
    const int n = __builtin_amdgcn_readfirstlane((int)max<int64_t>(0, min<int64_t>(16, T - t0)));
    const uint2 cur = cv;
    cv = codes_of(u1);                        // next batch, in flight meanwhile
    // No branch inside a batch: the stores are buffer stores whose resource holds the job's row slice,
    // with 0 bytes for a job past the run's last (the hardware drops an out-of-range store: no traffic,
    // no scratch row).  A batch is then one basic block -- job K + 1's plane reads overlap job K's
    // combines -- and the compiler's wait for the code load counts exactly the batch's 16 stores behind
    // it (with conditional stores it drained every store of the batch, vmcnt(0), once per batch).
    uint32_t p[16];
#pragma unroll
    for (int K = 0; K < 16; ++K) {
      const int64_t j = j0 + step * (t0 + K);
      auto entry = [&](int e) -> uint32_t {                           // u16 entry e of job K
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)((e & 2) ? cur.y : cur.x), 4 * K + e / 4);
        return (e & 1) ? d >> 16 : d & 0xFFFFu;
      };
      uint32_t f[W];
      slice_split<W>(plane_rd<W>(lds, entry(lds_need_slot(N4, N3, N2, N1)), lane), f);
#pragma unroll
      for (int fi = 0; fi < N4 + N3 + N2 + N1; ++fi) {          // unrolled: L and the entries are constants
        const int L = fi < N4 ? 4 : fi < N4 + N3 ? 3 : fi < N4 + N3 + N2 ? 2 : 1;
        const int o = lds_field_off(fi, N4, N3, N2);
        uint32_t a[W], g[W], h[W];
        slice_split<W>(plane_rd<W>(lds, entry(o), lane), a);
#pragma unroll
        for (int k = 1; k < L; ++k) {
          const uint32_t pk = entry(o + k);
#ifdef PE_LDS_OPAQUE_PAIR
          uint32_t ph = pk + 1;
          // W = 2: the compiler would fuse the two reads into one ds_read2st64_b64, which the LDS serves
          // at half the rate of two ds_read_b64 (8 vs 2 x 2 cycles: 128 vs 256 B/clk -- counted, the
          // fused form put the LDS array at 74 cycles per job instead of 42); an opaque index keeps them
          // apart for one extra address add
          if constexpr (W == 2) asm("" : "+s"(ph));
          slice_split<W>(plane_rd<W>(lds, pk, lane), g);
          slice_split<W>(plane_rd<W>(lds, ph, lane), h);
#else
          // W = 2: one address for the pair, GE(c + 1) read through the immediate offset (+512 B).  The
          // compiler would fuse the two reads into one ds_read2st64_b64, which the LDS serves at half
          // the rate of two ds_read_b64 (8 vs 2 x 2 cycles -- counted, the fused form put the LDS array at
          // 74 cycles per job instead of 42): a scheduling barrier that lets every instruction cross
          // (mask 0x7FF) sits between them, which the load/store merger does not merge across
          slice_split<W>(plane_rd<W>(lds, pk, lane), g);
          if constexpr (W == 2) __builtin_amdgcn_sched_barrier(0x7FF);
          slice_split<W>(plane_rd<W>(lds, pk + 1, lane), h);
#endif
#pragma unroll
          for (int i = 0; i < W; ++i) a[i] = h[i] | (g[i] & a[i]);
        }
#pragma unroll
        for (int i = 0; i < W; ++i) f[i] &= a[i];
      }
      const V fv = slice_join<W>(f);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(col0 + j * pitch_bytes), 0, K < n ? 256 * W : 0, 0x00020000);
      if constexpr (W == 1) __builtin_amdgcn_raw_buffer_store_b32(fv, rs, lane_off, 0, 0);
      else if constexpr (W == 2) __builtin_amdgcn_raw_buffer_store_b64(fv, rs, lane_off, 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(fv, rs, lane_off, 0, 0);
      p[K] = popc_vec<W>(fv);
    }
    const uint32_t F = reduce16x64(p, lane);
    if ((lane & 3) == 0 && sigma < (uint32_t)n && F) atomicAdd(&sl[t0 + sigma], F);
    u0 = u1;
    u1v = u2v;
  }
}

// Every field shape (N4, N3, N2, N1) with N4 + N3 + N2 + N1 <= LD_MAXF whose entries fit the code
// (4 N4 + 3 N3 + 2 N2 + N1 <= LD_NEED_SLOT): 35 without four-level fields, 34 with.
#define PE_LDS_SHAPES3(X, W)                                                                             \
  X(W, 0, 0, 0, 0) X(W, 0, 0, 0, 1) X(W, 0, 0, 0, 2) X(W, 0, 0, 0, 3) X(W, 0, 0, 0, 4) X(W, 0, 0, 1, 0)  \
  X(W, 0, 0, 1, 1) X(W, 0, 0, 1, 2) X(W, 0, 0, 1, 3) X(W, 0, 0, 2, 0) X(W, 0, 0, 2, 1) X(W, 0, 0, 2, 2)  \
  X(W, 0, 0, 3, 0) X(W, 0, 0, 3, 1) X(W, 0, 0, 4, 0) X(W, 0, 1, 0, 0) X(W, 0, 1, 0, 1) X(W, 0, 1, 0, 2)  \
  X(W, 0, 1, 0, 3) X(W, 0, 1, 1, 0) X(W, 0, 1, 1, 1) X(W, 0, 1, 1, 2) X(W, 0, 1, 2, 0) X(W, 0, 1, 2, 1)  \
  X(W, 0, 1, 3, 0) X(W, 0, 2, 0, 0) X(W, 0, 2, 0, 1) X(W, 0, 2, 0, 2) X(W, 0, 2, 1, 0) X(W, 0, 2, 1, 1)  \
  X(W, 0, 2, 2, 0) X(W, 0, 3, 0, 0) X(W, 0, 3, 0, 1) X(W, 0, 3, 1, 0) X(W, 0, 4, 0, 0)

#define PE_LDS_SHAPES4(X, W)                                                                             \
  X(W, 1, 0, 0, 0) X(W, 1, 0, 0, 1) X(W, 1, 0, 0, 2) X(W, 1, 0, 0, 3) X(W, 1, 0, 1, 0) X(W, 1, 0, 1, 1)  \
  X(W, 1, 0, 1, 2) X(W, 1, 0, 2, 0) X(W, 1, 0, 2, 1) X(W, 1, 0, 3, 0) X(W, 1, 1, 0, 0) X(W, 1, 1, 0, 1)  \
  X(W, 1, 1, 0, 2) X(W, 1, 1, 1, 0) X(W, 1, 1, 1, 1) X(W, 1, 1, 2, 0) X(W, 1, 2, 0, 0) X(W, 1, 2, 0, 1)  \
  X(W, 1, 2, 1, 0) X(W, 1, 3, 0, 0) X(W, 2, 0, 0, 0) X(W, 2, 0, 0, 1) X(W, 2, 0, 0, 2) X(W, 2, 0, 1, 0)  \
  X(W, 2, 0, 1, 1) X(W, 2, 0, 2, 0) X(W, 2, 1, 0, 0) X(W, 2, 1, 0, 1) X(W, 2, 1, 1, 0) X(W, 2, 2, 0, 0)  \
  X(W, 3, 0, 0, 0) X(W, 3, 0, 0, 1) X(W, 3, 0, 1, 0) X(W, 3, 1, 0, 0)

// The kernel of block size W for shape (n4, n3, n2, n1); nullptr for a shape outside the table
// (four-level shapes are built for W >= 2 only).
template <int W>
const void* lds_kernel_for(int n4, int n3, int n2, int n1) {
#define PE_LDS_PICK(W_, a, b, c, d) \
  if (n4 == a && n3 == b && n2 == c && n1 == d) return (const void*)fit_mask_lds_kernel<W_, a, b, c, d>;
  PE_LDS_SHAPES3(PE_LDS_PICK, W)
  if constexpr (W >= 2) {
    PE_LDS_SHAPES4(PE_LDS_PICK, W)
  }
#undef PE_LDS_PICK
  return nullptr;
}

const void* lds_kernel_w1(int n4, int n3, int n2, int n1);
const void* lds_kernel_w2(int n4, int n3, int n2, int n1);
const void* lds_kernel_w4(int n4, int n3, int n2, int n1);

}  // namespace pe
