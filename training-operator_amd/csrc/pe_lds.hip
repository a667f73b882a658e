// LDS digit-plane fit mask (gfx950): the exact fit path for batches with any number of distinct
// request values (pe_kernels.h, LdsSpec).  Two kernels per fit step:
//
//   node_ranks   per shard node and digit field: R = #{batch values <= residual} (binary search over
//                the field's sorted values), plus the folded single-value dimensions -> aux
//   fit_mask_lds one workgroup per (node block, job phase): builds the block's threshold planes in
//                LDS from the ranks, then 16 waves stream the jobs through them
//
// HBM traffic per step is the mask (written once, whole 128-B lines) plus the ranks (4 B per node
// and field, read by each of the R phases of a block) and the job codes (32 B per job, read by every
// block, mostly from L2): the same store-bound roofline as the bit-plane path.
#include "pe_kernels.h"
#include "pe_wave.h"

namespace pe {

__global__ __launch_bounds__(256) void node_ranks_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                         const uint32_t* __restrict__ labels, int64_t Ns, int64_t npad,
                                                         const LdsSpec* __restrict__ spp,
                                                         const int64_t* __restrict__ vals, uint32_t* __restrict__ ranks,
                                                         uint32_t* __restrict__ aux) {
  const LdsSpec& sp = *spp;
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= npad) return;
  const bool real = n < Ns;
  uint32_t ok = real ? 1u : 0u;
  for (int i = 0; i < sp.nfold; ++i) ok &= real && res[sp.fold_dim[i] * stride + n] >= sp.fold_val[i];
  aux[n] = ok;
  aux[npad + n] = real ? labels[n] : 0u;
  for (int f = 0; f < sp.nf; ++f) {
    uint32_t R = 0;
    if (real) {
      const int64_t x = res[sp.dim[f] * stride + n];
      const int64_t* v = vals + sp.voff[f];
      int64_t lo = 0, hi = sp.m[f];           // R = upper bound of x in v[0 .. m)
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (v[mid] <= x) lo = mid + 1;
        else hi = mid;
      }
      R = (uint32_t)lo;
    }
    ranks[f * npad + n] = R;
  }
}

hipError_t launch_node_ranks(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                             int64_t npad, const LdsSpec* spec, const int64_t* vals, uint32_t* ranks, uint32_t* aux) {
  if (npad <= 0) return hipSuccess;
  hipLaunchKernelGGL(node_ranks_kernel, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, res, stride, labels, Ns,
                     npad, spec, vals, ranks, aux);
  return hipGetLastError();
}

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

// Plane p's slice of lane `lane` (W u32 words: nodes 32 W lane .. +32 W - 1 of the block).
template <int W>
__device__ __forceinline__ typename LdVec<W>::T plane_rd(const uint32_t* lds, uint32_t p, int lane) {
  return *reinterpret_cast<const typename LdVec<W>::T*>(lds + p * (64u * W) + (uint32_t)lane * W);
}

// One workgroup = node block blk (S = 2048 W nodes) x job phase r.
//  1. zero the digit planes; scatter one equality bit per (node, field, level) into the plane of its
//     digit -- work items are (field, level, u32 word column), so no two threads write one word;
//  2. suffix OR per (field, level): GE(v) = E(v) | GE(v + 1), turning equality into threshold planes;
//     need planes by wave ballots (label test AND the folded dimensions);
//  3. waves stream jobs r + R (w + 16 t): per job the need plane AND, per field, the last level's
//     plane, then GE_k(c + 1) | (GE_k(c) & acc) per higher level; the slice is stored, its popcount
//     joins a 16-job batch that one column sum (reduce16x64) turns into 16 per-job atomics.
template <int W>
__global__ __launch_bounds__(LD_THREADS) void fit_mask_lds_kernel(const LdsSpec* __restrict__ spp,
                                                                  const uint32_t* __restrict__ ranks, int64_t npad,
                                                                  const uint32_t* __restrict__ aux, int64_t nblk,
                                                                  const uint2* __restrict__ codes, int64_t J,
                                                                  int64_t R, int64_t Tpad, int64_t pitch_bytes,
                                                                  uint8_t* __restrict__ mask,
                                                                  unsigned long long* __restrict__ counts) {
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
    for (int i = 0; i < sp.nneed; ++i) {
      const uint64_t b = __ballot(ok && (lab & sp.needs[i]) == sp.needs[i]);
      if (lane == 0) *reinterpret_cast<uint64_t*>(lds + (sp.need_pbase + i) * WPP + 2 * g) = b;
    }
  }
  __syncthreads();

  // 3. the jobs of this wave: j = r + R (wave + 16 t), t < T.  Their codes are contiguous (the t-major
  //    run of wave (r, wave), padded to 16 jobs): a 16-job batch is 512 B, one 8-B load per lane
  //    issued a batch ahead; lane 4K + i holds dwords 2i, 2i + 1 of batch job K (v_readlane).
  const int64_t j0 = r + R * wave, step = 16 * R;
  const int64_t T = j0 < J ? (J - j0 + step - 1) / step : 0;
  uint8_t* const col = mask + blk * (S / 8) + lane * (4 * W);
  const uint2* const cb = codes + (r * 16 + wave) * Tpad * (LD_CODE / 4);
  uint32_t sigma;
  {
    uint32_t probe[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) probe[k] = lane == 0 ? (uint32_t)k : 0u;
    sigma = reduce16x64(probe, lane);
  }
  const int nf = sp.nf;
  int Lf[LD_MAXF];
#pragma unroll
  for (int fi = 0; fi < LD_MAXF; ++fi) Lf[fi] = sp.L[fi];
  uint2 cv = T > 0 ? cb[lane] : make_uint2(0u, 0u);
  for (int64_t t0 = 0; t0 < T; t0 += 16) {
    const int n = (int)min<int64_t>(16, T - t0);
    const uint2 cur = cv;
    if (t0 + 16 < T) cv = cb[(t0 + 16) * (LD_CODE / 4) + lane];   // next batch, in flight meanwhile
    uint32_t p[16];
#pragma unroll
    for (int K = 0; K < 16; ++K) {
      p[K] = 0u;
      if (K < n) {
        const int64_t j = j0 + step * (t0 + K);
        auto entry = [&](int e) -> uint32_t {   // u16 entry e of job K
          const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)((e & 2) ? cur.y : cur.x), 4 * K + e / 4);
          return (e & 1) ? d >> 16 : d & 0xFFFFu;
        };
        V f = plane_rd<W>(lds, entry(LD_NEED_SLOT), lane);
#pragma unroll
        for (int fi = 0; fi < LD_MAXF; ++fi) {
          if (fi < nf) {
            V a = plane_rd<W>(lds, entry(3 * fi), lane);
#pragma unroll
            for (int k = 1; k < LD_MAXL; ++k) {
              if (k < Lf[fi]) {
                const uint32_t pi = entry(3 * fi + k);
                const V ge = plane_rd<W>(lds, pi, lane), gt = plane_rd<W>(lds, pi + 1, lane);
                a = gt | (ge & a);
              }
            }
            f &= a;
          }
        }
        *reinterpret_cast<V*>(col + j * pitch_bytes) = f;
        p[K] = popc_vec<W>(f);
      }
    }
    const uint32_t F = reduce16x64(p, lane);
    if ((lane & 3) == 0 && sigma < (uint32_t)n && F)
      atomicAdd(&counts[j0 + step * (t0 + sigma)], (unsigned long long)F);
  }
}

template <int W>
static hipError_t launch_w(hipStream_t s, size_t lds, dim3 grid, const LdsSpec* spec, const uint32_t* ranks,
                           int64_t npad, const uint32_t* aux, int64_t nblk, const uint2* codes,
                           int64_t J, int64_t R, int64_t Tpad, int64_t pitch_bytes, uint8_t* mask,
                           unsigned long long* counts) {
  hipError_t e = hipFuncSetAttribute((const void*)fit_mask_lds_kernel<W>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fit_mask_lds_kernel<W>, grid, dim3(LD_THREADS), lds, s, spec, ranks, npad, aux, nblk, codes, J,
                     R, Tpad, pitch_bytes, mask, counts);
  return hipGetLastError();
}

hipError_t launch_fit_mask_lds(hipStream_t s, int W, const LdsSpec* spec, int nplanes, const uint32_t* ranks,
                               int64_t npad, const uint32_t* aux, int64_t nblk,
                               const uint16_t* codes, int64_t J, int64_t R, int64_t Tpad, int64_t pitch_bytes,
                               uint8_t* mask, unsigned long long* counts) {
  if (J <= 0 || nblk <= 0 || R <= 0) return hipSuccess;
  const size_t lds = (size_t)nplanes * 2048 * W / 8;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(nblk * R));
  const uint2* c = reinterpret_cast<const uint2*>(codes);
  switch (W) {
    case 1: return launch_w<1>(s, lds, grid, spec, ranks, npad, aux, nblk, c, J, R, Tpad, pitch_bytes, mask, counts);
    case 2: return launch_w<2>(s, lds, grid, spec, ranks, npad, aux, nblk, c, J, R, Tpad, pitch_bytes, mask, counts);
    case 4: return launch_w<4>(s, lds, grid, spec, ranks, npad, aux, nblk, c, J, R, Tpad, pitch_bytes, mask, counts);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace pe
