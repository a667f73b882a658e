// Hand-written CDNA4 (gfx950) kernels of the gang-placement hot path.
//
//   pg_min_resources  v1 CalcPGMinResources / v2 CoScheduling.Build aggregation, one job per lane
//   fit_mask          J x N feasibility bitmask: node residuals streamed coalesced into VGPRs, the
//                     job's request is wave-uniform (scalar loads), one v_cmp per dimension turns
//                     into a 64-bit lane mask (the wave64 ballot IS the mask word)
//   scan              best-fit window scan: per lane top-2 over its nodes, wave bound, ballot
//                     compaction of the lane minima below the bound (exact per-wave candidates)
//   merge             per group: candidates below the min bound -> LDS -> bitonic sort -> top-K
//                     records (key + residual snapshot) for the host resolver
//   apply             scatter the resolver's residual updates back into the SoA
//
// Integer compare/reduce only: no MFMA (nothing is a contraction).  Roofline = HBM / VALU issue.
#include <type_traits>

#include "pe_kernels.h"
#include "pe_wave.h"

namespace pe {

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = umin64(v, __shfl_xor(v, off, 64));
  return v;
}

// ------------------------------------------------------------------ aggregation (sec. 8a a6/a10/a13)

__device__ __forceinline__ bool add_ovf(int64_t a, int64_t b, int64_t* r) { return __builtin_add_overflow(a, b, r); }
__device__ __forceinline__ bool mul_ovf(int64_t a, int64_t b, int64_t* r) { return __builtin_mul_overflow(a, b, r); }

// One job of CalcPGMinResources (V1) / CoScheduling.Build (V2): groups [g0, g1) of replicas rep[],
// containers of group g [gco[g], gco[g+1]) in req[][ND] / fl[].  Generic pointers: the segmented
// kernel runs it from LDS, the device-resident kernel from global memory.
// Key layouts (pe_kernels.h AggKeys): the fixed four engine dimensions (ND 4, u8 flags = presence bits
// 0-3 | kind << 4), or a per-call key table of up to 16 keys (ND 4 / 8 / 16, u32 flags = presence bits
// 0-15 | kind << 16; keys past the call's n_keys are never present).  Every key is summed exactly alike.
template <int ND>
struct AggJob {
  int64_t acc[ND];
  uint32_t pres, members;
  int32_t pod_cnt;
  bool ovf;
};

// Request readers: container c's value of key d.  ReqWide: the caller's int64 records; ReqNarrow: a
// narrowed segment section (pe_kernels.h agg_seg_layout), value = u32 << shift[d].
template <int ND>
struct ReqWide {
  const int64_t* p;
  __device__ __forceinline__ int64_t operator()(int64_t c, int d) const { return p[c * ND + d]; }
};
template <int ND>
struct ReqNarrow {
  const uint32_t* p;
  const uint8_t* sh;
  __device__ __forceinline__ int64_t operator()(int64_t c, int d) const {
    return (int64_t)((uint64_t)p[c * ND + d] << sh[d]);
  }
};

template <int ND, typename FT, typename RV = ReqWide<ND>>
__device__ __forceinline__ AggJob<ND> agg_job_t(int mode, int32_t mm, int32_t g0, int32_t g1, const int32_t* rep,
                                                const int32_t* gco, const RV req, const FT* fl) {
  constexpr int KS = sizeof(FT) == 1 ? 4 : 16;   // kind shift
  AggJob<ND> o;
#pragma unroll
  for (int d = 0; d < ND; ++d) o.acc[d] = 0;
  o.pres = 0;
  o.members = 0;
  o.pod_cnt = 0;
  o.ovf = false;
  for (int32_t g = g0; g < g1; ++g) {
    const int32_t r = rep[g];
    int64_t k;
    if (mode == 1) {                       // util.go:126-141: count pods until podCnt == minMember
      if (r <= 0) continue;                // Replicas == nil (-1) or an empty loop
      const int64_t room = (int64_t)mm - o.pod_cnt;
      if (room <= 0) continue;
      k = r < room ? r : room;
      o.pod_cnt += (int32_t)k;
    } else {                               // coscheduling.go:110-111: int32 members wrap like Go
      o.members += (uint32_t)r;
      k = r;
    }
    int64_t side[ND], initmax[ND], main_[ND], over[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) side[d] = initmax[d] = main_[d] = over[d] = 0;
    uint32_t pp = 0;
    for (int32_t c = gco[g]; c < gco[g + 1]; ++c) {
      const uint32_t f = fl[c];
      const uint32_t kind = (f >> KS) & 3u;
      if (mode == 1 && kind != 0) continue;  // v1 ignores init containers and overhead
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        if (!(f & (1u << d))) continue;
        const int64_t v = req(c, d);
        pp |= 1u << d;
        if (kind == 0) o.ovf |= add_ovf(main_[d], v, &main_[d]);
        else if (kind == 2) o.ovf |= add_ovf(side[d], v, &side[d]);
        else if (kind == 3) o.ovf |= add_ovf(over[d], v, &over[d]);
        else {                               // kueue: init_i + sidecars declared before it
          int64_t u;
          o.ovf |= add_ovf(side[d], v, &u);
          initmax[d] = u > initmax[d] ? u : initmax[d];
        }
      }
    }
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      if (!(pp & (1u << d))) continue;
      int64_t pod, t;
      o.ovf |= add_ovf(side[d], main_[d], &pod);          // v1: side/initmax/over are all 0
      pod = initmax[d] > pod ? initmax[d] : pod;
      o.ovf |= add_ovf(pod, over[d], &pod);
      o.ovf |= mul_ovf(pod, k, &t);
      o.ovf |= add_ovf(o.acc[d], t, &o.acc[d]);
    }
    o.pres |= pp;
  }
  return o;
}

__device__ __forceinline__ AggJob<D> agg_job(int mode, int32_t mm, int32_t g0, int32_t g1, const int32_t* rep,
                                             const int32_t* gco, const int64_t* req, const uint8_t* fl) {
  return agg_job_t<D, uint8_t>(mode, mm, g0, g1, rep, gco, ReqWide<D>{req}, fl);
}

__global__ __launch_bounds__(256) void pg_min_resources_kernel(
    int mode, int64_t n_jobs, const int32_t* __restrict__ job_group_off, const int32_t* __restrict__ min_member,
    const int32_t* __restrict__ group_replicas, const int32_t* __restrict__ group_cont_off,
    const int64_t* __restrict__ cont_req, const uint8_t* __restrict__ cont_flags, int64_t* __restrict__ out_res,
    uint8_t* __restrict__ out_present, int32_t* __restrict__ out_members, uint8_t* __restrict__ out_overflow) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_jobs) return;
  const AggJob<D> o = agg_job(mode, mode == 1 ? min_member[j] : 0, job_group_off[j], job_group_off[j + 1],
                              group_replicas, group_cont_off, cont_req, cont_flags);
#pragma unroll
  for (int d = 0; d < D; ++d) out_res[j * D + d] = o.ovf ? 0 : o.acc[d];   // no int64 answer: defined as 0
  out_present[j] = (uint8_t)o.pres;
  out_members[j] = mode == 1 ? o.pod_cnt : (int32_t)o.members;
  out_overflow[j] = o.ovf ? 1 : 0;
}

// Segmented form (pe_kernels.h AggSegHdr): block b = segment b.  The segment (<= AGG_SEG_BYTES)
// comes into LDS with one round of coalesced 16-B loads -- from pinned host memory over PCIe, so a
// one-job call costs one PCIe round trip for its inputs -- then lane t aggregates job t of the
// segment from LDS and writes its outputs into the (pinned) output buffer.
// One segment: stage [seg, seg + bytes) into LDS (8 16-B loads in flight per lane before the LDS
// stores: a 48 KB segment is 2 PCIe round trips, not 12), lane t aggregates job t from LDS and writes
// its outputs into `out`; with a flag, the last block to finish publishes the launch.
template <int ND, typename FT>
__device__ __forceinline__ void agg_segment(int mode, const uint8_t* seg, int64_t bytes, uint4* lds,
                                            uint8_t* __restrict__ out, int64_t J, uint32_t* flag, uint32_t flag_val,
                                            uint32_t* done_ctr) {
  using PT = typename std::conditional<sizeof(FT) == 1, uint8_t, uint16_t>::type;   // presence bits out
  if (bytes <= AGG_SEG_BYTES) {   // stage in LDS (else read in place: one oversized job)
    const uint4* src = reinterpret_cast<const uint4*>(seg);
    const int n16 = (int)(bytes >> 4);
    constexpr int U = 8;
    for (int i0 = 0; i0 < n16; i0 += U * AGG_SEG_JOBS) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * AGG_SEG_JOBS + threadIdx.x;
        if (i < n16) v[u] = src[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * AGG_SEG_JOBS + threadIdx.x;
        if (i < n16) lds[i] = v[u];
      }
    }
    __syncthreads();
    seg = reinterpret_cast<const uint8_t*>(lds);
  }
  const AggSegHdr h = *reinterpret_cast<const AggSegHdr*>(seg);
  const AggKeys ak{ND, (int)sizeof(FT)};
  int64_t off[7];
  agg_seg_layout(h.nj, h.ng, h.nc, mode == 1, off, ak, h.narrow != 0);
  const int t = threadIdx.x;
  if (t < h.nj) {
    const int32_t* jgo = reinterpret_cast<const int32_t*>(seg + off[0]);
    const int32_t mm = mode == 1 ? reinterpret_cast<const int32_t*>(seg + off[1])[t] : 0;
    // the offsets are the caller's (absolute): rebase the group and container sections instead
    const int32_t* rep = reinterpret_cast<const int32_t*>(seg + off[2]);
    const int32_t* gco = reinterpret_cast<const int32_t*>(seg + off[3]);
    const FT* fl = reinterpret_cast<const FT*>(seg + off[5]) - h.c0;
    const AggJob<ND> o =
        h.narrow ? agg_job_t<ND, FT>(mode, mm, jgo[t] - h.g0, jgo[t + 1] - h.g0, rep, gco,
                                     ReqNarrow<ND>{reinterpret_cast<const uint32_t*>(seg + off[4] + 16) -
                                                       (int64_t)h.c0 * ND,
                                                   seg + off[4]},
                                     fl)
                 : agg_job_t<ND, FT>(mode, mm, jgo[t] - h.g0, jgo[t + 1] - h.g0, rep, gco,
                                     ReqWide<ND>{reinterpret_cast<const int64_t*>(seg + off[4]) - (int64_t)h.c0 * ND},
                                     fl);
    int64_t oo[4];
    agg_out_layout(J, oo, ak);
    const int64_t j = h.j0 + t;
    int64_t* res = reinterpret_cast<int64_t*>(out + oo[0]) + j * ND;
#pragma unroll
    for (int d = 0; d < ND; d += 2)   // ND x 8 B per lane in 16-B stores
      reinterpret_cast<longlong2*>(res)[d / 2] = longlong2{o.ovf ? 0 : o.acc[d], o.ovf ? 0 : o.acc[d + 1]};
    reinterpret_cast<int32_t*>(out + oo[1])[j] = mode == 1 ? o.pod_cnt : (int32_t)o.members;
    reinterpret_cast<PT*>(out + oo[2])[j] = (PT)o.pres;
    out[oo[3] + j] = o.ovf ? 1 : 0;
  }
  if (flag) {   // latency launch: publish the outputs; the LAST block to finish stores the flag
    __threadfence_system();
    __syncthreads();
    if (t == 0) {
      const uint32_t nb = gridDim.x;
      const uint32_t done = nb == 1 ? 0u
                                    : __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
      if (done == nb - 1) {
        if (nb > 1) __hip_atomic_store(done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // for the next call
        __hip_atomic_store(flag, flag_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

template <int ND, typename FT>
__global__ __launch_bounds__(AGG_SEG_JOBS) void pg_agg_seg_kernel(int mode, const uint8_t* __restrict__ blob,
                                                                 const int64_t* __restrict__ seg_off, int64_t nbytes0,
                                                                 uint8_t* __restrict__ out, int64_t J, uint32_t* flag,
                                                                 uint32_t flag_val, uint32_t* done_ctr) {
  __shared__ uint4 lds[AGG_SEG_BYTES / 16];
  int64_t a = 0, e = nbytes0;
  if (seg_off) {
    a = seg_off[blockIdx.x];
    e = seg_off[blockIdx.x + 1];
  }
  agg_segment<ND, FT>(mode, blob + a, e - a, lds, out, J, flag, flag_val, done_ctr);
}

// A one-segment call of <= AGG_KARG_BYTES travels IN the kernel arguments (the blob is the first
// argument, so it sits at offset 0 of the kernarg segment): no zero-copy read of host memory, i.e.
// one PCIe round trip less on the operator's one-job call.
template <int ND, typename FT>
__global__ __launch_bounds__(AGG_SEG_JOBS) void pg_agg_karg_kernel(AggKarg blob, int mode, int64_t nbytes,
                                                                  uint8_t* __restrict__ out, int64_t J, uint32_t* flag,
                                                                  uint32_t flag_val) {
  __shared__ uint4 lds[AGG_KARG_BYTES / 16];
  const uint8_t* kp = (const uint8_t*)__builtin_amdgcn_kernarg_segment_ptr();   // (address space 4 -> generic)
  (void)blob;
  agg_segment<ND, FT>(mode, kp, nbytes, lds, out, J, flag, flag_val, nullptr);
}

// the kernel instance of a key layout: the fixed dimensions, or a key table of 4 / 8 / 16 keys
#define PE_AGG_DISPATCH(ak, KERNEL, ...)                                                                 \
  do {                                                                                                   \
    if ((ak).fb == 1 && (ak).nd == 4) hipLaunchKernelGGL((KERNEL<4, uint8_t>), __VA_ARGS__);              \
    else if ((ak).fb == 4 && (ak).nd == 4) hipLaunchKernelGGL((KERNEL<4, uint32_t>), __VA_ARGS__);        \
    else if ((ak).fb == 4 && (ak).nd == 8) hipLaunchKernelGGL((KERNEL<8, uint32_t>), __VA_ARGS__);        \
    else if ((ak).fb == 4 && (ak).nd == 16) hipLaunchKernelGGL((KERNEL<16, uint32_t>), __VA_ARGS__);      \
    else return hipErrorInvalidValue;                                                                    \
  } while (0)

hipError_t launch_pg_agg_karg(hipStream_t s, int mode, const AggKarg& blob, int64_t nbytes, uint8_t* out, int64_t J,
                              uint32_t* flag, uint32_t flag_val, AggKeys ak) {
  if (nbytes <= 0 || nbytes > AGG_KARG_BYTES || (nbytes & 15) || !flag) return hipErrorInvalidValue;
  PE_AGG_DISPATCH(ak, pg_agg_karg_kernel, dim3(1), dim3(AGG_SEG_JOBS), 0, s, blob, mode, nbytes, out, J, flag, flag_val);
  return hipGetLastError();
}

hipError_t launch_pg_agg_segments(hipStream_t s, int mode, const uint8_t* blob, const int64_t* seg_off, int64_t nseg,
                                  int64_t nbytes0, uint8_t* out, int64_t J, uint32_t* flag, uint32_t flag_val,
                                  uint32_t* done_ctr, AggKeys ak) {
  if (nseg <= 0) return hipSuccess;
  if ((!seg_off && nseg != 1) || (flag && nseg > 1 && !done_ctr)) return hipErrorInvalidValue;
  PE_AGG_DISPATCH(ak, pg_agg_seg_kernel, dim3((unsigned)nseg), dim3(AGG_SEG_JOBS), 0, s, mode, blob, seg_off, nbytes0,
                  out, J, flag, flag_val, done_ctr);
  return hipGetLastError();
}

hipError_t launch_pg_min_resources(hipStream_t s, int mode, int64_t n_jobs, const int32_t* job_group_off,
                                   const int32_t* min_member, const int32_t* group_replicas,
                                   const int32_t* group_cont_off, const int64_t* cont_req,
                                   const uint8_t* cont_flags, int64_t* out_res, uint8_t* out_present,
                                   int32_t* out_members, uint8_t* out_overflow) {
  if (n_jobs <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n_jobs + 255) / 256);
  hipLaunchKernelGGL(pg_min_resources_kernel, dim3(blocks), dim3(256), 0, s, mode, n_jobs, job_group_off,
                     min_member, group_replicas, group_cont_off, cont_req, cont_flags, out_res, out_present,
                     out_members, out_overflow);
  return hipGetLastError();
}

// ------------------------------------------------------------------ fit mask (config 5)
//
// Wave tile = FM_CH chunks of 64 nodes held in VGPRs (4 dims x int64 + labels) x FM_JT jobs.
// Per (job, chunk): 4 x v_cmp_le_i64 against SGPR requests (+ a label test only when the job
// needs labels) -> the 64-bit lane mask is the output word.  16 jobs x 4 chunks of words are
// gathered into one VGPR pair by v_writelane and leave as one 512-B store (16 rows x 32 B).
// Per-job popcounts: s_bcnt1 in SALU, accumulated lane-distributed across the wave's tiles,
// one global atomic per (job, wave).

// v_writelane_b32 with an immediate lane: the compiler's select->writelane fold hoists 64
// lane==k masks into SGPRs and spills them; the immediate form needs no mask and no SGPR.
template <int L>
__device__ __forceinline__ uint32_t writelane(uint32_t old, uint32_t uniform_val) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(uniform_val), "i"(L));
  return old;
}

template <int JJ>
__device__ __forceinline__ void wl4(int c, uint32_t& lo, uint32_t& hi, uint64_t w) {
  // c is a compile-time constant after unrolling; dispatch to the immediate-lane form
  switch (c) {
    case 0: lo = writelane<JJ * 4 + 0>(lo, (uint32_t)w); hi = writelane<JJ * 4 + 0>(hi, (uint32_t)(w >> 32)); break;
    case 1: lo = writelane<JJ * 4 + 1>(lo, (uint32_t)w); hi = writelane<JJ * 4 + 1>(hi, (uint32_t)(w >> 32)); break;
    case 2: lo = writelane<JJ * 4 + 2>(lo, (uint32_t)w); hi = writelane<JJ * 4 + 2>(hi, (uint32_t)(w >> 32)); break;
    default: lo = writelane<JJ * 4 + 3>(lo, (uint32_t)w); hi = writelane<JJ * 4 + 3>(hi, (uint32_t)(w >> 32)); break;
  }
}

template <class T> __device__ __forceinline__ T never_res();
template <> __device__ __forceinline__ int64_t never_res<int64_t>() { return NEVER; }
template <> __device__ __forceinline__ int32_t never_res<int32_t>() { return INT32_MIN; }

template <int JJ, class T, class JR>
__device__ __forceinline__ void fm_job(const JR* __restrict__ q, const T (&r)[FM_CH][D],
                                       const uint32_t (&lab)[FM_CH], uint32_t& col_lo, uint32_t& col_hi) {
  const T q0 = q->q[0], q1 = q->q[1], q2 = q->q[2], q3 = q->q[3];
  const uint32_t need = q->need;
  if (need) {
#pragma unroll
    for (int c = 0; c < FM_CH; ++c) {
      const uint64_t w = __builtin_amdgcn_ballot_w64((lab[c] & need) == need) & __builtin_amdgcn_ballot_w64(q0 <= r[c][0]) &
                         __builtin_amdgcn_ballot_w64(q1 <= r[c][1]) & __builtin_amdgcn_ballot_w64(q2 <= r[c][2]) &
                         __builtin_amdgcn_ballot_w64(q3 <= r[c][3]);
      wl4<JJ>(c, col_lo, col_hi, w);
    }
  } else {
#pragma unroll
    for (int c = 0; c < FM_CH; ++c) {
      // one ballot per compare: each folds into its v_cmp's SGPR mask, the AND runs on the SALU
      const uint64_t w = __builtin_amdgcn_ballot_w64(q0 <= r[c][0]) & __builtin_amdgcn_ballot_w64(q1 <= r[c][1]) &
                         __builtin_amdgcn_ballot_w64(q2 <= r[c][2]) & __builtin_amdgcn_ballot_w64(q3 <= r[c][3]);
      wl4<JJ>(c, col_lo, col_hi, w);
    }
  }
}

template <int JJ, class T, class JR>
__device__ __forceinline__ void fm_jobs(const JR* __restrict__ q, const T (&r)[FM_CH][D],
                                        const uint32_t (&lab)[FM_CH], uint32_t& col_lo, uint32_t& col_hi) {
  fm_job<JJ, T, JR>(q + JJ, r, lab, col_lo, col_hi);
  if constexpr (JJ + 1 < 16) fm_jobs<JJ + 1, T, JR>(q, r, lab, col_lo, col_hi);
}

// Wave tile = FM_CH chunks of 64 nodes held in VGPRs (4 dims x int64 + labels) x FM_JT jobs.
// Per (job, chunk): 4 x v_cmp_le_i64 against the job's SGPR request (+ a label test only for
// jobs that need labels); the AND of the lane masks (SALU) is the output word.  16 jobs x 4
// chunks of words are placed in one VGPR pair by v_writelane and leave as one 512-B store of
// whole 128-B lines (tile-major mask layout, pe_kernels.h).  Per-job popcounts come from the stored words (v_bcnt, 4-lane reduction,
// one permute into the lane-distributed counter) and leave with one atomic per (job, wave).
template <class T, class JR>
__global__ __launch_bounds__(256) void fit_mask_kernel(
    const T* __restrict__ res, int64_t stride, const uint32_t* __restrict__ labels, int64_t Ns, int64_t Wt,
    const JR* __restrict__ jobs, int64_t J, int64_t tiles_per_wave, uint64_t* __restrict__ mask,
    unsigned long long* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t node_base = wave_id * tiles_per_wave * (64 * FM_CH);
  if (node_base >= Ns) return;
  const int64_t j0 = (int64_t)blockIdx.y * FM_JT;
  unsigned cnt[FM_JT / 64];
#pragma unroll
  for (int kb = 0; kb < FM_JT / 64; ++kb) cnt[kb] = 0;

  for (int64_t t = 0; t < tiles_per_wave; ++t) {
    const int64_t tile0 = node_base + t * (64 * FM_CH);
    if (tile0 >= Ns) break;
    T r[FM_CH][D];
    uint32_t lab[FM_CH];
#pragma unroll
    for (int c = 0; c < FM_CH; ++c) {
      const int64_t n = tile0 + c * 64 + lane;
      const bool ok = n < Ns;
#pragma unroll
      for (int d = 0; d < D; ++d) r[c][d] = ok ? res[d * stride + n] : never_res<T>();
      lab[c] = ok ? labels[n] : 0u;
    }
    const int64_t chunk0 = tile0 >> 6;
#pragma unroll
    for (int kb = 0; kb < FM_JT / 64; ++kb) {
      for (int jg = 0; jg < 4; ++jg) {
        const int64_t jrow0 = j0 + kb * 64 + jg * 16;
        if (jrow0 >= J) break;                       // wave-uniform
        uint32_t col_lo = 0, col_hi = 0;
        fm_jobs<0, T, JR>(jobs + jrow0, r, lab, col_lo, col_hi);   // jobs padded to FM_JT on the device
        // tile-major layout: the 16 rows x 4 chunks of this collector are 512 contiguous bytes
        mask[((jrow0 >> 4) * Wt + (chunk0 >> 2)) * 64 + lane] = ((uint64_t)col_hi << 32) | col_lo;
        // popcount of this lane's word, summed over the 4 chunk lanes of each row (padding is 0)
        unsigned pc = (unsigned)(__popc(col_lo) + __popc(col_hi));
        pc += __shfl_xor(pc, 1, 64);
        pc += __shfl_xor(pc, 2, 64);
        // lane jg*16 + i of cnt[kb] counts job jrow0 + i, whose sum sits in lane 4i
        const int src = (lane & 15) * 4;
        const unsigned got = __shfl(pc, src, 64);
        if ((lane >> 4) == jg) cnt[kb] += got;
      }
    }
  }
#pragma unroll
  for (int kb = 0; kb < FM_JT / 64; ++kb) {
    const int64_t j = j0 + kb * 64 + lane;
    if (j < J && cnt[kb]) atomicAdd(&counts[j], (unsigned long long)cnt[kb]);
  }
}

hipError_t launch_fit_mask(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                           int64_t Wt, const ReqRec* jobs, int64_t J, int64_t tiles_per_wave, uint64_t* mask,
                           unsigned long long* counts) {
  if (J <= 0 || Ns <= 0) return hipSuccess;
  const int64_t span = tiles_per_wave * 64 * FM_CH;
  const int64_t waves = (Ns + span - 1) / span;
  dim3 grid((unsigned)((waves + 3) / 4), (unsigned)((J + FM_JT - 1) / FM_JT));
  hipLaunchKernelGGL((fit_mask_kernel<int64_t, ReqRec>), grid, dim3(256), 0, s, res, stride, labels, Ns, Wt, jobs, J,
                     tiles_per_wave, mask, counts);
  return hipGetLastError();
}

hipError_t launch_fit_mask32(hipStream_t s, const int32_t* res32, int64_t stride, const uint32_t* labels, int64_t Ns,
                             int64_t Wt, const ReqRec32* jobs, int64_t J, int64_t tiles_per_wave, uint64_t* mask,
                             unsigned long long* counts) {
  if (J <= 0 || Ns <= 0) return hipSuccess;
  const int64_t span = tiles_per_wave * 64 * FM_CH;
  const int64_t waves = (Ns + span - 1) / span;
  dim3 grid((unsigned)((waves + 3) / 4), (unsigned)((J + FM_JT - 1) / FM_JT));
  hipLaunchKernelGGL((fit_mask_kernel<int32_t, ReqRec32>), grid, dim3(256), 0, s, res32, stride, labels, Ns, Wt, jobs,
                     J, tiles_per_wave, mask, counts);
  return hipGetLastError();
}

struct Shift4 {
  int s[D];
};

__global__ __launch_bounds__(256) void compress_res_kernel(const int64_t* __restrict__ res, int32_t* __restrict__ res32,
                                                           int64_t stride, int64_t Ns, Shift4 sh) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= Ns) return;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int64_t v = res[d * stride + n] >> sh.s[d];          // arithmetic: floor(r / 2^s)
    res32[d * stride + n] = v < 0 ? -1 : (v > INT32_MAX ? INT32_MAX : (int32_t)v);
  }
}

hipError_t launch_compress_res(hipStream_t s, const int64_t* res, int32_t* res32, int64_t stride, int64_t Ns,
                               const int* shift) {
  if (Ns <= 0) return hipSuccess;
  Shift4 sh;
  for (int d = 0; d < D; ++d) sh.s[d] = shift[d];
  hipLaunchKernelGGL(compress_res_kernel, dim3((unsigned)((Ns + 255) / 256)), dim3(256), 0, s, res, res32, stride, Ns,
                     sh);
  return hipGetLastError();
}

// ------------------------------------------------------------------ coded fit mask (config 5)

__global__ __launch_bounds__(256) void encode_nodes_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                           const uint32_t* __restrict__ labels, int64_t Ns,
                                                           int64_t n_pad, CodeSpec spec,
                                                           const int64_t* __restrict__ vals,
                                                           const uint32_t* __restrict__ needs,
                                                           uint32_t* __restrict__ X) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_pad) return;
  if (n >= Ns) {              // padding node: every field at code 0 -> fails every job (ranks >= 1)
    X[n] = spec.therm ? 0u : spec.guard;
    return;
  }
  int code[CODE_FIELDS];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int64_t r = res[d * stride + n];
    const int64_t* v = vals + d * CODE_MAXV;
    int lo = 0, hi = spec.nvals[d];            // code = #{v <= r} (upper bound in sorted values)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (v[mid] <= r) lo = mid + 1;
      else hi = mid;
    }
    code[d] = lo;
  }
  const uint32_t lab = labels[n];
  int k = 0;                                    // needs form an inclusion chain: satisfied = prefix
  while (k < spec.nvals[4] && (needs[k] & lab) == needs[k]) ++k;
  code[4] = k;
  uint32_t x = 0;
#pragma unroll
  for (int f = 0; f < CODE_FIELDS; ++f) {
    // SWAR: code + guard bit; thermometer: code ones (job rank c fits <=> bit c-1 is set)
    const uint32_t fv = spec.therm ? (uint32_t)((1ull << code[f]) - 1) : ((uint32_t)code[f] | (1u << (spec.width[f] - 1)));
    x |= fv << spec.off[f];
  }
  X[n] = x;
}

hipError_t launch_encode_nodes(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                               int64_t n_pad, CodeSpec spec, const int64_t* vals, const uint32_t* needs, uint32_t* X) {
  if (n_pad <= 0) return hipSuccess;
  hipLaunchKernelGGL(encode_nodes_kernel, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), 0, s, res, stride, labels,
                     Ns, n_pad, spec, vals, needs, X);
  return hipGetLastError();
}

// One (job, chunk) step: tmp = (X - C) | ~M; carry = (tmp + 1 overflows) = fit for this lane;
// w = 2w + carry shifts the job's bit in, pc += popcount(carry) counts it.  The carry lives only
// inside the asm block: left to the scheduler, 16 carries (SGPR pairs) were computed ahead of their
// popcounts and spilled into VGPR lanes.  VALU->SALU SGPR reads are interlocked (no wait states).
__device__ __forceinline__ void fc_step(uint32_t x, uint32_t code, uint32_t not_guard, uint32_t& w, uint32_t& pc) {
  uint32_t tmp, t;
  uint64_t fit;
  asm("v_sub_u32_e64 %0, %5, %6\n\t"
      "v_or_b32_e32 %0, %7, %0\n\t"
      "v_add_co_u32_e64 %0, %1, %0, 1\n\t"
      "v_addc_co_u32_e64 %2, vcc, %2, %2, %1\n\t"
      "s_bcnt1_i32_b64 %4, %1\n\t"
      "s_add_u32 %3, %3, %4"
      : "=&v"(tmp), "=&s"(fit), "+v"(w), "+s"(pc), "=&s"(t)
      : "v"(x), "s"(code), "s"(not_guard)
      : "vcc", "scc");
}

// Thermometer step: tmp = X | ~Y; carry = (tmp + 1 overflows) = every field holds the job's bit.
__device__ __forceinline__ void ft_step(uint32_t x, uint32_t not_y, uint32_t& w, uint32_t& pc) {
  uint32_t tmp, t;
  uint64_t fit;
  asm("v_or_b32_e32 %0, %5, %6\n\t"
      "v_add_co_u32_e64 %0, %1, %0, 1\n\t"
      "v_addc_co_u32_e64 %2, vcc, %2, %2, %1\n\t"
      "s_bcnt1_i32_b64 %4, %1\n\t"
      "s_add_u32 %3, %3, %4"
      : "=&v"(tmp), "=&s"(fit), "+v"(w), "+s"(pc), "=&s"(t)
      : "s"(not_y), "v"(x)
      : "vcc", "scc");
}

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// 8 job codes per scalar load, issued inside the tile loop: a volatile load cannot be hoisted, so
// the 64 codes of the wave never sit in SGPRs at once (hoisting them spilled SGPRs into VGPR lanes).
__device__ __forceinline__ u32x8 load_codes8(const uint32_t* __restrict__ p) {
  u32x8 v;
  asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}

template <int THERM, int HALF, int JJ>
__device__ __forceinline__ void fc_jobs(const uint32_t* __restrict__ codes, const uint32_t (&x)[FC_CH],
                                        uint32_t not_guard, uint32_t (&w)[FC_CH], uint32_t& cnt, u32x8& c8) {
  // jobs are shifted in from the top of the half (JJ = 31 first) so job 32*HALF + jj ends in bit jj
  if constexpr (JJ % 8 == 7) c8 = load_codes8(codes + HALF * 32 + JJ - 7);
  const uint32_t code = c8[JJ % 8];
  uint32_t pc = 0;
#pragma unroll
  for (int c = 0; c < FC_CH; ++c) {
    if constexpr (THERM) ft_step(x[c], code, w[c], pc);
    else fc_step(x[c], code, not_guard, w[c], pc);
  }
  const unsigned prev = (unsigned)__builtin_amdgcn_readlane((int)cnt, HALF * 32 + JJ);
  cnt = writelane<HALF * 32 + JJ>(cnt, prev + pc);
  if constexpr (JJ > 0) fc_jobs<THERM, HALF, JJ - 1>(codes, x, not_guard, w, cnt, c8);
}

// Wave tile = FC_CH chunks x 64 nodes of code words (8 VGPRs) x FC_JT jobs whose code words are
// wave-uniform (scalar loads).  4 VALU per (job, chunk) = per 64 fit evaluations, the words leave
// as whole-line 512-B stores (bits over jobs), per-job counts are s_bcnt1 of the carry masks.
template <int THERM>
__global__ __launch_bounds__(256) void fit_mask_coded_kernel(const uint32_t* __restrict__ X, int64_t Ns,
                                                             int64_t node_stride, const uint32_t* __restrict__ jcode,
                                                             uint32_t not_guard, int64_t J, int64_t tiles_per_wave,
                                                             uint64_t* __restrict__ mask,
                                                             unsigned long long* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t node_base = wave_id * tiles_per_wave * (64 * FC_CH);
  if (node_base >= Ns) return;
  const int64_t jb = (int64_t)blockIdx.y * FC_JT;      // 64 jobs; codes padded with M (never fits)
  const int64_t ntile = min(tiles_per_wave, (Ns - node_base + 64 * FC_CH - 1) / (64 * FC_CH));
  uint32_t cnt = 0;                                    // lane i counts job jb + i
  uint64_t* row = mask + (jb >> 6) * node_stride + node_base + lane;
  for (int64_t t = 0; t < ntile; ++t) {
    uint32_t x[FC_CH];
#pragma unroll
    for (int c = 0; c < FC_CH; ++c) x[c] = X[node_base + t * (64 * FC_CH) + c * 64 + lane];   // padded
    uint32_t lo[FC_CH], hi[FC_CH];
#pragma unroll
    for (int c = 0; c < FC_CH; ++c) lo[c] = hi[c] = 0;
    u32x8 c8;
    fc_jobs<THERM, 0, 31>(jcode + jb, x, not_guard, lo, cnt, c8);
    fc_jobs<THERM, 1, 31>(jcode + jb, x, not_guard, hi, cnt, c8);
#pragma unroll
    for (int c = 0; c < FC_CH; ++c) row[t * (64 * FC_CH) + c * 64] = ((uint64_t)hi[c] << 32) | lo[c];
  }
  const int64_t j = jb + lane;
  if (j < J && cnt) atomicAdd(&counts[j], (unsigned long long)cnt);
}

hipError_t launch_fit_mask_coded(hipStream_t s, int therm, const uint32_t* X, int64_t Ns, int64_t node_stride,
                                 const uint32_t* jcode, uint32_t not_guard, int64_t J, int64_t tiles_per_wave,
                                 uint64_t* mask, unsigned long long* counts) {
  if (J <= 0 || Ns <= 0) return hipSuccess;
  const int64_t span = tiles_per_wave * 64 * FC_CH;
  const int64_t waves = (Ns + span - 1) / span;
  dim3 grid((unsigned)((waves + 3) / 4), (unsigned)((J + FC_JT - 1) / FC_JT));
  if (therm)
    hipLaunchKernelGGL(fit_mask_coded_kernel<1>, grid, dim3(256), 0, s, X, Ns, node_stride, jcode, not_guard, J,
                       tiles_per_wave, mask, counts);
  else
    hipLaunchKernelGGL(fit_mask_coded_kernel<0>, grid, dim3(256), 0, s, X, Ns, node_stride, jcode, not_guard, J,
                       tiles_per_wave, mask, counts);
  return hipGetLastError();
}

// ------------------------------------------------------------------ bit-plane fit mask

// Every plane set of a batch: the same planes as the encode above, set t = blockIdx.y (spec from
// device memory, uniform), planes of set t at planes + t * nblk * PL_MAX * 256.  One wave owns a
// segment of ES_G x 64 nodes = 2 ES_G plane words: it ballots the segment's node groups one after
// the other, parks word 2g / 2g+1 of plane p in lane 2g / 2g+1 of a per-plane VGPR (one select),
// then stores each plane's words with one contiguous 4 x 2 ES_G-byte store -- instead of a 2-lane
// 8-byte store per plane and 64 nodes (the per-set cost of that pattern was ~68 us at 1M nodes).
constexpr int ES_G = 8;                                   // node groups per wave: 16 words, 64 B
static_assert(PL_BLK % (64 * ES_G) == 0, "segments tile a block");
constexpr int64_t ES_SEGS_PER_BLK = PL_BLK / (64 * ES_G);
__device__ __forceinline__ void encode_segment(const int64_t* __restrict__ res, int64_t stride,
                                               const uint32_t* __restrict__ labels, int64_t Ns, int64_t nblk,
                                               const PlaneSpec& spec, int64_t t, int64_t seg,
                                               uint32_t* __restrict__ planes) {
  const int lane = threadIdx.x & 63;
  constexpr int64_t SEGS_PER_BLK = ES_SEGS_PER_BLK;
  const int np = spec.n;
  const int64_t blk = seg / SEGS_PER_BLK;
  const int64_t wbase = (seg % SEGS_PER_BLK) * (2 * ES_G);   // first plane word of the segment
  const int64_t nseg = blk * PL_BLK + wbase * 32;            // first node of the segment
  const uint32_t sh = (lane & 1) * 32;
  int64_t r[ES_G][D];                                       // the segment's residuals, loaded once
  uint32_t lab[ES_G];
  bool vld[ES_G];
#pragma unroll
  for (int g = 0; g < ES_G; ++g) {
    const int64_t n = nseg + g * 64 + lane;
    vld[g] = n < Ns;
#pragma unroll
    for (int d = 0; d < D; ++d) r[g][d] = vld[g] ? res[d * stride + n] : 0;
    lab[g] = vld[g] ? labels[n] : 0u;
  }
  uint32_t w[PL_MAX];
#pragma unroll
  for (int p = 0; p < PL_MAX; ++p) {                         // spec read once per plane
    w[p] = 0;
    if (p < np) {
      const int k = spec.kind[p];
      const int64_t v = spec.val[p];
#pragma unroll
      for (int g = 0; g < ES_G; ++g) {
        bool pr;                                              // k is wave-uniform: scalar branches
        switch (k) {
          case 0: pr = r[g][0] >= v; break;
          case 1: pr = r[g][1] >= v; break;
          case 2: pr = r[g][2] >= v; break;
          case 3: pr = r[g][3] >= v; break;
          default: pr = (lab[g] & (uint32_t)v) == (uint32_t)v; break;
        }
        const uint64_t b = __builtin_amdgcn_ballot_w64(vld[g] && pr);
        const uint32_t word = (uint32_t)(b >> sh);            // this lane's half of the ballot
        w[p] = (lane >> 1) == g ? word : w[p];                // lanes 2g, 2g+1 keep group g
      }
    }
  }
  if (lane < 2 * ES_G) {
    uint32_t* out = planes + (t * nblk + blk) * PL_MAX * (64 * PL_R) + wbase + lane;
#pragma unroll
    for (int p = 0; p < PL_MAX; ++p) out[p * (64 * PL_R)] = w[p];   // planes >= np stay zero
  }
}

__global__ __launch_bounds__(256) void encode_planes_sets_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                                 const uint32_t* __restrict__ labels, int64_t Ns,
                                                                 int64_t nblk, const PlaneSpec* __restrict__ specs,
                                                                 uint32_t* __restrict__ planes) {
  const int64_t seg = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (seg >= nblk * ES_SEGS_PER_BLK) return;
  encode_segment(res, stride, labels, Ns, nblk, specs[blockIdx.y], blockIdx.y, seg, planes);
}

// Single spec: one workgroup = 1024 nodes (16 waves of 64), whose 32 words per plane are parked
// in LDS by the ballots and stored as one full 128-B line per plane.  The spec's planes come
// grouped by field (dimension 0..3, then label needs), so each field is a plain loop whose plane
// value is read out of a VGPR (lane p holds plane p's value) and whose predicate is one compare:
// ~8 instructions per plane.  (The per-plane generic form -- kind selects behind branches, a scalar
// load and wait per plane, a 2-lane 8-byte store per plane and 64 nodes -- took 22 us alone and
// 31 us after the fit kernel at 1M nodes.)  Also zeroes the step's count slots (one launch fewer).
constexpr int EP_NODES = 1024;
static_assert(PL_BLK % EP_NODES == 0 && EP_NODES / 32 == 32, "a workgroup covers 32 words of every plane");
struct PlaneBounds {
  int32_t end[D + 1];   // end[f]: one past field f's last plane (end[D] = planes in use)
};
__global__ __launch_bounds__(EP_NODES) void encode_planes_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                                  const uint32_t* __restrict__ labels, int64_t Ns,
                                                                  const PlaneSpec* __restrict__ spec, PlaneBounds pb,
                                                                  uint32_t* __restrict__ planes,
                                                                  unsigned long long* __restrict__ zero,
                                                                  int64_t n_zero) {
  __shared__ uint32_t words[PL_MAX][EP_NODES / 32 + 1];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  for (int64_t i = (int64_t)blockIdx.x * EP_NODES + threadIdx.x; i < n_zero; i += (int64_t)gridDim.x * EP_NODES)
    zero[i] = 0;
  const int64_t n = (int64_t)blockIdx.x * EP_NODES + threadIdx.x;
  const bool valid = n < Ns;
  int64_t r[D];
#pragma unroll
  for (int d = 0; d < D; ++d) r[d] = valid ? res[d * stride + n] : 0;
  const uint32_t lab = valid ? labels[n] : 0u;
  const int64_t vl = lane < PL_MAX ? spec->val[lane] : 0;
  const int vlo = (int)(uint32_t)vl, vhi = (int)(uint32_t)((uint64_t)vl >> 32);
  int p = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    for (; p < pb.end[d]; ++p) {
      const int64_t v = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(vhi, p) << 32) |
                                  (uint32_t)__builtin_amdgcn_readlane(vlo, p));
      const uint64_t b = __builtin_amdgcn_ballot_w64(valid && r[d] >= v);
      if (lane < 2) words[p][2 * wv + lane] = (uint32_t)(lane ? b >> 32 : b);
    }
  }
  for (; p < pb.end[D]; ++p) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane(vlo, p);
    const uint64_t b = __builtin_amdgcn_ballot_w64(valid && (lab & v) == v);
    if (lane < 2) words[p][2 * wv + lane] = (uint32_t)(lane ? b >> 32 : b);
  }
  __syncthreads();
  const int64_t n0 = (int64_t)blockIdx.x * EP_NODES;
  const int q = threadIdx.x >> 5, w = threadIdx.x & 31;
  planes[(n0 / PL_BLK) * PL_MAX * (64 * PL_R) + q * (64 * PL_R) + (n0 % PL_BLK) / 32 + w] =
      q < pb.end[D] ? words[q][w] : 0u;
}

hipError_t launch_encode_planes_sets(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels,
                                     int64_t Ns, int64_t nblk, const PlaneSpec* specs, int nsets, uint32_t* planes) {
  if (nblk <= 0 || nsets <= 0) return hipSuccess;
  if (nsets > 65535) return hipErrorInvalidValue;
  const int64_t segs = nblk * ES_SEGS_PER_BLK;
  hipLaunchKernelGGL(encode_planes_sets_kernel, dim3((unsigned)((segs + 3) / 4), (unsigned)nsets), dim3(256), 0, s,
                     res, stride, labels, Ns, nblk, specs, planes);
  return hipGetLastError();
}

hipError_t launch_encode_planes(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels,
                                int64_t Ns, int64_t nblk, const PlaneSpec& spec, const PlaneSpec* spec_d,
                                uint32_t* planes, unsigned long long* zero, int64_t n_zero) {
  if (nblk <= 0) return hipSuccess;
  if (spec.n < 0 || spec.n > PL_MAX) return hipErrorInvalidValue;
  PlaneBounds pb{};
  for (int p = 0, f = 0; p <= spec.n; ++p) {   // fields in order 0..D, each a contiguous run
    const int k = p < spec.n ? spec.kind[p] : D + 1;
    if (k < f || k > D + 1) return hipErrorInvalidValue;
    for (; f < k && f <= D; ++f) pb.end[f] = p;
  }
  hipLaunchKernelGGL(encode_planes_kernel, dim3((unsigned)(nblk * (PL_BLK / EP_NODES))), dim3(EP_NODES), 0, s, res,
                     stride, labels, Ns, spec_d, pb, planes, zero, zero ? n_zero : 0);
  return hipGetLastError();
}

typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Sum over the 64 lanes, result wave-uniform: quad, half-row and row sums by DPP, then the rows
// by row_bcast:15 / row_bcast:31 into lane 63.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);   // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);   // row_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// v[lane] = x for one wave-uniform lane.  Data and lane select cannot both be SGPRs (one constant
// bus read), so the select goes through M0; 4 wait states after the VALU write of x.
__device__ __forceinline__ uint32_t writelane_s(uint32_t v, uint32_t x, uint32_t lane) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 3\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "s"(lane) : "m0");
  return v;
}

// Switching the indexed plane inside one gpr_idx region: PE_GPRIDX_CHAIN keeps the mode on and
// moves the index with s_set_gpr_idx_idx (one SALU instead of an off / on pair).
#ifdef PE_GPRIDX_CHAIN
#define PE_IDX_SWITCH(sel) sel "s_set_gpr_idx_idx %[t]\n\t"
#else
#define PE_IDX_SWITCH(sel) "s_set_gpr_idx_off\n\t" sel "s_set_gpr_idx_on %[t], gpr_idx(SRC0)\n\t"
#endif

// Plane registers.  Plane p = 8q + s lives in tuple q (pinned to v[32+32q : 63+32q]) at elements
// 4s..4s+3 = its 4 node words, i.e. word r of plane p is v(32 + 4p + r): one dwordx4 load per plane
// lands in place, and ONE gpr_idx region with index 4p addresses all four words (src0 = v32..v35
// + M0).  The compiler's own dynamic indexing opened a region per element (8 SALU per field).
__device__ __forceinline__ u32x32 load_planes8(const u32x4* __restrict__ p) {
  u32x32 r;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const u32x4 v = p[s * 64];
    r[4 * s] = v.x;
    r[4 * s + 1] = v.y;
    r[4 * s + 2] = v.z;
    r[4 * s + 3] = v.w;
  }
  return r;
}

// a = plane[idx4 / 4] (4 words)
__device__ __forceinline__ void plane_sel(u32x4& a, uint32_t idx4, const u32x32& A, const u32x32& B, const u32x32& C,
                                          const u32x32& Dq) {
  asm volatile("s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\t"
               "v_mov_b32_e32 %0, v32\n\tv_mov_b32_e32 %1, v33\n\tv_mov_b32_e32 %2, v34\n\tv_mov_b32_e32 %3, v35\n\t"
               "s_set_gpr_idx_off"
               : "=v"(a.x), "=v"(a.y), "=v"(a.z), "=v"(a.w)
               : "s"(idx4), "{v[32:63]}"(A), "{v[64:95]}"(B), "{v[96:127]}"(C), "{v[128:159]}"(Dq));
}

// a &= plane[idx4 / 4]
__device__ __forceinline__ void plane_and(u32x4& a, uint32_t idx4, const u32x32& A, const u32x32& B, const u32x32& C,
                                          const u32x32& Dq) {
  asm volatile("s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\t"
               "v_and_b32_e32 %0, v32, %0\n\tv_and_b32_e32 %1, v33, %1\n\tv_and_b32_e32 %2, v34, %2\n\t"
               "v_and_b32_e32 %3, v35, %3\n\ts_set_gpr_idx_off"
               : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w)
               : "s"(idx4), "{v[32:63]}"(A), "{v[64:95]}"(B), "{v[96:127]}"(C), "{v[128:159]}"(Dq));
}

// One wave = one 8192-node block (4 words x 32 nodes per lane, 32 planes in v32..v159) x a job
// range.  Per job: 5 planes selected by wave-uniform index (one gpr_idx region each, the AND folded
// into the indexed instruction: 20 VOP2 per 8192 pairs), one 16-B store per lane (1 KiB per wave,
// whole lines), the popcount summed over the wave; lane k gathers the count of the k-th job of each
// 64 and flushes them with one 64-lane atomic.  Output block-major (pe_kernels.h): the wave's
// stores form one sequential stream (1 KiB per job), which the HBM takes at ~5 TB/s where the
// same bytes scattered 1 KiB per 125 KB row ran at 3.6.
__global__ __launch_bounds__(256) void fit_mask_planes_kernel(const uint32_t* __restrict__ planes, int64_t nblk,
                                                              const uint64_t* __restrict__ jcode, int64_t J,
                                                              int64_t jobs_per_wave, uint32_t* __restrict__ mask,
                                                              unsigned long long* __restrict__ counts) {
  static_assert(PL_MAX == 32 && PL_R == 4, "register map assumes 32 planes x 4 words");
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = wave_id % nblk;
  const int64_t j0 = (wave_id / nblk) * jobs_per_wave;
  if (j0 >= J) return;
  const int64_t j1 = min(J, j0 + jobs_per_wave);
  const u32x4* pb = reinterpret_cast<const u32x4*>(planes + blk * PL_MAX * (64 * PL_R)) + lane;
  const u32x32 A = load_planes8(pb), B = load_planes8(pb + 8 * 64), C = load_planes8(pb + 16 * 64),
               Dq = load_planes8(pb + 24 * 64);
  u32x4* out = reinterpret_cast<u32x4*>(mask + blk * J * (64 * PL_R)) + lane;   // (blk, job 0, lane)
  uint32_t acc = 0;
  for (int64_t j = j0; j < j1; ++j) {
    const uint64_t c = jcode[j];                          // 5 x 7-bit fields = 4 x plane index
    u32x4 f;
    plane_sel(f, (uint32_t)c & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 7) & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 14) & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 21) & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 32) & 127, A, B, C, Dq);
    out[j * 64] = f;
    const uint32_t n = wave_sum(__popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w));
    const uint32_t k = (uint32_t)((j - j0) & 63);
    acc = writelane_s(acc, n, k);
    if (k == 63 || j + 1 == j1) {
      const int64_t jb = j - k;
      if ((uint32_t)lane <= k && acc) atomicAdd(&counts[jb + lane], (unsigned long long)acc);
      acc = 0;
    }
  }
}

typedef __attribute__((address_space(1))) u32x4 gu32x4;   // global (not flat) stores

// f = AND of the 5 planes of batch job K, whose code is lane K of (lo, hi): the code read-out and
// field extraction sit in the same asm block as the indexed ANDs, so the compiler cannot hoist 128
// readlanes of a batch into SGPRs (it did, and spilled them).  VALU -> SALU SGPR reads interlock.
template <int K>
__device__ __forceinline__ void plane_job(u32x4& f, uint32_t lo, uint32_t hi, const u32x32& A, const u32x32& B,
                                          const u32x32& C, const u32x32& Dq) {
  uint32_t c, c4, t;
  asm volatile(
      "v_readlane_b32 %[c], %[lo], %[k]\n\t"
      "v_readlane_b32 %[c4], %[hi], %[k]\n\t"
      "s_and_b32 %[t], %[c], 0x7f\n\t"
      "s_set_gpr_idx_on %[t], gpr_idx(SRC0)\n\t"
      "v_mov_b32_e32 %[f0], v32\n\tv_mov_b32_e32 %[f1], v33\n\tv_mov_b32_e32 %[f2], v34\n\tv_mov_b32_e32 %[f3], v35\n\t"
      PE_IDX_SWITCH("s_bfe_u32 %[t], %[c], 0x70007\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      PE_IDX_SWITCH("s_bfe_u32 %[t], %[c], 0x7000e\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      PE_IDX_SWITCH("s_bfe_u32 %[t], %[c], 0x70015\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      PE_IDX_SWITCH("s_and_b32 %[t], %[c4], 0x7f\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      "s_set_gpr_idx_off"
      : [f0] "=&v"(f.x), [f1] "=&v"(f.y), [f2] "=&v"(f.z), [f3] "=&v"(f.w), [c] "=&s"(c), [c4] "=&s"(c4),
        [t] "=&s"(t)
      : [lo] "v"(lo), [hi] "v"(hi), [k] "i"(K), "{v[32:63]}"(A), "{v[64:95]}"(B), "{v[96:127]}"(C),
        "{v[128:159]}"(Dq)
      : "scc");
}

// Jobs K .. 63 of a batch: select, store (row stride `step` u32x4), per-lane popcount into p[K].
// `row` is wave-uniform (kept in SGPRs by the empty asm, which also stops the compiler from
// precomputing 64 row offsets and spilling them); the store is row + lane.
template <int K>
__device__ __forceinline__ void rows_batch(uint32_t (&p)[64], uint32_t lo, uint32_t hi, const u32x32& A,
                                           const u32x32& B, const u32x32& C, const u32x32& Dq,
                                           __amdgpu_buffer_rsrc_t rs, uint32_t soff, uint32_t step,
                                           uint32_t lane_off) {
  u32x4 f;
  plane_job<K>(f, lo, hi, A, B, C, Dq);
  __builtin_amdgcn_raw_buffer_store_b128(f, rs, lane_off, soff, 0);
  p[K] = __popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w);
  if constexpr (K + 1 < 64) {
    soff += step;
    asm volatile("" : "+s"(soff));
    rows_batch<K + 1>(p, lo, hi, A, B, C, Dq, rs, soff, step, lane_off);
  }
}

// Row-major variant: the same per-job select, but the grid is ONE resident wave per SIMD
// (nblk x R waves, R job phases) and wave (blk, r) takes jobs r, r + R, r + 2R, ...  So at step i
// every wave writes into rows iR .. iR + R - 1: the chip's stores in flight cover one contiguous
// window of R x nblk KiB that sweeps the mask once, instead of ~2k independent streams (HBM takes
// the sweep at ~6.5 TB/s and the streams at ~5.3: profiles/r5_write_patterns.txt).  With one wave
// per SIMD nothing hides latency, so per 64 jobs: the codes come in one vector load issued a
// batch ahead (read out with v_readlane), and the per-job counts are one 64 x 64 column-sum
// (reduce64x64) instead of 64 dependent wave sums.  Mask layout row-major: u32 word w of row j at
// j * row_words + w, row_words = nblk * 256.
// Work units (ctr != nullptr): the waves of a block take (phase, 64-job batch) units from the
// block's counter, batch-major, instead of each working through its own phase.  The even and odd
// XCDs of a part do not write the mask at the same rate (per-wave finish times, one launch: XCDs
// 0/2/4/6 done at 1.82-1.97 ms, 1/3/5/7 at 2.20-2.31 ms), and a block's R waves sit on different
// XCDs -- so the fast ones take over the slow ones' batches and the launch ends near the mean.  The
// units in flight stay one contiguous window of rows (batch k of every phase = rows 64kR .. 64(k+1)R).
// A unit's index is fetched two batches ahead and its codes one batch ahead.
__global__ __launch_bounds__(256) void fit_mask_planes_rows_kernel(const uint32_t* __restrict__ planes, int64_t nblk,
                                                                   const uint64_t* __restrict__ jcode, int64_t J,
                                                                   int64_t R, int64_t Jr, uint32_t* __restrict__ mask,
                                                                   unsigned long long* __restrict__ counts,
                                                                   int64_t row_vec, unsigned long long* __restrict__ ctr) {
  static_assert(PL_MAX == 32 && PL_R == 4, "register map assumes 32 planes x 4 words");
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = wave_id % nblk;
  const int64_t r_own = wave_id / nblk;
  if (r_own >= R || r_own >= J) return;
  const u32x4* pb = reinterpret_cast<const u32x4*>(planes + blk * PL_MAX * (64 * PL_R)) + lane;
  const u32x32 A = load_planes8(pb), B = load_planes8(pb + 8 * 64), C = load_planes8(pb + 16 * 64),
               Dq = load_planes8(pb + 24 * 64);
  // row_vec: u32x4 per row (the pitch, >= nblk * 64)
  u32x4* const rows0 = reinterpret_cast<u32x4*>(mask) + blk * 64;   // this block's column, row 0
  u32x4* out = rows0 + lane;
  uint32_t sigma;                              // lane l of a batch sum counts batch job sigma
  {
    uint32_t probe[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) probe[k] = lane == 0 ? (uint32_t)k : 0u;
    sigma = reduce64x64(probe, lane);
  }
  const int64_t Rj = R < J ? R : J;            // phases that have jobs
  const int64_t nb = ((J + R - 1) / R + 63) / 64;   // batches of the longest phase
  const int64_t U = ctr ? Rj * nb : 0;         // units of the block (work-unit mode)
  // unit u: phase u % Rj, batch u / Rj; static mode: this wave's phase, batch by batch
  auto phase_of = [&](int64_t u) { return ctr ? u % Rj : r_own; };
  auto batch_of = [&](int64_t u) { return ctr ? u / Rj : u; };
  auto jobs_of = [&](int64_t r) { return (J - r + R - 1) / R; };
  const int64_t Ulast = ctr ? U : (jobs_of(r_own) + 63) / 64;
  auto grab = [&](int64_t& st) -> int64_t {    // static mode: the next batch; units: the counter
    if (!ctr) return st++;
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(ctr + blk, 1ull);
    return (int64_t)v;                         // (lane 0's; read out where used)
  };
  auto first = [&](int64_t v) { return (int64_t)__builtin_amdgcn_readfirstlane((int)v); };
  auto codes = [&](int64_t u) -> uint64_t {    // lane l: code of the unit's job l (0 past the end)
    if (u >= Ulast) return 0;
    const int64_t r = phase_of(u), i0 = batch_of(u) * 64;
    return i0 + lane < jobs_of(r) ? jcode[r * Jr + i0 + lane] : 0;
  };
  int64_t st = 0;
  int64_t u0 = first(grab(st));
  int64_t u1v = grab(st);                      // (the next unit: lane 0's value in flight)
  uint64_t c0 = codes(u0);
  while (u0 < Ulast) {
    const int64_t u1 = first(u1v);
    const int64_t u2v = grab(st);              // two ahead, in flight during this batch
    const uint64_t c1 = codes(u1);             // one ahead
    const int64_t r = phase_of(u0), i0 = batch_of(u0) * 64, ni = jobs_of(r);
    unsigned long long* cnt = counts + r * Jr;   // this phase's counts (the host un-permutes)
    if (i0 + 64 <= ni) {
      const uint32_t lo = (uint32_t)c0, hi = (uint32_t)(c0 >> 32);
      uint32_t p[64];
      // buffer stores: batch base in the resource, per-job advance in soffset (SALU), lane offset
      // in voffset -- no per-job VALU address arithmetic
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(rows0 + (r + i0 * R) * row_vec), 0, -1, 0x00020000);
      rows_batch<0>(p, lo, hi, A, B, C, Dq, rs, 0u, (uint32_t)(R * row_vec * 16), (uint32_t)lane * 16u);
      const uint32_t F = reduce64x64(p, lane);
      if (F) atomicAdd(&cnt[i0 + sigma], (unsigned long long)F);
    } else if (i0 < ni) {                      // a phase's last, short batch: per-job wave sums
      const uint64_t* jc = jcode + r * Jr;
      uint32_t acc = 0;
      for (int64_t i = i0; i < ni; ++i) {
        const uint64_t c = jc[i];
        u32x4 f;
        plane_sel(f, (uint32_t)c & 127, A, B, C, Dq);
        plane_and(f, (uint32_t)(c >> 7) & 127, A, B, C, Dq);
        plane_and(f, (uint32_t)(c >> 14) & 127, A, B, C, Dq);
        plane_and(f, (uint32_t)(c >> 21) & 127, A, B, C, Dq);
        plane_and(f, (uint32_t)(c >> 32) & 127, A, B, C, Dq);
        *(gu32x4*)(out + (r + i * R) * row_vec) = f;
        const uint32_t n = wave_sum(__popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w));
        acc = writelane_s(acc, n, (uint32_t)(i - i0));
      }
      if (lane < ni - i0 && acc) atomicAdd(&cnt[i0 + lane], (unsigned long long)acc);
    }
    u0 = u1;
    c0 = c1;
    u1v = u2v;
  }
}

hipError_t launch_fit_mask_planes_rows(hipStream_t s, const uint32_t* planes, int64_t nblk, const uint64_t* jcode,
                                       int64_t J, int64_t R, uint32_t* mask, unsigned long long* counts,
                                       int64_t pitch_blk, unsigned long long* unit_ctr) {
  if (J <= 0 || nblk <= 0 || R <= 0) return hipSuccess;
  if (pitch_blk < nblk) return hipErrorInvalidValue;
  const int64_t Jr = ((J + R - 1) / R + 3) / 4 * 4;   // phase stride (the engine pads codes alike)
  const int64_t waves = nblk * R;
  hipLaunchKernelGGL(fit_mask_planes_rows_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, planes, nblk,
                     jcode, J, R, Jr, mask, counts, pitch_blk * 64, unit_ctr);
  return hipGetLastError();
}

// plane_job with the job's mask row (code bits 40-63 = bits 8-31 of the high half) in an SGPR.
template <int K>
__device__ __forceinline__ void plane_job_row(u32x4& f, uint32_t& row, uint32_t lo, uint32_t hi, const u32x32& A,
                                              const u32x32& B, const u32x32& C, const u32x32& Dq) {
  uint32_t c, c4, t;
  asm volatile(
      "v_readlane_b32 %[c], %[lo], %[k]\n\t"
      "v_readlane_b32 %[c4], %[hi], %[k]\n\t"
      "s_and_b32 %[t], %[c], 0x7f\n\t"
      "s_set_gpr_idx_on %[t], gpr_idx(SRC0)\n\t"
      "v_mov_b32_e32 %[f0], v32\n\tv_mov_b32_e32 %[f1], v33\n\tv_mov_b32_e32 %[f2], v34\n\tv_mov_b32_e32 %[f3], v35\n\t"
      PE_IDX_SWITCH("s_bfe_u32 %[t], %[c], 0x70007\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      PE_IDX_SWITCH("s_bfe_u32 %[t], %[c], 0x7000e\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      PE_IDX_SWITCH("s_bfe_u32 %[t], %[c], 0x70015\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      PE_IDX_SWITCH("s_and_b32 %[t], %[c4], 0x7f\n\t")
      "v_and_b32_e32 %[f0], v32, %[f0]\n\tv_and_b32_e32 %[f1], v33, %[f1]\n\tv_and_b32_e32 %[f2], v34, %[f2]\n\tv_and_b32_e32 %[f3], v35, %[f3]\n\t"
      "s_set_gpr_idx_off\n\t"
      "s_lshr_b32 %[row], %[c4], 8"
      : [f0] "=&v"(f.x), [f1] "=&v"(f.y), [f2] "=&v"(f.z), [f3] "=&v"(f.w), [c] "=&s"(c), [c4] "=&s"(c4),
        [t] "=&s"(t), [row] "=&s"(row)
      : [lo] "v"(lo), [hi] "v"(hi), [k] "i"(K), "{v[32:63]}"(A), "{v[64:95]}"(B), "{v[96:127]}"(C),
        "{v[128:159]}"(Dq)
      : "scc");
}

// Jobs K .. 63 of a plane-set batch of n (<= 64, uniform) jobs: select, store to the job's own
// row, per-lane popcount into p[K] (0 past n).
template <int K>
__device__ __forceinline__ void sets_batch(uint32_t (&p)[64], uint32_t lo, uint32_t hi, const u32x32& A,
                                           const u32x32& B, const u32x32& C, const u32x32& Dq, u32x4* col,
                                           int64_t row_vec, int n) {
  p[K] = 0;
  if (K < n) {
    u32x4 f;
    uint32_t row;
    plane_job_row<K>(f, row, lo, hi, A, B, C, Dq);
    *(gu32x4*)(col + (int64_t)row * row_vec) = f;
    p[K] = __popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w);
  }
  if constexpr (K + 1 < 64) sets_batch<K + 1>(p, lo, hi, A, B, C, Dq, col, row_vec, n);
}

// Plane-set variant of the row sweep, every set in ONE launch: the rows kernel's grid (nblk x R
// resident waves, R common to all sets); wave (blk, r) walks the sets in turn, reloading its
// block's 32 planes of set t into the same registers, and takes set t's jobs r, r + R, ....  A
// job's mask row comes from its code (bits 40-63), so the store address is per job (row * pitch
// from SGPRs); counts per 64-job batch by the rows kernel's column sum (reduce64x64), one atomic.
// meta[t] = {first code / count slot, jobs, phase stride} of set t.
__global__ __launch_bounds__(256) void fit_mask_planes_sets_kernel(const uint32_t* __restrict__ planes, int64_t nblk,
                                                                   const uint64_t* __restrict__ jcode,
                                                                   const int64_t* __restrict__ meta, int nsets,
                                                                   int64_t R, uint32_t* __restrict__ mask,
                                                                   unsigned long long* __restrict__ counts,
                                                                   int64_t row_vec) {   // u32x4 per row (pitch)
  static_assert(PL_MAX == 32 && PL_R == 4, "register map assumes 32 planes x 4 words");
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = wave_id % nblk;
  const int64_t r = wave_id / nblk;
  if (r >= R) return;
  u32x4* const col = reinterpret_cast<u32x4*>(mask) + blk * 64 + lane;
  uint32_t sigma;                              // lane l of a batch sum counts batch job sigma
  {
    uint32_t probe[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) probe[k] = lane == 0 ? (uint32_t)k : 0u;
    sigma = reduce64x64(probe, lane);
  }
  for (int t = 0; t < nsets; ++t) {
    const int64_t off = meta[3 * t], J = meta[3 * t + 1], Jr = meta[3 * t + 2];
    if (r >= J) continue;
    const u32x4* pb = reinterpret_cast<const u32x4*>(planes + (t * nblk + blk) * PL_MAX * (64 * PL_R)) + lane;
    const u32x32 A = load_planes8(pb), B = load_planes8(pb + 8 * 64), C = load_planes8(pb + 16 * 64),
                 Dq = load_planes8(pb + 24 * 64);
    const uint64_t* jc = jcode + off + r * Jr;
    unsigned long long* cnt = counts + off + r * Jr;
    const int64_t ni = (J - r + R - 1) / R;    // jobs of this phase in set t
    for (int64_t i0 = 0; i0 < ni; i0 += 64) {
      const int n = (int)min<int64_t>(64, ni - i0);
      const uint64_t cv = lane < n ? jc[i0 + lane] : 0;   // lane l: code of batch job l
      uint32_t p[64];
      sets_batch<0>(p, (uint32_t)cv, (uint32_t)(cv >> 32), A, B, C, Dq, col, row_vec, n);
      const uint32_t F = reduce64x64(p, lane);
      if (F) atomicAdd(&cnt[i0 + sigma], (unsigned long long)F);
    }
  }
}

hipError_t launch_fit_mask_planes_sets(hipStream_t s, const uint32_t* planes, int64_t nblk, const uint64_t* jcode,
                                       const int64_t* meta, int nsets, int64_t R, uint32_t* mask,
                                       unsigned long long* counts, int64_t pitch_blk) {
  if (nblk <= 0 || R <= 0 || nsets <= 0) return hipSuccess;
  if (pitch_blk < nblk) return hipErrorInvalidValue;
  const int64_t waves = nblk * R;
  hipLaunchKernelGGL(fit_mask_planes_sets_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, planes, nblk,
                     jcode, meta, nsets, R, mask, counts, pitch_blk * 64);
  return hipGetLastError();
}

hipError_t launch_fit_mask_planes(hipStream_t s, const uint32_t* planes, int64_t nblk, const uint64_t* jcode,
                                  int64_t J, int64_t jobs_per_wave, uint32_t* mask, unsigned long long* counts) {
  if (J <= 0 || nblk <= 0) return hipSuccess;
  const int64_t waves = nblk * ((J + jobs_per_wave - 1) / jobs_per_wave);
  hipLaunchKernelGGL(fit_mask_planes_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, planes, nblk, jcode, J,
                     jobs_per_wave, mask, counts);
  return hipGetLastError();
}

// ------------------------------------------------------------------ best-fit scan (configs 2-4)

// Appendix B key: fit ? (score << 24) | gid : NO_KEY, score = min(a+b+c+d, 2^40-1) with
// a = left_cpu, b = left_mem >> 20, c = left_gpu << 20, d = left_eph >> 24, each term saturated.
__device__ __forceinline__ uint64_t node_key(int64_t r0, int64_t r1, int64_t r2, int64_t r3, uint32_t lab,
                                             int64_t q0, int64_t q1, int64_t q2, int64_t q3, uint32_t need,
                                             uint64_t gid) {
  const bool fit = ((lab & need) == need) & (q0 <= r0) & (q1 <= r1) & (q2 <= r2) & (q3 <= r3);
  const uint64_t a = (uint64_t)r0 - (uint64_t)q0;
  const uint64_t b = ((uint64_t)r1 - (uint64_t)q1) >> 20;
  const uint64_t c = (uint64_t)r2 - (uint64_t)q2;
  const uint64_t d = ((uint64_t)r3 - (uint64_t)q3) >> 24;
  const bool big = (a > SCORE_MAX) | (b > SCORE_MAX) | (c >= (1ull << 20)) | (d > SCORE_MAX);
  const uint64_t sum = a + b + (c << 20) + d;      // < 2^42 whenever !big
  const uint64_t score = (big | (sum > SCORE_MAX)) ? SCORE_MAX : sum;
  return fit ? ((score << 24) | gid) : NO_KEY;
}

// Node-only part of the Appendix-B score, kept per node for the scan:
//   S(n) = r0 + (r1 >> 20) + (r2 << 20) + (r3 >> 24),   K(n) = (S << 24) | gid.
// For a fitting request q and a node whose terms cannot saturate (r0 <= SCORE_MAX, r1 < 2^60,
// r2 < 2^20, S < SCORE_MAX) the score is exactly
//   score = S(n) - s(q) - [lo20(r1) < lo20(q1)] - [lo24(r3) < lo24(q3)]
// (floor((r - q) / 2^k) = (r >> k) - (q >> k) - borrow), so key = K(n) - (s(q) << 24) - borrows << 24.
// Nodes with a negative residual fit nothing (requests are >= 0): K = 0.  The rest: K = KEY_SLOW
// and the scan evaluates node_key() for them.
constexpr uint64_t KEY_SLOW = ~0ull;

__device__ __forceinline__ void node_prep(int64_t r0, int64_t r1, int64_t r2, int64_t r3, uint64_t gid, uint64_t& K,
                                          uint32_t& l1, uint32_t& l3) {
  l1 = (uint32_t)r1 & 0xFFFFFu;
  l3 = (uint32_t)r3 & 0xFFFFFFu;
  if ((r0 | r1 | r2 | r3) < 0) {
    K = 0;
  } else if ((uint64_t)r0 > SCORE_MAX || r1 >= (1ll << 60) || r2 >= (1ll << 20)) {
    K = KEY_SLOW;
  } else {
    const uint64_t S = (uint64_t)r0 + ((uint64_t)r1 >> 20) + ((uint64_t)r2 << 20) + ((uint64_t)r3 >> 24);
    K = S < SCORE_MAX ? (S << 24) | gid : KEY_SLOW;
  }
}

__global__ __launch_bounds__(256) void prep_nodes_kernel(const int64_t* __restrict__ res, int64_t stride, int64_t Ns,
                                                         uint64_t id_base, uint64_t* __restrict__ kn,
                                                         uint32_t* __restrict__ lo) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= stride) return;
  uint64_t K = 0;
  uint32_t l1 = 0, l3 = 0;
  if (n < Ns) node_prep(res[n], res[stride + n], res[2 * stride + n], res[3 * stride + n], id_base + (uint64_t)n, K, l1, l3);
  kn[n] = K;
  lo[n] = l1;
  lo[stride + n] = l3;
}

hipError_t launch_prep_nodes(hipStream_t s, const int64_t* res, int64_t stride, int64_t Ns, uint64_t id_base,
                             uint64_t* kn, uint32_t* lo) {
  if (stride <= 0) return hipSuccess;
  hipLaunchKernelGGL(prep_nodes_kernel, dim3((unsigned)((stride + 255) / 256)), dim3(256), 0, s, res, stride, Ns,
                     id_base, kn, lo);
  return hipGetLastError();
}

#ifndef PE_SCAN_ASM
#define PE_SCAN_ASM 1
#endif
// One group's key on the fast path, scheduled by hand: the compiler lowered the 5-way fit AND of
// groups 2.. into v_cndmask / v_bitop3 chains and put the key under an exec branch (~40 VALU per
// group and chunk).  Here: 4 x v_cmp_le_i64 + label test combined by s_and into the fit mask,
// borrow masks, K - Q - borrows << 24 in a 32-bit carry chain, NO_KEY where the mask is clear.
// 19 VALU + 4 SALU; the s_nop pairs keep 2 wait states between a VALU carry/mask write and its
// VALU read (gfx950 hazard; the compiler inserts the same).
__device__ __forceinline__ uint64_t fast_key(int64_t r0, int64_t r1, int64_t r2, int64_t r3, uint32_t lab, uint64_t K,
                                             uint32_t l1, uint32_t l3, int64_t q0, int64_t q1, int64_t q2, int64_t q3,
                                             uint32_t need, uint64_t Q, uint32_t ql1, uint32_t ql3, uint32_t c24) {
  uint32_t klo, khi, x, y;
  uint64_t f, t, b1, b3, c;
  asm volatile(
      "v_cmp_le_i64_e64 %[f], %[q0], %[r0]\n\t"
      "v_cmp_le_i64_e64 %[t], %[q1], %[r1]\n\t"
      "v_and_b32_e32 %[x], %[need], %[lab]\n\t"
      "s_and_b64 %[f], %[f], %[t]\n\t"
      "v_cmp_le_i64_e64 %[t], %[q2], %[r2]\n\t"
      "v_cmp_lt_u32_e64 %[b1], %[l1], %[ql1]\n\t"
      "s_and_b64 %[f], %[f], %[t]\n\t"
      "v_cmp_le_i64_e64 %[t], %[q3], %[r3]\n\t"
      "v_cmp_lt_u32_e64 %[b3], %[l3], %[ql3]\n\t"
      "s_and_b64 %[f], %[f], %[t]\n\t"
      "v_cmp_eq_u32_e64 %[t], %[need], %[x]\n\t"
      "v_sub_co_u32_e64 %[klo], %[c], %[Klo], %[Qlo]\n\t"
      "s_and_b64 %[f], %[f], %[t]\n\t"
      "v_cndmask_b32_e64 %[x], 0, %[c24], %[b1]\n\t"
      "v_cndmask_b32_e64 %[y], 0, %[c24], %[b3]\n\t"
      "v_subb_co_u32_e64 %[khi], %[c], %[Khi], %[Qhi], %[c]\n\t"
      "v_add_u32_e32 %[x], %[x], %[y]\n\t"
      "s_nop 1\n\t"
      "v_sub_co_u32_e64 %[klo], %[c], %[klo], %[x]\n\t"
      "s_nop 1\n\t"
      "v_subbrev_co_u32_e64 %[khi], %[c], 0, %[khi], %[c]\n\t"
      "v_cndmask_b32_e64 %[klo], -1, %[klo], %[f]\n\t"
      "v_cndmask_b32_e64 %[khi], -1, %[khi], %[f]"
      : [klo] "=&v"(klo), [khi] "=&v"(khi), [x] "=&v"(x), [y] "=&v"(y), [f] "=&s"(f), [t] "=&s"(t), [b1] "=&s"(b1),
        [b3] "=&s"(b3), [c] "=&s"(c)
      : [r0] "v"(r0), [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [lab] "v"(lab), [Klo] "v"((uint32_t)K),
        [Khi] "v"((uint32_t)(K >> 32)), [l1] "v"(l1), [l3] "v"(l3), [q0] "s"(q0), [q1] "s"(q1), [q2] "s"(q2),
        [q3] "s"(q3), [need] "s"(need), [Qlo] "v"((uint32_t)Q), [Qhi] "v"((uint32_t)(Q >> 32)), [ql1] "v"(ql1),
        [ql3] "v"(ql3), [c24] "v"(c24)
      : "scc");
  return ((uint64_t)khi << 32) | klo;
}

// Grid: one block per 1024-node span (SC_WPB waves), wave w of the block takes group tile
// blockIdx.y * SC_WPB + w.  All waves of a block read the same node chunks at about the same
// time, so the node data comes from HBM once per window and the re-reads for the other group
// tiles hit the CU's L1 (a grid of spans x tiles re-read it from MALL once per tile).
__global__ __launch_bounds__(64 * SC_WPB) void scan_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                   const uint32_t* __restrict__ labels, const uint64_t* __restrict__ kn,
                                                   const uint32_t* __restrict__ lo, int64_t Ns, uint64_t id_base,
                                                   const ReqRec* __restrict__ groups, int Wg,
                                                   uint64_t* __restrict__ cand, int32_t* __restrict__ cnt,
                                                   uint64_t* __restrict__ bound, int nwaves) {
  const int lane = threadIdx.x & 63;
  const int wave_id = blockIdx.x;                                              // node span
  const int g0 = (blockIdx.y * SC_WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * SC_GT;
  if (g0 >= Wg) return;
  int64_t q[SC_GT][D];
  uint32_t need[SC_GT], ql1[SC_GT], ql3[SC_GT];
  uint64_t Q[SC_GT];
#pragma unroll
  for (int g = 0; g < SC_GT; ++g) {                // groups padded to SC_GT on the device
    const ReqRec& gr = groups[g0 + g];
#pragma unroll
    for (int d = 0; d < D; ++d) q[g][d] = gr.q[d];
    need[g] = gr.need;
    ql1[g] = (uint32_t)q[g][1] & 0xFFFFFu;
    ql3[g] = (uint32_t)q[g][3] & 0xFFFFFFu;
    // s(q) << 24 with the terms clamped where no fast-path node can fit anyway (r0 <= SCORE_MAX,
    // r1 < 2^60, r2 < 2^20 for every K(n) != KEY_SLOW)
    const uint64_t t0 = (uint64_t)q[g][0] > SCORE_MAX ? SCORE_MAX : (uint64_t)q[g][0];
    const uint64_t t1 = (uint64_t)q[g][1] >> 20;
    const uint64_t t2 = (uint64_t)q[g][2] >= (1ull << 20) ? (1ull << 20) : (uint64_t)q[g][2];
    Q[g] = (t0 + (t1 > SCORE_MAX ? SCORE_MAX : t1) + (t2 << 20) + ((uint64_t)q[g][3] >> 24)) << 24;
    // wave-uniform, but kept in VGPRs: the group requests (q, need) already take most of the SGPR
    // budget, and scalar spills inside the node loop cost more than VGPR operands
    asm volatile("" : "+v"(Q[g]), "+v"(ql1[g]), "+v"(ql3[g]));
  }
  uint64_t m[SC_GT], s2[SC_GT];
#pragma unroll
  for (int g = 0; g < SC_GT; ++g) m[g] = s2[g] = NO_KEY;
  uint32_t c24 = 1u << 24;                          // a VGPR operand (one SGPR per VALU op)
  asm volatile("" : "+v"(c24));
  const int64_t base = (int64_t)wave_id * SC_SPAN;
  // stride is a multiple of 64, so a 64-node chunk is wholly inside [0, stride) or wholly past it:
  // a wave-uniform bound, no per-lane masks.  Nodes in [Ns, stride) are padding (residual NEVER,
  // K = 0): they fit nothing.
  const int nchunk = (int)min((int64_t)SC_M, (stride - base) / 64);
  // chunk i+1's node data is loaded while chunk i is scored (the loads' latency was exposed)
  struct Chunk {
    int64_t r0, r1, r2, r3;
    uint64_t K;
    uint32_t lab, l1, l3;
  };
  auto load_chunk = [&](int i) {
    const int64_t n = base + i * 64 + lane;
    return Chunk{res[n], res[stride + n], res[2 * stride + n], res[3 * stride + n], kn[n], labels[n], lo[n],
                 lo[stride + n]};
  };
  Chunk nxt = nchunk > 0 ? load_chunk(0) : Chunk{};
  for (int i = 0; i < nchunk; ++i) {
    const Chunk c = nxt;
    if (i + 1 < nchunk) nxt = load_chunk(i + 1);
    const int64_t n = base + i * 64 + lane;
    const int64_t r0 = c.r0, r1 = c.r1, r2 = c.r2, r3 = c.r3;
    const uint32_t lab = c.lab;
    const uint64_t K = c.K;
    const uint32_t l1 = c.l1, l3 = c.l3;
    const uint64_t gid = id_base + (uint64_t)n;
    if (__builtin_expect(__ballot(K == KEY_SLOW) == 0, 1)) {   // wave-uniform: no saturating node here
#pragma unroll
      for (int g = 0; g < SC_GT; ++g) {
#if PE_SCAN_ASM
        const uint64_t k = fast_key(r0, r1, r2, r3, lab, K, l1, l3, q[g][0], q[g][1], q[g][2], q[g][3], need[g], Q[g],
                                    ql1[g], ql3[g], c24);
#else
        const bool fit = ((lab & need[g]) == need[g]) & (q[g][0] <= r0) & (q[g][1] <= r1) & (q[g][2] <= r2) &
                         (q[g][3] <= r3);
        const uint64_t borrow = ((uint64_t)(l1 < ql1[g]) + (uint64_t)(l3 < ql3[g])) << 24;
        const uint64_t k = fit ? K - Q[g] - borrow : NO_KEY;
#endif
        const bool lt_m = k < m[g];
        const bool lt_s = k < s2[g];
        s2[g] = lt_m ? m[g] : (lt_s ? k : s2[g]);
        m[g] = lt_m ? k : m[g];
      }
    } else {
      const bool slow = K == KEY_SLOW;
#pragma unroll
      for (int g = 0; g < SC_GT; ++g) {
        const bool fit = ((lab & need[g]) == need[g]) & (q[g][0] <= r0) & (q[g][1] <= r1) & (q[g][2] <= r2) &
                         (q[g][3] <= r3);
        const uint64_t borrow = ((uint64_t)(l1 < ql1[g]) + (uint64_t)(l3 < ql3[g])) << 24;
        const uint64_t k = !fit ? NO_KEY
                           : slow ? node_key(r0, r1, r2, r3, lab, q[g][0], q[g][1], q[g][2], q[g][3], need[g], gid)
                                  : K - Q[g] - borrow;
        const bool lt_m = k < m[g];
        const bool lt_s = k < s2[g];
        s2[g] = lt_m ? m[g] : (lt_s ? k : s2[g]);
        m[g] = lt_m ? k : m[g];
      }
    }
  }
#pragma unroll
  for (int g = 0; g < SC_GT; ++g) {
    if (g0 + g >= Wg) break;
    const uint64_t B = wave_min_u64(s2[g]);        // every key < B in this wave is some lane's minimum
    const bool take = m[g] < B;
    const uint64_t bal = __ballot(take);
    const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
    const size_t slot = (size_t)(g0 + g) * (size_t)nwaves + (size_t)wave_id;
    if (take) cand[slot * 64 + pos] = m[g];
    if (lane == 0) {
      cnt[slot] = __popcll(bal);
      bound[slot] = B;
    }
  }
}

hipError_t launch_scan(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, const uint64_t* kn,
                       const uint32_t* lo, int64_t Ns, uint64_t id_base, const ReqRec* groups, int Wg, uint64_t* cand,
                       int32_t* cnt, uint64_t* bound, int nwaves) {
  if (Wg <= 0 || nwaves <= 0) return hipSuccess;
  const int tiles = (Wg + SC_GT - 1) / SC_GT;
  dim3 grid((unsigned)nwaves, (unsigned)((tiles + SC_WPB - 1) / SC_WPB));
  hipLaunchKernelGGL(scan_kernel, grid, dim3(64 * SC_WPB), 0, s, res, stride, labels, kn, lo, Ns, id_base, groups, Wg,
                     cand, cnt, bound, nwaves);
  return hipGetLastError();
}

// ------------------------------------------------------------------ merge: per-group exact top-K

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = umax64(v, __shfl_xor(v, off, 64));
  return v;
}

// LDS working set of one top-K block (merge or walk), MG_THREADS threads.
struct TopkShared {
  uint64_t keys[MG_CAP];
  uint64_t sel[MG_SEL];
  uint64_t red[2 * (MG_THREADS / 64)];
  int hist[256];
  int total, sel_n, sel_bin;
  int sel_c;   // topk_sort's one-level gather count (zeroed with the histogram, no barrier pair of its own)
};

// Wave-aggregated append of the lanes' keys with `take` to s.keys: one LDS atomic per wave
// (ballot / mbcnt ranks).  Keys past MG_CAP are counted in s.total but dropped.
__device__ __forceinline__ void topk_append(TopkShared& s, uint64_t k, bool take) {
  const uint64_t bal = __ballot(take);
  if (bal == 0) return;
  const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
  int base = 0;
  if (take && rank == 0) base = atomicAdd(&s.total, __popcll(bal));
  base = __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
  if (take && base + rank < MG_CAP) s.keys[base + rank] = k;
}

// Histogram add, wave-wide (every lane calls it; b < 0: nothing to count): each run of consecutive
// lanes with the same bin adds its length with one LDS atomic from its first lane.
__device__ __forceinline__ void hist_add_runs(int* hist, int b, int lane) {
  const int bp = __shfl_up(b, 1, 64);
  const bool edge = lane == 0 || bp != b;
  const uint64_t bal = __ballot(edge);
  const uint64_t above = lane == 63 ? 0ull : bal & (~0ull << (lane + 1));   // run ends at the next edge
  const int next = above ? __ffsll((unsigned long long)above) - 1 : 64;
  if (edge && b >= 0) atomicAdd(&hist[b], next - lane);
}

// 256-bin histogram cut (block-wide, wave 0 scans): with s.hist filled, the first bin whose
// inclusive count reaches `need` (255 if none) -> s.sel_bin, and the count of the bins before it
// -> s.sel_n.  Ends with a barrier.
__device__ void hist_cut(TopkShared& s, int need) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 64) {                          // inclusive scan of 256 bins, 4 per lane
    int h[4], sum = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      h[u] = s.hist[lane * 4 + u];
      sum += h[u];
    }
    int incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    int run = incl - sum, cut = 1 << 30, before = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (run + h[u] >= need && cut == (1 << 30)) {
        cut = lane * 4 + u;
        before = run;
      }
      run += h[u];
    }
    const uint64_t bal = __ballot(cut != (1 << 30));   // first lane holding a cut bin
    const int first = __ffsll((unsigned long long)bal) - 1;
    const int cb = __shfl(cut, first < 0 ? 0 : first, 64);
    const int bf = __shfl(before, first < 0 ? 0 : first, 64);
    if (lane == 0) {
      s.sel_bin = first < 0 ? 255 : cb;
      s.sel_n = first < 0 ? incl : bf;   // (no cut: every key counted, the bin is the last)
    }
  }
  __syncthreads();
}

// Block-wide: the K + 1 smallest of s.keys[0..T) (or all T if fewer), ascending, at the front of
// the returned array.  Only the K + 1 smallest matter (K records + the limit).  For T > 2(K+1):
// a 256-bin histogram of (key - min) >> shift over [min, max] finds the bin holding the (K+1)-th
// smallest, a second 256-bin histogram inside that bin narrows it, and the C keys up to the
// narrowed cut (C ~ K + 1 + a sub-bin) are placed by rank -- each thread counts the selected keys
// below its own (keys are unique: the node id is in the low bits) -- instead of a bitonic sort
// with ~50 block barriers.  T <= 2(K+1) keys are rank-placed directly; a cut that still holds
// > MG_SEL keys falls back to the bitonic sort of all T.  T <= MG_CAP.  Starts and ends with a
// block barrier.
// Rank placement: the C unique keys of s.sel, each thread t < C counts the keys below its own and
// writes it to s.keys[rank] if rank <= K.  The count loop reads 16 keys per step (every lane the same
// address: LDS broadcast) before comparing, so 16 reads are in flight instead of one read latency per
// key (the one-at-a-time loop was ~11 us of the walk's ~30 us per group at C ~ 300).
// P threads per key when C x P fits the block (P = 2..16, lanes of one wave): each counts a 1/P slice
// of the keys, the slices' counts are summed by lane shuffles -- the count loop is P times shorter
// (C ~ 240 -> 4 threads per key).  PE_RANK_ONE=1 at build time: one thread per key (A/B).
__device__ __forceinline__ void rank_place(TopkShared& s, int C, int K) {
#ifndef PE_RANK_ONE
  int P = 1;   // (block-uniform)
  while (P < 16 && C * (P * 2) <= MG_THREADS) P *= 2;
  if (P > 1) {
    const int t = threadIdx.x / P, part = threadIdx.x & (P - 1);
    const bool live = t < C;
    const uint64_t k = live ? s.sel[t] : 0;
    const int j0 = (int)((int64_t)C * part / P), j1 = (int)((int64_t)C * (part + 1) / P);
    int rank = 0, j = j0;
    if (live) {
      for (; j + 8 <= j1; j += 8) {
        uint64_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = s.sel[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) rank += v[u] < k;
      }
      for (; j < j1; ++j) rank += s.sel[j] < k;
    }
    for (int off = P >> 1; off >= 1; off >>= 1) rank += __shfl_xor(rank, off, 64);
    if (live && part == 0 && rank <= K) s.keys[rank] = k;
    return;
  }
#endif
  for (int t = threadIdx.x; t < C; t += MG_THREADS) {
    const uint64_t k = s.sel[t];
    int rank = 0, j = 0;
    for (; j + 16 <= C; j += 16) {
      uint64_t v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = s.sel[j + u];
#pragma unroll
      for (int u = 0; u < 16; ++u) rank += v[u] < k;
    }
    for (; j < C; ++j) rank += s.sel[j] < k;
    if (rank <= K) s.keys[rank] = k;
  }
}

// Block-wide: the C <= MG_SEL unique keys of s.sel ranked, the K + 1 smallest written ascending to the
// front of s.keys.  Wave w < ceil(C / 64) sorts s.sel[64w, 64w + 64) in registers (a bitonic network
// over lane shuffles; NO_KEY pads the last chunk) and writes it back; then thread t < C takes the
// t-th sorted key: its rank is its index in its own chunk plus, per other chunk, the count of keys
// below it (a 7-read binary search over the chunk's 64 sorted keys) -- one thread per key and
// ~7 x chunks LDS reads, against rank_place's count over every selected key.  The caller's barrier
// after s.sel was written precedes it; ends with a barrier.  (PE_RANK_PLACE=1 at build time: rank_place.)
__device__ __forceinline__ void sort_rank(TopkShared& s, int C, int K) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nch = (C + 63) >> 6;
  if (wave < nch) {
    const int i = (wave << 6) + lane;
    uint64_t v = i < C ? s.sel[i] : NO_KEY;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const uint64_t o = __shfl_xor(v, j, 64);
        // the lower lane of a pair keeps the smaller key in an ascending run, the larger in a descending one
        v = (((lane & j) == 0) == ((lane & k) == 0)) ? umin64(v, o) : umax64(v, o);
      }
    }
    s.sel[i] = v;
  }
  __syncthreads();
  if (tid < C) {
    const uint64_t k = s.sel[tid];
    int rank = lane;   // keys are unique: its index in its own sorted chunk
    for (int c = 0; c < nch; ++c) {   // (the chunks' searches interleaved step by step measured slower:
      if (c == wave) continue;        // rank 4.2 vs 2.7 us per call, profiles/r57_topk_ab.txt)
      const uint64_t* ch = s.sel + (c << 6);
      int pos = ch[31] < k ? 32 : 0;
      pos += ch[pos + 15] < k ? 16 : 0;
      pos += ch[pos + 7] < k ? 8 : 0;
      pos += ch[pos + 3] < k ? 4 : 0;
      pos += ch[pos + 1] < k ? 2 : 0;
      pos += ch[pos] < k ? 1 : 0;
      pos += ch[pos] < k ? 1 : 0;   // (all 64 below: pos 63 -> 64)
      rank += pos;
    }
    if (rank <= K) s.keys[rank] = k;
  }
  __syncthreads();
}

__device__ __forceinline__ void place_ranked(TopkShared& s, int C, int K) {
#ifdef PE_RANK_PLACE
  rank_place(s, C, K);
  __syncthreads();
#else
  sort_rank(s, C, K);
#endif
}

#ifdef PE_WALK_PROF   // topk_sort breakdown (diagnostics build): calls, T, C, bitonic fallbacks, phase ticks
__device__ unsigned long long topk_prof[8];
#define TKP(i, v) (threadIdx.x == 0 ? (void)atomicAdd(&topk_prof[i], (unsigned long long)(v)) : (void)0)
#define TKT(n) unsigned long long tkt##n = wall_clock64()
#else
#define TKP(i, v)
#define TKT(n)
#endif
// bound: keys >= bound can be ignored (the caller knows >= K + 1 keys lie below it; NO_KEY = none)
__device__ uint64_t* topk_sort(TopkShared& s, int T, int K, uint64_t bound = NO_KEY) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  __syncthreads();
  TKT(0);
  TKP(0, 1);
  TKP(1, T);
  if (T <= 2 * (K + 1) && T <= MG_SEL) {   // few keys: rank-place them all (no histogram, no bitonic)
    for (int i = tid; i < T; i += MG_THREADS) s.sel[i] = s.keys[i];
    __syncthreads();
    place_ranked(s, T, K);
    return s.keys;
  }
  if (K + 1 <= MG_SEL) {
    uint64_t mn = NO_KEY, mx = 0;
    for (int i = tid; i < T; i += MG_THREADS) {
      const uint64_t k = s.keys[i];
      if (k < bound) {
        mn = umin64(mn, k);
        mx = umax64(mx, k);
      }
    }
    mn = wave_min_u64(mn);
    mx = wave_max_u64(mx);
    if (lane == 0) {
      s.red[wave] = mn;
      s.red[MG_THREADS / 64 + wave] = mx;
    }
    for (int i = tid; i < 256; i += MG_THREADS) s.hist[i] = 0;
    if (tid == 0) s.sel_c = 0;
    __syncthreads();
    uint64_t kmin = NO_KEY, kmax = 0;
#pragma unroll
    for (int i = 0; i < MG_THREADS / 64; ++i) {
      kmin = umin64(kmin, s.red[i]);
      kmax = umax64(kmax, s.red[MG_THREADS / 64 + i]);
    }
    const int bits = 64 - __clzll((long long)((kmax - kmin) | 1));
    const int sh = bits > 8 ? bits - 8 : 0;
#ifdef PE_HIST_PLAIN   // (A/B: one LDS atomic per key)
    for (int i = tid; i < T; i += MG_THREADS) {
      const uint64_t k = s.keys[i];
      if (k < bound) atomicAdd(&s.hist[(int)((k - kmin) >> sh)], 1);
    }
#else
    // one LDS atomic per run of equal bins across a wave's lanes: the walk appends its keys round by
    // round, nearly sorted, so neighbouring lanes mostly share a bin (one atomic per key serialises there)
    for (int i0 = 0; i0 < T; i0 += MG_THREADS) {   // (block-uniform trip count: shuffles and ballots)
      const int i = i0 + tid;
      const uint64_t k = i < T ? s.keys[i] : NO_KEY;
      const int b = k < bound ? (int)((k - kmin) >> sh) : -1;
      hist_add_runs(s.hist, b, lane);
    }
#endif
    __syncthreads();
    hist_cut(s, K + 1);
    const int cb = s.sel_bin;
    const int before = s.sel_n;
#ifndef PE_TOPK_TWO_LEVEL
    // one level when it suffices: every key below the bound in bins <= cb (the (K+1)-th smallest lies
    // in bin cb), appended wave by wave; up to MG_SEL of them are ranked directly (the second histogram,
    // its cut and three barriers saved), more fall through to the second level below
    // (s.sel_c was zeroed before the first histogram's barrier; hist_cut's sel_n / sel_bin are read above)
    for (int i0 = 0; i0 < T; i0 += MG_THREADS) {   // (block-uniform trip count: the ballot is wave-wide)
      const int i = i0 + tid;
      const uint64_t k = i < T ? s.keys[i] : NO_KEY;
      const bool take = i < T && k < bound && (int)((k - kmin) >> sh) <= cb;
      const uint64_t bal = __ballot(take);
      if (bal) {
        const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        int base = 0;
        if (take && r == 0) base = atomicAdd(&s.sel_c, __popcll(bal));
        base = __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
        if (take && base + r < MG_SEL) s.sel[base + r] = k;
      }
    }
    __syncthreads();
    if (s.sel_c <= MG_SEL) {
      const int C1 = s.sel_c;
      TKT(1);
      TKP(3, C1);
      TKP(4, tkt1 - tkt0);
      place_ranked(s, C1, K);
      TKT(2);
      TKP(5, tkt2 - tkt1);
      return s.keys;
    }
#endif
    // level 2 inside bin cb: keys in [base, base + 2^sh), 256 sub-bins of 2^sh2
    const uint64_t base = kmin + ((uint64_t)cb << sh);
    const int sh2 = sh > 8 ? sh - 8 : 0;
    int cb2 = 255;
    if (sh > 0) {
      __syncthreads();                     // every thread has read sel_bin / sel_n
      for (int i = tid; i < 256; i += MG_THREADS) s.hist[i] = 0;
      __syncthreads();
#ifdef PE_HIST_PLAIN
      for (int i = tid; i < T; i += MG_THREADS) {
        const uint64_t k = s.keys[i];
        if (k < bound && (int)((k - kmin) >> sh) == cb) atomicAdd(&s.hist[(int)((k - base) >> sh2)], 1);
      }
#else
      for (int i0 = 0; i0 < T; i0 += MG_THREADS) {
        const int i = i0 + tid;
        const uint64_t k = i < T ? s.keys[i] : NO_KEY;
        const int b = k < bound && (int)((k - kmin) >> sh) == cb ? (int)((k - base) >> sh2) : -1;
        hist_add_runs(s.hist, b, lane);
      }
#endif
      __syncthreads();
      hist_cut(s, K + 1 - before);
      cb2 = s.sel_bin;
    }
    // selected: below bin cb, or in bin cb up to sub-bin cb2
    __syncthreads();
    if (tid == 0) s.sel_n = 0;
    __syncthreads();
    for (int i = tid; i < T; i += MG_THREADS) {
      const uint64_t k = s.keys[i];
      const int b1 = k < bound ? (int)((k - kmin) >> sh) : 256;
      if (b1 < cb || (b1 == cb && (int)((k - base) >> sh2) <= cb2)) {
        const int pos = atomicAdd(&s.sel_n, 1);
        if (pos < MG_SEL) s.sel[pos] = k;
      }
    }
    __syncthreads();
    const int C = s.sel_n;
    TKT(1);
    TKP(3, C);
    TKP(4, tkt1 - tkt0);
    if (C <= MG_SEL) {
      place_ranked(s, C, K);               // into s.keys (its old contents are no longer needed)
      TKT(2);
      TKP(5, tkt2 - tkt1);
      return s.keys;
    }
  }
  // bitonic sort of all T keys
  TKP(2, 1);
  uint64_t* sk = s.keys;
  int P = 2;
  while (P < T) P <<= 1;
  for (int i = T + tid; i < P; i += MG_THREADS) sk[i] = NO_KEY;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += MG_THREADS) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = sk[i], c = sk[ixj];
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            sk[i] = c;
            sk[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  return sk;
}

// Group blob: header + the first nout keys of sk.  gen != 0 (walk windows written straight into
// pinned host memory): the group is SIGNALLED -- keys, n and limit first, every thread's stores
// made visible at system scope, then header.flags = gen as the last store -- so the host can take
// each group as soon as its block is done instead of waiting for the whole launch.
__device__ void write_group(const uint64_t* sk, int nout, int flags, uint64_t limit, int K, int g,
                            uint8_t* __restrict__ out, uint32_t gen = 0) {
  uint8_t* og = out + (size_t)g * cand_group_bytes(K);
  uint64_t* keys = reinterpret_cast<uint64_t*>(og + sizeof(CandHdr));
  for (int i = threadIdx.x; i < nout; i += blockDim.x) keys[i] = sk[i];
  CandHdr* hp = reinterpret_cast<CandHdr*>(og);
  if (gen == 0) {
    if (threadIdx.x == 0) {
      CandHdr h;
      h.n = nout;
      h.flags = flags;
      h.limit = limit;
      *hp = h;
    }
    return;
  }
  if (threadIdx.x == 0) {
    hp->n = nout;
    hp->limit = limit;
  }
  // the waves that stored (keys: threads < nout; header: thread 0) wait until their stores have
  // left the CU (vmcnt 0), the block agrees, and thread 0's system-scope release (L2 write-back,
  // then the flag store) publishes the generation after all of them
#ifdef PE_SIGNAL_FULL_FENCE
  if ((int)(threadIdx.x & ~63u) < nout || threadIdx.x < 64) __threadfence_system();
#else
  if ((int)(threadIdx.x & ~63u) < nout || threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  __syncthreads();
#ifdef PE_SIGNAL_RELAXED   // (A/B: no L2 write-back before the flag -- the list went to uncached host memory)
  if (threadIdx.x == 0) __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  if (threadIdx.x == 0) __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
}

__global__ __launch_bounds__(MG_THREADS) void merge_kernel(const uint64_t* __restrict__ cand,
                                                           const int32_t* __restrict__ cnt,
                                                           const uint64_t* __restrict__ bound, int nwaves, int K,
                                                           uint8_t* __restrict__ out) {
  __shared__ TopkShared s;
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t gbase = (size_t)g * (size_t)nwaves;

  // Phase A+B in one round trip: each thread loads its wave list's bound, count and first PRE
  // keys together (independent loads; list slots always exist); G = block min of the bounds; the
  // loaded keys below G are appended to LDS with one atomic per wave (ballot/mbcnt ranks).
  constexpr int PRE = 8;
  uint64_t b = NO_KEY;
  int c0 = 0;
  uint64_t k0[PRE];
  {
    const bool has = tid < nwaves;
    b = has ? bound[gbase + tid] : NO_KEY;
    c0 = has ? cnt[gbase + tid] : 0;
    const uint64_t* lst = cand + (gbase + (has ? tid : 0)) * 64;
#pragma unroll
    for (int u = 0; u < PRE; ++u) k0[u] = lst[u];
  }
  for (int w = tid + MG_THREADS; w < nwaves; w += MG_THREADS) b = umin64(b, bound[gbase + w]);
  b = wave_min_u64(b);
  if (lane == 0) s.red[wave] = b;
  if (tid == 0) s.total = 0;
  __syncthreads();
  uint64_t G = NO_KEY;
#pragma unroll
  for (int i = 0; i < MG_THREADS / 64; ++i) G = umin64(G, s.red[i]);
#pragma unroll
  for (int u = 0; u < PRE; ++u) topk_append(s, k0[u], u < c0 && k0[u] < G);
  // the rest of longer lists, and lists beyond the first MG_THREADS
  for (int w = tid; w < nwaves; w += MG_THREADS) {
    const int c = w == tid ? c0 : cnt[gbase + w];
    const uint64_t* lst = cand + (gbase + w) * 64;
    for (int i0 = w == tid ? PRE : 0; i0 < c; i0 += 8) {
      uint64_t k[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) k[u] = i0 + u < c ? lst[i0 + u] : NO_KEY;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k[u] < G) {
          const int pos = atomicAdd(&s.total, 1);
          if (pos < MG_CAP) s.keys[pos] = k[u];
        }
    }
  }
  __syncthreads();
  const int T = s.total;
  if (T > MG_CAP) {
    // Overflow (pathological): keep only the exact minimum over every candidate.
    uint64_t mn = NO_KEY;
    for (int w = tid; w < nwaves; w += MG_THREADS) {
      const int c = cnt[gbase + w];
      for (int i = 0; i < c; ++i) mn = umin64(mn, cand[(gbase + w) * 64 + i]);
    }
    mn = wave_min_u64(mn);
    __syncthreads();                       // every thread has read G from s.red
    if (lane == 0) s.red[wave] = mn;
    __syncthreads();
    mn = NO_KEY;
#pragma unroll
    for (int i = 0; i < MG_THREADS / 64; ++i) mn = umin64(mn, s.red[i]);
    if (tid == 0) s.keys[0] = mn;
    __syncthreads();
    write_group(s.keys, 1, 1, mn + 1, K, g, out);
    return;
  }
  const uint64_t* sk = topk_sort(s, T, K);
  // sk holds the K + 1 smallest of all T in order; keys >= G were never listed
  write_group(sk, T < K ? T : K, 0, T > K ? sk[K] : G, K, g, out);
}

// Shard merge (multi-rank greedy): after the all-gather every rank holds each shard's list of each
// window group (world consecutive blobs, group g of shard r at r * Wg * gb + g * gb).  One block per
// group keeps the keys below L = the smallest shard limit (every shard lists all its keys below its
// own limit, so every key below L is there), selects the K + 1 smallest and writes ONE list with
// limit = the (K+1)-th key, or L -- the unsharded window's blob, signalled (gen) when the host takes
// groups as they arrive.  world * K <= MG_CAP (the host checks).
__global__ __launch_bounds__(MG_THREADS) void merge_shards_kernel(const uint8_t* __restrict__ gath, int world, int Wg,
                                                                  int K, uint8_t* __restrict__ out, uint32_t gen,
                                                                  int64_t rank_stride,
                                                                  const uint64_t* __restrict__ xstatus) {
  __shared__ TopkShared s;
  const int g = blockIdx.x;
  const int tid = threadIdx.x;
  const size_t gb = cand_group_bytes(K);
  const size_t shard_bytes = rank_stride > 0 ? (size_t)rank_stride : (size_t)Wg * gb;
  if (xstatus && *xstatus != 0) {   // zero-copy exchange: a rank's lists never arrived (xwait_kernel)
    if (tid == 0) {
      CandHdr* hp = reinterpret_cast<CandHdr*>(out + (size_t)g * gb);
      hp->n = -1;   // the host raises on it (pe_resolver.cpp parse_group_keys) and reports the limit
      hp->limit = *xstatus;
      __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  // The shards' lists may sit in host memory written by other processes' kernels (host exchange):
  // read them with system-scope loads, which go to memory past the GPU caches (no acquire: that
  // would invalidate L2 under every kernel on the GPU).  Headers once per block, through LDS.
  __shared__ uint64_t hl[MG_THREADS / 64];
  __shared__ int hn[MG_THREADS / 64];
  __shared__ int bad;
  if (tid == 0) {
    s.total = 0;
    bad = 0;
  }
  __syncthreads();
  if (tid < world) {
    const CandHdr* h = reinterpret_cast<const CandHdr*>(gath + tid * shard_bytes + (size_t)g * gb);
    hl[tid] = __hip_atomic_load(&h->limit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int n = __hip_atomic_load(&h->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    hn[tid] = n < 0 ? 0 : (n > K ? K : n);
    if (n < 0 || n > K) bad = 1;   // a shard list is corrupt: the merged group says so (never read past it)
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) {
      CandHdr* hp = reinterpret_cast<CandHdr*>(out + (size_t)g * gb);
      hp->n = CAND_CORRUPT;
      hp->limit = 0;
      __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  uint64_t L = NO_KEY;
  for (int r = 0; r < world; ++r) L = umin64(L, hl[r]);
  for (int r = 0; r < world; ++r) {
    const uint8_t* base = gath + r * shard_bytes + (size_t)g * gb;
    const int n = hn[r];
    const uint64_t* keys = reinterpret_cast<const uint64_t*>(base + sizeof(CandHdr));
    for (int i0 = 0; i0 < n; i0 += MG_THREADS) {   // block-uniform bound: topk_append is wave-collective
      const int i = i0 + tid;
      const uint64_t k = i < n ? __hip_atomic_load(&keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : NO_KEY;
      topk_append(s, k, k < L);
    }
  }
  __syncthreads();
  const int T = s.total;
  const uint64_t* sk = topk_sort(s, T, K);
  write_group(sk, T < K ? T : K, 0, T > K ? sk[K] : L, K, g, out, gen);
}

hipError_t launch_merge_shards(hipStream_t s, const uint8_t* gath, int world, int Wg, int K, uint8_t* out, uint32_t gen,
                               int64_t rank_stride, const uint64_t* xstatus, bool /*sys_scope: always*/) {
  if (Wg <= 0) return hipSuccess;
  if (world < 1 || world > MG_THREADS / 64 || K < 1 || (int64_t)world * K > MG_CAP) return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_shards_kernel, dim3(Wg), dim3(MG_THREADS), 0, s, gath, world, Wg, K, out, gen, rank_stride,
                     xstatus);
  return hipGetLastError();
}

// Zero-copy exchange wait (pe_hostx.h): ONE small block polls every (rank, group) header of the
// window's slots until it carries in_gen, then the shard merge runs behind it on the stream.  The
// wait is one block, not the merge's 1024-thread blocks: with several ranks on one GPU, merges that
// spun while holding a CU's registers each could take every CU a peer's walk needs (a 3-rank run on
// one card did exactly that).  A peer that never writes: after timeout_ticks of wall_clock64 (100
// MHz) *xstatus = 1 << 63 | rank << 32 | the generation seen, which the merge reports per group.
__global__ __launch_bounds__(XW_THREADS) void xwait_kernel(const uint8_t* __restrict__ gath, int world, int Wg, int K,
                                                           int64_t rank_stride, uint32_t in_gen, int64_t timeout_ticks,
                                                           uint64_t* __restrict__ xstatus) {
  __shared__ unsigned long long late;
  if (threadIdx.x == 0) late = 0;
  __syncthreads();
  const size_t gb = cand_group_bytes(K);
  const long long t0 = wall_clock64();
  for (int i = threadIdx.x; i < world * Wg; i += XW_THREADS) {
    const int r = i / Wg, g = i - r * Wg;
    const CandHdr* h = reinterpret_cast<const CandHdr*>(gath + (size_t)r * rank_stride + (size_t)g * gb);
    // relaxed system-scope polls: each reads memory, past the caches, without an acquire's cache
    // invalidation (an acquire per poll invalidated L2 under every kernel of the GPU: the walks
    // sharing it slowed down ~1.5x).  The merge behind this kernel reads the lists the same way.
    int32_t f;
    while ((f = __hip_atomic_load(&h->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != (int32_t)in_gen) {
      if (__hip_atomic_load(&late, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0) break;
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > timeout_ticks) {
        atomicCAS(&late, 0ull, (1ull << 63) | ((unsigned long long)r << 32) | (uint32_t)f);
        break;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) *xstatus = late;
}

hipError_t launch_xwait(hipStream_t s, const uint8_t* gath, int world, int Wg, int K, int64_t rank_stride,
                        uint32_t in_gen, int64_t timeout_ticks, uint64_t* xstatus) {
  if (Wg <= 0) return hipSuccess;
  if (world < 1 || rank_stride < (int64_t)Wg * (int64_t)cand_group_bytes(K) || in_gen == 0 || timeout_ticks <= 0 || !xstatus)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(xwait_kernel, dim3(1), dim3(XW_THREADS), 0, s, gath, world, Wg, K, rank_stride, in_gen,
                     timeout_ticks, xstatus);
  return hipGetLastError();
}

// Rank merge (same output as merge_shards_kernel), the default shard merge: one 256-thread block
// per group holds the shards' lists in LDS (world x K keys) and places the merged list's keys by
// their rank in the union.  Only a cut of each list is ranked: with c = ceil((K+1) / world), every
// list's first min(c, keys below L) keys hold >= K + 1 keys in all (unless the lists have fewer below
// L than that, when every key below L is ranked), so the K + 1 smallest are at or below U = the
// largest of those heads -- the candidates are each list's keys <= U (a downward-closed set: ~1.3
// (K+1) keys at 8 ranks instead of 8 K).  A candidate's rank is its index in its own list plus, per
// other list, the count of that list's candidates below it: lock-step branchless binary searches
// over every other list, one step of each per round (independent LDS reads in flight, no sort, no
// histogram, one barrier).  Keys are unique across shards (the node id is in their low bits).
// Ranks < K land in an LDS output list copied out coalesced; rank K is the new limit.
// SYS: the lists sit in host memory written by other processes' kernels (host exchange): read with
// system-scope relaxed loads (see merge_shards_kernel).  !SYS: the all-gather's device buffer,
// written by an earlier kernel of the stream -- plain loads.
__device__ __forceinline__ int lds_lower_bound(const uint64_t* a, int n, uint64_t k) {
  int lo = 0;
  while (n > 0) {
    const int h = n >> 1;
    if (a[lo + h] < k) {
      lo += h + 1;
      n -= h + 1;
    } else {
      n = h;
    }
  }
  return lo;
}

template <bool SYS>
__device__ __forceinline__ uint64_t merge_load(const uint64_t* p) {
  if constexpr (SYS) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return *p;
}

template <bool SYS>
__global__ __launch_bounds__(RM_THREADS) void merge_ranked_kernel(const uint8_t* __restrict__ gath, int world, int Wg,
                                                                  int K, uint8_t* __restrict__ out, uint32_t gen,
                                                                  int64_t rank_stride,
                                                                  const uint64_t* __restrict__ xstatus) {
  extern __shared__ uint64_t lk[];   // shard r's keys at lk[r * K ...]; the merged list at lk[world * K ...]
  __shared__ uint64_t hl[RM_MAX_WORLD];
  __shared__ int hn[RM_MAX_WORLD], cnt[RM_MAX_WORLD], mc[RM_MAX_WORLD];
  __shared__ int bad;
  const int g = blockIdx.x;
  const int tid = threadIdx.x;
  const size_t gb = cand_group_bytes(K);
  const size_t shard_bytes = rank_stride > 0 ? (size_t)rank_stride : (size_t)Wg * gb;
  uint8_t* og = out + (size_t)g * gb;
  CandHdr* hp = reinterpret_cast<CandHdr*>(og);
  if (xstatus && *xstatus != 0) {   // zero-copy exchange: a rank's lists never arrived (xwait_kernel)
    if (tid == 0) {
      hp->n = -1;
      hp->limit = *xstatus;
      __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  if (tid == 0) bad = 0;
  __syncthreads();
  if (tid < world) {
    const CandHdr* h = reinterpret_cast<const CandHdr*>(gath + tid * shard_bytes + (size_t)g * gb);
    int n;
    if constexpr (SYS) {
      hl[tid] = __hip_atomic_load(&h->limit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      n = __hip_atomic_load(&h->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      hl[tid] = h->limit;
      n = h->n;
    }
    hn[tid] = max(0, min(n, K));
    if (n < 0 || n > K) bad = 1;   // (as merge_shards_kernel: a corrupt shard list marks the group)
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) {
      hp->n = CAND_CORRUPT;
      hp->limit = 0;
      __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  // every list into LDS: 8 loads per thread in flight at once (the lists are at most K keys each)
  const int span = world * K;
  for (int base = 0; base < span; base += 8 * RM_THREADS) {
    uint64_t v[8];
    int at[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * RM_THREADS + tid;
      const int r = i / K, j = i - r * K;
      at[u] = i < span && j < hn[r] ? i : -1;
      v[u] = at[u] >= 0 ? merge_load<SYS>(reinterpret_cast<const uint64_t*>(gath + r * shard_bytes + (size_t)g * gb +
                                                                               sizeof(CandHdr)) + j)
                        : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (at[u] >= 0) lk[at[u]] = v[u];
  }
  uint64_t L = NO_KEY;
  for (int r = 0; r < world; ++r) L = umin64(L, hl[r]);
  __syncthreads();
  if (tid < world) cnt[tid] = lds_lower_bound(lk + tid * K, hn[tid], L);   // keys below L
  __syncthreads();
  const int c = (K + 1 + world - 1) / world;
  int T = 0, have = 0;
  uint64_t U = 0;
  for (int r = 0; r < world; ++r) {
    const int hd = min(cnt[r], c);
    T += cnt[r];
    have += hd;
    if (hd > 0) U = umax64(U, lk[r * K + hd - 1]);
  }
  if (tid < world)   // the candidates: keys <= U (when the heads hold K + 1 keys), else every key below L
    mc[tid] = have >= K + 1 ? lds_lower_bound(lk + tid * K, cnt[tid], U + 1) : cnt[tid];
  __syncthreads();
  int M = 0, mx = 0, mq[RM_MAX_WORLD];
#pragma unroll
  for (int q = 0; q < RM_MAX_WORLD; ++q) {
    mq[q] = q < world ? mc[q] : 0;
    M += mq[q];
    mx = max(mx, mq[q]);
  }
  int top = 1;   // the largest power of two <= mx (the binary searches' first step)
  while (top * 2 <= mx) top *= 2;
  uint64_t* ok = lk + (size_t)world * K;   // the merged list (K + 1 keys: the list and the new limit)
  for (int t = tid; t < M; t += RM_THREADS) {
    int r = 0, idx = t;
    while (idx >= mc[r]) {   // (t < M: some list holds it; LDS, not the register copy: r is not static)
      idx -= mc[r];
      ++r;
    }
    const uint64_t k = lk[r * K + idx];
    int pos[RM_MAX_WORLD];
#pragma unroll
    for (int q = 0; q < RM_MAX_WORLD; ++q) pos[q] = 0;
    for (int st = top; st > 0; st >>= 1) {
#pragma unroll
      for (int q = 0; q < RM_MAX_WORLD; ++q) {
        const int p = pos[q] + st;
        if (q < world && q != r && p <= mq[q] && lk[q * K + p - 1] < k) pos[q] = p;
      }
    }
    int rank = idx;
#pragma unroll
    for (int q = 0; q < RM_MAX_WORLD; ++q) rank += pos[q];
    if (rank <= K) ok[rank] = k;
  }
  __syncthreads();
  const int nout = T < K ? T : K;
  uint64_t* dst = reinterpret_cast<uint64_t*>(og + sizeof(CandHdr));
  for (int i = tid; i < nout; i += RM_THREADS) dst[i] = ok[i];
  if (tid == 0) {
    hp->n = nout;
    hp->limit = T > K ? ok[K] : L;
    if (gen == 0) hp->flags = 0;
  }
  // as write_group: every store has left the CU, the block agrees, then the signal (release)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 && gen != 0) __hip_atomic_store(&hp->flags, (int32_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

size_t merge_ranked_lds(int world, int K) { return ((size_t)world * K + K + 1) * sizeof(uint64_t); }

hipError_t launch_merge_ranked(hipStream_t s, const uint8_t* gath, int world, int Wg, int K, uint8_t* out, uint32_t gen,
                               int64_t rank_stride, const uint64_t* xstatus, bool sys_scope) {
  if (Wg <= 0) return hipSuccess;
  if (world < 1 || world > RM_MAX_WORLD || K < 1 || merge_ranked_lds(world, K) > RM_MAX_LDS) return hipErrorInvalidValue;
  if (sys_scope)
    hipLaunchKernelGGL(merge_ranked_kernel<true>, dim3(Wg), dim3(RM_THREADS), merge_ranked_lds(world, K), s, gath, world,
                       Wg, K, out, gen, rank_stride, xstatus);
  else
    hipLaunchKernelGGL(merge_ranked_kernel<false>, dim3(Wg), dim3(RM_THREADS), merge_ranked_lds(world, K), s, gath, world,
                       Wg, K, out, gen, rank_stride, xstatus);
  return hipGetLastError();
}

// Empty lists (an empty node shard's window in a zero-copy exchange), signalled like a walk's.
__global__ __launch_bounds__(64) void empty_groups_kernel(int Wg, int K, uint8_t* __restrict__ out, uint32_t gen) {
  write_group(nullptr, 0, 0, NO_KEY, K, blockIdx.x, out, gen);
}

__global__ __launch_bounds__(64) void stall_kernel(int64_t ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

hipError_t launch_stall(hipStream_t s, int64_t ticks) {
  if (ticks <= 0 || ticks > (int64_t)30 * 100000000) return hipErrorInvalidValue;   // at most 30 s
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}

hipError_t launch_empty_groups(hipStream_t s, int Wg, int K, uint8_t* out, uint32_t gen) {
  if (Wg <= 0) return hipSuccess;
  hipLaunchKernelGGL(empty_groups_kernel, dim3(Wg), dim3(64), 0, s, Wg, K, out, gen);
  return hipGetLastError();
}

hipError_t launch_merge(hipStream_t s, const uint64_t* cand, const int32_t* cnt, const uint64_t* bound, int nwaves,
                        int K, uint8_t* out, int Wg) {
  if (Wg <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_kernel, dim3(Wg), dim3(MG_THREADS), 0, s, cand, cnt, bound, nwaves, K, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ sorted walk (greedy default)

// Appends local node n with state (r, lab) and node-only key Kn to the overlay (slot, state copy,
// membership).
__device__ __forceinline__ void overlay_add(const WalkIndex& w, int64_t n, const int64_t (&r)[D], uint32_t lab,
                                            uint64_t Kn) {
  const int32_t i = atomicAdd(w.ovl_n, 1);
  w.ovl[i] = (int32_t)n;
  w.ovl_idx[n] = (uint32_t)i;
#pragma unroll
  for (int d = 0; d < D; ++d) w.ovl_res[d * w.sstride + i] = r[d];
  w.ovl_lab[i] = lab;
  w.ovl_kn[i] = Kn;
}

__global__ __launch_bounds__(256) void walk_prep_kernel(const int64_t* __restrict__ res, int64_t stride, int64_t Ns,
                                                        const uint64_t* __restrict__ kn,
                                                        const uint32_t* __restrict__ labels, uint64_t* __restrict__ kin,
                                                        WalkIndex w, uint32_t* __restrict__ slow) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= Ns) return;
  const int64_t r[D] = {res[n], res[stride + n], res[2 * stride + n], res[3 * stride + n]};
  const bool neg = (r[0] | r[1] | r[2] | r[3]) < 0;
  const uint64_t K = kn[n];
  uint64_t k = K;
  if (neg) {
    k = WK_INVALID;                  // fits nothing
  } else if (K == KEY_SLOW) {
    k = WK_INVALID;                  // saturating terms: evaluated in full through the overlay
    if (slow) {
      slow[n] = 1u;                  // (side-stream rebuild: walk_switch adds it)
    } else {
      w.in_ovl[n] = 1u;
      overlay_add(w, n, r, labels[n], KEY_SLOW);
    }
  }
  kin[n] = k;
}

hipError_t launch_walk_prep(hipStream_t s, const int64_t* res, int64_t stride, int64_t Ns, const uint64_t* kn,
                            const uint32_t* labels, uint64_t* kin, const WalkIndex& w, uint32_t* slow) {
  if (Ns <= 0) return hipSuccess;
  hipLaunchKernelGGL(walk_prep_kernel, dim3((unsigned)((Ns + 255) / 256)), dim3(256), 0, s, res, stride, Ns, kn, labels,
                     kin, w, slow);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void walk_switch_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                          const uint32_t* __restrict__ labels, int64_t Ns,
                                                          const uint32_t* __restrict__ slow, WalkIndex nx) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= Ns) return;
  if (nx.in_ovl[n]) {                // updated during the rebuild: its overlay entry is current
    const uint32_t p = nx.pos[n];
    if (p != ~0u) {
      nx.sk[p] = WK_INVALID;
      nx.pos[n] = ~0u;
    }
  } else if (slow[n]) {
    const int64_t r[D] = {res[n], res[stride + n], res[2 * stride + n], res[3 * stride + n]};
    nx.in_ovl[n] = 1u;
    overlay_add(nx, n, r, labels[n], KEY_SLOW);
  }
}

hipError_t launch_walk_switch(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                              const uint32_t* slow, const WalkIndex& nx) {
  if (Ns <= 0) return hipSuccess;
  hipLaunchKernelGGL(walk_switch_kernel, dim3((unsigned)((Ns + 255) / 256)), dim3(256), 0, s, res, stride, labels, Ns,
                     slow, nx);
  return hipGetLastError();
}

// One block per round: gather the sorted SoA copy, pos[], and the round's summary.
__global__ __launch_bounds__(WK_ROUND) void walk_build_kernel(const int64_t* __restrict__ res, int64_t stride,
                                                              const uint32_t* __restrict__ labels, int64_t Ns,
                                                              uint64_t id_base, WalkIndex w) {
  __shared__ int64_t mx[D][WK_ROUND / 64];
  __shared__ uint32_t orl[WK_ROUND / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r = blockIdx.x;
  const int64_t i = r * WK_ROUND + tid;
  const uint64_t K = i < Ns ? w.sk[i] : WK_INVALID;
  int64_t v[D] = {INT64_MIN, INT64_MIN, INT64_MIN, INT64_MIN};
  uint32_t lab = 0;
  if (K != WK_INVALID) {
    const int64_t n = (int64_t)((K & 0xFFFFFFull) - id_base);
    w.pos[n] = (uint32_t)i;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = res[d * stride + n];
      w.sr[d * w.sstride + i] = v[d];
    }
    lab = labels[n];
    w.sl[i] = lab;
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    for (int off = 32; off >= 1; off >>= 1) {
      const int64_t o = __shfl_xor(v[d], off, 64);
      v[d] = o > v[d] ? o : v[d];
    }
  for (int off = 32; off >= 1; off >>= 1) lab |= __shfl_xor(lab, off, 64);
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) mx[d][wave] = v[d];
    orl[wave] = lab;
  }
  __syncthreads();
  if (tid < D) {
    int64_t m = INT64_MIN;
    for (int k = 0; k < WK_ROUND / 64; ++k) m = mx[tid][k] > m ? mx[tid][k] : m;
    w.rmax[tid * w.nr + r] = m;
  } else if (tid == D) {
    uint32_t o = 0;
    for (int k = 0; k < WK_ROUND / 64; ++k) o |= orl[k];
    w.ror[r] = o;
    w.rmin[r] = w.sk[r * WK_ROUND];       // sorted: the round's smallest key
  }
}

hipError_t launch_walk_build(hipStream_t s, const int64_t* res, int64_t stride, const uint32_t* labels, int64_t Ns,
                             uint64_t id_base, const WalkIndex& w) {
  if (Ns <= 0) return hipSuccess;
  hipLaunchKernelGGL(walk_build_kernel, dim3((unsigned)w.nr), dim3(WK_ROUND), 0, s, res, stride, labels, Ns, id_base,
                     w);
  return hipGetLastError();
}

// Appends of one walk step: positions from the block-uniform total T0 of the keys before the step
// plus a per-step counter (one LDS atomic per wave).  The walk rotates three counters so that no
// barrier is needed between reading a step's count and the next step's appends: step t appends to
// wcnt[t % 3], every thread reads it after step t's barrier (before reaching the next one), and
// thread 0 zeroes wcnt[(t + 1) % 3] -- last read before step t - 1's barrier -- during step t.  (With
// one shared total, a thread that skipped the stop test could append the next step's keys before a
// slower wave had read the step's total: the threads' views of T diverged.)  Keys past MG_CAP are
// counted but dropped, as in topk_append.
__device__ __forceinline__ void step_append(TopkShared& s, int T0, int* cnt, uint64_t k, bool take) {
  const uint64_t bal = __ballot(take);
  if (bal == 0) return;
  const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
  int base = 0;
  if (take && rank == 0) base = atomicAdd(cnt, __popcll(bal));
  base = T0 + __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
  if (take && base + rank < MG_CAP) s.keys[base + rank] = k;
}

#ifdef PE_WALK_PROF   // phase timings of walk_kernel (wall clock ticks, summed over blocks), diagnostics build only
__device__ unsigned long long walk_prof[32];
#define WPT(i) unsigned long long wpt##i = wall_clock64()
#else
#define WPT(i)
#endif

// One block of WK_ROUND threads per group of the window:
//  1. per round (all rounds at once): can it hold a fit (q <= max residual per dimension, need in
//     the OR of labels)?  -> LDS bitmap; and how many rounds start below s(q) << 24 -> the first
//     round worth walking;
//  2. the overlay in full (current residuals);
//  3. the candidate rounds in sorted order, one node per thread, until >= K + 1 collected keys lie
//     below X = rmin(next round) - ((s(q) + 2) << 24), a lower bound of every key the unvisited
//     rounds can produce (their K(n) >= rmin, key = K(n) - ((s(q) + borrows) << 24)).
// Then the same exact selection and blob as merge: top-K records, limit = the (K+1)-th key (or
// NO_KEY once every candidate round was walked and at most K fit).
__global__ __launch_bounds__(WK_ROUND) void walk_kernel(const ReqRec* __restrict__ groups, int K, int Kst, WalkIndex w,
                                                        const int64_t* __restrict__ res, int64_t stride,
                                                        const uint32_t* __restrict__ labels, int64_t Ns,
                                                        uint64_t id_base, uint8_t* __restrict__ out, uint32_t gen) {
  static_assert(WK_ROUND == MG_THREADS, "the walk uses the merge's block-wide selection");
  __shared__ TopkShared s;
  __shared__ uint32_t cbits[WK_MAXR / 32];
  __shared__ int start_cnt, below[2], wcnt[3];
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  WPT(0);
  const ReqRec rq = groups[g];
  const int64_t q0 = rq.q[0], q1 = rq.q[1], q2 = rq.q[2], q3 = rq.q[3];
  const uint32_t need = rq.need;
  // s(q), saturated: a walkable node has S(n) < SCORE_MAX, so s(q) >= SCORE_MAX fits none of them
  uint64_t sq = (uint64_t)q0 + ((uint64_t)q1 >> 20) + ((uint64_t)q3 >> 24);
  sq = (uint64_t)q0 > SCORE_MAX || (uint64_t)q2 >= (1ull << 20) || sq >= SCORE_MAX ? SCORE_MAX : sq;
  sq = sq < SCORE_MAX ? sq + ((uint64_t)q2 << 20) : sq;
  const bool walk = sq < SCORE_MAX;
  const uint64_t KQ = walk ? sq << 24 : 0;
  const uint64_t KQ2 = !walk ? 0 : sq + 2 >= (1ull << 40) ? ~0ull : (sq + 2) << 24;   // (s(q) + 2) << 24, saturated
  const int64_t nr = w.nr;
  const int nwords = (int)((nr + 31) / 32);
  for (int i = tid; i < nwords; i += WK_ROUND) cbits[i] = 0u;
  if (tid == 0) {
    s.total = 0;
    start_cnt = 0;
    below[0] = below[1] = 0;
    wcnt[0] = wcnt[1] = wcnt[2] = 0;
  }
  __syncthreads();
  if (walk) {
    int cnt = 0;
    for (int64_t r0 = 0; r0 < nr; r0 += WK_ROUND) {   // (block-uniform bound: the ballot is wave-wide)
      const int64_t r = r0 + tid;
      bool can = false;
      if (r < nr) {
        cnt += w.rmin[r] < KQ;
        can = q0 <= w.rmax[r] && q1 <= w.rmax[nr + r] && q2 <= w.rmax[2 * nr + r] && q3 <= w.rmax[3 * nr + r] &&
              (w.ror[r] & need) == need;
      }
#ifdef PE_PREPASS_ATOMIC   // (A/B: one LDS atomic per round, 32 lanes of a wave on one word)
      if (can) atomicOr(&cbits[r >> 5], 1u << (r & 31));
#else
      // the wave's 64 rounds are two whole bitmap words, owned by this wave: one ballot, two stores
      const uint64_t bal = __ballot(can);
      const int64_t wr = r0 + (tid & ~63);
      if (lane == 0 && wr < nr) {
        cbits[wr >> 5] = (uint32_t)bal;
        if (wr + 32 < nr) cbits[(wr >> 5) + 1] = (uint32_t)(bal >> 32);
      }
#endif
    }
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane == 0 && cnt) atomicAdd(&start_cnt, cnt);
  }
  __syncthreads();   // (start_cnt and the candidate-round bitmap, read block-uniformly below)
  WPT(1);
  // The sorted rounds first, the overlay after them.  The walk stops once >= K + 1 of ITS keys lie
  // below X (every unvisited round's keys are >= X); the overlay then appends only keys below that
  // xstop -- a key >= xstop can never be among the K + 1 smallest -- instead of every fitting overlay
  // node ahead of the walk (round 4: 7.3k overlay entries per group, about half of the keys the
  // selection sorted).  Exact either way: the K + 1 smallest keys of (walked rounds + overlay) are
  // all below xstop, and every key below it is collected.
  //
  // Stop test without rescanning every collected key (it was O(T) per step, quadratic in the long
  // walks that set a launch's length): a round r's keys are <= rmin(next candidate round) - KQ
  // (K(n) <= every later sorted key, key <= K(n) - (s(q) << 24)), so once a step's bound lies below
  // the test's X, every key that step appended is below every later X too (X only grows): it is
  // counted once (cnt_certain) and not read again.  Only the keys of the last few steps, whose bound
  // is not below X yet, are compared -- they sit at [lo_idx, T), appended after the certain ones.
  bool done = !walk;
  int rounds = 0;
  int64_t r = walk ? (start_cnt > 0 ? start_cnt - 1 : 0) : nr;
  auto next_round = [&](int64_t from) -> int64_t {   // first candidate round >= from (uniform)
    int64_t wi = from >> 5;
    if (wi >= nwords) return nr;
    uint32_t bits = cbits[wi] & (~0u << (from & 31));
    while (bits == 0) {
      if (++wi >= nwords) return nr;
      bits = cbits[wi];
    }
    return wi * 32 + __ffs(bits) - 1;
  };
  if (!done) r = next_round(r);
  uint64_t xstop = NO_KEY;
  int tests = 0;
  int lo_idx = 0, cnt_certain = 0;   // keys [0, lo_idx): below every X from now on (block-uniform)
  constexpr int PEND = 4;            // pending steps, oldest first: end index and key bound
  int pend_n = 0;
  int pend_end[PEND];
  uint64_t pend_b[PEND];
  auto pend_push = [&](int end, uint64_t b) {
    if (pend_n == PEND) {            // merge the two oldest (contiguous ranges, bounds ascending)
#pragma unroll
      for (int i = 0; i + 1 < PEND; ++i) {
        pend_end[i] = pend_end[i + 1];
        pend_b[i] = pend_b[i + 1];
      }
      --pend_n;
    }
#pragma unroll
    for (int i = 0; i < PEND; ++i)
      if (i == pend_n) {
        pend_end[i] = end;
        pend_b[i] = b;
      }
    ++pend_n;
  };
  int Tcur = 0;      // keys collected so far (block-uniform)
  int step = 0;      // append steps so far (walk and overlay): counter wcnt[step % 3]
  auto compact = [&]() {   // keep the K + 1 smallest of the Tcur keys; ends with a barrier
    const int T2 = Tcur < MG_CAP ? Tcur : MG_CAP;
    const uint64_t* sk = topk_sort(s, T2, K);
    const int m = T2 < K + 1 ? T2 : K + 1;
    uint64_t v = tid < m ? sk[tid] : 0;
    __syncthreads();
    if (tid < m) s.keys[tid] = v;
    __syncthreads();
    Tcur = m;
    return m;
  };
  auto step_begin = [&]() -> int* {   // this step's counter; the one after the next zeroed
    if (tid == 0) wcnt[(step + 1) % 3] = 0;
    return &wcnt[step % 3];
  };
  auto step_end = [&]() {             // after the step's barrier
    Tcur += wcnt[step % 3];
    ++step;
  };
  // the next step's first round and its smallest key are found during the current step (the load
  // in flight with the step's node loads): the stop test does not wait for its own load
  uint64_t rm_r = !done && r < nr ? w.rmin[r] : 0;
  while (!done && r < nr) {
    const int T = Tcur < MG_CAP ? Tcur : MG_CAP;
    if (T >= K + 1) {                      // stop once K + 1 keys lie below every unvisited key
#ifdef PE_WALK_NO_RM_PREFETCH   // (A/B)
      const uint64_t rm = w.rmin[r];
#else
      const uint64_t rm = rm_r;
#endif
      const uint64_t X = rm > KQ2 ? rm - KQ2 : 0;
      while (pend_n > 0 && pend_b[0] < X) {   // a whole step below X: certain from now on
        cnt_certain += pend_end[0] - lo_idx;
        lo_idx = pend_end[0];
#pragma unroll
        for (int i = 0; i + 1 < PEND; ++i) {
          pend_end[i] = pend_end[i + 1];
          pend_b[i] = pend_b[i + 1];
        }
        --pend_n;
      }
#ifdef PE_WALK_CHECK
      if (cnt_certain >= K + 1) {
        __shared__ int full2;
        if (tid == 0) full2 = 0;
        __syncthreads();
        int cf = 0;
        for (int i = tid; i < T; i += WK_ROUND) cf += s.keys[i] < X;
        for (int off = 32; off >= 1; off >>= 1) cf += __shfl_xor(cf, off, 64);
        if (lane == 0 && cf) atomicAdd(&full2, cf);
        __syncthreads();
        if (tid == 0 && full2 < cnt_certain)
          printf("walk check: g %d early full %d < certain %d (lo_idx %d T %d X %llx)\n", g, full2, cnt_certain, lo_idx, T,
                 (unsigned long long)X);
        __syncthreads();
      }
#endif
      if (cnt_certain >= K + 1) {
        xstop = X;
        break;
      }
      int c = 0;
      for (int i = lo_idx + tid; i < T; i += WK_ROUND) c += s.keys[i] < X;
      for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
      // two counters used in turn: the one for the next test is zeroed after this test's barrier (every
      // thread read it at the previous test, and an append barrier lies between) -- one barrier per test
      if (lane == 0 && c) atomicAdd(&below[tests & 1], c);
      __syncthreads();
      const int nb = below[tests & 1];
      if (tid == 0) below[(tests + 1) & 1] = 0;
      ++tests;
#ifdef PE_WALK_CHECK   // (diagnostics: the incremental count equals a full count)
      {
        __shared__ int full;
        if (tid == 0) full = 0;
        __syncthreads();
        int cf = 0;
        for (int i = tid; i < T; i += WK_ROUND) cf += s.keys[i] < X;
        for (int off = 32; off >= 1; off >>= 1) cf += __shfl_xor(cf, off, 64);
        if (lane == 0 && cf) atomicAdd(&full, cf);
        __syncthreads();
        if (tid == 0 && full != cnt_certain + nb)
          printf("walk check: g %d full %d != certain %d + %d (lo_idx %d T %d pend %d X %llx)\n", g, full, cnt_certain,
                 nb, lo_idx, T, pend_n, (unsigned long long)X);
        __syncthreads();
      }
#endif
      if (cnt_certain + nb >= K + 1) {
        xstop = X;                         // >= K + 1 collected keys lie below it: the rest never matter
        break;
      }
    }
    // the rounds of this step: r, and once the walk is long (WK_MULTI_AFTER rounds walked: requests
    // few nodes fit, the launch's slowest blocks) up to WK_MULTI - 1 more candidate rounds, their loads
    // all in flight together -- one memory latency and one barrier per step instead of per round.
    // Walking a round more than needed is harmless (the stop bound only ever needs >= K + 1 keys).
    int64_t rr[WK_MULTI];
    int nstep = 1;
    rr[0] = r;
    if (rounds >= WK_MULTI_AFTER)
      for (; nstep < WK_MULTI; ++nstep) {
        const int64_t nx = next_round(rr[nstep - 1] + 1);
        if (nx >= nr) break;
        rr[nstep] = nx;
      }
    const int64_t r_next = next_round(rr[nstep - 1] + 1);
    const uint64_t rm_next = r_next < nr ? w.rmin[r_next] : 0;
    uint64_t k[WK_MULTI];
#pragma unroll
    for (int u = 0; u < WK_MULTI; ++u) {
      k[u] = NO_KEY;
      const int64_t i = rr[u < nstep ? u : 0] * WK_ROUND + tid;
      if (u < nstep && i < Ns) {
#ifdef PE_WALK_COND_LOAD   // (A/B: the state loads behind the sorted key's validity test)
        const uint64_t Kn = w.sk[i];
        if (Kn != WK_INVALID)
          k[u] = node_key(w.sr[i], w.sr[w.sstride + i], w.sr[2 * w.sstride + i], w.sr[3 * w.sstride + i], w.sl[i], q0,
                          q1, q2, q3, need, Kn & 0xFFFFFFull);
#else   // all six loads in flight at once (one memory latency per step, not two); an invalid
        // entry's state is read and dropped
        const uint64_t Kn = w.sk[i];
        const int64_t s0 = w.sr[i], s1 = w.sr[w.sstride + i], s2 = w.sr[2 * w.sstride + i], s3 = w.sr[3 * w.sstride + i];
        const uint32_t sl = w.sl[i];
        const uint64_t kk = node_key(s0, s1, s2, s3, sl, q0, q1, q2, q3, need, Kn & 0xFFFFFFull);
        k[u] = Kn != WK_INVALID ? kk : NO_KEY;
#endif
      }
    }
    int* const cnt = step_begin();
#pragma unroll
    for (int u = 0; u < WK_MULTI; ++u)
      if (u < nstep) step_append(s, Tcur, cnt, k[u], k[u] != NO_KEY);
    __syncthreads();
    step_end();
    // this step's keys: [previous total, Tcur), each <= rmin(r_next) - KQ (the last round has no
    // bound: its keys stay pending)
    pend_push(Tcur, r_next < nr ? (rm_next > KQ ? rm_next - KQ : 0) : NO_KEY);
    // (room for the next step's appends.  Cutting long walks' keys to K + 1 early, at 1024 or 2048,
    // with later appends filtered below the (K+1)-th, was measured slower: 62-64 vs 52 us per launch)
    if (Tcur > MG_CAP - WK_MULTI * WK_ROUND) {
      const int m = compact();
      lo_idx = cnt_certain = pend_n = 0;   // the kept keys, ascending: pending up to the largest
      pend_push(m, m > 0 ? s.keys[m - 1] : 0);
    }
    r = r_next;
    rm_r = rm_next;
    rounds += nstep;
  }
  WPT(2);
  // overlay: every node changed since the sort (and the saturating ones), current values; only keys
  // below xstop.  OV entries per thread between barriers (the overlay holds up to resort_nodes
  // entries, and up to ~1.5 x resort_nodes while a side-stream rebuild is pending: one barrier,
  // append and compaction check per 4096 instead of per 1024)
  // An entry is read in full only when its node-only key allows a key below xstop: a fit needs
  // K(n) >= KQ, and its key is >= K(n) - KQ2 (KEY_SLOW entries always) -- 8 B per entry instead of
  // 44 (the overlay phase streamed ~300 KB per group: CU-bandwidth-bound, not latency-bound).
#ifndef WK_OV
#define WK_OV 8   // (4: the same within noise; 8 halves the barriers of a long overlay)
#endif
  constexpr int OV = WK_OV;
  const int no = *w.ovl_n;
  const uint64_t klim = xstop > NO_KEY - KQ2 ? NO_KEY : xstop + KQ2;   // (NO_KEY: no bound)
  for (int i0 = 0; i0 < no; i0 += OV * WK_ROUND) {
    uint64_t kn[OV];
#pragma unroll
    for (int u = 0; u < OV; ++u) {
      const int i = i0 + u * WK_ROUND + tid;
      kn[u] = i < no ? w.ovl_kn[i] : 0;
    }
    uint64_t k[OV];
#pragma unroll
    for (int u = 0; u < OV; ++u) {
      const int i = i0 + u * WK_ROUND + tid;
      k[u] = NO_KEY;
      if (i < no && (kn[u] == KEY_SLOW || (kn[u] >= KQ && kn[u] < klim)))   // the overlay keeps its own state copy
        k[u] = node_key(w.ovl_res[i], w.ovl_res[w.sstride + i], w.ovl_res[2 * w.sstride + i],
                        w.ovl_res[3 * w.sstride + i], w.ovl_lab[i], q0, q1, q2, q3, need, id_base + (uint64_t)w.ovl[i]);
    }
    // room for this step's appends BEFORE them: the walk leaves up to MG_CAP - WK_MULTI * WK_ROUND keys,
    // and one overlay step appends up to OV * WK_ROUND (more than that room) -- keys past MG_CAP would be
    // dropped, and the dropped ones may be the group's best (changed nodes are the tight ones).
    // (Tcur is block-uniform; the step's keys wait in registers across the compaction.)
    if (Tcur > MG_CAP - OV * WK_ROUND) compact();
    int* const cnt = step_begin();
#pragma unroll
    for (int u = 0; u < OV; ++u) step_append(s, Tcur, cnt, k[u], k[u] < xstop);   // (NO_KEY never is)
    __syncthreads();
    step_end();
  }
  __syncthreads();
  WPT(3);
  const int T = Tcur < MG_CAP ? Tcur : MG_CAP;
  const uint64_t* sk = topk_sort(s, T, K, xstop);
  WPT(4);
  write_group(sk, T < K ? T : K, 0, T > K ? sk[K] : NO_KEY, Kst, g, out, gen);   // (stride: Kst keys)
  if (tid == 0 && w.stat) {
    atomicAdd(&w.stat[0], (unsigned long long)rounds);
    atomicAdd(&w.stat[1], (unsigned long long)no);
  }
#ifdef PE_WALK_PROF
  __syncthreads();
  WPT(5);
  if (tid == 0) {
    atomicAdd(&walk_prof[0], wpt1 - wpt0);
    atomicAdd(&walk_prof[1], wpt2 - wpt1);
    atomicAdd(&walk_prof[2], wpt3 - wpt2);
    atomicAdd(&walk_prof[3], wpt4 - wpt3);
    atomicAdd(&walk_prof[4], wpt5 - wpt4);
    atomicAdd(&walk_prof[5], 1ull);
    atomicAdd(&walk_prof[6], (unsigned long long)no);
    atomicAdd(&walk_prof[7], (unsigned long long)rounds);
    atomicAdd(&walk_prof[8], (unsigned long long)T);
    atomicMax(&walk_prof[9], wpt5 - wpt0);
    atomicMax(&walk_prof[10], wpt2 - wpt1);
    atomicMax(&walk_prof[11], wpt3 - wpt2);
    atomicMax(&walk_prof[12], wpt4 - wpt3);
    atomicMax(&walk_prof[13], (unsigned long long)rounds);
    atomicMax(&walk_prof[14], (unsigned long long)T);
    atomicMax(&walk_prof[15], wpt1 - wpt0);
    if (wpt5 - wpt0 > 3500) {   // slow blocks (> 35 us): where their time goes
      atomicAdd(&walk_prof[16], 1ull);
      atomicAdd(&walk_prof[17], wpt1 - wpt0);
      atomicAdd(&walk_prof[18], wpt2 - wpt1);
      atomicAdd(&walk_prof[19], wpt3 - wpt2);
      atomicAdd(&walk_prof[20], wpt4 - wpt3);
      atomicAdd(&walk_prof[21], wpt5 - wpt4);
      atomicAdd(&walk_prof[22], (unsigned long long)rounds);
      atomicAdd(&walk_prof[23], (unsigned long long)T);
      atomicAdd(&walk_prof[24], (unsigned long long)no);
      atomicAdd(&walk_prof[25], (unsigned long long)tests);
    }
  }
#endif
}

hipError_t launch_walk(hipStream_t s, const ReqRec* groups, int Wg, int K, const WalkIndex& w, const int64_t* res,
                       int64_t stride, const uint32_t* labels, int64_t Ns, uint64_t id_base, uint8_t* out,
                       uint32_t gen, int K_stride) {
  if (Wg <= 0) return hipSuccess;
  const int Kst = K_stride > 0 ? K_stride : K;
  if (w.nr > WK_MAXR || K + 1 > WK_ROUND || K > Kst) return hipErrorInvalidValue;
  hipLaunchKernelGGL(walk_kernel, dim3((unsigned)Wg), dim3(WK_ROUND), 0, s, groups, K, Kst, w, res, stride, labels, Ns,
                     id_base, out, gen);
#ifdef PE_WALK_PROF
  static int launches = 0;
  if (++launches % 500 == 0) {
    unsigned long long p[32];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(p, HIP_SYMBOL(walk_prof), sizeof(p));
    const double n = (double)p[5], us = 100.0;   // wall_clock64 runs at 100 MHz: ticks / 100 = us
    fprintf(stderr, "walk prof over %.0f blocks (us/block): setup+prepass %.2f walk %.2f overlay %.2f sort %.2f write %.2f"
                    " | overlay %.0f rounds %.2f T %.0f\n", n, p[0] / n / us, p[1] / n / us, p[2] / n / us,
            p[3] / n / us, p[4] / n / us, p[6] / n, p[7] / n, p[8] / n);
    fprintf(stderr, "walk prof max: block %.2f us setup %.2f walk %.2f overlay %.2f sort %.2f | rounds %llu T %llu\n",
            p[9] / us, p[15] / us, p[10] / us, p[11] / us, p[12] / us, p[13], p[14]);
    const double ns = (double)(p[16] ? p[16] : 1);
    fprintf(stderr, "walk prof slow blocks (> 35 us): %.0f (%.2f%%): setup %.2f walk %.2f overlay %.2f sort %.2f write %.2f"
                    " us | rounds %.2f T %.0f overlay %.0f tests %.2f\n", (double)p[16], 100.0 * p[16] / n, p[17] / ns / us,
            p[18] / ns / us, p[19] / ns / us, p[20] / ns / us, p[21] / ns / us, p[22] / ns, p[23] / ns, p[24] / ns, p[25] / ns);
    unsigned long long t[8];
    (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(topk_prof), sizeof(t));
    const double c = (double)t[0];
    fprintf(stderr, "topk_sort: %.0f calls, T %.0f, C %.0f, bitonic %.0f, hist+select %.2f us, rank %.2f us per call\n",
            c, t[1] / c, t[3] / c, (double)t[2], t[4] / c / us, t[5] / c / us);
  }
#endif
  return hipGetLastError();
}

// ------------------------------------------------------------------ apply residual updates

__global__ __launch_bounds__(256) void apply_kernel(int64_t* __restrict__ res, int64_t stride,
                                                    const int64_t* __restrict__ upd, int64_t n, uint64_t id_base,
                                                    uint64_t* __restrict__ kn, uint32_t* __restrict__ lo,
                                                    const uint32_t* __restrict__ labels, WalkIndex w, int walk,
                                                    WalkIndex nx, int pend) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t* u = upd + i * (D + 1);
  const int64_t node = u[0];
#pragma unroll
  for (int d = 0; d < D; ++d) res[d * stride + node] = u[1 + d];
  uint64_t K;                                 // the node-only key of the new state
  uint32_t l1, l3;
  node_prep(u[1], u[2], u[3], u[4], id_base + (uint64_t)node, K, l1, l3);
  if (kn) {                                   // keep the scan's node-only score terms current
    kn[node] = K;
    lo[node] = l1;
    lo[stride + node] = l3;
  }
  if (walk) {                                 // leave the sorted walk, join the overlay (once)
    const uint32_t p = w.pos[node];
    if (p != ~0u) {
      w.sk[p] = WK_INVALID;
      w.pos[node] = ~0u;
    }
    const int64_t r[D] = {u[1], u[2], u[3], u[4]};
    if (atomicExch(&w.in_ovl[node], 1u) == 0u) {
      overlay_add(w, node, r, labels[node], K);
    } else {                                  // already there: refresh its state copy
      const uint32_t i = w.ovl_idx[node];
#pragma unroll
      for (int d = 0; d < D; ++d) w.ovl_res[d * w.sstride + i] = r[d];
      w.ovl_kn[i] = K;
    }
    if (pend) {                               // the index being rebuilt: overlay only (walk_switch
      if (atomicExch(&nx.in_ovl[node], 1u) == 0u) {   // drops its sorted entry)
        overlay_add(nx, node, r, labels[node], K);
      } else {
        const uint32_t i = nx.ovl_idx[node];
#pragma unroll
        for (int d = 0; d < D; ++d) nx.ovl_res[d * nx.sstride + i] = r[d];
        nx.ovl_kn[i] = K;
      }
    }
  }
}

hipError_t launch_apply(hipStream_t s, int64_t* res, int64_t stride, const int64_t* upd, int64_t n, uint64_t id_base,
                        uint64_t* kn, uint32_t* lo, const uint32_t* labels, const WalkIndex* w,
                        const WalkIndex* nx) {
  if (n <= 0) return hipSuccess;
  const WalkIndex none{};
  hipLaunchKernelGGL(apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, res, stride, upd, n, id_base,
                     kn, lo, labels, w ? *w : none, w ? 1 : 0, (w && nx) ? *nx : none, (w && nx) ? 1 : 0);
  return hipGetLastError();
}

// ------------------------------------------------------------------ inventory deltas (sec. 8f row 3)

__global__ __launch_bounds__(256) void scatter_nodes_kernel(int64_t* __restrict__ res, int64_t* __restrict__ res0,
                                                            int64_t stride, uint32_t* __restrict__ labels,
                                                            int32_t* __restrict__ island,
                                                            const NodeUpd* __restrict__ upd, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const NodeUpd u = upd[i];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    res[d * stride + u.local] = u.res[d];
    res0[d * stride + u.local] = u.res[d];
  }
  labels[u.local] = u.labels;
  island[u.local] = u.island;
}

hipError_t launch_scatter_nodes(hipStream_t s, int64_t* res, int64_t* res0, int64_t stride, uint32_t* labels,
                                int32_t* island, const NodeUpd* upd, int64_t n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_nodes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, res, res0, stride,
                     labels, island, upd, n);
  return hipGetLastError();
}

}  // namespace pe
