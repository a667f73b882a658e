// LDS digit-plane fit mask (gfx950): the exact fit path for batches with any number of distinct
// request values (pe_kernels.h, LdsSpec).  Two kernels per fit step:
//
//   node_ranks   per shard node and digit field: R = #{batch values <= residual} (binary search over
//                the field's sorted values), plus the folded single-value dimensions -> aux
//   fit_mask_lds one workgroup per (node block, job phase): builds the block's threshold planes in
//                LDS from the ranks, then 16 waves stream the jobs through them
//
// The fit kernel itself is in pe_lds_kernel.h (instantiated per block size in pe_lds_w{1,2,4}.hip).
// HBM traffic per step is the mask (written once, whole 128-B lines) plus the ranks (4 B per node
// and field, read by each of the R phases of a block) and the job codes (32 B per job, read by every
// block, mostly from L2): the same store-bound roofline as the bit-plane path.
#include "pe_lds_kernel.h"

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
  for (int f = 0; f < sp.nf + sp.nx; ++f) {   // digit fields, then the crossed ones
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

// The fit kernel of the batch's shape and block size (pe_lds_kernel.h, one translation unit per W).
hipError_t launch_fit_mask_lds(hipStream_t s, int W, const int shape[4], const LdsSpec* spec, int nplanes,
                               const uint32_t* ranks, int64_t npad, const uint32_t* aux, int64_t nblk,
                               const uint16_t* codes, int64_t J, int64_t R, int64_t Tpad, int64_t pitch_bytes,
                               uint8_t* mask, uint32_t* slots, uint32_t* units) {
  if (J <= 0 || nblk <= 0 || R <= 0) return hipSuccess;
  const size_t lds = (size_t)nplanes * 2048 * W / 8;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const void* fn = W == 1   ? lds_kernel_w1(shape[0], shape[1], shape[2], shape[3])
                   : W == 2 ? lds_kernel_w2(shape[0], shape[1], shape[2], shape[3])
                   : W == 4 ? lds_kernel_w4(shape[0], shape[1], shape[2], shape[3])
                            : nullptr;
  if (!fn) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const uint2* c = reinterpret_cast<const uint2*>(codes);
  void* args[] = {(void*)&spec, (void*)&ranks, (void*)&npad, (void*)&aux,         (void*)&nblk,   (void*)&c,
                  (void*)&J,    (void*)&R,     (void*)&Tpad, (void*)&pitch_bytes, (void*)&mask,   (void*)&slots,
                  (void*)&units};
  e = hipLaunchKernel(fn, dim3((unsigned)(nblk * R)), dim3(LD_THREADS), args, lds, s);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

// Per-job counts from the fit kernel's count slots: slot s holds job rows[s] (~0: an empty slot).
__global__ __launch_bounds__(256) void lds_counts_kernel(const uint32_t* __restrict__ slots,
                                                         const uint32_t* __restrict__ rows, int64_t nslots,
                                                         unsigned long long* __restrict__ counts) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
  const uint32_t j = rows[s];
  if (j != ~0u) counts[j] = slots[s];
}

hipError_t launch_lds_counts(hipStream_t s, const uint32_t* slots, const uint32_t* rows, int64_t nslots,
                             unsigned long long* counts) {
  if (nslots <= 0) return hipSuccess;
  hipLaunchKernelGGL(lds_counts_kernel, dim3((unsigned)((nslots + 255) / 256)), dim3(256), 0, s, slots, rows, nslots,
                     counts);
  return hipGetLastError();
}

}  // namespace pe
