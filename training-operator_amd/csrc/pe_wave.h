// Wave-level building blocks shared by the fit-mask kernels (device code only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pe {

// Column sums of a 64 x 64 block: p[k] holds, per lane, a partial count of job k; returns F with
// F[l] = sum over all 64 lanes of p[sigma(l)] for a fixed permutation sigma of 0..63 (find it by
// reducing a probe, p[k] = (lane == 0) ? k : 0).  Six halving levels, each pairing two registers
// into one that carries both jobs on half the lanes: permlane32_swap (halves), permlane16_swap
// (rows), then DPP row_ror:8, row_half_mirror, quad_perm [2,3,0,1], [1,0,3,2] with a lane select.
// 141 VALU per 64 jobs, no dependent chains: 2.2 per job where a per-job wave sum costs ~12.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_pair(uint32_t x, uint32_t y, bool take_y) {
  const uint32_t tx = x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
  const uint32_t ty = y + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, CTRL, 0xf, 0xf, false);
  return take_y ? ty : tx;
}

__device__ __forceinline__ uint32_t reduce64x64(const uint32_t (&p)[64], int lane) {
  uint32_t s1[32], s2[16], s3[8], s4[4], s5[2];
#pragma unroll
  for (int m = 0; m < 32; ++m) {
    const auto r = __builtin_amdgcn_permlane32_swap(p[2 * m], p[2 * m + 1], false, false);
    s1[m] = r[0] + r[1];
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const auto r = __builtin_amdgcn_permlane16_swap(s1[2 * m], s1[2 * m + 1], false, false);
    s2[m] = r[0] + r[1];
  }
  const bool b8 = lane & 8, b4 = lane & 4, b2 = lane & 2, b1 = lane & 1;
#pragma unroll
  for (int m = 0; m < 8; ++m) s3[m] = dpp_pair<0x128>(s2[2 * m], s2[2 * m + 1], b8);   // row_ror:8
#pragma unroll
  for (int m = 0; m < 4; ++m) s4[m] = dpp_pair<0x141>(s3[2 * m], s3[2 * m + 1], b4);   // row_half_mirror
#pragma unroll
  for (int m = 0; m < 2; ++m) s5[m] = dpp_pair<0x4e>(s4[2 * m], s4[2 * m + 1], b2);   // quad_perm [2,3,0,1]
  return dpp_pair<0xb1>(s5[0], s5[1], b1);                                          // quad_perm [1,0,3,2]
}

// 16-job form of reduce64x64: p[k] per-lane partial counts of job k (k < 16); returns F with F[l] =
// the wave-wide sum of job sigma(l), the same on the four lanes of a quad (find sigma with the
// probe p[k] = (lane == 0) ? k : 0).  Four halving levels (permlane32_swap, permlane16_swap, DPP
// row_ror:8, row_half_mirror) then two quad adds: 41 VALU per 16 jobs, 16 registers of partials.
__device__ __forceinline__ uint32_t reduce16x64(const uint32_t (&p)[16], int lane) {
  uint32_t s1[8], s2[4], s3[2];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const auto r = __builtin_amdgcn_permlane32_swap(p[2 * m], p[2 * m + 1], false, false);
    s1[m] = r[0] + r[1];
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const auto r = __builtin_amdgcn_permlane16_swap(s1[2 * m], s1[2 * m + 1], false, false);
    s2[m] = r[0] + r[1];
  }
  const bool b8 = lane & 8, b4 = lane & 4;
#pragma unroll
  for (int m = 0; m < 2; ++m) s3[m] = dpp_pair<0x128>(s2[2 * m], s2[2 * m + 1], b8);   // row_ror:8
  uint32_t x = dpp_pair<0x141>(s3[0], s3[1], b4);                                     // row_half_mirror
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4e, 0xf, 0xf, false);         // quad_perm [2,3,0,1]
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xb1, 0xf, 0xf, false);         // quad_perm [1,0,3,2]
  return x;
}

}  // namespace pe
