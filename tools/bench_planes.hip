// Variant bench of the bit-plane fit kernel (what bounds it: store, count reduction, code loads?).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench_planes.hip -o tools/bench_planes && tools/bench_planes
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x32 load_planes8(const u32x4* __restrict__ p) {
  u32x32 r;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const u32x4 v = p[s * 64];
    r[4 * s] = v.x; r[4 * s + 1] = v.y; r[4 * s + 2] = v.z; r[4 * s + 3] = v.w;
  }
  return r;
}
__device__ __forceinline__ void plane_sel(u32x4& a, uint32_t idx4, const u32x32& A, const u32x32& B, const u32x32& C,
                                          const u32x32& Dq) {
  asm volatile("s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\t"
               "v_mov_b32_e32 %0, v32\n\tv_mov_b32_e32 %1, v33\n\tv_mov_b32_e32 %2, v34\n\tv_mov_b32_e32 %3, v35\n\t"
               "s_set_gpr_idx_off"
               : "=v"(a.x), "=v"(a.y), "=v"(a.z), "=v"(a.w)
               : "s"(idx4), "{v[32:63]}"(A), "{v[64:95]}"(B), "{v[96:127]}"(C), "{v[128:159]}"(Dq));
}
__device__ __forceinline__ void plane_and(u32x4& a, uint32_t idx4, const u32x32& A, const u32x32& B, const u32x32& C,
                                          const u32x32& Dq) {
  asm volatile("s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\t"
               "v_and_b32_e32 %0, v32, %0\n\tv_and_b32_e32 %1, v33, %1\n\tv_and_b32_e32 %2, v34, %2\n\t"
               "v_and_b32_e32 %3, v35, %3\n\ts_set_gpr_idx_off"
               : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w)
               : "s"(idx4), "{v[32:63]}"(A), "{v[64:95]}"(B), "{v[96:127]}"(C), "{v[128:159]}"(Dq));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t writelane_s(uint32_t v, uint32_t x, uint32_t lane) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 3\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "s"(lane) : "m0");
  return v;
}

// MODE bits: 1 store, 2 count, 4 nontemporal store, 8 batch-of-8 code loads, 16 block-major layout
template <int MODE>
__global__ __launch_bounds__(256) void k(const uint32_t* __restrict__ planes, int64_t nblk, const uint64_t* __restrict__ jcode,
                                         int64_t J, int64_t jpw, int64_t row_words, uint32_t* __restrict__ mask,
                                         unsigned long long* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = wave_id % nblk;
  const int64_t j0 = (wave_id / nblk) * jpw;
  if (j0 >= J) return;
  const int64_t j1 = min(J, j0 + jpw);
  const u32x4* pb = reinterpret_cast<const u32x4*>(planes + blk * 32 * 256) + lane;
  const u32x32 A = load_planes8(pb), B = load_planes8(pb + 8 * 64), C = load_planes8(pb + 16 * 64),
               Dq = load_planes8(pb + 24 * 64);
  const int64_t col = blk * 256 + lane * 4;
  const bool in_row = col < row_words;
  u32x4* out = (MODE & 16) ? reinterpret_cast<u32x4*>(mask + blk * J * 256) + lane
                           : reinterpret_cast<u32x4*>(mask + col);
  const int64_t row4 = (MODE & 16) ? 64 : row_words / 4;
  uint32_t acc = 0, sink = 0;
  auto one = [&](int64_t j, uint64_t c) {
    u32x4 f;
    plane_sel(f, (uint32_t)c & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 7) & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 14) & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 21) & 127, A, B, C, Dq);
    plane_and(f, (uint32_t)(c >> 28) & 127, A, B, C, Dq);
    if (MODE & 1) {
      if (in_row) {
        if (MODE & 4) __builtin_nontemporal_store(f, out + j * row4);
        else out[j * row4] = f;
      }
    } else {
      sink ^= f.x ^ f.y ^ f.z ^ f.w;
    }
    if (MODE & 2) {
      const uint32_t n = wave_sum(__popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w));
      const uint32_t kk = (uint32_t)((j - j0) & 63);
      acc = writelane_s(acc, n, kk);
      if (kk == 63 || j + 1 == j1) {
        const int64_t jb = j - kk;
        if ((uint32_t)lane <= kk && acc) atomicAdd(&counts[jb + lane], (unsigned long long)acc);
        acc = 0;
      }
    }
  };
  if (MODE & 8) {
    for (int64_t jj = j0; jj < j1; jj += 8) {
      uint64_t c[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = jcode[jj + i];   // codes padded by 8
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (jj + i < j1) one(jj + i, c[i]);
    }
  } else {
    for (int64_t j = j0; j < j1; ++j) one(j, jcode[j]);
  }
  if (!(MODE & 1) && sink == 0x12345) mask[0] = sink;
}

template <int MODE>
float run(const uint32_t* planes, int64_t nblk, const uint64_t* jc, int64_t J, int64_t row_words, uint32_t* mask,
          unsigned long long* counts) {
  const int64_t ranges = (16384 + nblk - 1) / nblk;
  const int64_t jpw = ((J + ranges - 1) / ranges + 7) / 8 * 8;
  const int64_t waves = nblk * ((J + jpw - 1) / jpw);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<MODE>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, planes, nblk, jc, J, jpw, row_words, mask, counts);
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(k<MODE>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, planes, nblk, jc, J, jpw, row_words, mask, counts);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int64_t N = 1000000, J = 100000;
  const int64_t nblk = (N + 8191) / 8192, row_words = ((N + 31) / 32 + 3) / 4 * 4;
  std::vector<uint32_t> hp((size_t)nblk * 32 * 256);
  uint64_t x = 88172645463325252ull;
  for (auto& v : hp) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x | (uint32_t)(x >> 32); }
  std::vector<uint64_t> hj((size_t)J + 8);
  for (auto& c : hj) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    c = 0;
    for (int f = 0; f < 5; ++f) c |= (uint64_t)(4 * ((x >> (5 * f)) & 31)) << (7 * f);
  }
  uint32_t *planes, *mask;
  uint64_t* jc;
  unsigned long long* counts;
  hipMalloc(&planes, hp.size() * 4);
  hipMalloc(&jc, hj.size() * 8);
  hipMalloc(&mask, (size_t)J * nblk * 256 * 4);
  hipMalloc(&counts, (size_t)J * 8);
  hipMemcpy(planes, hp.data(), hp.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(jc, hj.data(), hj.size() * 8, hipMemcpyHostToDevice);
  const double bytes = (double)J * row_words * 4;
  auto rep = [&](const char* name, float ms) { printf("%-28s %7.3f ms  %6.2f TB/s of mask\n", name, ms, bytes / ms / 1e9); };
  rep("store+count", run<3>(planes, nblk, jc, J, row_words, mask, counts));
  rep("store only", run<1>(planes, nblk, jc, J, row_words, mask, counts));
  rep("count only (no store)", run<2>(planes, nblk, jc, J, row_words, mask, counts));
  rep("select only", run<0>(planes, nblk, jc, J, row_words, mask, counts));
  rep("store+count nt", run<7>(planes, nblk, jc, J, row_words, mask, counts));
  rep("store nt", run<5>(planes, nblk, jc, J, row_words, mask, counts));
  rep("store+count batch8", run<11>(planes, nblk, jc, J, row_words, mask, counts));
  rep("store batch8", run<9>(planes, nblk, jc, J, row_words, mask, counts));
  rep("store nt batch8", run<13>(planes, nblk, jc, J, row_words, mask, counts));
  rep("select batch8", run<8>(planes, nblk, jc, J, row_words, mask, counts));
  rep("blockmajor store+count", run<19>(planes, nblk, jc, J, row_words, mask, counts));
  rep("blockmajor store", run<17>(planes, nblk, jc, J, row_words, mask, counts));
  rep("blockmajor store nt", run<21>(planes, nblk, jc, J, row_words, mask, counts));
  rep("blockmajor store+count nt", run<23>(planes, nblk, jc, J, row_words, mask, counts));
  // plain store roofline: hipMemsetD32 of the mask
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipMemsetD32((hipDeviceptr_t)mask, 0, (size_t)J * row_words);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipMemsetD32((hipDeviceptr_t)mask, r, (size_t)J * row_words);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  rep("hipMemsetD32 (write roofline)", ms / 5);
  return 0;
}
