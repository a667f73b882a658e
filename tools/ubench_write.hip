// HBM write-pattern microbenchmark for the fit-mask output (12.6 GB per launch at cfg5).
// What bounds the planes kernel's stores: the pattern (one sequential stream per wave vs a
// chip-wide linear sweep), the occupancy (waves per CU), the cache policy, the store spacing?
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_write.hip -o tools/ubench_write && tools/ubench_write
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int POL>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (POL == 0) *p = v;
  else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
  else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// delay: DLY dependent VALU ops between stores (the real kernel issues ~40 VALU per store)
template <int DLY>
__device__ __forceinline__ u32x4 spin(u32x4 v) {
#pragma unroll
  for (int i = 0; i < DLY; ++i) asm volatile("v_xor_b32 %0, 1, %0" : "+v"(v.x));
  return v;
}

// Each wave owns `chunk` consecutive KiB and writes them in order (the block-major fit pattern).
template <int POL, int DLY>
__global__ __launch_bounds__(256) void streams(u32x4* __restrict__ out, int64_t nwaves, int64_t chunk) {
  extern __shared__ int occ[];
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nwaves) return;
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  u32x4* p = out + w * chunk * 64 + lane;
  for (int64_t i = 0; i < chunk; ++i) {
    v = spin<DLY>(v);
    st<POL>(p + i * 64, v);
  }
  if (v.x == 0xdeadbeef) occ[0] = 1;
}

// Persistent waves sweep the buffer linearly: iteration i of wave w writes KiB i*W + w.
template <int POL, int DLY>
__global__ __launch_bounds__(256) void linear(u32x4* __restrict__ out, int64_t nwaves, int64_t kib) {
  extern __shared__ int occ[];
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  for (int64_t k = w; k < kib; k += nwaves) {
    v = spin<DLY>(v);
    st<POL>(out + k * 64 + lane, v);
  }
  if (v.x == 0xdeadbeef) occ[0] = 1;
}

// Block-major fit pattern, exactly: wave (blk, range) writes jobs [j0, j1) of slab blk.
template <int POL, int DLY>
__global__ __launch_bounds__(256) void fitlike(u32x4* __restrict__ out, int64_t nblk, int64_t J, int64_t jpw) {
  extern __shared__ int occ[];
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t blk = wave_id % nblk;
  const int64_t j0 = (wave_id / nblk) * jpw;
  if (j0 >= J) return;
  const int64_t j1 = j0 + jpw < J ? j0 + jpw : J;
  u32x4 v = {(uint32_t)wave_id, 1u, 2u, 3u};
  u32x4* p = out + blk * J * 64 + lane;
  for (int64_t j = j0; j < j1; ++j) {
    v = spin<DLY>(v);
    st<POL>(p + j * 64, v);
  }
  if (v.x == 0xdeadbeef) occ[0] = 1;
}

// One-shot waves: wave w writes K KiB; group of G consecutive waves interleave (G = 1: each wave
// its own K contiguous KiB).  KiB i of wave w (group q = w / G, member m = w % G) lands at
// q*G*K + i*G + m.
template <int POL, int DLY>
__global__ __launch_bounds__(256) void oneshot(u32x4* __restrict__ out, int64_t kib, int64_t K, int64_t G) {
  extern __shared__ int occ[];
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t q = w / G, m = w % G;
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  for (int64_t i = 0; i < K; ++i) {
    const int64_t k = q * G * K + i * G + m;
    if (k >= kib) break;
    v = spin<DLY>(v);
    st<POL>(out + k * 64 + lane, v);
  }
  if (v.x == 0xdeadbeef) occ[0] = 1;
}

// Persistent linear sweep with a soft grid barrier: every S steps a wave adds 1 to one of 16
// counters (own cache lines); before step t it waits until the counters' sum shows that every
// wave finished step t - D.  Bounds the drift between waves, i.e. the width of the written window.
template <int POL>
__global__ __launch_bounds__(256) void linear_sync(u32x4* __restrict__ out, int64_t nwaves, int64_t kib, int S, int D,
                                                   unsigned* __restrict__ ctr) {
  extern __shared__ int occ[];
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  int64_t step = 0;
  for (int64_t k = w; k < kib; k += nwaves, ++step) {
    if (step >= D && step % S == 0) {
      const unsigned need = (unsigned)(nwaves * ((step - D) / S));
      for (;;) {
        unsigned c = lane < 16 ? __hip_atomic_load(&ctr[lane * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
        c = __shfl(c, 0, 64);
        if (c >= need) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    st<POL>(out + k * 64 + lane, v);
    if (step % S == S - 1 && lane == 0)
      __hip_atomic_fetch_add(&ctr[(w % 16) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (v.x == 0xdeadbeef) occ[0] = 1;
}

// One-shot waves with a per-wave read of R KiB from an L2-resident 4 MB buffer (the plane load),
// then K KiB written with G-wave interleave (oneshot's layout).
template <int DW>
__global__ __launch_bounds__(256) void readwrite(u32x4* __restrict__ out, int64_t kib, int64_t K, int64_t G,
                                                 const u32x4* __restrict__ src, int R) {
  extern __shared__ int occ[];
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t q = w / G, m = w % G;
  const u32x4* s = src + (w % 4096) * (int64_t)R * 64 + lane;   // 4096 distinct slices
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  for (int r = 0; r < R; ++r) v ^= s[r * 64];
  for (int64_t i = 0; i < K; ++i) {
    const int64_t k = q * G * K + i * G + m;
    if (k >= kib) break;
    if constexpr (DW == 4) {
      out[k * 64 + lane] = v;
    } else {
      // K counts 1-KiB units; each unit = 4 dword stores of 256 B (2048-node waves)
      uint32_t* o = reinterpret_cast<uint32_t*>(out + k * 64);
      o[lane] = v.x;
      o[64 + lane] = v.y;
      o[128 + lane] = v.z;
      o[192 + lane] = v.w;
    }
    v.x += 1;
  }
  if (v.x == 0xdeadbeef) occ[0] = 1;
}

// Linear sweep with a workgroup barrier every S steps: the 4 waves of a CU stay in lockstep.
template <int S>
__global__ __launch_bounds__(256) void linear_bar(u32x4* __restrict__ out, int64_t nwaves, int64_t kib) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  const int64_t steps = (kib + nwaves - 1) / nwaves;
  for (int64_t i = 0; i < steps; ++i) {
    const int64_t k = i * nwaves + w;
    v = spin<40>(v);
    if (k < kib) out[k * 64 + lane] = v;
    if (i % S == S - 1) __syncthreads();
  }
}

// The rows fit pattern: wave (blk, r) writes KiB (r + i*R) * pitch + blk for its jobs i (row pitch
// `pitch` KiB, `nblk` KiB written per row; pitch > nblk leaves a hole at the end of every row).
__global__ __launch_bounds__(256) void rows(u32x4* __restrict__ out, int64_t nblk, int64_t pitch, int64_t J,
                                            int64_t R) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t blk = w % nblk, r = w / nblk;
  if (r >= R) return;
  u32x4 v = {(uint32_t)w, 1u, 2u, 3u};
  for (int64_t j = r; j < J; j += R) {
    v = spin<40>(v);
    out[(j * pitch + blk) * 64 + lane] = v;
  }
}

static float time_it(void (*launch)(void*), void* arg, hipEvent_t a, hipEvent_t b, int reps = 5) {
  launch(arg);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a, 0);
    launch(arg);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best;
}

struct Arg {
  u32x4* out;
  int64_t kib, nwaves, chunk, nblk, J, jpw;
  int lds;
  int kind, pol, dly;
  int S, D;
  unsigned* ctr;
  const u32x4* src;
  int R;
};

template <int POL, int DLY>
static void go(const Arg& a) {
  if (a.kind == 0) {
    hipLaunchKernelGGL((streams<POL, DLY>), dim3((unsigned)((a.nwaves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.nwaves,
                       a.chunk);
  } else if (a.kind == 1) {
    hipLaunchKernelGGL((linear<POL, DLY>), dim3((unsigned)((a.nwaves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.nwaves,
                       a.kib);
  } else if (a.kind == 4) {
    hipMemsetAsync(a.ctr, 0, 16 * 32 * 4, 0);
    hipLaunchKernelGGL((linear_sync<POL>), dim3((unsigned)((a.nwaves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.nwaves,
                       a.kib, a.S, a.D, a.ctr);
  } else if (a.kind == 5 || a.kind == 6) {
    const int64_t waves = (a.kib + a.chunk - 1) / a.chunk;
    if (a.kind == 5)
      hipLaunchKernelGGL((readwrite<4>), dim3((unsigned)((waves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.kib, a.chunk,
                         a.nwaves, a.src, a.R);
    else
      hipLaunchKernelGGL((readwrite<1>), dim3((unsigned)((waves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.kib, a.chunk,
                         a.nwaves, a.src, a.R);
  } else if (a.kind == 7) {
    const dim3 g((unsigned)((a.nwaves + 3) / 4));
    if (a.S == 1) hipLaunchKernelGGL(linear_bar<1>, g, dim3(256), a.lds, 0, a.out, a.nwaves, a.kib);
    else if (a.S == 4) hipLaunchKernelGGL(linear_bar<4>, g, dim3(256), a.lds, 0, a.out, a.nwaves, a.kib);
    else hipLaunchKernelGGL(linear_bar<16>, g, dim3(256), a.lds, 0, a.out, a.nwaves, a.kib);
  } else if (a.kind == 8) {
    hipLaunchKernelGGL(rows, dim3((unsigned)((a.nblk * a.R + 3) / 4)), dim3(256), a.lds, 0, a.out, a.nblk, a.chunk,
                       a.J, (int64_t)a.R);
  } else if (a.kind == 3) {
    const int64_t waves = (a.kib + a.chunk - 1) / a.chunk;
    hipLaunchKernelGGL((oneshot<POL, DLY>), dim3((unsigned)((waves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.kib,
                       a.chunk, a.nwaves);
  } else {
    const int64_t waves = a.nblk * ((a.J + a.jpw - 1) / a.jpw);
    hipLaunchKernelGGL((fitlike<POL, DLY>), dim3((unsigned)((waves + 3) / 4)), dim3(256), a.lds, 0, a.out, a.nblk, a.J,
                       a.jpw);
  }
}

static void launch(void* p) {
  const Arg& a = *(const Arg*)p;
  switch (a.pol * 100 + a.dly) {
    case 0: go<0, 0>(a); break;
    case 40: go<0, 40>(a); break;
    case 100: go<1, 0>(a); break;
    case 140: go<1, 40>(a); break;
    case 200: go<2, 0>(a); break;
    case 240: go<2, 40>(a); break;
  }
}

static void memset_launch(void* p) {
  const Arg& a = *(const Arg*)p;
  hipMemsetD32((hipDeviceptr_t)a.out, 0, (size_t)a.kib * 256);
}

int main() {
  const int64_t nblk = 123, J = 100000;
  const int64_t kib = nblk * J;   // 12.6 GB
  const double bytes = (double)kib * 1024.0;
  u32x4* out;
  CHK(hipMalloc(&out, (size_t)(132 * J) * 1024));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  Arg g{};
  g.out = out;
  g.kib = kib;
  g.nblk = nblk;
  g.J = J;
  auto rep = [&](const char* name, float ms) { printf("%-58s %7.3f ms  %5.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12); };
  rep("hipMemsetD32", time_it(memset_launch, &g, a, b));
  char name[160];
  g.lds = 98304;   // one workgroup (4 waves) per CU, like the rows kernel
  g.pol = 0;
  g.dly = 40;
  struct RowCase { int64_t nblk, pitch, R; };
  for (int pass = 0; pass < 2; ++pass)
    for (RowCase c : {RowCase{123, 123, 8}, RowCase{123, 128, 8}, RowCase{128, 128, 8}, RowCase{123, 123, 16},
                      RowCase{123, 128, 16}, RowCase{128, 128, 16}, RowCase{123, 124, 8}, RowCase{123, 132, 8}}) {
      g.kind = 8;
      g.nblk = c.nblk;
      g.chunk = c.pitch;
      g.R = (int)c.R;
      g.lds = c.R == 8 ? 98304 : 0;
      const float ms = time_it(launch, &g, a, b);
      snprintf(name, sizeof name, "rows nblk=%ld pitch=%ld R=%ld (bytes/written %.3f)", (long)c.nblk, (long)c.pitch,
               (long)c.R, (double)c.nblk / 123.0);
      // rate over the bytes actually written
      printf("%-58s %7.3f ms  %5.2f TB/s written\n", name, ms, bytes * (double)c.nblk / 123.0 / (ms * 1e-3) / 1e12);
    }
  rep("hipMemsetD32 again", time_it(memset_launch, &g, a, b));
  hipFree(out);
  return 0;
}
