// Micro-benchmark: issue cost of the instructions the fit/scan kernels are built from (gfx950).
// hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu && tools/ubench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2000
#define REP8(x) x x x x x x x x

__global__ __launch_bounds__(256) void k_cmp64(int64_t* out, int64_t a0, int64_t b0) {
  int64_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t m0, m1, m2, m3;
    REP8(asm volatile("v_cmp_le_i64_e64 %0, %4, %5\n v_cmp_le_i64_e64 %1, %5, %4\n v_cmp_lt_i64_e64 %2, %4, %5\n v_cmp_gt_i64_e64 %3, %4, %5"
                      : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(a), "v"(b));)
    acc ^= m0 ^ m1 ^ m2 ^ m3;
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_cmp32(int64_t* out, int a0, int b0) {
  int a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t m0, m1, m2, m3;
    REP8(asm volatile("v_cmp_le_i32_e64 %0, %4, %5\n v_cmp_le_i32_e64 %1, %5, %4\n v_cmp_lt_i32_e64 %2, %4, %5\n v_cmp_gt_i32_e64 %3, %4, %5"
                      : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(a), "v"(b));)
    acc ^= m0 ^ m1 ^ m2 ^ m3;
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_cmp64_sgpr(int64_t* out, int64_t a0, int64_t b0) {
  int64_t a = a0 + threadIdx.x;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    uint64_t m0, m1, m2, m3;
    REP8(asm volatile("v_cmp_le_i64_e64 %0, %4, %5\n v_cmp_le_i64_e64 %1, %4, %5\n v_cmp_lt_i64_e64 %2, %4, %5\n v_cmp_gt_i64_e64 %3, %4, %5"
                      : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "s"(b0), "v"(a));)
    acc ^= m0 ^ m1 ^ m2 ^ m3;
  }
  if (acc == 0x1234567) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_writelane(int64_t* out, int a0) {
  uint32_t v0 = threadIdx.x, v1 = 0, v2 = 0, v3 = 0;
  uint32_t s = a0;
  for (int i = 0; i < ITERS; ++i) {
    REP8(asm volatile("v_writelane_b32 %0, %4, 3\n v_writelane_b32 %1, %4, 9\n v_writelane_b32 %2, %4, 17\n v_writelane_b32 %3, %4, 33"
                      : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s));)
  }
  if ((v0 ^ v1 ^ v2 ^ v3) == 0x1234567) out[0] = v0;
}

__global__ __launch_bounds__(256) void k_addc(int64_t* out, int a0) {
  uint32_t v0 = threadIdx.x, v1 = 1, v2 = 2, v3 = 3;
  uint64_t m = (uint64_t)a0 * 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < ITERS; ++i) {
    REP8(asm volatile("v_addc_co_u32_e64 %0, s[60:61], %0, %0, %4\n v_addc_co_u32_e64 %1, s[60:61], %1, %1, %4\n "
                      "v_addc_co_u32_e64 %2, s[60:61], %2, %2, %4\n v_addc_co_u32_e64 %3, s[60:61], %3, %3, %4"
                      : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(m) : "s60", "s61");)
  }
  if ((v0 ^ v1 ^ v2 ^ v3) == 0x1234567) out[0] = v0;
}

__global__ __launch_bounds__(256) void k_add32(int64_t* out, int a0) {
  uint32_t v0 = threadIdx.x, v1 = 1, v2 = 2, v3 = 3;
  for (int i = 0; i < ITERS; ++i) {
    REP8(asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                      : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(a0));)
  }
  if ((v0 ^ v1 ^ v2 ^ v3) == 0x1234567) out[0] = v0;
}

__global__ __launch_bounds__(256) void k_salu_and(int64_t* out, int a0) {
  uint64_t s0 = a0, s1 = 3, s2 = 5, s3 = 7;
  for (int i = 0; i < ITERS; ++i) {
    REP8(asm volatile("s_and_b64 %0, %0, %1\n s_and_b64 %1, %1, %2\n s_and_b64 %2, %2, %3\n s_and_b64 %3, %3, %0"
                      : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));)
  }
  if ((s0 ^ s1 ^ s2 ^ s3) == 0x1234567) out[0] = s0;
}

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  int64_t* out;
  hipMalloc(&out, 64);
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  for (int wps = 1; wps <= 8; wps *= 2) {     // waves per SIMD
    const int blocks = cus * wps;             // 256-thread blocks = 4 waves = one per SIMD
    const double instrs = (double)blocks * 4 * ITERS * 32;  // wave-instructions
    const double per_simd = instrs / (cus * 4);
    auto rep = [&](const char* name, float ms) {
      printf("wps=%d %-14s %8.3f ms  %6.2f cycles/instr/SIMD @2.4GHz\n", wps, name, ms, ms * 1e-3 * 2.4e9 / per_simd);
    };
    rep("v_cmp_i64", timeit([&] { hipLaunchKernelGGL(k_cmp64, blocks, 256, 0, 0, out, 5, 7); }));
    rep("v_cmp_i64_sgpr", timeit([&] { hipLaunchKernelGGL(k_cmp64_sgpr, blocks, 256, 0, 0, out, 5, 7); }));
    rep("v_cmp_i32", timeit([&] { hipLaunchKernelGGL(k_cmp32, blocks, 256, 0, 0, out, 5, 7); }));
    rep("v_writelane", timeit([&] { hipLaunchKernelGGL(k_writelane, blocks, 256, 0, 0, out, 5); }));
    rep("v_addc_co", timeit([&] { hipLaunchKernelGGL(k_addc, blocks, 256, 0, 0, out, 5); }));
    rep("v_add_u32", timeit([&] { hipLaunchKernelGGL(k_add32, blocks, 256, 0, 0, out, 5); }));
    rep("s_and_b64", timeit([&] { hipLaunchKernelGGL(k_salu_and, blocks, 256, 0, 0, out, 5); }));
  }
  return 0;
}
