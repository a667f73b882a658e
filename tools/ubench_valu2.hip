// Micro-benchmark 2: is integer VALU issue 2 or 4 cycles per wave64 instruction on a SIMD-32?
// 8 independent chains per wave; VGPR-only vs SGPR operands; f32 vs int; the fit-mask step.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_valu2.hip -o tools/ubench_valu2 && tools/ubench_valu2
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 1000
#define REP4(x) x x x x

// 8 ops per asm block, ITERS*4 blocks -> 32*ITERS wave-instructions per wave
#define K8(name, fmt, cons)                                                                              \
  __global__ __launch_bounds__(256) void name(int64_t* out, uint32_t s) {                               \
    uint32_t v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, \
             v7 = v0 + 7, b = v0 * 3;                                                                    \
    for (int i = 0; i < ITERS; ++i) {                                                                    \
      REP4(asm volatile(fmt : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6),      \
                        "+v"(v7) : cons(b), "s"(s) : "s60", "s61", "vcc");)                              \
    }                                                                                                    \
    if ((v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7) == 0x1234567) out[0] = v0;                              \
  }
#define VV "v"
#define OPS8(op, src) op " %0, %0, " src "\n " op " %1, %1, " src "\n " op " %2, %2, " src "\n " op " %3, %3, " src "\n " \
  op " %4, %4, " src "\n " op " %5, %5, " src "\n " op " %6, %6, " src "\n " op " %7, %7, " src

K8(k_add_vv, OPS8("v_add_u32", "%8"), VV)
K8(k_add_vs, OPS8("v_add_u32", "%9"), VV)
K8(k_or_vv, OPS8("v_or_b32", "%8"), VV)
K8(k_xor_vs, OPS8("v_xor_b32", "%9"), VV)
K8(k_fadd_vv, OPS8("v_add_f32", "%8"), VV)
K8(k_fma_vv, "v_fma_f32 %0, %0, %8, %0\n v_fma_f32 %1, %1, %8, %1\n v_fma_f32 %2, %2, %8, %2\n v_fma_f32 %3, %3, %8, %3\n "
             "v_fma_f32 %4, %4, %8, %4\n v_fma_f32 %5, %5, %8, %5\n v_fma_f32 %6, %6, %8, %6\n v_fma_f32 %7, %7, %8, %7", VV)
K8(k_pkadd_u16, OPS8("v_pk_add_u16", "%8"), VV)
K8(k_addco_vv, "v_add_co_u32_e64 %0, s[60:61], %0, %8\n v_add_co_u32_e64 %1, s[60:61], %1, %8\n "
               "v_add_co_u32_e64 %2, s[60:61], %2, %8\n v_add_co_u32_e64 %3, s[60:61], %3, %8\n "
               "v_add_co_u32_e64 %4, s[60:61], %4, %8\n v_add_co_u32_e64 %5, s[60:61], %5, %8\n "
               "v_add_co_u32_e64 %6, s[60:61], %6, %8\n v_add_co_u32_e64 %7, s[60:61], %7, %8", VV)
K8(k_addco_vcc, "v_add_co_u32_e32 %0, vcc, %0, %8\n v_add_co_u32_e32 %1, vcc, %1, %8\n "
                "v_add_co_u32_e32 %2, vcc, %2, %8\n v_add_co_u32_e32 %3, vcc, %3, %8\n "
                "v_add_co_u32_e32 %4, vcc, %4, %8\n v_add_co_u32_e32 %5, vcc, %5, %8\n "
                "v_add_co_u32_e32 %6, vcc, %6, %8\n v_add_co_u32_e32 %7, vcc, %7, %8", VV)
K8(k_cmp_vv, "v_cmp_le_u32_e64 s[60:61], %0, %8\n v_cmp_le_u32_e64 s[60:61], %1, %8\n v_cmp_le_u32_e64 s[60:61], %2, %8\n "
             "v_cmp_le_u32_e64 s[60:61], %3, %8\n v_cmp_le_u32_e64 s[60:61], %4, %8\n v_cmp_le_u32_e64 s[60:61], %5, %8\n "
             "v_cmp_le_u32_e64 s[60:61], %6, %8\n v_cmp_le_u32_e64 s[60:61], %7, %8", VV)

// the thermometer fit step, 8 independent chunks: or, add_co (carry->SGPR), addc shift-in, s_bcnt, s_add
__global__ __launch_bounds__(256) void k_ftstep(int64_t* out, uint32_t s) {
  uint32_t x[8], w[8];
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * (c + 3), w[c] = 0;
  uint32_t pc = 0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t ny = s + i + r;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        uint32_t tmp, t;
        uint64_t fit;
        asm volatile("v_or_b32_e32 %0, %5, %6\n\t"
                     "v_add_co_u32_e64 %0, %1, %0, 1\n\t"
                     "v_addc_co_u32_e64 %2, vcc, %2, %2, %1\n\t"
                     "s_bcnt1_i32_b64 %4, %1\n\t"
                     "s_add_u32 %3, %3, %4"
                     : "=&v"(tmp), "=&s"(fit), "+v"(w[c]), "+s"(pc), "=&s"(t)
                     : "s"(ny), "v"(x[c])
                     : "vcc", "scc");
      }
    }
  }
  uint32_t a = pc;
  for (int c = 0; c < 8; ++c) a ^= w[c];
  if (a == 0x1234567) out[0] = a;
}

// the same step without the SALU count (3 VALU only)
__global__ __launch_bounds__(256) void k_ftstep_nosalu(int64_t* out, uint32_t s) {
  uint32_t x[8], w[8];
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * (c + 3), w[c] = 0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t ny = s + i + r;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        uint32_t tmp;
        uint64_t fit;
        asm volatile("v_or_b32_e32 %0, %3, %4\n\t"
                     "v_add_co_u32_e64 %0, %1, %0, 1\n\t"
                     "v_addc_co_u32_e64 %2, vcc, %2, %2, %1"
                     : "=&v"(tmp), "=&s"(fit), "+v"(w[c])
                     : "s"(ny), "v"(x[c])
                     : "vcc");
      }
    }
  }
  uint32_t a = 0;
  for (int c = 0; c < 8; ++c) a ^= w[c];
  if (a == 0x1234567) out[0] = a;
}

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  int64_t* out;
  hipMalloc(&out, 64);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("CUs %d, clock %d kHz\n", cus, p.clockRate);
  for (int wps = 2; wps <= 8; wps *= 2) {
    const int blocks = cus * wps;
    auto rep = [&](const char* name, float ms, double instr_per_wave) {
      const double per_simd = (double)blocks * 4 * instr_per_wave / (cus * 4);
      printf("wps=%d %-16s %8.3f ms  %6.2f cyc/wave-instr/SIMD @2.4GHz\n", wps, name, ms, ms * 1e-3 * 2.4e9 / per_simd);
    };
    const double n8 = 32.0 * ITERS;
#define RUN(k) rep(#k, timeit([&] { hipLaunchKernelGGL(k, blocks, 256, 0, 0, out, 5u); }), n8)
    RUN(k_add_vv);
    RUN(k_add_vs);
    RUN(k_or_vv);
    RUN(k_xor_vs);
    RUN(k_fadd_vv);
    RUN(k_fma_vv);
    RUN(k_pkadd_u16);
    RUN(k_addco_vv);
    RUN(k_addco_vcc);
    RUN(k_cmp_vv);
    rep("ftstep(per step)", timeit([&] { hipLaunchKernelGGL(k_ftstep, blocks, 256, 0, 0, out, 5u); }), 32.0 * ITERS);
    rep("ftstep_nosalu", timeit([&] { hipLaunchKernelGGL(k_ftstep_nosalu, blocks, 256, 0, 0, out, 5u); }), 32.0 * ITERS);
  }
  return 0;
}
