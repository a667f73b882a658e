// Micro-benchmark 3: issue cost of all-VGPR candidates for the fit step (inline constants, 3-input ops)
// hipcc --offload-arch=gfx950 -O3 tools/ubench_valu3.hip -o tools/ubench_valu3 && tools/ubench_valu3
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

#define OPS8I(op, tail) op " %0, %0, " tail "\n " op " %1, %1, " tail "\n " op " %2, %2, " tail "\n " op " %3, %3, " tail "\n " \
  op " %4, %4, " tail "\n " op " %5, %5, " tail "\n " op " %6, %6, " tail "\n " op " %7, %7, " tail
#define OPS8U(op, tail) op " %0, " tail "\n " op " %1, " tail "\n " op " %2, " tail "\n " op " %3, " tail "\n " \
  op " %4, " tail "\n " op " %5, " tail "\n " op " %6, " tail "\n " op " %7, " tail

K8(k_add_inl, OPS8I("v_add_u32", "1"), VV)
K8(k_alignbit, OPS8I("v_alignbit_b32", "%8, 31"), VV)
K8(k_andor, OPS8I("v_and_or_b32", "%8, %8"), VV)
K8(k_lshlor, OPS8I("v_lshl_or_b32", "1, %8"), VV)
K8(k_add3, OPS8I("v_add3_u32", "%8, 1"), VV)
K8(k_bitop3, OPS8I("v_bitop3_b32", "%8, %8 bitop3:0x6c"), VV)
K8(k_ffbl, OPS8U("v_ffbl_b32", "%8"), VV)
K8(k_min, OPS8I("v_min_u32", "%8"), VV)
K8(k_xad, OPS8I("v_xad_u32", "%8, 1"), VV)

// new thermometer step, codes in VGPRs: t = x | ny ; u = t + 1 ; w = alignbit(w, u, 31)
template <int SG>
__global__ __launch_bounds__(256) void k_step3(int64_t* out, uint32_t s) {
  uint32_t x[8], w[8];
  for (int c = 0; c < 8; ++c) x[c] = threadIdx.x * (c + 3), w[c] = 0;
  uint32_t nyv[4];
  for (int r = 0; r < 4; ++r) nyv[r] = s + r + (threadIdx.x >> 6);
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        uint32_t t;
        if constexpr (SG)
          asm volatile("v_or_b32_e32 %0, %2, %3\n\tv_add_u32_e32 %0, 1, %0\n\tv_alignbit_b32 %1, %1, %0, 31"
                       : "=&v"(t), "+v"(w[c]) : "s"(s + r), "v"(x[c]));
        else
          asm volatile("v_or_b32_e32 %0, %2, %3\n\tv_add_u32_e32 %0, 1, %0\n\tv_alignbit_b32 %1, %1, %0, 31"
                       : "=&v"(t), "+v"(w[c]) : "v"(nyv[r]), "v"(x[c]));
      }
    }
    nyv[i & 3] ^= w[0];
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
  for (int wps = 4; wps <= 8; wps *= 2) {
    const int blocks = cus * wps;
    auto rep = [&](const char* name, float ms, double instr_per_wave) {
      const double per_simd = (double)blocks * 4 * instr_per_wave / (cus * 4);
      printf("wps=%d %-18s %8.3f ms  %6.2f cyc/unit/SIMD @2.4GHz\n", wps, name, ms, ms * 1e-3 * 2.4e9 / per_simd);
    };
    const double n8 = 32.0 * ITERS;
#define RUN(k) rep(#k, timeit([&] { hipLaunchKernelGGL(k, blocks, 256, 0, 0, out, 5u); }), n8)
    RUN(k_add_vv);
    RUN(k_add_inl);
    RUN(k_alignbit);
    RUN(k_andor);
    RUN(k_lshlor);
    RUN(k_add3);
    RUN(k_bitop3);
    RUN(k_ffbl);
    RUN(k_min);
    RUN(k_xad);
    rep("step3_vgpr(/step)", timeit([&] { hipLaunchKernelGGL(k_step3<0>, blocks, 256, 0, 0, out, 5u); }), n8);
    rep("step3_sgpr(/step)", timeit([&] { hipLaunchKernelGGL(k_step3<1>, blocks, 256, 0, 0, out, 5u); }), n8);
  }
  return 0;
}
