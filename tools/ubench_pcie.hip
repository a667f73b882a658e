// Host <-> device microbenchmark for the aggregation call path (pe_pg_min_resources): what a call
// of the operator's size (one job, a few hundred bytes) and a 1M-job batch (~170 MB) can cost.
//   - launch + hipStreamSynchronize of an empty kernel; launch + spin on a flag the kernel writes
//     into coherent pinned host memory
//   - one block reading B bytes zero-copy from pinned host memory into LDS, then the flag
//   - H2D of a small pinned buffer + kernel + sync
//   - bandwidths: DMA H2D / D2H pinned and pageable, zero-copy kernel reads / writes, host memcpy
//     into pinned memory on 1 and 8 threads, hipHostRegister of a 128 MB array
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread tools/ubench_pcie.hip -o tools/ubench_pcie && tools/ubench_pcie
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void empty_kernel() {}

__global__ void flag_kernel(uint32_t* flag, uint32_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one block: copy `bytes` from host memory into LDS (16 B per lane per step), sum it, write 64 B
// of output to host memory, then the flag
__global__ __launch_bounds__(256) void stage_kernel(const u32x4* __restrict__ in, int n16, uint32_t* out,
                                                    uint32_t* flag, uint32_t v) {
  __shared__ u32x4 lds[4096];
  for (int i = threadIdx.x; i < n16; i += blockDim.x) lds[i] = in[i];
  __syncthreads();
  uint32_t s = 0;
  for (int i = threadIdx.x; i < n16; i += blockDim.x) s += lds[i].x;
  if (threadIdx.x < 16) out[threadIdx.x] = s;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ in, int64_t n16, uint32_t* sink) {
  uint32_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    s += in[i].x;
  if (s == 0x9e3779b9u) sink[0] = s;
}

__global__ __launch_bounds__(256) void write_kernel(u32x4* __restrict__ out, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static void spin_flag(volatile uint32_t* f, uint32_t v) {
  while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != v) __builtin_ia32_pause();
}

int main() {
  CHK(hipSetDevice(0));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const unsigned zc = hipHostMallocCoherent | hipHostMallocMapped;
  uint32_t* hflag;
  CHK(hipHostMalloc((void**)&hflag, 64, zc));
  uint32_t* dflag;
  CHK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
  *hflag = 0;
  const int R = 2000;
  // 1. empty kernel + stream sync
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
  CHK(hipStreamSynchronize(s));
  std::vector<double> t;
  for (int i = 0; i < R; ++i) {
    const double a = now_us();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    CHK(hipStreamSynchronize(s));
    t.push_back(now_us() - a);
  }
  printf("launch+streamsync empty          median %.2f us  p10 %.2f\n", median(t), (std::sort(t.begin(), t.end()), t[R / 10]));
  // launch only (host side)
  t.clear();
  for (int i = 0; i < R; ++i) {
    const double a = now_us();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    t.push_back(now_us() - a);
    CHK(hipStreamSynchronize(s));
  }
  printf("launch call only (host)          median %.2f us\n", median(t));
  // 2. launch + flag spin
  t.clear();
  uint32_t v = 0;
  for (int i = 0; i < R; ++i) {
    const double a = now_us();
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, ++v);
    spin_flag(hflag, v);
    t.push_back(now_us() - a);
  }
  CHK(hipStreamSynchronize(s));
  printf("launch+flag spin                 median %.2f us  p10 %.2f\n", median(t), (std::sort(t.begin(), t.end()), t[R / 10]));
  // 2b. launch + flag spin, then also stream sync (is the stream ready right after?)
  t.clear();
  for (int i = 0; i < R; ++i) {
    const double a = now_us();
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, dflag, ++v);
    spin_flag(hflag, v);
    CHK(hipStreamSynchronize(s));
    t.push_back(now_us() - a);
  }
  printf("launch+flag spin+streamsync      median %.2f us\n", median(t));
  // 3. staged reads of B bytes
  uint8_t* hin;
  CHK(hipHostMalloc((void**)&hin, 1 << 20, zc));
  memset(hin, 1, 1 << 20);
  uint8_t* din;
  CHK(hipHostGetDevicePointer((void**)&din, hin, 0));
  uint32_t* hout;
  CHK(hipHostMalloc((void**)&hout, 4096, zc));
  uint32_t* dout;
  CHK(hipHostGetDevicePointer((void**)&dout, hout, 0));
  for (int bytes : {64, 256, 1024, 4096, 16384, 65536}) {
    t.clear();
    for (int i = 0; i < R; ++i) {
      const double a = now_us();
      hipLaunchKernelGGL(stage_kernel, dim3(1), dim3(256), 0, s, (const u32x4*)din, bytes / 16, dout, dflag, ++v);
      spin_flag(hflag, v);
      t.push_back(now_us() - a);
    }
    CHK(hipStreamSynchronize(s));
    printf("launch+zero-copy stage %6d B    median %.2f us\n", bytes, median(t));
  }
  // 4. small H2D memcpy + kernel + sync
  uint8_t* dbuf;
  CHK(hipMalloc((void**)&dbuf, 256 << 20));
  t.clear();
  for (int i = 0; i < R; ++i) {
    const double a = now_us();
    CHK(hipMemcpyAsync(dbuf, hin, 256, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    CHK(hipMemcpyAsync(hin + 4096, dbuf, 64, hipMemcpyDeviceToHost, s));
    CHK(hipStreamSynchronize(s));
    t.push_back(now_us() - a);
  }
  printf("H2D 256B + kernel + D2H 64B + sync median %.2f us\n", median(t));
  std::vector<uint8_t> page(256);
  t.clear();
  for (int i = 0; i < R; ++i) {
    const double a = now_us();
    for (int k = 0; k < 6; ++k) CHK(hipMemcpyAsync(dbuf + k * 4096, page.data(), 32, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    for (int k = 0; k < 4; ++k) CHK(hipMemcpyAsync(page.data() + 64 + k * 8, dbuf + k * 4096, 8, hipMemcpyDeviceToHost, s));
    CHK(hipStreamSynchronize(s));
    t.push_back(now_us() - a);
  }
  printf("6 pageable H2D + kernel + 4 D2H + sync (r2 path) median %.2f us\n", median(t));
  // 5. bandwidths
  const size_t BIG = 128ull << 20;
  uint8_t* hpin;
  CHK(hipHostMalloc((void**)&hpin, BIG, hipHostMallocDefault));
  uint8_t* hzc;
  CHK(hipHostMalloc((void**)&hzc, BIG, zc));
  uint8_t* dzc;
  CHK(hipHostGetDevicePointer((void**)&dzc, hzc, 0));
  std::vector<uint8_t> pg(BIG, 3);
  memset(hpin, 2, BIG);
  memset(hzc, 2, BIG);
  auto bw = [&](const char* what, auto f, size_t bytes) {
    f();
    CHK(hipStreamSynchronize(s));
    std::vector<double> tt;
    for (int i = 0; i < 5; ++i) {
      const double a = now_us();
      f();
      CHK(hipStreamSynchronize(s));
      tt.push_back(now_us() - a);
    }
    const double m = median(tt);
    printf("%-44s %8.1f us  %6.1f GB/s\n", what, m, bytes / m / 1e3);
  };
  bw("DMA H2D 128MB pinned", [&] { CHK(hipMemcpyAsync(dbuf, hpin, BIG, hipMemcpyHostToDevice, s)); }, BIG);
  bw("DMA H2D 128MB pageable", [&] { CHK(hipMemcpyAsync(dbuf, pg.data(), BIG, hipMemcpyHostToDevice, s)); }, BIG);
  bw("DMA D2H 40MB pinned", [&] { CHK(hipMemcpyAsync(hpin, dbuf, 40 << 20, hipMemcpyDeviceToHost, s)); }, 40 << 20);
  bw("DMA D2H 40MB pageable", [&] { CHK(hipMemcpyAsync(pg.data(), dbuf, 40 << 20, hipMemcpyDeviceToHost, s)); }, 40 << 20);
  for (int blocks : {256, 1024, 4096}) {
    char nm[96];
    snprintf(nm, sizeof nm, "zero-copy kernel read 128MB (%d blocks)", blocks);
    bw(nm, [&] { hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(256), 0, s, (const u32x4*)dzc, (int64_t)(BIG / 16), (uint32_t*)dbuf); }, BIG);
    snprintf(nm, sizeof nm, "zero-copy kernel write 40MB (%d blocks)", blocks);
    bw(nm, [&] { hipLaunchKernelGGL(write_kernel, dim3(blocks), dim3(256), 0, s, (u32x4*)dzc, (int64_t)((40 << 20) / 16)); }, 40 << 20);
  }
  auto host_bw = [&](const char* what, int nt, uint8_t* dst, const uint8_t* src, size_t bytes) {
    std::vector<double> tt;
    for (int i = 0; i < 5; ++i) {
      const double a = now_us();
      std::vector<std::thread> th;
      for (int k = 0; k < nt; ++k)
        th.emplace_back([&, k] { memcpy(dst + bytes * k / nt, src + bytes * k / nt, bytes * (k + 1) / nt - bytes * k / nt); });
      for (auto& x : th) x.join();
      tt.push_back(now_us() - a);
    }
    const double m = median(tt);
    printf("%-44s %8.1f us  %6.1f GB/s\n", what, m, bytes / m / 1e3);
  };
  host_bw("host memcpy pageable->pinned 128MB x1", 1, hzc, pg.data(), BIG);
  host_bw("host memcpy pageable->pinned 128MB x4", 4, hzc, pg.data(), BIG);
  host_bw("host memcpy pageable->pinned 128MB x8", 8, hzc, pg.data(), BIG);
  host_bw("host memcpy pinned->pageable 40MB x1", 1, pg.data(), hzc, 40 << 20);
  host_bw("host memcpy pinned->pageable 40MB x8", 8, pg.data(), hzc, 40 << 20);
  {
    std::vector<uint8_t> reg(BIG, 1);
    const double a = now_us();
    CHK(hipHostRegister(reg.data(), BIG, hipHostRegisterDefault));
    const double b = now_us();
    void* dp;
    CHK(hipHostGetDevicePointer(&dp, reg.data(), 0));
    bw("DMA H2D 128MB registered", [&] { CHK(hipMemcpyAsync(dbuf, reg.data(), BIG, hipMemcpyHostToDevice, s)); }, BIG);
    const double c = now_us();
    CHK(hipHostUnregister(reg.data()));
    const double d = now_us();
    printf("hipHostRegister 128MB %.1f us, unregister %.1f us\n", b - a, d - c);
  }
  printf("done\n");
  return 0;
}
