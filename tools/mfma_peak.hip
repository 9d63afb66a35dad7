// Calibration micro-benchmark: achievable bf16 MFMA rate on this MI355X with random operands in
// registers (no memory traffic in the loop), one or two waves per SIMD, and the in-kernel clock
// (s_memtime / s_memrealtime at 100 MHz, stamped by wave 0 of each block around the loop).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o tools/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// MODE 0: 16x16x32, 1: 32x32x16, 2: 16x16x32 as inline asm with the A operand in AGPRs (the
// projection GEMM's form); operands: 8 random bf16x8 per lane from `src`
template <int MODE, int THREADS>
__global__ __launch_bounds__(THREADS, 1) void k(const bf16x8* __restrict__ src, float* out, long long* stamps,
                                                int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
  const bf16x8* s = src + ((size_t)blockIdx.x * THREADS + threadIdx.x) * 8;
  for (int i = 0; i < 4; ++i) { a[i] = s[i]; b[i] = s[4 + i]; }
  long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  float sum = 0;
  if constexpr (MODE == 0) {
    f32x4 c[16];
    for (int i = 0; i < 16; ++i) c[i] = (f32x4){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 3], b[i >> 2], c[i], 0, 0, 0);
    for (int i = 0; i < 16; ++i) sum += c[i][0] + c[i][3];
  } else if constexpr (MODE == 2) {
    f32x4 c[16];
    for (int i = 0; i < 16; ++i) c[i] = (f32x4){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c[i]) : "a"(a[i & 3]), "v"(b[i >> 2]));
    for (int i = 0; i < 16; ++i) sum += c[i][0] + c[i][3];
  } else {
    f32x16 c[8];
    for (int i = 0; i < 8; ++i) for (int r = 0; r < 16; ++r) c[i][r] = 0;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i & 1], b[i >> 1], c[i], 0, 0, 0);
    for (int i = 0; i < 8; ++i) sum += c[i][0] + c[i][5];
  }
  out[(size_t)blockIdx.x * THREADS + threadIdx.x] = sum;
  if (threadIdx.x == 0) {
    stamps[blockIdx.x * 2] = __builtin_amdgcn_s_memtime() - t0;
    stamps[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  (void)lane;
}

template <int MODE, int THREADS>
void run(const char* name, int blocks, int iters) {
  const size_t n = (size_t)blocks * THREADS * 8;
  std::vector<uint16_t> h(n * 8);
  uint32_t x = 12345;
  for (auto& v : h) {   // random bf16 in roughly N(0,1) magnitudes: sign, exponent 2^-2..2^1, random mantissa
    x = x * 1664525u + 1013904223u;
    v = (uint16_t)(((x >> 31) << 15) | ((125 + ((x >> 8) & 3)) << 7) | ((x >> 12) & 127));
  }
  bf16x8* src; float* out; long long* st;
  hipMalloc(&src, n * 16); hipMalloc(&out, (size_t)blocks * THREADS * 4); hipMalloc(&st, blocks * 16);
  hipMemcpy(src, h.data(), n * 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 20; ++w) k<MODE, THREADS><<<blocks, THREADS>>>(src, out, st, iters);   // >= 2 s warm
  hipEventRecord(e0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) k<MODE, THREADS><<<blocks, THREADS>>>(src, out, st, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> hs(blocks * 2);
  hipMemcpy(hs.data(), st, blocks * 16, hipMemcpyDeviceToHost);
  std::vector<double> clk(blocks);
  for (int b = 0; b < blocks; ++b) clk[b] = hs[2 * b] * 100.0 / std::max(1LL, hs[2 * b + 1]);   // MHz
  std::sort(clk.begin(), clk.end());
  const double flop_per_iter_wave = MODE != 1 ? 16.0 * 16 * 16 * 32 * 2 : 8.0 * 32 * 32 * 16 * 2;
  const double flops = flop_per_iter_wave * iters * (THREADS / 64.0) * blocks * reps;
  printf("%-40s %8.1f TFLOP/s   in-kernel clock median %.0f MHz\n", name, flops / (ms * 1e-3) / 1e12, clk[blocks / 2]);
  hipFree(src); hipFree(out); hipFree(st);
}

int main() {
  run<0, 256>("16x16x32 bf16, 1 wave/SIMD, random", 256, 20000);
  run<0, 512>("16x16x32 bf16, 2 waves/SIMD, random", 256, 10000);
  run<1, 256>("32x32x16 bf16, 1 wave/SIMD, random", 256, 20000);
  run<1, 512>("32x32x16 bf16, 2 waves/SIMD, random", 256, 10000);
  run<2, 256>("16x16x32 bf16 asm, A in AGPRs, 1 wave/SIMD", 256, 20000);
  run<2, 512>("16x16x32 bf16 asm, A in AGPRs, 2 waves/SIMD", 256, 10000);
  return 0;
}
