// Calibration micro-benchmark: achievable bf16 MFMA rate on this MI355X (random operands in
// registers, no memory traffic), and the same loop with ds_read_b128 operand refills at the
// projection GEMM's ratio.  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>   // 0: 16x16x32 regs only; 1: 32x32x16 regs only; 2: 32x32x16 + 6 ds_read_b128 per 8 MFMA
__global__ __launch_bounds__(512, 1) void k(float* out, int iters, float seed) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) { a[i][e] = (__bf16)(seed * (lane + i + e)); b[i][e] = (__bf16)(seed * (lane - i * e)); }
  for (int i = threadIdx.x; i < 65536 / 4; i += 512) ((float*)lds)[i] = seed * i;
  __syncthreads();
  if constexpr (MODE == 0) {
    f32x4 c[16];
    for (int i = 0; i < 16; ++i) c[i] = (f32x4){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 3], b[i >> 2], c[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < 16; ++i) s += c[i][0] + c[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  } else {
    f32x16 c[8];
    for (int i = 0; i < 8; ++i) for (int r = 0; r < 16; ++r) c[i][r] = 0;
    const int off = (threadIdx.x >> 6) * 4096 + lane * 16;
    for (int it = 0; it < iters; ++it) {
      if constexpr (MODE == 2) {
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = *(const bf16x8*)(lds + ((off + i * 1024 + it * 64) & 65535));
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = *(const bf16x8*)(lds + ((off + 2048 + i * 1024 + it * 64) & 65535));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i & 1], b[i >> 1], c[i], 0, 0, 0);
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][5];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  }
}

template <int MODE>
void run(const char* name, int blocks, int iters) {
  float* out;
  hipMalloc(&out, blocks * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) k<MODE><<<blocks, 512>>>(out, iters, 0.001f);
  hipEventRecord(e0);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) k<MODE><<<blocks, 512>>>(out, iters, 0.001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flop_per_iter_wave = MODE == 0 ? 16.0 * 16 * 16 * 32 * 2 : 8.0 * 32 * 32 * 16 * 2;
  const double flops = flop_per_iter_wave * iters * 8.0 * blocks * reps;
  printf("%-44s %8.1f TFLOP/s\n", name, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  run<0>("16x16x32 bf16, regs only, 2 waves/SIMD", 256, 20000);
  run<1>("32x32x16 bf16, regs only, 2 waves/SIMD", 256, 20000);
  run<2>("32x32x16 bf16 + 6 ds_read_b128 / 8 MFMA", 256, 20000);
  return 0;
}
