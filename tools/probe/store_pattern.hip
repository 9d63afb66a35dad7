// Store-pattern probe: write a [M, N] bf16 matrix (746 MB, FFN hidden shape) with 16-B-per-lane
// stores whose 64 lanes cover R rows x (1024/R) bytes per instruction, 256 persistent blocks of
// 512 threads (GEMM-like residency).  Prints GB/s per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int R>
__global__ __launch_bounds__(512) void st_kernel(char* out, int M, int ldb /*bytes*/, int tiles_n) {
  // a "tile" = 256 rows x 512 bytes (256 bf16 cols); wave w of 8 covers 128 rows x 128 B like the GEMM
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;
  constexpr int SEG = 1024 / R;          // bytes per row per instruction
  const int r_in = lane / (SEG / 16), c_in = (lane % (SEG / 16)) * 16;
  const int T = (M / 256) * tiles_n;
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    const int tm = t / tiles_n, tn = t % tiles_n;
    char* base = out + (size_t)(tm * 256 + wm * 128) * ldb + tn * 512 + wn * 128;
    // wave region: 128 rows x 128 B = 16 KB = 16 instructions
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      // instruction k covers rows (k*R .. k*R+R) when SEG == 128... general: region split in 16 pieces
      const int piece_rows = R, pieces_per_rowband = 128 / SEG;
      const int band = k / pieces_per_rowband, pc = k % pieces_per_rowband;
      char* p = base + (size_t)(band * piece_rows + r_in) * ldb + pc * SEG + c_in;
      *reinterpret_cast<u32x4*>(p) = (u32x4){(unsigned)t, (unsigned)k, 1u, 2u};
    }
  }
}

int main() {
  const int M = 182016, N = 2048, ldb = N * 2;
  char* out;
  hipMalloc(&out, (size_t)M * ldb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, M, ldb, N / 256);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, M, ldb, N / 256);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 10;
    printf("%-28s %8.1f us  %7.1f GB/s\n", name, ms * 1e3, (double)M * ldb / ms / 1e6);
  };
  run(st_kernel<16>, "16 rows x 64 B / instr");
  run(st_kernel<8>, "8 rows x 128 B / instr");
  run(st_kernel<64>, "64 rows x 16 B / instr");
  return 0;
}
