// LDS-DMA throughput probe (GEMM operand streaming without MFMA / LDS reads / stores).
// 256 persistent blocks of 512 threads; each block streams NT tiles: per K-step the 8 waves move
// a [256 x BK] A slab (A = [M, K] bf16 row-major, K = 2048: the FFN w2 operand) and a [256 x BK]
// W slab (W = [512, K], L2-resident) into an R-slot LDS ring with counted vmcnt + s_barrier.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16;

template <int BK, int R, int D, bool BAR, bool WONLY>
__device__ __forceinline__ void dma_body(const bf16* A, const bf16* W, int M, int K, int tiles_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int SLOT = 256 * BK * 2 * 2;       // A + W
  static_assert(R * SLOT <= 160 * 1024, "lds");
  constexpr int ROWB = BK * 2;                  // bytes per row per step
  constexpr int LPR = ROWB / 16;                // lanes per row
  constexpr int RPI = 64 / LPR;                 // rows per instruction
  constexpr int NI = 256 / RPI / 8;             // instructions per wave per operand per step
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nk = K / BK;
  int voff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) voff[i] = ((wid * NI + i) * RPI + lane / LPR) * K * 2 + (lane % LPR) * 16;
  const int Y = tiles_per_block * nk;
  int t = blockIdx.x, k = 0;
  auto rA = [&](int tt) { return __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)((tt * 256) % (M - 255)) * K), (short)0, 256 * K * 2, 0x00020000); };
  auto rW = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, 256 * K * 2, 0x00020000);
  __amdgpu_buffer_rsrc_t ra = rA(t);
  auto issue = [&](int slot) {
    char* sb = smem + slot * SLOT + wid * (NI * 1024);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (!WONLY)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(sb + i * 1024), 16, voff[i], k * ROWB, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (__attribute__((address_space(3))) void*)(sb + SLOT / 2 + i * 1024), 16, voff[i], k * ROWB, 0, 0);
    }
    if (++k == nk) { k = 0; t += gridDim.x; ra = rA(t); }
  };
  for (int p = 0; p < D; ++p) issue(p % R);
  int slot = D % R;
  for (int y = 0; y < Y; ++y) {
    if (y + D < Y) issue(slot);
    slot = slot + 1 == R ? 0 : slot + 1;
    if constexpr (WONLY) {
      if (D == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * NI) : "memory");
    } else {
      if (D == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(6 * NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 * NI) : "memory");
    }
    if (BAR) { asm volatile("s_barrier" ::: "memory"); asm volatile("s_barrier" ::: "memory"); }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


#define KDEF(NAME, BK, R, D, BAR, WO) \
  __global__ __launch_bounds__(512, 1) void NAME(const void* A, const void* W, int M, int K, int tpb) { \
    dma_body<BK, R, D, BAR, WO>((const bf16*)A, (const bf16*)W, M, K, tpb); }
KDEF(k0, 32, 5, 3, true, false) KDEF(k1, 32, 5, 3, false, false) KDEF(k2, 64, 2, 1, true, false)
KDEF(k3, 64, 2, 1, false, false) KDEF(k4, 32, 5, 3, true, true) KDEF(k5, 32, 5, 3, false, true) KDEF(k6, 64, 2, 1, false, true)

int main() {
  const int M = 182080, K = 2048;
  bf16 *A, *W;
  (void)hipMalloc(&A, (size_t)M * K * 2);
  (void)hipMalloc(&W, (size_t)512 * K * 2);
  (void)hipMemset(A, 0, (size_t)M * K * 2);
  (void)hipMemset(W, 0, (size_t)512 * K * 2);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int tpb = 5;   // 1280 tiles of 256 rows ~ the w2 column-tile count / CU
#define CFG(...) __VA_ARGS__
#define RUN(KERN, name, wonly) (void)hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); run([&]() { hipLaunchKernelGGL(KERN, dim3(256), dim3(512), 160 * 1024, 0, (const void*)A, (const void*)W, M, K, tpb); }, name, wonly)
  auto run = [&](auto launch, const char* name, bool wonly) {
    for (int i = 0; i < 2; ++i) launch();
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    const double bytes = 256.0 * tpb * 256 * K * 2 * (wonly ? 1 : 2);
    printf("%-40s %8.1f us  %7.1f GB/s per CU  %6.2f TB/s chip\n", name, ms * 1e3, bytes / 256 / ms / 1e6, bytes / ms / 1e9);
  };
  RUN(k0, "BK32 R5 D3 barrier A+W", false);
  RUN(k1, "BK32 R5 D3 nobarrier A+W", false);
  RUN(k2, "BK64 R2 D1 barrier A+W", false);
  RUN(k3, "BK64 R2 D1 nobarrier A+W", false);
  RUN(k4, "BK32 R5 D3 barrier W only (L2)", true);
  RUN(k5, "BK32 R5 D3 nobarrier W only (L2)", true);
  RUN(k6, "BK64 R2 D1 nobarrier W only (L2)", true);
  return 0;
}
