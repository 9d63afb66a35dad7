// bf16 MFMA GEMM for K = 512 with the weight tile held in registers ("W-stationary").
//
//   C[M, N] = A[M, K] . W[N, K]^T   (bf16 in, f32 accumulate), K == 512, N % 256 == 0
//
// Why: the 256 x 256 LDS-DMA kernel (gemm_bf16.hip) streams BOTH operands through LDS, 128 FLOP per
// byte filled, and its per-CU L2 -> LDS fill rate caps it well below the MFMA rate.  With K = 512 a
// 256-column weight tile is 256 KiB of bf16: spread over the 4 waves of a CU (one wave per SIMD,
// 512 registers each) it fits in registers, 256 per lane.  Only A is streamed, 64 rows x 512 per
// 64 x 256 output tile: 256 FLOP per byte filled, and a 16-slot LDS ring keeps 15 K-steps
// (120 KiB) of A in flight per CU.
//
//   * block = 4 waves (256 threads), one per CU; wave w owns output columns 64w .. 64w+63 of the
//     block's column tile: W fragments wf[n-block 0..3][k32 0..15] (bf16x8), loaded once;
//   * a tile = 64 rows x 256 columns, 8 K-steps of 64; per K-step each wave reads 4 x 2 A
//     fragments (ds_read_b128, swizzled conflict-free image) and issues 32
//     v_mfma_f32_16x16x32_bf16 (MFMA A operand = W fragment, B = A fragment: the accumulator holds
//     C^T, so the shared swapped-operand epilogue of gemm_bf16_epi.h stores 16-B bf16 row pieces);
//   * A staging: LDS-DMA (global_load_lds_dwordx4), 2 x 1 KiB per wave per step, lane-linear LDS
//     destination with the 16-B chunk swizzle applied on the source address; one barrier per step;
//   * placement: the row tiles are cut into 8 XCD ranges; on one XCD the column tiles of a row
//     range run on different CUs at the same pace, so each A tile comes from HBM once and is
//     re-read from that XCD's L2 by the other column tiles (blockIdx % 8 = XCD is a speed
//     assumption only, never a correctness one).
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "gemm_bf16_epi.h"
#include <cstdlib>

namespace cfm {

namespace {
constexpr int WST_K = 512;
constexpr int WST_MT = 64;              // rows per tile
constexpr int WST_KS = 64;              // K per step
constexpr int WST_NK = WST_K / WST_KS;  // 8 steps per tile
constexpr int WST_SLOT = WST_MT * WST_KS * 2;   // 8 KiB
constexpr int WST_NSLOT = 16;
constexpr int WST_DEPTH = WST_NSLOT - 1;         // steps in flight ahead of the one being read
}  // namespace

#define WST_VMCNT(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

// acc += W-fragment (AGPR, "a") x A-fragment (VGPR): the 256 weight registers per lane live in the
// AGPR half of the register file and feed the MFMA directly (with the builtin, hipcc keeps them in
// AGPRs but copies each one to VGPRs before use).  asm volatile keeps program order with the
// explicit LDS waits; the VALU <-> MFMA hazards around it are padded by hand (s_nop) where the
// accumulators are seeded (VALU write -> MFMA srcC) and read back (MFMA write -> VALU read).
CFM_DEV void mfma_wa(f32x4& acc, const bf16x8& w, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
}

// DIAG (timing experiments, CFM_GEMM_DIAG): 1 = no MFMAs, 3 = no epilogue, 4 = epilogue without activation,
// 6 = A stream only (no MFMAs, no epilogue), 2 = no DMA waits / barriers (stale LDS), 7 = no DMA in the loop
template <int EPI, int ACT, int DIAG = 0>
__global__ __launch_bounds__(256, 1) void gemm_wst_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ W, int ldw, int M, int N,
                                                          EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[WST_NSLOT * WST_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;

  // ---- block -> (column tile, row-tile range)
  const int nbn = N >> 8, nbm = (M + WST_MT - 1) / WST_MT;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per = gridDim.x >> 3;
  const int cpx = per / nbn;   // CUs per column tile on one XCD
  if (cpx == 0 || j >= cpx * nbn) return;
  const int ct = j % nbn, sub = j / nbn;
  const int xr0 = (int)((long long)xcd * nbm / 8), xr1 = (int)((long long)(xcd + 1) * nbm / 8);
  const int r0 = xr0 + (int)((long long)sub * (xr1 - xr0) / cpx);
  const int r1 = xr0 + (int)((long long)(sub + 1) * (xr1 - xr0) / cpx);
  if (r0 >= r1) return;
  const int Y = (r1 - r0) * WST_NK;   // K-steps of this block

  // ---- A DMA: step y -> tile r0 + y / 8, K slice y % 8, ring slot y % 16.  Wave wv, instruction i
  // covers tile rows (2 wv + i) * 8 + lane / 8; 16-B chunk (lane & 7) of the LDS row holds source
  // chunk (lane & 7) ^ ((row >> 1) & 7)
  const int drow[2] = {(2 * wv) * 8 + (lane >> 3), (2 * wv + 1) * 8 + (lane >> 3)};
  const int dcol[2] = {((lane & 7) ^ ((drow[0] >> 1) & 7)) * 8, ((lane & 7) ^ ((drow[1] >> 1) & 7)) * 8};
  auto issue = [&](int yy) {
    const int rt = r0 + yy / WST_NK, ks = yy % WST_NK, slot = yy % WST_NSLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = min(rt * WST_MT + drow[i], M - 1);
      const bf16* src = A + (size_t)row * lda + ks * WST_KS + dcol[i];
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + slot * WST_SLOT +
                                                                                 (2 * wv + i) * 1024),
                                       16, 0, 0);
    }
  };
  // prologue DMA first (its latency covers the weight loads)
  for (int p = 0; p < WST_DEPTH; ++p)
    if (p < Y) issue(p);

  // ---- weight tile -> registers: lane (fr, g) of fragment (nb, kk) = W[col0 + 16 nb + fr][32 kk + 8 g ..]
  const int col0 = ct * 256 + wv * 64;
  bf16x8 wf[4][16];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const bf16* wp = W + (size_t)(col0 + 16 * nb + fr) * ldw + 8 * g;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) wf[nb][kk] = *reinterpret_cast<const bf16x8*>(wp + 32 * kk);
  }
  asm volatile("s_nop 7" ::: "memory");   // weight AGPR writes -> first MFMA reads
  float bias4[4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const f32x4 b = ep.bias ? *reinterpret_cast<const f32x4*>(ep.bias + col0 + 16 * nb + 4 * g)
                            : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) bias4[nb][r] = b[r];
  }

  // fragment read offsets in a slot: row 16 mb + fr, chunk 4 kh + g at its swizzled position
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  const int key = (fr >> 1) & 7;
  const unsigned foff[2] = {(unsigned)(fr * 128 + ((g ^ key) << 4)), (unsigned)(fr * 128 + (((4 + g) ^ key) << 4))};

  auto read_frags = [&](int yy, bf16x8 (&af)[4][2]) {
    const unsigned sb = lds_base + (unsigned)((yy % WST_NSLOT) * WST_SLOT);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      af[0][kh] = lds_read_b128<0>(sb + foff[kh]);
      af[1][kh] = lds_read_b128<2048>(sb + foff[kh]);
      af[2][kh] = lds_read_b128<4096>(sb + foff[kh]);
      af[3][kh] = lds_read_b128<6144>(sb + foff[kh]);
    }
  };
  // A fragments double-buffered: step y's MFMAs run on fragments read during step y-1, so the
  // barrier and LDS latency of step y+1 hide behind them
  bf16x8 afr[2][4][2];
  if (Y > WST_DEPTH - 1) WST_VMCNT(28); else WST_VMCNT(0);   // DMA of step 0 landed
  asm volatile("s_barrier" ::: "memory");
  read_frags(0, afr[0]);

  f32x4 acc[4][4];
  int y = 0;
  for (int rt = r0; rt < r1; ++rt) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[nb][mb] = (f32x4){bias4[nb][0], bias4[nb][1], bias4[nb][2], bias4[nb][3]};
    asm volatile("s_nop 4" ::: "memory");   // seed writes (VALU) -> MFMA srcC reads
#pragma unroll
    for (int ks = 0; ks < WST_NK; ++ks, ++y) {
      bf16x8 (&cur)[4][2] = afr[ks & 1];
      bf16x8 (&nxt)[4][2] = afr[(ks + 1) & 1];
      // step y+1's DMA landed for this wave (younger: steps y+2 .. y+DEPTH-1, 2 each), then for every
      // wave (barrier).  Every wave has also finished reading slot y-1 (its reads were waited on
      // before step y-1's MFMAs), the slot the DMA below refills.
      if (y + 1 < Y) {
        if constexpr (DIAG != 2) {
          if (y + WST_DEPTH <= Y) WST_VMCNT(26); else WST_VMCNT(0);
          asm volatile("s_barrier" ::: "memory");
        }
        read_frags(y + 1, nxt);
      }
      if (DIAG != 7 && y + WST_DEPTH < Y) issue(y + WST_DEPTH);
      // step y's fragments (issued one step ago) are in; step y+1's 8 reads may still be in flight
      if (y + 1 < Y) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (DIAG == 1 || DIAG == 6) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) asm volatile("" ::"v"(cur[mb][kh]));
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) mfma_wa(acc[nb][mb], wf[nb][2 * ks + kh], cur[mb][kh]);
      }
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // last MFMA writes -> epilogue VALU reads
    if constexpr (DIAG == 3 || DIAG == 6) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) asm volatile("" ::"v"(acc[nb][mb]));
    } else {
      wave_epilogue<EPI, DIAG == 4 ? ACT_NONE : ACT, 4>(acc, rt * WST_MT + fr, col0, g, M, ep);
    }
  }
}

static int wst_enabled() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("CFM_GEMM_WST"); v = e ? atoi(e) : 0; }
  return v;
}

template <int EPI, int ACT>
static int launch_wst(const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep,
                      hipStream_t st) {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
    n_cu = n_cu / 8 * 8;
  }
  static int diag = -1;
  if (diag < 0) { const char* e = getenv("CFM_GEMM_DIAG"); diag = e ? atoi(e) : 0; }
  if (diag == 1)
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 1>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  else if (diag == 3)
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 3>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  else if (diag == 2)
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 2>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  else if (diag == 7)
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 7>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  else if (diag == 6)
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 6>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  else if (diag == 4)
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 4>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  else
    hipLaunchKernelGGL((gemm_wst_kernel<EPI, ACT, 0>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep);
  CFM_CHECK_LAUNCH();
  return 0;
}

// -1 = not eligible (caller uses the 256 x 256 kernel)
int gemm_bf16_wst(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st) {
  if (!wst_enabled() || K != WST_K || N % 256 || lda % 8 || ldw % 8 || M <= 0) return -1;
  // enough rows for every CU of an XCD's column tiles to own several tiles
  if ((M + WST_MT - 1) / WST_MT < 8 * 32 * 2) return -1;
  if (N / 256 > 32) return -1;
  switch (epi) {
    case EPI_STORE:
      if (act == ACT_RELU) return launch_wst<EPI_STORE, ACT_RELU>(A, lda, W, ldw, M, N, ep, st);
      if (act == ACT_SILU) return launch_wst<EPI_STORE, ACT_SILU>(A, lda, W, ldw, M, N, ep, st);
      return launch_wst<EPI_STORE, ACT_NONE>(A, lda, W, ldw, M, N, ep, st);
    case EPI_QKV: return launch_wst<EPI_QKV, ACT_NONE>(A, lda, W, ldw, M, N, ep, st);
    case EPI_GLU:
      if (ep.bias == nullptr) return -1;
      return launch_wst<EPI_GLU, ACT_NONE>(A, lda, W, ldw, M, N, ep, st);
  }
  return -1;
}

}  // namespace cfm
