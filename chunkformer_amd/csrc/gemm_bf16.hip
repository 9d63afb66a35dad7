// bf16 MFMA GEMM, 256 x 256 tiles, LDS-DMA (global_load_lds_dwordx4) staging.
//
//   C[M, N] = A[M, K] . W[N, K]^T   (bf16 in, f32 accumulate), N % 256 == 0, K % 64 == 0
//
// Structure (cdna_hip_programming.md §5 "glds, 2 LDS buffers, BK=64"):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns 128 (M) x 64 (N);
//   * per K-step of 64 the block moves A 256x64 and W 256x64 (32 KiB each) by
//     LDS-DMA: each wave issues 4+4 `global_load_lds_dwordx4` (1 KiB each, lane-
//     linear LDS destination); the 16-B chunk swizzle of a 128-B LDS row,
//     pos = chunk ^ ((row >> 1) & 7), is applied on the per-lane SOURCE address, so
//     the 16-row ds_read_b128 fragment reads are bank-conflict free;
//   * LDS rings: A 3 x 32 KiB, W 2 x 32 KiB (all 160 KiB of the CU, one __shared__
//     array): at step s the block issues W(s+1) then A(s+2) before its MFMAs and
//     ends the step with a counted `s_waitcnt vmcnt(4)` + raw s_barrier, so the A
//     stream (HBM) keeps two K-steps in flight across barriers (Little's law: the
//     per-CU DMA rate is bytes-in-flight / latency) and W (L2-resident) one;
//   * two wave groups (waves 0-3 / 4-7, one wave of each per SIMD) run one barrier
//     segment apart: each 32-MFMA segment of one group overlaps the other group's
//     LDS fragment reads, DMA issue and tile epilogue (ping-pong);
//   * operands are swapped (MFMA A = W fragment, B = A fragment) so the 16x16
//     accumulator holds C^T: lane (fr, g) owns C[m = fr][n = 4g .. 4g+3], i.e. each
//     epilogue store is 4 consecutive columns (8 B bf16 / 16 B f32) per lane;
//   * persistent (one block per CU) with an XCD-aware tile walk: the column tiles of
//     one A row panel run on one XCD back to back, so the panel is fetched from HBM
//     once and re-read from L2; the first K-step DMA of the next tile is in flight
//     while the current tile's epilogue runs.
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "gemm_bf16_epi.h"
#include <cstdlib>

namespace cfm {

#ifndef G256_FULLROW
#define G256_FULLROW 1   // EPI_STORE epilogue through LDS as full 128-B row stores (A/B: 0 = 64-B pieces)
#endif
// DIAG: 0 = normal; 1 = skip MFMAs (DMA + epilogue only); 2 = skip DMA inside the loop (MFMA on stale LDS);
// 3 = skip the epilogue (no bias/activation/stores)
template <int EPI, int ACT, int DIAG = 0, int FMT = 0>
__global__ __launch_bounds__(512, 1) void gemm_bf16_256_kernel(const bf16* __restrict__ A, int lda,
                                                               const bf16* __restrict__ W, int ldw, int M, int N,
                                                               int K, EpiArgs ep) {
  // LDS: A ring of 3 x 32 KiB (two K-steps of A in flight) + W ring of 2 x 32 KiB = 160 KiB
  __shared__ __attribute__((aligned(16))) char smem[5 * 32768];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, g = lane >> 4;
  // wave groups: waves 0-3 (wm = 0) and 4-7 (wm = 1) hold one wave on every SIMD each; group 1 runs
  // one barrier segment behind group 0, so on every SIMD one wave's MFMA segment overlaps the
  // other wave's LDS-read / DMA-issue / epilogue segment (ping-pong).
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2);

  const int nbn = N >> 8, nbm = (M + 255) >> 8, T = nbn * nbm;
  // tile order: column groups of cgw tiles, then rows, then the columns of the group
  const int cgw = (ep.col_group > 0 && nbn % ep.col_group == 0) ? ep.col_group : nbn;
  auto tile_m = [&](int t) { return (t % (nbm * cgw)) / cgw; };
  auto tile_n = [&](int t) { return (t / (nbm * cgw)) * cgw + t % cgw; };
  const int G = gridDim.x;
  int t_first, t_step, t_end;
  if (G >= T) {   // one tile per block: bijective XCD remap
    const int b = blockIdx.x, xcd = b & 7, q8 = T >> 3, r8 = T & 7;
    t_first = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    t_step = T;
    t_end = T;
  } else {        // G % 8 == 0: the blocks of one XCD walk one contiguous eighth of the tiles
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per = T >> 3, rem = T & 7;
    const int start = xcd * per + min(xcd, rem), size = per + (xcd < rem ? 1 : 0);
    t_first = start + j;
    t_step = G >> 3;
    t_end = start + size;
  }
  if (t_first >= t_end) return;
  const int nk = K >> 6;

  // ---- LDS-DMA: wave w, instruction i covers tile rows (w*4+i)*8 .. +8 (1 KiB, lane-linear);
  // row = (w*4+i)*8 + lane/8, its XOR key (row>>1)&7 = (4i + lane/16) & 7 (pre-swizzled source)
  auto stage_a = [&](int t, int kt, int slot) {
    const int tm = tile_m(t);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int srow = (wid * 4 + i) * 8 + (lane >> 3);
      const int scol = ((lane & 7) ^ ((4 * i + (lane >> 4)) & 7)) * 8;
      const bf16* ap = A + (size_t)min(tm * 256 + srow, M - 1) * lda + kt * 64 + scol;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ap,
                                       (__attribute__((address_space(3))) void*)(smem + slot * 32768 + (wid * 4 + i) * 1024),
                                       16, 0, 0);
    }
  };
  auto stage_w = [&](int t, int kt, int slot) {
    const int tn = tile_n(t);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int srow = (wid * 4 + i) * 8 + (lane >> 3);
      const int scol = ((lane & 7) ^ ((4 * i + (lane >> 4)) & 7)) * 8;
      const bf16* wp = W + (size_t)(tn * 256 + srow) * ldw + kt * 64 + scol;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)wp,
                                       (__attribute__((address_space(3))) void*)(smem + (3 + slot) * 32768 + (wid * 4 + i) * 1024),
                                       16, 0, 0);
    }
  };

  f32x4 acc[4][8];   // seeded with the bias at every tile's first K-step

  const int key = (fr >> 1) & 7;   // XOR key of fragment rows (row & 15 == fr)
  const int wrow = (wn * 64 + fr) * 128, arow = (wm * 128 + fr) * 128;
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  bf16x8 wf[4], af[8];

  // step cursor: (t1, k1) = step s+1, (t2, k2) = step s+2
  int t1 = t_first, k1 = 0, t2 = t_first, k2 = 0;
  auto advance = [&](int& t, int& k) { if (++k == nk) { k = 0; t += t_step; } };
  // prologue: W(0), A(0), A(1); all of step 0 resident before the first barrier
  stage_w(t_first, 0, 0);
  stage_a(t_first, 0, 0);
  advance(t1, k1);
  t2 = t1; k2 = k1;
  if (t1 < t_end) {
    stage_a(t1, k1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  advance(t2, k2);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");   // stagger group 1 by one segment
  if constexpr (DIAG == 6) { if (grp == 1) __builtin_amdgcn_s_setprio(1); }   // static priority, later half

  // pending epilogue (tile finished in the previous MFMA segment), executed in the next LOAD segment
  int epi_t = -1;
  int s = 0;
  for (int t = t_first; t < t_end; t += t_step) {
    for (int kt = 0; kt < nk; ++kt, ++s) {
      const bool has1 = t1 < t_end, has2 = t2 < t_end;
      const char* as = smem + (s % 3) * 32768;
      const char* ws = smem + (3 + (s & 1)) * 32768;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        // ================= LOAD segment: (epilogue of the previous tile), fragments of (s, ss), DMA issue
        if (ss == 0 && kt == 0) {
          if (epi_t >= 0) {
            if constexpr (DIAG != 3) {
              if constexpr (EPI == EPI_STORE && G256_FULLROW)
                // staging in A slot (s + 2) % 3: A(s - 1) there was read by both groups' last LOAD
                // segments, and A(s + 2) is issued only in the ss = 1 LOAD segment, after the barrier
                // that ends this segment for both groups
                wave_epilogue_fullrow<ACT, FMT>(acc, tile_m(epi_t) * 256 + wm * 128, tile_n(epi_t) * 256 + wn * 64, fr, g,
                                           lane, M, ep, lds_base + (unsigned)(((s + 2) % 3) * 32768 + wid * 2304));
              else
                tile_epilogue<EPI, ACT, false, FMT>(acc, tile_m(epi_t), tile_n(epi_t), wm, wn, fr, g, M, ep);
            }
            epi_t = -1;
          }
          seed_bias(acc, ep.bias, tile_n(t), wn, g);
        }
        const int pos = ((ss * 4 + g) ^ key) << 4;
        const unsigned wa = lds_base + (unsigned)(ws - smem) + wrow + pos;
        const unsigned aa = lds_base + (unsigned)(as - smem) + arow + pos;
        wf[0] = lds_read_b128<0>(wa); wf[1] = lds_read_b128<2048>(wa);
        wf[2] = lds_read_b128<4096>(wa); wf[3] = lds_read_b128<6144>(wa);
        af[0] = lds_read_b128<0>(aa); af[1] = lds_read_b128<2048>(aa);
        af[2] = lds_read_b128<4096>(aa); af[3] = lds_read_b128<6144>(aa);
        af[4] = lds_read_b128<8192>(aa); af[5] = lds_read_b128<10240>(aa);
        af[6] = lds_read_b128<12288>(aa); af[7] = lds_read_b128<14336>(aa);
        if (ss == 0) {
          if (DIAG != 2 && has1) stage_w(t1, k1, (s + 1) & 1);
        } else {
          if (DIAG != 2 && has2) {
            stage_a(t2, k2, (s + 2) % 3);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // W(s+1), A(s+1) of this wave landed
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // keep segments intact: hipcc moves register-only
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // MFMAs across asm barriers
        __builtin_amdgcn_sched_barrier(0);
        // ================= MFMA segment
        if constexpr (DIAG == 1) {
#pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(wf[i]));
#pragma unroll
          for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(af[j]));
        } else {
          if constexpr (DIAG == 5) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
              acc[i][j] = mfma16x32<FMT>(wf[i], af[j], acc[i][j]);
          if constexpr (DIAG == 5) __builtin_amdgcn_s_setprio(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      if (kt + 1 == nk) epi_t = t;
      advance(t1, k1);
      advance(t2, k2);
    }
  }
  // last tile's epilogue (no MFMA partner left), then rebalance the barrier count
  if (epi_t >= 0 && DIAG != 3) {
    if constexpr (EPI == EPI_STORE && G256_FULLROW) {
      // every DMA has landed and been read; the other group only runs MFMAs from here on
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wave_epilogue_fullrow<ACT, FMT>(acc, tile_m(epi_t) * 256 + wm * 128, tile_n(epi_t) * 256 + wn * 64, fr, g, lane, M,
                                 ep, lds_base + (unsigned)(((s + 2) % 3) * 32768 + wid * 2304));
    } else {
      tile_epilogue<EPI, ACT, false, FMT>(acc, tile_m(epi_t), tile_n(epi_t), wm, wn, fr, g, M, ep);
    }
  }
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
}

template <int EPI, int ACT>
static int launch256(const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K, const EpiArgs& ep,
                     hipStream_t st) {
  const int tiles = ((M + 255) / 256) * (N / 256);
  const int n_cu = (cu_count() + 7) / 8 * 8;
  const int grid = tiles <= n_cu ? tiles : n_cu;   // persistent: one 512-thread block per CU
  // ep.diag (timing diagnostics, model option "gemm_diag"): 1 no MFMA, 2 no DMA in the loop, 3 no
  // epilogue, 5 / 6 wave-group priorities
#define G256(D)                                                                                                   \
  do {                                                                                                            \
    if (ep.f16)                                                                                                   \
      hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, D, 1>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep); \
    else                                                                                                          \
      hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, D, 0>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep); \
  } while (0)
#ifdef CFM_GEMM_DIAG
  switch (ep.diag) {
    case 1: G256(1); break;
    case 2: G256(2); break;
    case 3: G256(3); break;
    case 5: G256(5); break;
    case 6: G256(6); break;
    default: G256(0); break;
  }
#else
  G256(0);
#endif
#undef G256
  CFM_CHECK_LAUNCH();
  return 0;
}

// returns -1 when the shape is not eligible (caller falls back to the 128x128 kernel)
int gemm_bf16_wst(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st);

int gemm_bf16_big(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st) {
  if (M <= 0) return 0;
  if (ep.wst) {
    const int r = gemm_bf16_wst(epi, act, A, lda, W, ldw, M, N, K, ep, st);   // K = 512: weight tile in registers
    if (r != -1) return r;
  }
  if (N % 256 || K % 64 || lda % 8 || ldw % 8) return -1;
  if (((M + 255) / 256) * (N / 256) < ep.big_min_tiles) return -1;   // too few tiles to fill the chip
  if (epi == EPI_GLU && ep.bias == nullptr) return -1;
  switch (epi) {
    case EPI_STORE:
      if (act == ACT_RELU) return launch256<EPI_STORE, ACT_RELU>(A, lda, W, ldw, M, N, K, ep, st);
      if (act == ACT_SILU) return launch256<EPI_STORE, ACT_SILU>(A, lda, W, ldw, M, N, K, ep, st);
      if (act == ACT_SILU_L2E) return launch256<EPI_STORE, ACT_SILU_L2E>(A, lda, W, ldw, M, N, K, ep, st);
      return launch256<EPI_STORE, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_STORE_F32: return launch256<EPI_STORE_F32, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_RESID: return launch256<EPI_RESID, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_QKV: return launch256<EPI_QKV, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_GLU:
      if (act == ACT_SILU_L2E) return launch256<EPI_GLU, ACT_SILU_L2E>(A, lda, W, ldw, M, N, K, ep, st);
      return launch256<EPI_GLU, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
  }
  return -1;
}

}  // namespace cfm
