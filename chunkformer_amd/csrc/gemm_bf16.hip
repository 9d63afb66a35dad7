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

// DIAG: 0 = normal; 1 = skip MFMAs (DMA + epilogue only); 2 = skip DMA inside the loop (MFMA on stale LDS);
// 3 = skip the epilogue (no bias/activation/stores)
template <int EPI, int ACT, int DIAG = 0>
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
            if constexpr (DIAG != 3) tile_epilogue<EPI, ACT>(acc, tile_m(epi_t), tile_n(epi_t), wm, wn, fr, g, M, ep);
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
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
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
  if (epi_t >= 0 && DIAG != 3) tile_epilogue<EPI, ACT>(acc, tile_m(epi_t), tile_n(epi_t), wm, wn, fr, g, M, ep);
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
}

// =====================================================================================
// Ring variant: 5-slot LDS ring of K = 32 half-steps, buffer_load ... lds staging.
//
//   * a slot = A [256][32] + W [256][32] bf16 = 32 KiB; 5 slots = the CU's 160 KiB.  Each
//     wave stages 2 + 2 KiB of a slot (4 `buffer_load_dwordx4 ... lds`), four slots ahead of
//     the one being read, so three slots (96 KiB) stay in flight across barriers: Little's law
//     on the per-CU DMA rate, which capped the 3+2-slot K = 64 ring (gemm_bf16_256_kernel);
//   * DMA addressing is fixed per lane (a 32-bit voffset per operand block), the K step is
//     the scalar soffset and the tile the descriptor base: no per-step VALU address math.
//     Rows past M fall outside the A descriptor's range and read as 0;
//   * LDS image of a [256][32] operand: row r at 64 r bytes, 16-B chunk c at position
//     c ^ f((r >> 2) & 3), f(q) = (4 - q) & 3: every ds_read_b128 lane group of a 16-row
//     fragment read covers the 64 banks once (conflict free); the DMA pre-swizzles the
//     per-lane SOURCE chunk (LDS destination stays lane-linear);
//   * same two ping-pong wave groups, tile walk, swapped-operand accumulators and tile
//     epilogue as gemm_bf16_256_kernel; the bias seeds the accumulators through scalar loads
//     (lgkmcnt), so the vector-memory counter only ever holds DMA and epilogue stores and
//     every wait is a counted vmcnt (never a drain in the steady state).
// =====================================================================================
typedef int i32x4_t __attribute__((ext_vector_type(4)));

// bias of this wave's 64 columns -> accumulator seeds; col0 wave-uniform
CFM_DEV void seed_bias_smem(f32x4 (&acc)[4][8], const float* bias, int col0, int g) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 b = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (bias) {
      const float* bp = bias + col0 + 16 * i;
      i32x4_t s0, s1, s2, s3;
      asm volatile("s_load_dwordx4 %0, %4, 0x0\n\ts_load_dwordx4 %1, %4, 0x10\n\t"
                   "s_load_dwordx4 %2, %4, 0x20\n\ts_load_dwordx4 %3, %4, 0x30\n\ts_waitcnt lgkmcnt(0)"
                   : "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&s"(s3)
                   : "s"(bp)
                   : "memory");
      const i32x4_t lo = (g & 1) ? s1 : s0, hi = (g & 1) ? s3 : s2;
      const i32x4_t v = (g & 2) ? hi : lo;
      b = __builtin_bit_cast(f32x4, v);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = b;
  }
}

template <int EPI> struct EpiStores { static constexpr int n = 16; };   // bf16 out: 2 x 8 16-B stores
template <> struct EpiStores<EPI_STORE_F32> { static constexpr int n = 32; };
template <> struct EpiStores<EPI_GLU> { static constexpr int n = 8; };

#define CFM_VMCNT(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

template <int EPI, int ACT, int DIAG = 0>
__global__ __launch_bounds__(512, 1) void gemm_bf16_ring_kernel(const bf16* __restrict__ A, int lda,
                                                                const bf16* __restrict__ W, int ldw, int M, int N,
                                                                int K, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[5 * 32768];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, g = lane >> 4;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int grp = wid_u >> 2;
  const int wn_u = wid_u & 3;

  const int nbn = N >> 8, nbm = (M + 255) >> 8, T = nbn * nbm;
  const int G = gridDim.x;
  int t_first, t_step, t_end;
  if (G >= T) {
    const int b = blockIdx.x, xcd = b & 7, q8 = T >> 3, r8 = T & 7;
    t_first = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    t_step = T;
    t_end = T;
  } else {
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per = T >> 3, rem = T & 7;
    const int start = xcd * per + min(xcd, rem), size = per + (xcd < rem ? 1 : 0);
    t_first = start + j;
    t_step = G >> 3;
    t_end = start + size;
  }
  if (t_first >= t_end) return;
  const int nk = K >> 5;                                          // K-32 steps per tile (>= 4)
  const int n_mine = (t_end - t_first + t_step - 1) / t_step;    // tiles of this block
  const int Y = n_mine * nk;                                      // ring steps

  // ---- per-lane DMA offsets: wave w stages rows 32w + 16i + lane/4 of A and W, chunk pre-swizzled
  const int drow = lane >> 2;
  const int dch = (lane & 3) ^ ((4 - (lane >> 4)) & 3);
  int voffA[2], voffW[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 32 * wid + 16 * i + drow;
    voffA[i] = (row * lda + 8 * dch) * 2;
    voffW[i] = (row * ldw + 8 * dch) * 2;
  }
  // issue cursor: step (it, ik) with descriptors of tile it
  int it = t_first, ik = 0;
  __amdgpu_buffer_rsrc_t rA, rW;
  auto set_rsrc = [&](int t) {
    const int tm = t / nbn, tn = t - tm * nbn;
    const int rows = min(256, M - tm * 256);
    rA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)tm * 256 * lda), (short)0, rows * lda * 2, 0x00020000);
    rW = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)tn * 256 * ldw), (short)0, 256 * ldw * 2, 0x00020000);
  };
  auto issue = [&](int slot) {
    char* sb = smem + slot * 32768 + wid_u * 2048;
    const int soff = ik * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (__attribute__((address_space(3))) void*)(sb + i * 1024), 16,
                                               voffA[i], soff, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (__attribute__((address_space(3))) void*)(sb + 16384 + i * 1024),
                                               16, voffW[i], soff, 0, 0);
    if (++ik == nk) {
      ik = 0;
      it += t_step;
      if (it < t_end) set_rsrc(it);
    }
  };

  f32x4 acc[4][8];
  // fragment read offsets: row (16-row block base) + fr, chunk g at its swizzled position
  const int cpos = (g ^ ((4 - ((fr >> 2) & 3)) & 3)) << 4;
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  const unsigned offW = 16384 + (wn * 64 + fr) * 64 + cpos;
  const unsigned offA = (wm * 128 + fr) * 64 + cpos;
  bf16x8 wf[4], af[8];

  // prologue: slots 0..3
  set_rsrc(it);
#pragma unroll
  for (int p = 0; p < 4; ++p)
    if (p < Y) issue(p);
  if (Y >= 4) CFM_VMCNT(12); else CFM_VMCNT(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");

  int epi_t = -1;
  bool epi_full = false;   // the last epilogue stored every row (counted stores outstanding)
  int y = 0, slot = 0, slot4 = 4;
  for (int t = t_first; t < t_end; t += t_step) {
    for (int kc = 0; kc < nk; ++kc, ++y) {
      // ================= LOAD segment
      const unsigned sa = lds_base + (unsigned)slot * 32768u;
      const unsigned wa = sa + offW, aa = sa + offA;
      wf[0] = lds_read_b128<0>(wa); wf[1] = lds_read_b128<1024>(wa);
      wf[2] = lds_read_b128<2048>(wa); wf[3] = lds_read_b128<3072>(wa);
      af[0] = lds_read_b128<0>(aa); af[1] = lds_read_b128<1024>(aa);
      af[2] = lds_read_b128<2048>(aa); af[3] = lds_read_b128<3072>(aa);
      af[4] = lds_read_b128<4096>(aa); af[5] = lds_read_b128<5120>(aa);
      af[6] = lds_read_b128<6144>(aa); af[7] = lds_read_b128<7168>(aa);
      if (y + 4 < Y) {
        if (DIAG != 2) issue(slot4);
        // slot y+1 landed: younger are y+2..y+4 (12) and, for 3 steps after a full epilogue, its stores
        if (DIAG != 2 && epi_full && kc >= 1 && kc <= 3) {
          if constexpr (EpiStores<EPI>::n == 32) CFM_VMCNT(44);
          else if constexpr (EpiStores<EPI>::n == 16) CFM_VMCNT(28);
          else CFM_VMCNT(20);
        } else if (DIAG != 2) {
          CFM_VMCNT(12);
        }
      } else {
        CFM_VMCNT(0);
      }
      if (kc == 0) {
        epi_full = false;
        if (epi_t >= 0) {
          const int etm = epi_t / nbn;
          tile_epilogue<EPI, DIAG == 4 ? ACT_NONE : ACT, DIAG == 3>(acc, etm, epi_t - etm * nbn, wm, wn, fr, g, M, ep);
          epi_full = DIAG != 3 && etm * 256 + 256 <= M;
          epi_t = -1;
        }
        seed_bias_smem(acc, ep.bias, (t % nbn) * 256 + wn_u * 64, g);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // ================= MFMA segment
      if constexpr (DIAG == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(wf[i]));
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(af[j]));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      slot = slot == 4 ? 0 : slot + 1;
      slot4 = slot4 == 4 ? 0 : slot4 + 1;
    }
    epi_t = t;
  }
  if (epi_t >= 0) tile_epilogue<EPI, DIAG == 4 ? ACT_NONE : ACT, DIAG == 3>(acc, epi_t / nbn, epi_t % nbn, wm, wn, fr, g, M, ep);
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
}

// =====================================================================================
// Spread-store variant of the ring kernel (bf16 outputs, K % 512 == 0).
//
// The bunched tile epilogue issues 16 KiB of stores per wave in one segment; the CU's store
// path takes them at ~10-20 B/cycle, so the partner wave group idles at the next barrier for
// several MFMA segments (no-store diagnostic: FFN w1 582 -> 427 us).  Here the finished tile
// is packed to bf16 at once (64 VGPRs per lane: activation, permlane16 swap into 16-B row
// pieces) and its 16 stores are issued one per load segment across the next tile's first 16
// K-steps, beside the other group's MFMAs.  Stores go through a buffer descriptor per output
// block, so rows past M are dropped by the range check while the instruction still issues:
// every load segment's store count is exact and the DMA waits stay counted
// (vmcnt = 12 + stores issued in the three previous load segments).
// =====================================================================================
// entries kept packed in registers and stored one per load segment (the rest of the tile is stored at
// once at the tile end: VGPR budget 2 waves/SIMD = 256 with the 128-register accumulator)
// s_waitcnt vmcnt(n) for the counts the spread kernel uses (n folds to a constant per unrolled step)
CFM_DEV void wait_vm(int n) {
  switch (n) {
#define CFM_VMCASE(N) case N: CFM_VMCNT(N); break;
    CFM_VMCASE(13) CFM_VMCASE(14) CFM_VMCASE(15) CFM_VMCASE(16) CFM_VMCASE(17) CFM_VMCASE(18) CFM_VMCASE(19)
    CFM_VMCASE(20) CFM_VMCASE(21) CFM_VMCASE(22) CFM_VMCASE(23) CFM_VMCASE(24) CFM_VMCASE(25) CFM_VMCASE(26)
    CFM_VMCASE(27) CFM_VMCASE(28) CFM_VMCASE(29) CFM_VMCASE(30) CFM_VMCASE(31)
#undef CFM_VMCASE
    default: CFM_VMCNT(12); break;
  }
}


template <int EPI> struct PendN {
  static constexpr int total = EPI == EPI_GLU ? 8 : 16;   // 16-B stores per wave per tile
  static constexpr int n = 4;                              // of which spread (the rest at the tile end)
};

// packs the finished tile: GLU -> pend[0..7] (one 16-B store per row block j); STORE / QKV:
// half p = 0 -> pend[0..7], half p = 1 stored now through rO[1]
template <int EPI, int ACT>
CFM_DEV void pack_tile(f32x4 (&acc)[4][8], u32x4 (&pend)[PendN<EPI>::n], __amdgpu_buffer_rsrc_t r0,
                       __amdgpu_buffer_rsrc_t r1, int ld0, int ld1, int rowq, int col_g) {
  constexpr int NP = PendN<EPI>::n;
  if constexpr (EPI == EPI_GLU) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      u32x2_t o[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const f32x4 a = acc[2 * p][j], gt = acc[2 * p + 1][j];
        o[p] = (u32x2_t){pack_bf16x2(a[0] * fast_sigmoid(gt[0]), a[1] * fast_sigmoid(gt[1])),
                         pack_bf16x2(a[2] * fast_sigmoid(gt[2]), a[3] * fast_sigmoid(gt[3]))};
      }
      const auto s0 = __builtin_amdgcn_permlane16_swap(o[0][0], o[1][0], false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(o[0][1], o[1][1], false, false);
      const u32x4 v = (u32x4){s0[0], s1[0], s0[1], s1[1]};
      if (j < NP) {
        pend[j] = v;
      } else {
        int r = rowq;
        asm volatile("" : "+v"(r));
        __builtin_amdgcn_raw_buffer_store_b128(v, r0, ((r + 16 * j) * ld0 + col_g) * 2, 0, 0);
      }
    }
  } else {
#pragma unroll
    for (int p = 1; p >= 0; --p)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 v0 = act4<ACT>(acc[2 * p][j]), v1 = act4<ACT>(acc[2 * p + 1][j]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v1[0], v1[1]), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[2], v1[3]), false, false);
        const u32x4 v = (u32x4){s0[0], s1[0], s0[1], s1[1]};
        if (p == 0 && j < NP) {
          pend[j] = v;
        } else {
          int r = rowq;
          asm volatile("" : "+v"(r));   // recompute the offset here: hoisted, 16 such offsets spill
          __builtin_amdgcn_raw_buffer_store_b128(v, p ? r1 : r0, ((r + 16 * j) * (p ? ld1 : ld0) + col_g) * 2, 0, 0);
        }
      }
  }
}

template <int EPI, int ACT>
__global__ __launch_bounds__(512, 1) void gemm_bf16_spread_kernel(const bf16* __restrict__ A, int lda,
                                                                  const bf16* __restrict__ W, int ldw, int M, int N,
                                                                  int K, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[5 * 32768];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, g = lane >> 4;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int grp = wid_u >> 2;
  const int wn_u = wid_u & 3;
  constexpr int NP = PendN<EPI>::n;

  const int nbn = N >> 8, nbm = (M + 255) >> 8, T = nbn * nbm;
  const int G = gridDim.x;
  int t_first, t_step, t_end;
  if (G >= T) {
    const int b = blockIdx.x, xcd = b & 7, q8 = T >> 3, r8 = T & 7;
    t_first = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    t_step = T;
    t_end = T;
  } else {
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per = T >> 3, rem = T & 7;
    const int start = xcd * per + min(xcd, rem), size = per + (xcd < rem ? 1 : 0);
    t_first = start + j;
    t_step = G >> 3;
    t_end = start + size;
  }
  if (t_first >= t_end) return;
  const int nk = K >> 5;                                          // K-32 steps per tile, % 16 == 0
  const int n_mine = (t_end - t_first + t_step - 1) / t_step;
  const int Y = n_mine * nk;

  const int drow = lane >> 2;
  const int dch = (lane & 3) ^ ((4 - (lane >> 4)) & 3);
  int voffA[2], voffW[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 32 * wid + 16 * i + drow;
    voffA[i] = (row * lda + 8 * dch) * 2;
    voffW[i] = (row * ldw + 8 * dch) * 2;
  }
  int it = t_first, ik = 0;
  __amdgpu_buffer_rsrc_t rA, rW;
  auto set_rsrc = [&](int t) {
    const int tm = t / nbn, tn = t - tm * nbn;
    const int rows = min(256, M - tm * 256);
    rA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)tm * 256 * lda), (short)0, rows * lda * 2, 0x00020000);
    rW = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)tn * 256 * ldw), (short)0, 256 * ldw * 2, 0x00020000);
  };
  auto issue = [&](int slot) {
    char* sb = smem + slot * 32768 + wid_u * 2048;
    const int soff = ik * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (__attribute__((address_space(3))) void*)(sb + i * 1024), 16,
                                               voffA[i], soff, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (__attribute__((address_space(3))) void*)(sb + 16384 + i * 1024),
                                               16, voffW[i], soff, 0, 0);
    if (++ik == nk) {
      ik = 0;
      it += t_step;
      if (it < t_end) set_rsrc(it);
    }
  };

  // output descriptors of the pending (packed) tile, one per 32-column half p (GLU: one)
  __amdgpu_buffer_rsrc_t rO[2];
  int ldO[2];
  auto set_out = [&](int t) {
    const int tm = t / nbn, tn = t - tm * nbn;
    const int rows = min(256, M - tm * 256);
    const int nw = tn * 256 + wn_u * 64;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      bf16* base;
      int ld;
      if constexpr (EPI == EPI_GLU) {
        base = reinterpret_cast<bf16*>(ep.out) + (size_t)(ep.row_off + tm * 256) * ep.ldo + nw / 2;
        ld = ep.ldo;
      } else if constexpr (EPI == EPI_QKV) {
        const int n = nw + 32 * p, d = ep.d;
        if (n < d) {
          base = reinterpret_cast<bf16*>(ep.out) + (size_t)tm * 256 * d + n;
          ld = d;
        } else {
          const int c2 = n - d, which = c2 >= d ? 1 : 0, cc = c2 - which * d;
          base = reinterpret_cast<bf16*>(ep.out2) + (size_t)(ep.row_off + tm * 256) * 2 * d + qkv_kv_col(cc, which, ep.dk);
          ld = 2 * d;
        }
      } else {
        base = reinterpret_cast<bf16*>(ep.out) + (size_t)(ep.row_off + tm * 256) * ep.ldo + nw + 32 * p;
        ld = ep.ldo;
      }
      rO[p] = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, rows * ld * 2, 0x00020000);
      ldO[p] = ld;
    }
  };
  const int col_g = 16 * (g & 1) + 8 * (g >> 1);
  const int rowq = wm * 128 + fr;

  f32x4 acc[4][8];
  u32x4 pend[NP];
  const int cpos = (g ^ ((4 - ((fr >> 2) & 3)) & 3)) << 4;
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  const unsigned offW = 16384 + (wn * 64 + fr) * 64 + cpos;
  const unsigned offA = (wm * 128 + fr) * 64 + cpos;
  bf16x8 wf[4], af[8];

  set_rsrc(it);
#pragma unroll
  for (int p = 0; p < 4; ++p)
    if (p < Y) issue(p);
  if (Y >= 4) CFM_VMCNT(12); else CFM_VMCNT(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");

  int epi_t = -1;
  bool pend_on = false;   // this tile's first 16-step block stores the previous tile (packed at e = 0)
  int y = 0, slot = 0, slot4 = 4;
  for (int t = t_first; t < t_end; t += t_step) {
    for (int kc0 = 0; kc0 < nk; kc0 += 16) {
#pragma unroll
      for (int e = 0; e < 16; ++e, ++y) {
        // ================= LOAD segment
        if (e == 0 && kc0 == 0) {
          pend_on = false;
          if (epi_t >= 0) {
            set_out(epi_t);
            pack_tile<EPI, ACT>(acc, pend, rO[0], rO[1], ldO[0], ldO[1], rowq, col_g);
            pend_on = true;
            epi_t = -1;
          }
          seed_bias_smem(acc, ep.bias, (t % nbn) * 256 + wn_u * 64, g);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the pack's temporaries out of the fragment reads
        const unsigned sa = lds_base + (unsigned)slot * 32768u;
        const unsigned wa = sa + offW, aa = sa + offA;
        wf[0] = lds_read_b128<0>(wa); wf[1] = lds_read_b128<1024>(wa);
        wf[2] = lds_read_b128<2048>(wa); wf[3] = lds_read_b128<3072>(wa);
        af[0] = lds_read_b128<0>(aa); af[1] = lds_read_b128<1024>(aa);
        af[2] = lds_read_b128<2048>(aa); af[3] = lds_read_b128<3072>(aa);
        af[4] = lds_read_b128<4096>(aa); af[5] = lds_read_b128<5120>(aa);
        af[6] = lds_read_b128<6144>(aa); af[7] = lds_read_b128<7168>(aa);
        if (y + 4 < Y) {
          issue(slot4);
          // slot y+1 landed.  Younger than its DMA (issued 3 segments back, before that segment's
          // spread store): 12 DMA + the spread stores of segments y-3..y-1 + the 8 tile-end stores
          // if the tile was packed in segments y-2..y.  Spread stores run at e = 0..7 of a packed
          // tile's first 16-step block, so the count is a constant per unrolled e.
          const bool sp = pend_on && kc0 == 0;
          const int n_sp = !sp ? 0 : max(0, min(e, NP) - max(0, e - 3));
          const int n_b = (sp && e <= 2) ? PendN<EPI>::total - NP : 0;
          wait_vm(12 + n_sp + n_b);
        } else {
          CFM_VMCNT(0);
        }
        if (e < NP && pend_on && kc0 == 0) {
          int r = rowq;
          asm volatile("" : "+v"(r));   // (see pack_tile)
          __builtin_amdgcn_raw_buffer_store_b128(pend[e], rO[0], ((r + 16 * e) * ldO[0] + col_g) * 2, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // ================= MFMA segment
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], af[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        slot = slot == 4 ? 0 : slot + 1;
        slot4 = slot4 == 4 ? 0 : slot4 + 1;
      }
    }
    epi_t = t;
  }
  if (epi_t >= 0) tile_epilogue<EPI, ACT>(acc, epi_t / nbn, epi_t % nbn, wm, wn, fr, g, M, ep);
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
}

// A/B switch for in-process experiments ("gemm_variant" model option): 5 = s_setprio(1) around each
// MFMA segment, 6 = static priority 1 for the later wave group (MI355X_MICROARCH.md, two waves per SIMD)
static int g_gemm_variant = 0;
void gemm_set_variant(int v) { g_gemm_variant = v; }

static int ring_mode() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("CFM_GEMM_RING"); v = e ? atoi(e) : 0; }
  return v;
}

template <int EPI, int ACT>
static int launch256(const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K, const EpiArgs& ep_in,
                     hipStream_t st) {
  const int tiles = ((M + 255) / 256) * (N / 256);
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
    n_cu = (n_cu + 7) / 8 * 8;
  }
  const int grid = tiles <= n_cu ? tiles : n_cu;   // persistent: one 512-thread block per CU
  static int diag_env = -1;
  if (diag_env < 0) { const char* e = getenv("CFM_GEMM_DIAG"); diag_env = e ? atoi(e) : 0; }
  const int diag = g_gemm_variant ? g_gemm_variant : diag_env;
  EpiArgs ep = ep_in;
  static int store_env = -1;
  if (store_env < 0) { const char* e = getenv("CFM_STORE_MODE"); store_env = e ? atoi(e) : 0; }
  if (store_env) ep.store_mode = store_env;
  static int cg_env = -1;
  if (cg_env < 0) { const char* e = getenv("CFM_GEMM_COLGROUP"); cg_env = e ? atoi(e) : 0; }
  if (cg_env) ep.col_group = cg_env;
  if constexpr (EPI == EPI_STORE || EPI == EPI_QKV || EPI == EPI_GLU) {
    if (ring_mode() == 2 && diag == 0 && K % 512 == 0 && (size_t)256 * ldw * 2 < (1u << 31) &&
        (size_t)256 * lda * 2 < (1u << 31)) {
      hipLaunchKernelGGL((gemm_bf16_spread_kernel<EPI, ACT>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
      CFM_CHECK_LAUNCH();
      return 0;
    }
  }
  if constexpr (EPI != EPI_RESID) {
    if (ring_mode() == 1 && K % 128 == 0 && (size_t)256 * ldw * 2 < (1u << 31) && (size_t)256 * lda * 2 < (1u << 31)) {
      if (diag == 1)
        hipLaunchKernelGGL((gemm_bf16_ring_kernel<EPI, ACT, 1>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
      else if (diag == 3)
        hipLaunchKernelGGL((gemm_bf16_ring_kernel<EPI, ACT, 3>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
      else if (diag == 4)
        hipLaunchKernelGGL((gemm_bf16_ring_kernel<EPI, ACT, 4>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
      else if (diag == 2)
        hipLaunchKernelGGL((gemm_bf16_ring_kernel<EPI, ACT, 2>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
      else
        hipLaunchKernelGGL((gemm_bf16_ring_kernel<EPI, ACT, 0>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
      CFM_CHECK_LAUNCH();
      return 0;
    }
  }
  if (diag == 1)
    hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, 1>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
  else if (diag == 2)
    hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, 2>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
  else if (diag == 5)
    hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, 5>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
  else if (diag == 6)
    hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, 6>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
  else
    hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, ACT, 0>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, N, K, ep);
  CFM_CHECK_LAUNCH();
  return 0;
}

// returns -1 when the shape is not eligible (caller falls back to the 128x128 kernel)
int gemm_bf16_wst(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st);

int gemm_bf16_big(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st) {
  if (M <= 0) return 0;
  {
    EpiArgs e2 = ep;
    const int r = gemm_bf16_wst(epi, act, A, lda, W, ldw, M, N, K, e2, st);   // K = 512: weight tile in registers
    if (r != -1) return r;
  }
  if (N % 256 || K % 64 || lda % 8 || ldw % 8) return -1;
  if (epi == EPI_GLU && ep.bias == nullptr) return -1;
  switch (epi) {
    case EPI_STORE:
      if (act == ACT_RELU) return launch256<EPI_STORE, ACT_RELU>(A, lda, W, ldw, M, N, K, ep, st);
      if (act == ACT_SILU) return launch256<EPI_STORE, ACT_SILU>(A, lda, W, ldw, M, N, K, ep, st);
      return launch256<EPI_STORE, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_STORE_F32: return launch256<EPI_STORE_F32, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_RESID: return launch256<EPI_RESID, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_QKV: return launch256<EPI_QKV, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_GLU: return launch256<EPI_GLU, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
  }
  return -1;
}

}  // namespace cfm
