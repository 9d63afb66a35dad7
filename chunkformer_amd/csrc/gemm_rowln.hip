// Row-owning bf16 MFMA GEMM for the N = d_model = 512 outputs of an encoder layer, with the residual
// add and the LayerNorm(s) that follow each of them fused into its epilogue.
//
//   C[M, 512] = A[M, K] . W[512, K]^T + b     (bf16 in, f32 accumulate), K % 64 == 0
//
// Why: each of a layer's four branch outputs (FFN w2 of both FFNs, linear_out, pointwise_conv2) feeds a
// LayerNorm over the whole 512-column row (encoder_layer.py:155-248).  Unfused, every branch output y
// makes a round trip through HBM (bf16 write, read back by a LayerNorm kernel) and the LayerNorm kernels
// run at the copy ceiling (8.2 ms per 240-min step, 50 GB).  Here one workgroup owns whole rows, so the
// residual stream is read, updated, normalised and the next GEMM's operand h written in the epilogue of
// the GEMM that produced the branch, beside the MFMA work of the other row group.
//
// Structure (gemm_bf16.hip's ping-pong, re-cut for full rows):
//   * tile = 128 rows x 512 columns; 512 threads = 8 waves = 2 row groups (grp: rows 64 grp ..) x 4
//     column quarters (wn: columns 128 wn ..); each wave owns 64 x 128 of C, acc[8 n-blocks][4 m-blocks],
//     with swapped operands (MFMA A = W fragment), so lane (fr, g) holds C[16 mb + fr][16 nb + 4g .. +3];
//   * per K-step of 64: A 128 x 64 (16 KiB) and W 512 x 64 (64 KiB) by LDS-DMA into two-slot rings (all
//     160 KiB of the CU); 128-B rows with the 16-B chunk swizzle chunk ^ ((row >> 1) & 7) applied on the
//     source address, so the ds_read_b128 fragment reads are conflict-free; each row group stages its own
//     64 A rows, W is staged by group 0 (16 pieces per wave); step s + 1 is issued in step s's first LOAD segment and
//     waited behind its last MFMA segment;
//   * the two row groups run one barrier segment apart (ping-pong): one group's MFMA segments overlap the
//     other group's LDS reads, DMA issue and epilogue;
//   * epilogue (per row group, its 64 rows x 512 columns): v = bf16(acc) (the rounding the unfused bf16
//     branch output had), the residual terms, then per LayerNorm ONE extra barrier segment: Welford
//     partials (mean, M2 over the lane's 32 columns) merged over the 4 lanes of a row (xor 16, 32) and
//     over the group's 4 waves through a 2 KiB exchange in the group's own 64 rows of the A slot just
//     consumed (nothing reads or refills them until that group's next DMA issue).
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "gemm_bf16_epi.h"

namespace cfm {

namespace {
constexpr int RL_N = 512, RL_MT = 128, RL_KS = 64;
constexpr int RL_ASLOT = RL_MT * RL_KS * 2;   // 16 KiB
constexpr int RL_WSLOT = RL_N * RL_KS * 2;    // 64 KiB
typedef bf16 rl_bf16x4 __attribute__((ext_vector_type(4)));

CFM_DEV f32x4 round_bf16x4(f32x4 v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (float)(bf16)v[e];
  return v;
}
// merge the Welford partials (mean m, M2 q) of two equal-count parts of n each (lanes l and l ^ X):
// symmetric, so both lanes end with bit-identical values
template <int X>
CFM_DEV void welford_xor(float& m, float& q, float n) {
  const float mo = __shfl_xor(m, X, 64), qo = __shfl_xor(q, X, 64);
  const float d = m - mo;
  q = (q + qo) + (0.5f * n) * (d * d);
  m = 0.5f * (m + mo);
}
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
// the four words of a raw buffer resource (base, num_records bytes; the flags of make_buffer_rsrc below),
// wave-uniform, as an SGPR quad for inline asm
CFM_DEV u32x4 rs_words(const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)p;
  return (u32x4){(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                 (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32)) & 0xffffu,
                 (unsigned)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}
}  // namespace

// site flags (compile time: only the arrays a site uses cost registers)
enum { RF_Y1 = 1, RF_YOUT = 2, RF_XOUT = 4, RF_FOUT = 8, RF_ACCMASK = 16, RF_Y1MASK = 32, RF_HMASK = 64, RF_NT = 128 };

template <int NX, int FL, int R, int DIAG = 0>
__global__ __launch_bounds__(512, 1) void gemm_rowln_kernel(const bf16* __restrict__ A, int lda,
                                                            const bf16* __restrict__ W, int ldw, int M, int K,
                                                            RowLnArgs ra_) {
  // a local copy: the lambdas below capture by reference, and a reference to the by-value kernel argument
  // would keep it in a private (scratch) copy
  const RowLnArgs ra = ra_;
  __shared__ __attribute__((aligned(16))) char smem[2 * RL_ASLOT + 2 * RL_WSLOT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2), wn = __builtin_amdgcn_readfirstlane(wid & 3);
  const int fr = lane & 15, g = lane >> 4;
  const int T = (M + RL_MT - 1) / RL_MT;
  const int t_first = blockIdx.x, t_step = gridDim.x;
  if (t_first >= T) return;
  const int nk = K / RL_KS;

  // ---- LDS-DMA of step (t, kt) into ring slot `slot`: piece p = rows 8p .. 8p + 7 (1 KiB, lane-linear),
  // row 8p + lane / 8, XOR key (row >> 1) & 7 = (4p + lane / 16) & 7 (pre-swizzled source chunk)
  // buffer LDS-DMA: per-lane 32-bit offsets (row, swizzled chunk) fixed for the whole kernel, the K slice
  // in soffset, A by a per-tile descriptor (rows past M read as 0)
  unsigned voffA[2], voffW[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {   // this group's A rows: pieces 8 grp + 2 wn + i
    const int srow = 8 * (8 * grp + 2 * wn + i) + (lane >> 3);
    voffA[i] = (unsigned)(srow * lda + ((lane & 7) ^ ((4 * i + (lane >> 4)) & 7)) * 8) * 2u;
  }
  // W is staged by group 0 alone (16 pieces per wave: rows 128 wn + 8 i ..), which waits for it at the end
  // of its step and so before group 1 reads it one segment later; piece i's row offset 8 i rows goes in
  // soffset, its chunk swizzle depends on i & 1 only
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int srow = 128 * wn + (lane >> 3);
    voffW[i] = (unsigned)(srow * ldw + ((lane & 7) ^ ((4 * i + (lane >> 4)) & 7)) * 8) * 2u;
  }
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, RL_N * ldw * 2, 0x00020000);
  auto stage = [&](int t, int kt, int slot) __attribute__((always_inline)) {
    const int rows = __builtin_amdgcn_readfirstlane(min(RL_MT, M - t * RL_MT));
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)t * RL_MT * lda), (short)0, rows * lda * 2, 0x00020000);
    const int soff = __builtin_amdgcn_readfirstlane(kt * RL_KS * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + slot * RL_ASLOT + (8 * grp + 2 * wn + i) * 1024), 16,
          voffA[i], soff, 0, 0);
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsW,
            (__attribute__((address_space(3))) void*)(smem + 2 * RL_ASLOT + slot * RL_WSLOT + (16 * wn + i) * 1024),
            16, voffW[i & 1], soff + i * 16 * ldw, 0, 0);
    }
  };

  f32x4 acc[8][4];
  bf16x8 wf[8], af[4];
  const int key = (fr >> 1) & 7;
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  const unsigned arow = (unsigned)((64 * grp + fr) * 128);
  const unsigned wrow = (unsigned)(2 * RL_ASLOT + (128 * wn + fr) * 128);
  const int col0 = 128 * wn + 4 * g;   // column of this lane's n-block 0

  // bias seed of every tile's accumulators, re-loaded per tile (L2 hits) through an opaque offset: hoisted
  // out of the tile loop (loop-invariant), the 32 bias registers stayed live across the K-loop
  auto seed = [&]() __attribute__((always_inline)) {
    unsigned bo = (unsigned)col0;
    asm volatile("" : "+v"(bo));
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const f32x4 b = ra.bias ? *reinterpret_cast<const f32x4*>(ra.bias + (bo + 16u * nb)) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) acc[nb][mb] = b;
    }
  };

  // ---- tile end: v = bf16(acc) (the rounding the unfused branch output had) to ybuf, 8 contiguous columns
  // per lane after a permlane16 swap of n-block pairs; a descriptor over the group's valid rows drops the
  // stores past M.  The offset is opaque per tile (hoisted, every constant sum became a VGPR of its own).
  bf16* const ybuf = (FL & RF_YOUT) ? ra.y_out : ra.ybuf;
  auto store_y = [&](int tp) __attribute__((always_inline)) {
    const int grow = tp * RL_MT + 64 * grp;
    const int nrow = __builtin_amdgcn_readfirstlane(max(0, min(64, M - grow)));
    if constexpr (NX == 0 && (FL & RF_FOUT) != 0) {   // plain GEMM, f32 output alpha * (acc + bias)
      const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc((void*)(ra.f_out + (size_t)grow * RL_N),
                                                                         (short)0, nrow * RL_N * 4, 0x00020000);
      unsigned vo = (unsigned)(fr * RL_N + col0) * 4u;
      asm volatile("" : "+v"(vo));
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ra.alpha * acc[nb][mb]), rf, vo + 64u * nb,
                                                 mb * 16 * RL_N * 4, 0);
      return;
    }
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void*)(ybuf + (size_t)grow * RL_N), (short)0, nrow * RL_N * 2, 0x00020000);
    unsigned vo = (unsigned)(fr * RL_N + 128 * wn + 16 * (g & 1) + 8 * (g >> 1)) * 2u;
    asm volatile("" : "+v"(vo));
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const f32x4 a = acc[2 * p][mb], b = acc[2 * p + 1][mb];
        const auto r0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(a[0], a[1]), pack_bf16x2(b[0], b[1]), false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(a[2], a[3]), pack_bf16x2(b[2], b[3]), false, false);
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){r0[0], r1[0], r0[1], r1[1]}, ry, vo + 64u * p,
                                               mb * 16 * RL_N * 2, NX == 0 && (FL & RF_NT) ? 2 : 0);
      }
  };

  // ---- the residual add and LayerNorm(s) of one row by one wave (lane l: columns 8l .. 8l + 7), the
  // arithmetic of norm.hip's ln_kernel / ln2_kernel (two-pass statistics by DPP wave sums)
  struct RowIn {
    f32x4 x0, x1;
    u32x4 y, y1;
    float am, a1m;
  };
  auto load_row = [&](int row, RowIn& r) __attribute__((always_inline)) {
    const size_t e = (size_t)row * RL_N + 8 * lane;
    r.x0 = *reinterpret_cast<const f32x4*>(ra.x + e);
    r.x1 = *reinterpret_cast<const f32x4*>(ra.x + e + 4);
    r.y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ybuf + e));
    if (FL & RF_Y1) r.y1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ra.y1 + e));
    r.am = ra.alpha * ((FL & RF_ACCMASK) ? (float)ra.accmask[row] : 1.f);
    r.a1m = ra.a1 * ((FL & RF_Y1MASK) ? (float)ra.y1mask[row] : 1.f);
  };
  auto ln8 = [&](float (&v)[8], const float* w, const float* b) __attribute__((always_inline)) {
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += v[e];
    const float mean = wave_sum_dpp(sum) / RL_N;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = v[e] - mean;
      q += t * t;
    }
    const float rstd = rsqrtf(wave_sum_dpp(q) / RL_N + ra.eps);
    // weights through an opaque offset: loop-invariant, hipcc hoisted them out of the tile loop (type-based
    // alias analysis lets f32 loads pass the bf16 stores) and held 16 / 32 VGPRs for the whole kernel
    unsigned wo = 8u * lane;
    asm volatile("" : "+v"(wo));
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + wo), w1 = *reinterpret_cast<const f32x4*>(w + wo + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + wo), b1 = *reinterpret_cast<const f32x4*>(b + wo + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = (v[e] - mean) * rstd * w0[e] + b0[e];
      v[e + 4] = (v[e + 4] - mean) * rstd * w1[e] + b1[e];
    }
  };
  auto process_row = [&](int row, const RowIn& r) __attribute__((always_inline)) {
    const size_t e = (size_t)row * RL_N + 8 * lane;
    float v[8] = {r.x0[0], r.x0[1], r.x0[2], r.x0[3], r.x1[0], r.x1[1], r.x1[2], r.x1[3]};
    if (FL & RF_Y1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = fmaf(r.a1m, __builtin_bit_cast(float, r.y1[k] << 16), v[2 * k]);
        v[2 * k + 1] = fmaf(r.a1m, __builtin_bit_cast(float, r.y1[k] & 0xffff0000u), v[2 * k + 1]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = fmaf(r.am, __builtin_bit_cast(float, r.y[k] << 16), v[2 * k]);
      v[2 * k + 1] = fmaf(r.am, __builtin_bit_cast(float, r.y[k] & 0xffff0000u), v[2 * k + 1]);
    }
    if (NX == 1 && (FL & RF_XOUT)) {
      __builtin_nontemporal_store((f32x4){v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(ra.x_out + e));
      __builtin_nontemporal_store((f32x4){v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(ra.x_out + e + 4));
    }
    ln8(v, ra.g1, ra.b1);
    if constexpr (NX == 2) {
      if (FL & RF_XOUT) {
        __builtin_nontemporal_store((f32x4){v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(ra.x_out + e));
        __builtin_nontemporal_store((f32x4){v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(ra.x_out + e + 4));
      }
      ln8(v, ra.g2, ra.b2);
    }
    if (FL & RF_FOUT) {
      *reinterpret_cast<f32x4*>(ra.f_out + e) = (f32x4){v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(ra.f_out + e + 4) = (f32x4){v[4], v[5], v[6], v[7]};
    } else {
      u32x4 o = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
      if ((FL & RF_HMASK) && !ra.hmask[row]) o = (u32x4){0u, 0u, 0u, 0u};
      __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(ra.h_out + e));
    }
  };

  auto seg_barrier = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  int t1 = t_first, k1 = 0;   // step s + 1
  auto advance = [&](int& t, int& k) __attribute__((always_inline)) {
    if (++k == nk) {
      k = 0;
      t += t_step;
    }
  };
  stage(t_first, 0, 0);
  advance(t1, k1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");   // stagger group 1 by one segment

  // LayerNorm pipeline of the previous tile's rows: this wave owns rows lr0 + i, i < 16 (16 rows of its row
  // group).  Tile t's y is stored in tile t + 1's first LOAD segment; from step 1 on (the stores are waited
  // at the end of step 0, and only this row group's waves wrote these rows) R rows are loaded per step and
  // processed one step later, after the end-of-step wait, beside the other group's MFMA segments.
  int lr0 = -1, nload = 16, nproc = 16;
  RowIn rin[R];
  int s = 0, prev_t = -1;
  for (int t = t_first; t < T; t += t_step) {
    for (int kt = 0; kt < nk; ++kt, ++s) {
      const bool has1 = t1 < T;
      const unsigned slot = (unsigned)(s & 1);
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        // ================= LOAD segment: (tile end), fragments of (s, ss), LayerNorm rows, DMA
        if (ss == 0 && kt == 0) {
          if (prev_t >= 0) {
            if constexpr (DIAG != 1) store_y(prev_t);
            lr0 = prev_t * RL_MT + 64 * grp + 16 * wn;
            nload = nproc = 0;
          }
          seed();
        }
        if (NX > 0 && ss == 0) {
          if constexpr (DIAG != 1) {
            // the rows loaded one step ago; then the next rows, spread evenly over steps 1 .. nk - 2 (every
            // CU's LayerNorm traffic beside its K-loop, not in one burst), issued before the DMA pieces
#pragma unroll
            for (int r = 0; r < R; ++r)
              if (nproc < nload) {
                if (lr0 + nproc < M) process_row(lr0 + nproc, rin[r]);
                ++nproc;
              }
            if (kt >= 1) {
#pragma unroll
              for (int r = 0; r < R; ++r)
                if (nload < 16 && nload * (nk - 2) < kt * 16) {   // row i at step 1 + floor(i (nk - 2) / 16) <= nk - 2
                  if (lr0 + nload < M) load_row(lr0 + nload, rin[r]);
                  ++nload;
                }
            }
          }
        }
        // fragments after the LayerNorm rows: not live across them (register pressure)
        const unsigned pos = (unsigned)(((ss * 4 + g) ^ key) << 4);
        const unsigned aa = lds_base + slot * RL_ASLOT + arow + pos;
        const unsigned wa = lds_base + slot * RL_WSLOT + wrow + pos;
        af[0] = lds_read_b128<0>(aa);
        af[1] = lds_read_b128<2048>(aa);
        af[2] = lds_read_b128<4096>(aa);
        af[3] = lds_read_b128<6144>(aa);
        wf[0] = lds_read_b128<0>(wa);
        wf[1] = lds_read_b128<2048>(wa);
        wf[2] = lds_read_b128<4096>(wa);
        wf[3] = lds_read_b128<6144>(wa);
        wf[4] = lds_read_b128<8192>(wa);
        wf[5] = lds_read_b128<10240>(wa);
        wf[6] = lds_read_b128<12288>(wa);
        wf[7] = lds_read_b128<14336>(wa);
        if (ss == 0 && has1) stage(t1, k1, (s + 1) & 1);
        seg_barrier();
        // ================= MFMA segment
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
            acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nb], af[mb], acc[nb][mb], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // step s + 1 of this wave landed, and its LayerNorm loads / stores (waited behind the MFMAs just
        // issued; the barrier then covers every wave's pieces before the next LOAD segment reads them)
        if (ss == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      advance(t1, k1);
    }
    prev_t = t;
  }
  // drain: the rows still in flight, the last tile's y, then its rows (four at a time)
  if constexpr (DIAG != 1) {
    if constexpr (NX > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (nproc < nload) {
          if (lr0 + nproc < M) process_row(lr0 + nproc, rin[r]);
          ++nproc;
        }
      for (; nload < 16; ++nload)
        if (lr0 + nload < M) {
          load_row(lr0 + nload, rin[0]);
          process_row(lr0 + nload, rin[0]);
        }
    }
    store_y(prev_t);
  }
  if constexpr (NX > 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");   // every wave's y stores of its row group landed
    if constexpr (DIAG != 1) {
      lr0 = prev_t * RL_MT + 64 * grp + 16 * wn;
      for (int i0 = 0; i0 < 16; i0 += 4) {
        RowIn rd[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (lr0 + i0 + i < M) load_row(lr0 + i0 + i, rd[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (lr0 + i0 + i < M) process_row(lr0 + i0 + i, rd[i]);
      }
    }
  }
  if (grp == 0) asm volatile("s_barrier" ::: "memory");
}

int gemm_rowln_bf16(const bf16* A, int lda, const bf16* W, int ldw, int M, int K, const RowLnArgs& ra, hipStream_t st) {
  if (M <= 0) return 0;
  const int nk = K / RL_KS;
  if (K <= 0 || K % RL_KS || nk < 8 || lda % 8 || ldw % 8) return -1;
  if (ra.g1) {   // the fused forms
    if (!ra.x || !ra.b1 || (!ra.h_out == !ra.f_out) || (ra.g2 == nullptr) != (ra.b2 == nullptr) || (!ra.y_out && !ra.ybuf))
      return -1;
  } else if (!ra.y_out == !ra.f_out) {
    return -1;
  }
  const int fl = (ra.y1 ? RF_Y1 : 0) | (ra.y_out ? RF_YOUT : 0) | (ra.x_out ? RF_XOUT : 0) | (ra.f_out ? RF_FOUT : 0) |
                 (ra.accmask ? RF_ACCMASK : 0) | (ra.y1mask ? RF_Y1MASK : 0) | (ra.hmask ? RF_HMASK : 0) |
                 (!ra.g1 && ra.y_out && ra.nt ? RF_NT : 0);
  const int tiles = (M + RL_MT - 1) / RL_MT;
  const int grid = tiles < cu_count() ? tiles : cu_count();
  // rows per LayerNorm slot: a wave's 16 rows loaded in steps 1 .. nk - 2 (R (nk - 2) >= 16)
  const bool r1 = nk >= 18;
#define RL_GO(NX, FL, RR, D) hipLaunchKernelGGL((gemm_rowln_kernel<NX, FL, RR, D>), dim3(grid), dim3(512), 0, st, A, lda, W, ldw, M, K, ra)
#ifdef CFM_GEMM_DIAG
#define RL_LAUNCH(NX, FL)                                  \
  do {                                                     \
    if (ra.diag == 1) {                                    \
      if (r1) RL_GO(NX, FL, 1, 1); else RL_GO(NX, FL, 3, 1); \
    } else {                                               \
      if (r1) RL_GO(NX, FL, 1, 0); else RL_GO(NX, FL, 3, 0); \
    }                                                      \
  } while (0)
#else
#define RL_LAUNCH(NX, FL)                                  \
  do {                                                     \
    if (r1) RL_GO(NX, FL, 1, 0); else RL_GO(NX, FL, 3, 0);   \
  } while (0)
#endif
  // the sites of an encoder layer (ModelT::encode): FFN_mac w2, linear_out (masked / padded), pointwise_conv2,
  // FFN w2 (inner layer / last layer)
  if (!ra.g1) {   // plain GEMM (gemm_n512_bf16)
    if (fl == RF_YOUT) RL_LAUNCH(0, RF_YOUT);
    else if (fl == (RF_YOUT | RF_NT)) RL_LAUNCH(0, RF_YOUT | RF_NT);
    else if (fl == RF_FOUT) RL_LAUNCH(0, RF_FOUT);
    else return -1;
  } else if (!ra.g2) {
    switch (fl) {
      case RF_YOUT: RL_LAUNCH(1, RF_YOUT); break;
      case RF_YOUT | RF_ACCMASK: RL_LAUNCH(1, RF_YOUT | RF_ACCMASK); break;
      case RF_Y1 | RF_XOUT: RL_LAUNCH(1, RF_Y1 | RF_XOUT); break;
      case RF_Y1 | RF_XOUT | RF_HMASK: RL_LAUNCH(1, RF_Y1 | RF_XOUT | RF_HMASK); break;
      default: return -1;
    }
  } else {
    switch (fl) {
      case RF_Y1 | RF_Y1MASK | RF_XOUT: RL_LAUNCH(2, RF_Y1 | RF_Y1MASK | RF_XOUT); break;
      case RF_Y1 | RF_Y1MASK | RF_FOUT: RL_LAUNCH(2, RF_Y1 | RF_Y1MASK | RF_FOUT); break;
      default: return -1;
    }
  }
#undef RL_LAUNCH
#undef RL_GO
  CFM_CHECK_LAUNCH();
  return 0;
}

}  // namespace cfm
