// Convolution module middle: overlapping-chunk window -> mask -> depthwise
// conv k=15 (valid) -> LayerNorm(channels) -> SiLU.
//
// Reference: ChunkConvolutionModule.forward_parallel_chunk (convolution.py:224-249)
// and, with other descriptors, the dynamic-chunk padded `forward`
// (convolution.py:133-186).  pointwise_conv1+GLU runs in the GEMM epilogue and
// writes a flat GLU stream; pointwise_conv2 (+ output mask) is the next GEMM.
//
// Descriptor (cfm_common.h CD_*): output row i of the block reads stream rows
// SRC_ROW0 + i + t, t = 0..14, i.e. window columns j = i + t; columns outside
// [J_LO, J_HI) are zero (torch.where(mask_pad, x, 0) / zero padding).
// One wave per output row, lane l owns channels [l*VPL, l*VPL+VPL); the LN
// statistics are wave reductions.  Depthwise weights are stored tap-major
// [15][d] so every tap is one coalesced vector load.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

template <typename T, int VPL> struct VecIO;
template <int VPL> struct VecIO<float, VPL> {
  static CFM_DEV void load(const float* p, float (&v)[VPL]) {
#pragma unroll
    for (int e = 0; e < VPL; e += 2) {
      typedef float f2 __attribute__((ext_vector_type(2)));
      const f2 t = *reinterpret_cast<const f2*>(p + e);
      v[e] = t[0]; v[e + 1] = t[1];
    }
  }
  static CFM_DEV void store(float* p, const float (&v)[VPL]) {
#pragma unroll
    for (int e = 0; e < VPL; e += 2) {
      typedef float f2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<f2*>(p + e) = (f2){v[e], v[e + 1]};
    }
  }
};
template <typename H, int VPL> struct VecIO16 {   // bf16 / f16 streams
  typedef H h2 __attribute__((ext_vector_type(2)));
  static CFM_DEV void load(const H* p, float (&v)[VPL]) {
#pragma unroll
    for (int e = 0; e < VPL; e += 2) {
      const h2 t = *reinterpret_cast<const h2*>(p + e);
      v[e] = (float)t[0]; v[e + 1] = (float)t[1];
    }
  }
  static CFM_DEV void store(H* p, const float (&v)[VPL]) {
#pragma unroll
    for (int e = 0; e < VPL; e += 2) *reinterpret_cast<h2*>(p + e) = (h2){(H)v[e], (H)v[e + 1]};
  }
};
template <int VPL> struct VecIO<bf16, VPL> : VecIO16<bf16, VPL> {};
template <int VPL> struct VecIO<f16, VPL> : VecIO16<f16, VPL> {};

template <typename T, int VPL>
__global__ __launch_bounds__(256) void conv_dw_ln_silu_kernel(const T* __restrict__ glu, const int32_t* __restrict__ desc,
                                                              const float* __restrict__ wdw, const float* __restrict__ bdw,
                                                              const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                              float eps, T* __restrict__ out) {
  constexpr int d = VPL * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t* D = desc + (size_t)blockIdx.x * CD_INTS;
  const int out_row0 = D[CD_OUT_ROW0], nout = D[CD_NOUT], src0 = D[CD_SRC_ROW0];
  const int jlo = D[CD_J_LO], jhi = D[CD_J_HI];
  const int c0 = lane * VPL;
  float bias[VPL];
#pragma unroll
  for (int e = 0; e < VPL; ++e) bias[e] = bdw[c0 + e];
  for (int i = blockIdx.y * 4 + w; i < nout; i += 4 * gridDim.y) {
    float acc[VPL];
#pragma unroll
    for (int e = 0; e < VPL; ++e) acc[e] = bias[e];
    const int tlo = max(0, jlo - i), thi = min(15, jhi - i);
    for (int t = tlo; t < thi; ++t) {
      float xv[VPL], wv[VPL];
      VecIO<T, VPL>::load(glu + (size_t)(src0 + i + t) * d + c0, xv);
      VecIO<float, VPL>::load(wdw + t * d + c0, wv);
#pragma unroll
      for (int e = 0; e < VPL; ++e) acc[e] = fmaf(xv[e], wv[e], acc[e]);
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < VPL; ++e) s += acc[e];
    const float mean = wave_sum(s) / d;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < VPL; ++e) { const float t = acc[e] - mean; q += t * t; }
    const float rstd = rsqrtf(wave_sum(q) / d + eps);
#pragma unroll
    for (int e = 0; e < VPL; ++e) acc[e] = silu_f((acc[e] - mean) * rstd * lnw[c0 + e] + lnb[c0 + e]);
    VecIO<T, VPL>::store(out + (size_t)(out_row0 + i) * d + c0, acc);
  }
}

// bf16: one block per descriptor.  The window's GLU rows are staged once into LDS with
// 16-B loads (rows outside the unmasked columns [j_lo, j_hi) are zero there, which is the
// reference's where(mask_pad, x, 0)), so each HBM row is read by one block instead of by
// every output-row wave on whichever XCD it lands.  Each wave then produces 8 consecutive
// output rows: per tap one weight vector load and 8 LDS row reads, LayerNorm statistics
// as wave reductions, SiLU, one vector store per row.
template <int VPL>
__global__ __launch_bounds__(512) void conv_dw_ln_silu_lds_kernel(const bf16* __restrict__ glu,
                                                                  const int32_t* __restrict__ desc,
                                                                  const float* __restrict__ wdw,
                                                                  const float* __restrict__ bdw,
                                                                  const float* __restrict__ lnw,
                                                                  const float* __restrict__ lnb, float eps,
                                                                  bf16* __restrict__ out) {
  constexpr int d = VPL * 64;
  constexpr int MAXJ = 64 + 14;
  constexpr int RW = 8;   // output rows per wave
  typedef bf16 bvec __attribute__((ext_vector_type(VPL)));
  __shared__ __attribute__((aligned(16))) bf16 win[MAXJ * d];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int32_t* D = desc + (size_t)blockIdx.x * CD_INTS;
  const int out_row0 = D[CD_OUT_ROW0], nout = D[CD_NOUT], src0 = D[CD_SRC_ROW0];
  const int nj = nout + 14;
  const int jlo = max(D[CD_J_LO], 0), jhi = min(D[CD_J_HI], nj);
  constexpr int V8 = d / 8;   // 16-B vectors per row
  for (int idx = tid; idx < nj * V8; idx += 512) {
    const int j = idx / V8, v = idx % V8;
    u32x4 val = (u32x4){0u, 0u, 0u, 0u};
    if (j >= jlo && j < jhi) val = *reinterpret_cast<const u32x4*>(glu + (size_t)(src0 + j) * d + v * 8);
    *reinterpret_cast<u32x4*>(win + j * d + v * 8) = val;
  }
  __syncthreads();
  const int i0 = w * RW;
  if (i0 >= nout) return;
  const int c0 = lane * VPL;
  float acc[RW][VPL];
#pragma unroll
  for (int e = 0; e < VPL; ++e) {
    const float bv = bdw[c0 + e];
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r][e] = bv;
  }
  for (int t = 0; t < 15; ++t) {
    float wv[VPL];
    VecIO<float, VPL>::load(wdw + t * d + c0, wv);
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const bvec x = *reinterpret_cast<const bvec*>(win + min(i0 + r + t, nj - 1) * d + c0);
#pragma unroll
      for (int e = 0; e < VPL; ++e) acc[r][e] = fmaf((float)x[e], wv[e], acc[r][e]);
    }
  }
  float lw[VPL], lb[VPL];
#pragma unroll
  for (int e = 0; e < VPL; ++e) {
    lw[e] = lnw[c0 + e];
    lb[e] = lnb[c0 + e];
  }
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    if (i0 + r >= nout) break;
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < VPL; ++e) sum += acc[r][e];
    const float mean = wave_sum(sum) / d;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < VPL; ++e) { const float t = acc[r][e] - mean; q += t * t; }
    const float rstd = rsqrtf(wave_sum(q) / d + eps);
    bvec o;
#pragma unroll
    for (int e = 0; e < VPL; ++e) o[e] = (bf16)silu_f((acc[r][e] - mean) * rstd * lw[e] + lb[e]);
    *reinterpret_cast<bvec*>(out + (size_t)(out_row0 + i0 + r) * d + c0) = o;
  }
}

// bf16, VPL even (d = 128 / 256 / 512): the k = 15 depthwise conv as bf16 dot products over TAP
// PAIRS -- v_dot2_f32_bf16 adds x[j] w[t] + x[j+1] w[t+1] to an f32 accumulator in one
// instruction (bf16 taps: what conv1d runs on under the reference's bf16 autocast), instead of
// one bf16 -> f32 conversion plus one FMA per tap.  Lane l owns channels [VPL l, VPL l + VPL);
// a wave owns 8 output rows i0 + r.  The row pair (i0 + j, i0 + j + 1) is packed once per
// channel pair (v_perm_b32) and feeds every output r whose tap t = j - r is even; tap 14 pairs
// with w[15] = 0 on the window's extra zero row.  LayerNorm statistics by DPP / permlane
// reductions (no LDS round trips), SiLU as v_exp + v_rcp.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
// E = bf16: v_dot2_f32_bf16; E = f16 (fp16 mode): v_dot2_f32_f16 on f16 taps
template <typename E>
CFM_DEV float dot2e(unsigned a, unsigned b, float c) {
  if constexpr (std::is_same<E, f16>::value)
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, a), __builtin_bit_cast(f16x2_t, b), c, false);
  else
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
template <typename E>
CFM_DEV unsigned pke(float lo, float hi) {
  typedef E e2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, (e2){(E)lo, (E)hi});
}
// the compute half of the dot2 kernels: wave w's RW output rows from the staged window `win`
// (`w` indexes RW-row groups of the chunk; the staged window starts at window row win_row0)
template <int VPL, typename E>
CFM_DEV void conv_dot2_rows(const E* __restrict__ win, int nout, int out_row0, const float* __restrict__ wdw,
                            const float* __restrict__ bdw, const float* __restrict__ lnw,
                            const float* __restrict__ lnb, float eps, E* __restrict__ out, int w, int lane,
                            int win_row0 = 0) {
  constexpr int d = VPL * 64, NW = VPL / 2;
  constexpr int RW = 8;
  typedef E bvec __attribute__((ext_vector_type(VPL)));
  const int i0 = w * RW;
  if (i0 >= nout) return;
  win -= (size_t)win_row0 * d;   // rows below win_row0 are never read
  const int c0 = lane * VPL;
  // tap-pair weights: wp[p][e] = (w[2p][c0 + e], w[2p + 1][c0 + e]) as bf16x2, w[15] = 0
  unsigned wp[8][VPL];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    float lo[VPL], hi[VPL];
    VecIO<float, VPL>::load(wdw + (2 * p) * d + c0, lo);
    if (p < 7) {
      VecIO<float, VPL>::load(wdw + (2 * p + 1) * d + c0, hi);
    } else {
#pragma unroll
      for (int e = 0; e < VPL; ++e) hi[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < VPL; ++e) wp[p][e] = pke<E>(lo[e], hi[e]);
  }
  float acc[RW][VPL];
#pragma unroll
  for (int e = 0; e < VPL; ++e) {
    const float bv = bdw[c0 + e];
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[r][e] = bv;
  }
  auto ld = [&](unsigned (&x)[NW], int row) {
    const unsigned* p = reinterpret_cast<const unsigned*>(win + row * d + c0);
    if constexpr (NW == 4) {
      const u32x4 t = *reinterpret_cast<const u32x4*>(p);
      x[0] = t[0]; x[1] = t[1]; x[2] = t[2]; x[3] = t[3];
    } else if constexpr (NW == 2) {
      typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
      const u32x2_ t = *reinterpret_cast<const u32x2_*>(p);
      x[0] = t[0]; x[1] = t[1];
    } else {
      x[0] = p[0];
    }
  };
  unsigned ra[NW], rb[NW];
  ld(ra, i0);
#pragma unroll
  for (int j = 0; j < RW + 14; ++j) {
    ld(rb, i0 + j + 1);
    unsigned pk[VPL];   // channel e: (row i0 + j, row i0 + j + 1)
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      pk[2 * k] = __builtin_amdgcn_perm(rb[k], ra[k], 0x05040100u);
      pk[2 * k + 1] = __builtin_amdgcn_perm(rb[k], ra[k], 0x07060302u);
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int t = j - r;
      if (t >= 0 && t <= 14 && (t & 1) == 0) {
#pragma unroll
        for (int e = 0; e < VPL; ++e) acc[r][e] = dot2e<E>(pk[e], wp[t >> 1][e], acc[r][e]);
      }
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) ra[k] = rb[k];
  }
  float lw[VPL], lb[VPL];
#pragma unroll
  for (int e = 0; e < VPL; ++e) {
    lw[e] = lnw[c0 + e];
    lb[e] = lnb[c0 + e];
  }
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    if (i0 + r >= nout) break;
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < VPL; ++e) sum += acc[r][e];
    const float mean = wave_sum_dpp(sum) / d;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < VPL; ++e) { const float t = acc[r][e] - mean; q += t * t; }
    const float rstd = rsqrtf(wave_sum_dpp(q) / d + eps);
    bvec o;
#pragma unroll
    for (int e = 0; e < VPL; ++e) {
      const float y = (acc[r][e] - mean) * rstd * lw[e] + lb[e];
      o[e] = (E)(y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * y)));
    }
    // non-temporal: read once, by pw2 (A/B x3: this kernel 1.72 -> 1.66 ms/step, pw2 1.13 -> 1.09)
    __builtin_nontemporal_store(o, reinterpret_cast<bvec*>(out + (size_t)(out_row0 + i0 + r) * d + c0));
  }
}

template <int VPL, typename E>
__global__ __launch_bounds__(512) void conv_dw_ln_silu_dot2_kernel(const E* __restrict__ glu,
                                                                   const int32_t* __restrict__ desc,
                                                                   const float* __restrict__ wdw,
                                                                   const float* __restrict__ bdw,
                                                                   const float* __restrict__ lnw,
                                                                   const float* __restrict__ lnb, float eps,
                                                                   E* __restrict__ out, int dma) {
  constexpr int d = VPL * 64, NW = VPL / 2;   // NW dwords (channel pairs) per lane per row
  constexpr int MAXJ = 64 + 15;               // window rows + the zero row of the w[15] = 0 tap
  constexpr int RW = 8;                       // output rows per wave
  typedef E bvec __attribute__((ext_vector_type(VPL)));
  __shared__ __attribute__((aligned(16))) E win[MAXJ * d];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int32_t* D = desc + (size_t)blockIdx.x * CD_INTS;
  const int out_row0 = D[CD_OUT_ROW0], nout = D[CD_NOUT], src0 = D[CD_SRC_ROW0];
  const int nj = nout + 14;
  const int jlo = max(D[CD_J_LO], 0), jhi = min(D[CD_J_HI], nj);
  constexpr int V8 = d / 8;   // 16-B vectors per row
  if (VPL == 8 && dma) {
    // d = 512: a row is 1 KiB = one LDS-DMA instruction (64 lanes x 16 B, lane-linear), all of the
    // window in flight at once; rows outside [jlo, jhi) are zeroed instead
    for (int j = __builtin_amdgcn_readfirstlane(w); j < MAXJ; j += 8) {
      if (j >= jlo && j < jhi)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(glu + (size_t)(src0 + j) * d + lane * 8),
                                         (__attribute__((address_space(3))) void*)(win + j * d), 16, 0, 0);
      else
        *reinterpret_cast<u32x4*>(win + j * d + lane * 8) = (u32x4){0u, 0u, 0u, 0u};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int idx = tid; idx < MAXJ * V8; idx += 512) {
      const int j = idx / V8, v = idx % V8;
      u32x4 val = (u32x4){0u, 0u, 0u, 0u};
      if (j >= jlo && j < jhi) val = *reinterpret_cast<const u32x4*>(glu + (size_t)(src0 + j) * d + v * 8);
      *reinterpret_cast<u32x4*>(win + j * d + v * 8) = val;
    }
  }
  __syncthreads();
  conv_dot2_rows<VPL, E>(win, nout, out_row0, wdw, bdw, lnw, lnb, eps, out, w, lane);
}


// Half-chunk blocks: the dot2 kernel needs 243 VGPRs (2 waves per SIMD), so one 8-wave block holds
// a whole CU and every chunk's window DMA waits with no other work on the CU.  Here a 4-wave block
// takes 32 output rows of a chunk (window rows 32h .. 32h + 46, 47 KiB), two blocks share a CU and
// one block's window DMA overlaps the other's arithmetic; the 14 overlap rows are read twice.
template <int VPL, int QR, typename E>
__global__ __launch_bounds__(QR * 8) void conv_dw_ln_silu_dot2h_kernel(const E* __restrict__ glu,
                                                                    const int32_t* __restrict__ desc,
                                                                    const float* __restrict__ wdw,
                                                                    const float* __restrict__ bdw,
                                                                    const float* __restrict__ lnw,
                                                                    const float* __restrict__ lnb, float eps,
                                                                    E* __restrict__ out) {
  constexpr int d = VPL * 64, NWV = QR / 8;
  constexpr int HJ = QR + 15;   // window rows of the block (+ the zero row of the w[15] = 0 tap)
  __shared__ __attribute__((aligned(16))) E win[HJ * d];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int half = blockIdx.y;
  const int32_t* D = desc + (size_t)blockIdx.x * CD_INTS;
  const int out_row0 = D[CD_OUT_ROW0], nout = D[CD_NOUT], src0 = D[CD_SRC_ROW0];
  if (QR * half >= nout) return;
  const int nj = nout + 14;
  const int jlo = max(D[CD_J_LO], 0), jhi = min(D[CD_J_HI], nj);
  const int r0 = QR * half;
  if (VPL == 8) {
    for (int jj = __builtin_amdgcn_readfirstlane(w); jj < HJ; jj += NWV) {
      const int j = r0 + jj;
      if (j >= jlo && j < jhi)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(glu + (size_t)(src0 + j) * d + lane * 8),
                                         (__attribute__((address_space(3))) void*)(win + jj * d), 16, 0, 0);
      else
        *reinterpret_cast<u32x4*>(win + jj * d + lane * 8) = (u32x4){0u, 0u, 0u, 0u};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    constexpr int V8 = d / 8;
    for (int idx = tid; idx < HJ * V8; idx += QR * 8) {
      const int jj = idx / V8, v = idx % V8, j = r0 + jj;
      u32x4 val = (u32x4){0u, 0u, 0u, 0u};
      if (j >= jlo && j < jhi) val = *reinterpret_cast<const u32x4*>(glu + (size_t)(src0 + j) * d + v * 8);
      *reinterpret_cast<u32x4*>(win + jj * d + v * 8) = val;
    }
  }
  __syncthreads();
  conv_dot2_rows<VPL, E>(win, nout, out_row0, wdw, bdw, lnw, lnb, eps, out, NWV * half + w, lane, r0);
}

template <typename T>
int conv_dw_ln_silu(const T* glu, const int32_t* desc, int nblk, int d, const float* wdw_t, const float* bdw,
                    const float* lnw, const float* lnb, float eps, T* out, hipStream_t st, int dot2, int dma) {
  if (nblk <= 0) return 0;
  // dot2 = 0: the per-tap f32 kernel; dma = 0: stage the window through registers (A/B, model options)
  if constexpr (sizeof(T) == 2) {   // bf16 / f16 (the non-dot2 LDS kernel: bf16 only)
    if (dot2 >= 2 && d == 512) {   // half-chunk blocks (conv_dot2 = 2), quarter-chunk blocks (3)
      if (dot2 == 3)
        hipLaunchKernelGGL((conv_dw_ln_silu_dot2h_kernel<8, 16, T>), dim3(nblk, 4), dim3(128), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
      else
        hipLaunchKernelGGL((conv_dw_ln_silu_dot2h_kernel<8, 32, T>), dim3(nblk, 2), dim3(256), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
      CFM_CHECK_LAUNCH();
      return 0;
    }
    if (dot2) {
      if (d == 128) hipLaunchKernelGGL((conv_dw_ln_silu_dot2_kernel<2, T>), dim3(nblk), dim3(512), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out, dma);
      else if (d == 256) hipLaunchKernelGGL((conv_dw_ln_silu_dot2_kernel<4, T>), dim3(nblk), dim3(512), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out, dma);
      else if (d == 512) hipLaunchKernelGGL((conv_dw_ln_silu_dot2_kernel<8, T>), dim3(nblk), dim3(512), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out, dma);
      else return (int)hipErrorInvalidValue;
      CFM_CHECK_LAUNCH();
      return 0;
    }
    if constexpr (std::is_same<T, bf16>::value) {
      if (d == 128) hipLaunchKernelGGL((conv_dw_ln_silu_lds_kernel<2>), dim3(nblk), dim3(512), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
      else if (d == 256) hipLaunchKernelGGL((conv_dw_ln_silu_lds_kernel<4>), dim3(nblk), dim3(512), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
      else if (d == 512) hipLaunchKernelGGL((conv_dw_ln_silu_lds_kernel<8>), dim3(nblk), dim3(512), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
      else return (int)hipErrorInvalidValue;
      CFM_CHECK_LAUNCH();
      return 0;
    }
  }
  const dim3 grid(nblk, 4);   // 4 x 4 waves stride over the (<= 64) rows of a block
  if (d == 128) hipLaunchKernelGGL((conv_dw_ln_silu_kernel<T, 2>), grid, dim3(256), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
  else if (d == 256) hipLaunchKernelGGL((conv_dw_ln_silu_kernel<T, 4>), grid, dim3(256), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
  else if (d == 512) hipLaunchKernelGGL((conv_dw_ln_silu_kernel<T, 8>), grid, dim3(256), 0, st, glu, desc, wdw_t, bdw, lnw, lnb, eps, out);
  else return (int)hipErrorInvalidValue;
  CFM_CHECK_LAUNCH();
  return 0;
}

template int conv_dw_ln_silu<float>(const float*, const int32_t*, int, int, const float*, const float*, const float*,
                                    const float*, float, float*, hipStream_t, int, int);
template int conv_dw_ln_silu<bf16>(const bf16*, const int32_t*, int, int, const float*, const float*, const float*,
                                   const float*, float, bf16*, hipStream_t, int, int);
template int conv_dw_ln_silu<f16>(const f16*, const int32_t*, int, int, const float*, const float*, const float*,
                                   const float*, float, f16*, hipStream_t, int, int);

}  // namespace cfm
