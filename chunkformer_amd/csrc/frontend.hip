// 8x depthwise-striding front-end (the parts that are not GEMMs).
//
// Reference: GlobalCMVN (cmvn.py:32-43) applied to the packed windows
// (encoder.py:615-616), then DepthwiseConvSubsampling.conv (subsampling.py:69-112):
//   conv0 Conv2d(1->d, 3x3, s2) + ReLU -> dw Conv2d(d, 3x3, s2, groups=d) -> pw 1x1 + ReLU
//   -> dw 3x3 s2 -> pw 1x1 + ReLU -> flatten (c*9+f) -> Linear(9d -> d) (x sqrt(d), embedding.py:509)
// The pointwise convs and the output Linear are GEMMs (gemm.hip); this file
// holds conv0+ReLU+dw1 fused (conv0's [d, 4C+3, 39] output never reaches HBM:
// it is produced tile by tile in LDS) and dw2.  Activations are channels-last
// ([window][t][f][d]) so the pointwise convs are plain row-major GEMMs.
//
// A "window" is one packed chunk (masked batch, W = 8C+7 rows) or one whole
// padded utterance (forward_encoder, W = T); its rows come from the feature
// buffer at meta[PM_SRC_ROW], rows >= meta[PM_NVALID] are zero padding, and
// CMVN is applied after padding exactly like the reference (padding rows
// become -mean*istd).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

constexpr int FE_T2_TILE = 8;                 // dw1 output rows per block
constexpr int FE_T1_ROWS = 2 * FE_T2_TILE + 1;  // conv0 rows per block
constexpr int FE_IN_ROWS = 2 * FE_T1_ROWS + 1;  // input rows per block
constexpr int FE_F0 = 80, FE_F1 = 39, FE_F2 = 19, FE_F3 = 9;
constexpr int FE_CG = 16;                     // channels per LDS pass

// First feature row of a window: packed mode (feats = the utterances concatenated, plan row
// PM_SRC_ROW) or table mode (tab[utt] = that utterance's own [T, 80] rows, window c at row c * step),
// so forward_parallel_chunk's caller-owned tensors are read in place, with no concatenation copy.
__device__ __forceinline__ const float* window_rows(const float* feats, const float* const* tab, int step,
                                                   const int32_t* m) {
  return tab ? tab[m[PM_UTT]] + (size_t)m[PM_CHUNK] * step * FE_F0 : feats + (size_t)m[PM_SRC_ROW] * FE_F0;
}

template <typename T>
__global__ __launch_bounds__(256) void fe_conv0_dw_kernel(const float* __restrict__ feats, const float* const* __restrict__ tab,
                                                          int step, const int32_t* __restrict__ meta,
                                                          int meta_stride, int W, int T2, const float* __restrict__ cm,
                                                          const float* __restrict__ ci, const float* __restrict__ w0,
                                                          const float* __restrict__ b0, const float* __restrict__ w1,
                                                          const float* __restrict__ b1, int d, T* __restrict__ out) {
  __shared__ float xin[FE_IN_ROWS * FE_F0];
  __shared__ float c0[FE_CG * FE_T1_ROWS * FE_F1];
  const int tid = threadIdx.x;
  const int win = blockIdx.y;
  const int t2_0 = blockIdx.x * FE_T2_TILE;
  const int nt2 = min(FE_T2_TILE, T2 - t2_0);
  const int T1 = (W - 3) / 2 + 1;
  const float* xsrc = window_rows(feats, tab, step, meta + (size_t)win * meta_stride);
  const int nvalid = meta[(size_t)win * meta_stride + PM_NVALID];
  const int r0 = 4 * t2_0;   // first input row
  for (int idx = tid; idx < FE_IN_ROWS * FE_F0; idx += 256) {
    const int r = idx / FE_F0, f = idx - r * FE_F0, gr = r0 + r;
    float v = (gr < nvalid && gr < W) ? xsrc[(size_t)gr * FE_F0 + f] : 0.f;
    if (cm) v = (v - cm[f]) * ci[f];
    xin[idx] = v;
  }
  __syncthreads();
  // conv0 positions of this block (t1 local in [0, 17), f1 in [0, 39)); 663 <= 3 * 256
  const int n1 = min(FE_T1_ROWS, T1 - 2 * t2_0) * FE_F1;
  float xp[3][9];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int p = tid + 256 * k;
    const int tl = p / FE_F1, f1 = p - tl * FE_F1;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int v = 0; v < 3; ++v)
        xp[k][u * 3 + v] = xin[min((2 * tl + u) * FE_F0 + 2 * f1 + v, FE_IN_ROWS * FE_F0 - 1)];
  }
  const int nout = nt2 * FE_F2 * FE_CG;
  for (int cg = 0; cg < d; cg += FE_CG) {
    for (int c = 0; c < FE_CG; ++c) {
      const float* wc = w0 + (size_t)(cg + c) * 9;
      const float bc = b0[cg + c];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int p = tid + 256 * k;
        float a = bc;
#pragma unroll
        for (int e = 0; e < 9; ++e) a = fmaf(wc[e], xp[k][e], a);
        if (p < n1) c0[c * (FE_T1_ROWS * FE_F1) + p] = fmaxf(a, 0.f);
      }
    }
    __syncthreads();
    for (int o = tid; o < nout; o += 256) {
      const int c = o & (FE_CG - 1), pos = o >> 4;
      const int tl = pos / FE_F2, f2 = pos - tl * FE_F2;
      const float* wc = w1 + (size_t)(cg + c) * 9;
      const float* cb = c0 + c * (FE_T1_ROWS * FE_F1) + (2 * tl) * FE_F1 + 2 * f2;
      float a = b1[cg + c];
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) a = fmaf(wc[u * 3 + v], cb[u * FE_F1 + v], a);
      out[(((size_t)win * T2 + t2_0 + tl) * FE_F2 + f2) * d + cg + c] = from_f32<T>(a);
    }
    __syncthreads();
  }
}

// bf16 mode: conv0 + ReLU + dw1 fused on MFMA with no LDS round trip.  For a dw1 output
// position (t2, f2) and channel c:
//   out1 = b1[c] + sum_{s=(u,v)} w1[c][s] * relu(b0[c] + sum_e w0[c][e] * X[4t2+2u+e/3][4f2+2v+e%3])
// Each wave owns 32 dw1 positions (MFMA rows) and sweeps all channels in tiles of 32 (MFMA
// columns).  For each of the 9 dw1 taps s one v_mfma_f32_32x32x16_bf16 (K = the 9 conv0
// taps, zero-padded to 16; bias-seeded accumulator) yields conv0 at the tap's positions,
// and the VALU folds relu * w1[c][s] into the dw1 accumulator.  conv0 is recomputed per dw1
// tap (2.25x its FLOPs, free on MFMA), which removes the conv0 tile in LDS, the barriers
// between the two convolutions and the partial-row stores of a channel-split grid.
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int FE_POS_BLOCK = 128;                     // dw1 positions per block (4 waves x 32)
constexpr int FE_XROWS = 4 * ((FE_POS_BLOCK - 1) / FE_F2 + 2) + 3;   // staged input rows (>= 4*span + 7)

// v_mfma_f32_32x32x16_{bf16,f16} on 8-element fragments of E
template <typename E, typename V>
CFM_DEV f32x16 mfma32x16(const V& a, const V& b, const f32x16& c) {
  if constexpr (std::is_same<E, f16>::value) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <typename E>
__global__ __launch_bounds__(256, 3) void fe_conv0_dw_mfma_kernel(const float* __restrict__ feats,
                                                               const float* const* __restrict__ tab, int step,
                                                               const int32_t* __restrict__ meta, int meta_stride,
                                                               int W, int T2, const float* __restrict__ cm,
                                                               const float* __restrict__ ci,
                                                               const float* __restrict__ wpack, int d,
                                                               E* __restrict__ out) {
  typedef E ex8 __attribute__((ext_vector_type(8)));   // bf16 / f16 (fp16 mode) operands
  __shared__ float xin[FE_XROWS * FE_F0];
  // per-wave output staging [32 positions][64 channels] E, 144-B rows: the MFMA layout gives
  // each lane one channel; two channel tiles are gathered here and leave as full 128-B rows
  constexpr int OPITCH = 144;
  __shared__ __attribute__((aligned(16))) char ostage[4][32 * OPITCH];
  const int tid = threadIdx.x;
  const int win = blockIdx.y;
  const int P = T2 * FE_F2;
  const int p0 = blockIdx.x * FE_POS_BLOCK;
  const int r0 = 4 * (p0 / FE_F2);   // first staged input row
  const float* xsrc = window_rows(feats, tab, step, meta + (size_t)win * meta_stride);
  const int nvalid = min(meta[(size_t)win * meta_stride + PM_NVALID], W);
  for (int idx = tid; idx < FE_XROWS * FE_F0; idx += 256) {
    const int r = idx / FE_F0, f = idx - r * FE_F0, gr = r0 + r;
    float v = gr < nvalid ? xsrc[(size_t)gr * FE_F0 + f] : 0.f;
    if (cm) v = (v - cm[f]) * ci[f];   // CMVN after padding, like cmvn.py:32-43 on the padded window
    xin[idx] = v;
  }
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6, hh = lane >> 5, n = lane & 31;
  const int pw = p0 + wv * 32;   // this wave's first position
  if (pw >= P) return;
  // A fragments: row m = n -> position pw + n; k = 8*hh + j = conv0 tap e (e < 9)
  ex8 xa[9];
  {
    const int pos = min(pw + n, P - 1);   // rows past P are computed and discarded
    const int t2 = pos / FE_F2, f2 = pos - t2 * FE_F2;
    const float* xb = xin + (4 * t2 - r0) * FE_F0 + 4 * f2;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const float* xs = xb + 2 * (s / 3) * FE_F0 + 2 * (s % 3);
      if (hh == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) xa[s][j] = (E)xs[(j / 3) * FE_F0 + j % 3];
      } else {
        xa[s][0] = (E)xs[2 * FE_F0 + 2];
        xa[s][1] = (E)1.f;   // k = 9: the conv0 bias row (B holds b0 there; E as under autocast)
#pragma unroll
        for (int j = 2; j < 8; ++j) xa[s][j] = (E)0.f;
      }
    }
  }
  // per-channel-tile weights, software-pipelined one tile ahead: load_w only issues the raw
  // 16-B loads; they are unpacked when the next tile starts, so their wait lands a whole tile
  // later.  (The compiler's wait at the top of a pass also covers the previous pass's stores --
  // loads and stores share vmcnt in issue order; hand-counted waits on inline-asm loads that
  // leave those stores in flight measured within 2%, not kept.)
  f32x4 qw[5];
  auto load_w = [&](int c) {
    const f32x4* wp = reinterpret_cast<const f32x4*>(wpack + (size_t)c * FE_WPACK);
#pragma unroll
    for (int i = 0; i < 5; ++i) qw[i] = wp[i];
  };
  load_w(n);
  // the window's output range as a wave-uniform buffer descriptor (readfirstlane: SGPRs, so the
  // stores need no waterfall loop)
  const unsigned long long obase = (unsigned long long)(out + (size_t)win * P * d);
  const unsigned long long obu = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(obase >> 32)) << 32) |
                                 (unsigned)__builtin_amdgcn_readfirstlane((unsigned)obase);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)obu, (short)0, __builtin_amdgcn_readfirstlane(P * d * 2), 0x00020000);
  unsigned voff[4];   // byte offsets of this lane's 16-B store chunks at channel 0
#pragma unroll
  for (int k = 0; k < 4; ++k) voff[k] = (unsigned)(((pw + (lane >> 3) + 8 * k) * d + (lane & 7) * 8) * 2);
  // two 32-channel tiles per iteration, then one unconditional store pass of the 64 staged
  // channels
  for (int ct = 0; ct < d; ct += 64) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      // lanes of the upper half need only conv0 tap 8 (k = 8) and the bias b0 (k = 9); the rest
      // of K is zero, so the conv0 MFMAs start from a zero accumulator
      const float t[9] = {qw[0][0], qw[0][1], qw[0][2], qw[0][3], qw[1][0], qw[1][1], qw[1][2], qw[1][3], qw[2][0]};
      ex8 wcur;
#pragma unroll
      for (int j = 0; j < 8; ++j) wcur[j] = (E)(hh ? (j == 0 ? t[8] : j == 1 ? qw[4][2] : 0.f) : t[j]);
      const float wkc[9] = {qw[2][1], qw[2][2], qw[2][3], qw[3][0], qw[3][1], qw[3][2], qw[3][3], qw[4][0], qw[4][1]};
      const f32x16 seed = {};
      f32x16 o;
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] = qw[4][3];
      load_w(min(ct + 32 * half + 32 + n, d - 1));   // past the last tile: a harmless reload
      // taps are software-pipelined one deep: MFMA s+1 is issued before tap s's relu/FMA work
      // (scheduling barriers pin the order: without them the compiler sinks MFMA s+1 below tap
      // s's VALU and both accumulator sets share registers, serialising MFMA and VALU per wave)
      f32x16 acc = mfma32x16<E>(xa[0], wcur, seed);
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        f32x16 nxt;
        if (s + 1 < 9) nxt = mfma32x16<E>(xa[s + 1], wcur, seed);
        __builtin_amdgcn_sched_barrier(0);
        // one v_max_f32 + one v_fma_f32 per value (IEEE mode off in build.py: no canonicalising
        // max in front; no SLP packing: a v_pk_fma_f32 beside MFMAs issues slower than two v_fma_f32)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = fmaf(fmaxf(acc[r], 0.f), wkc[s], o[r]);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < 9) acc = nxt;
      }
      char* os = ostage[wv];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 8 * (r >> 2) + 4 * hh + (r & 3);
        *reinterpret_cast<E*>(os + m * OPITCH + (32 * half + n) * 2) = (E)o[r];
      }
    }
    // 64 channels staged: lane -> 16-B chunk (lane & 7) of positions (lane >> 3) + 8k, buffer
    // stores against the window's range (positions past P fall outside it and are dropped by
    // the hardware), so the store needs no branch
    const char* os = ostage[wv];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(os + ((lane >> 3) + 8 * k) * OPITCH + (lane & 7) * 16);
#ifndef CFM_FE_DIAG_NOSTORE   // timing-only build: no output stores
      __builtin_amdgcn_raw_buffer_store_b128(v, ors, voff[k], ct * 2, 0);
#else
      asm volatile("" ::"v"(v));
#endif
    }
  }
}

// bf16 mode, channel-stationary (the default, "fe_conv" 2): dw1 on MFMA as well.  Each wave owns
// 32 channels for a run of FE2_POS-position chunks, so its weights are loop-invariant registers.
//  - conv0 is computed transposed, X^T[channel][position] = W0 . im2col (A = the wave's W0 rows with
//    b0 at k = 9, B = the position's conv0 patch), so its accumulator has the position on the lane
//    and 16 channels in registers;
//  - ReLU + bf16 rounding (autocast rounds conv0's output to bf16 too) turn registers 8t..8t+7 into
//    the B operand of k-step t of a second 32x32x16 MFMA with no lane movement: k = 8h + j holds
//    channel 16t + 8(j>>2) + 4h + (j&3);
//  - dw1 is that MFMA against a diagonal A (row c: w1[c][s] at its own channel's k), accumulated
//    over the 9 taps on top of a b1-seeded accumulator.
// Per tap and 32x32 tile: 3 MFMAs (96 cycles) and 16 packed VALU ops (8 cvt_pk + 8 pk_max_i16),
// against 1 MFMA and 32 f32 VALU ops (max + fma per value) in the kernel above.
// conv0 patches are built once per chunk as bf16 im2col rows in LDS (taps 0..7 in the "lo" image,
// tap 8 + 1.0 + zeros in the "hi" image, 16 B each, even and odd conv0 columns in separate planes so
// the 32 lanes of a tap read consecutive 16-B slots), so a tap's B fragment is one ds_read_b128 at a
// constant offset.  The next chunk's input rows are loaded into registers while this chunk computes.
#ifndef FE2_POS_DEF
#define FE2_POS_DEF 256
#endif
#ifndef FE2_WAVES
#define FE2_WAVES 4   // waves (32-channel tiles) per workgroup sharing one im2col build: 4 (2 workgroups per CU) or 8
#endif
#ifndef FE2_PRIO
#define FE2_PRIO 0
#endif
#ifndef FE2_STG
#define FE2_STG 1   // output staging buffers per wave (2: a tile's outputs leave during the next tile; 2.709 vs 2.688 ms)
#endif
constexpr int FE2_POS = FE2_POS_DEF;                                  // dw1 positions per chunk
constexpr int FE2_T1ROWS = 2 * ((FE_F2 - 1 + FE2_POS - 1) / FE_F2) + 3;   // conv0 rows a chunk can touch
constexpr int FE2_XROWS = 2 * FE2_T1ROWS + 1;                         // input rows behind them
constexpr int FE2_SLOTS = (FE_F1 + 1) / 2;                            // conv0 columns per parity plane
// slot of conv0 row t1, column pair i within a parity plane: each pair of rows is padded by 11 slots
// so that one dw1 row (2 conv0 rows) spans 51 = 3 (mod 16) slots and 16 consecutive positions fall in
// 16 different 16-B bank groups even across a row boundary (18 -> 0: +33 slots)
__host__ __device__ constexpr int fe2_slot(int t1, int i) { return t1 * FE2_SLOTS + (t1 >> 1) * 11 + i; }
constexpr int FE2_PLANE = fe2_slot(FE2_T1ROWS - 1, FE2_SLOTS - 1) + 1;  // slots per parity plane
constexpr int FE2_IMG = 2 * FE2_PLANE * 16;                           // one image (lo or hi), bytes
constexpr int FE2_OPITCH = 80;                                        // output staging row (32 ch bf16 + pad)
constexpr int FE2_NQ = FE2_XROWS * (FE_F0 / 4);                        // float4 loads per chunk
constexpr int FE2_NT = 64 * FE2_WAVES;                                // threads per workgroup
constexpr int FE2_QPT = (FE2_NQ + FE2_NT - 1) / FE2_NT;               // ... per thread
typedef short short2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef bf16 bf16x2v __attribute__((ext_vector_type(2)));

#ifndef FE2_CLAMP
#define FE2_CLAMP 1   // ReLU as the clamp modifier of the conversion (see fe2_relu_pk); 0: v_pk_max_i16
#endif
template <typename E>
__device__ __forceinline__ unsigned fe2_relu_pk(float a, float b) {
  if constexpr (std::is_same<E, f16>::value) {   // f16: RNE pack, then the ReLU as a packed int16 max
    typedef f16 h2v __attribute__((ext_vector_type(2)));
    short2v v = __builtin_bit_cast(short2v, __builtin_convertvector((f32x2v){a, b}, h2v));
    v = __builtin_elementwise_max(v, (short2v){0, 0});
    return __builtin_bit_cast(unsigned, v);
  }
#if FE2_CLAMP
  // W0 and b0 enter the fragments scaled by 2^-24 and w1 by 2^24 (exact: powers of two), so conv0's
  // accumulator is the true value times 2^-24 and, for |conv0| < 2^24, the conversion's clamp to
  // [0, 1] is exactly the ReLU: one instruction per pair instead of two (saturation to [0, 1], NaN to 0,
  // probed on gfx950: tools/probe/cvt_clamp.hip).  Front-end conv0 outputs of CMVN-normalised
  // features are orders of magnitude below 2^24.
  unsigned u;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2 clamp" : "=v"(u) : "v"(a), "v"(b));
  return u;
#endif
  const bf16x2v pr = __builtin_convertvector((f32x2v){a, b}, bf16x2v);   // one v_cvt_pk_bf16_f32
  short2v v = __builtin_bit_cast(short2v, pr);
  v = __builtin_elementwise_max(v, (short2v){0, 0});   // v_pk_max_i16: a negative bf16 is a negative int16
  return __builtin_bit_cast(unsigned, v);
}

// 8 f32 -> the 16-bit format (RNE), as a bf16x8 container of raw lanes
template <typename E>
__device__ __forceinline__ bf16x8 pk8(float a, float b, float c, float d_, float e, float f, float g, float h) {
  typedef E e8v __attribute__((ext_vector_type(8)));
  return __builtin_bit_cast(bf16x8, (e8v){(E)a, (E)b, (E)c, (E)d_, (E)e, (E)f, (E)g, (E)h});
}
// 32x32x16 MFMA on the 16-bit format's raw lanes (bf16x8 containers)
template <typename E>
__device__ __forceinline__ f32x16 fe2_mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  if constexpr (std::is_same<E, f16>::value)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <typename E>
__global__ __launch_bounds__(FE2_NT, 8 / FE2_WAVES) void fe_conv0_dw_mfma2_kernel(const float* __restrict__ feats,
                                                                const float* const* __restrict__ tab, int step,
                                                                const int32_t* __restrict__ meta, int meta_stride,
                                                                int W, int T2, const float* __restrict__ cm,
                                                                const float* __restrict__ ci,
                                                                const float* __restrict__ wfrag, int d,
                                                                E* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char im2col[2 * FE2_IMG];
  // the chunk's input rows (f32, CMVN applied) while im2col is built; then the waves' output staging
  constexpr int XBYTES = FE2_XROWS * FE_F0 * 4, OBYTES = FE2_STG * FE2_WAVES * 32 * FE2_OPITCH;   // output staging
  __shared__ __attribute__((aligned(16))) char xstage[XBYTES > OBYTES ? XBYTES : OBYTES];
  __shared__ __attribute__((aligned(16))) float cmvn[2][FE_F0];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6, h = lane >> 5, n = lane & 31;
  if (cm && tid < 2 * FE_F0) cmvn[tid / FE_F0][tid % FE_F0] = (tid < FE_F0 ? cm : ci)[tid % FE_F0];
  const int win = blockIdx.z;
  const int P = T2 * FE_F2;
  const int ct = blockIdx.y * FE2_WAVES + wv;   // this wave's 32-channel tile (waves past d only help build)
  // FE2_PRIO (A/B): static priority for one of a SIMD's two partner waves (MI355X_MICROARCH.md, two waves per
  // SIMD, item 4): waves 4-7 of an 8-wave workgroup, or the odd channel groups' workgroups
  if constexpr (FE2_PRIO) {
    if (FE2_WAVES == 8 ? wv >= 4 : (blockIdx.y & 1) != 0) __builtin_amdgcn_s_setprio(1);
  }
  const bool active = ct * 32 < d;
  // loop-invariant operands (host-built per-lane fragments, model.hip), loaded first so their latency
  // overlaps the first chunk's input loads: W0 rows (+ b0 at k = 9), the diagonal dw1 fragments, the
  // b1 seed
  bf16x8 a0, a1[9][2];
  f32x16 seed;
  {
    const u32x4* fr = reinterpret_cast<const u32x4*>(wfrag) + (size_t)(active ? ct : 0) * FE2_NFRAG * 64 + lane;
    a0 = __builtin_bit_cast(bf16x8, fr[0]);
#pragma unroll
    for (int s = 0; s < 9; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) a1[s][t] = __builtin_bit_cast(bf16x8, fr[(1 + 2 * s + t) * 64]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 v = __builtin_bit_cast(f32x4, fr[(19 + i) * 64]);
#pragma unroll
      for (int r = 0; r < 4; ++r) seed[4 * i + r] = v[r];
    }
  }
  const float* xsrc = window_rows(feats, tab, step, meta + (size_t)win * meta_stride);
  const int nvalid = min(meta[(size_t)win * meta_stride + PM_NVALID], W);
  const int nck = (P + FE2_POS - 1) / FE2_POS;
  // the window's chunks split evenly over the gridDim.x workgroups of its row (counts differ by <= 1)
  const int c_beg = (int)((long long)blockIdx.x * nck / gridDim.x), c_end = (int)((long long)(blockIdx.x + 1) * nck / gridDim.x);
  f32x4 pv[FE2_QPT];   // a chunk's input rows in flight; rows at or past nvalid are padding (zeros before CMVN)
  auto prefetch = [&](int c) {
    const int r0 = 4 * ((c * FE2_POS) / FE_F2);
#pragma unroll
    for (int i = 0; i < FE2_QPT; ++i) {
      const int q = tid + FE2_NT * i, r = q / (FE_F0 / 4), gr = r0 + r;
      pv[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (q < FE2_NQ && gr < nvalid)
        pv[i] = *reinterpret_cast<const f32x4*>(xsrc + (size_t)gr * FE_F0 + 4 * (q % (FE_F0 / 4)));
    }
  };
  if (c_beg < c_end) prefetch(c_beg);
  const unsigned long long obase = (unsigned long long)(out + (size_t)win * P * d);
  const unsigned long long obu = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(obase >> 32)) << 32) |
                                 (unsigned)__builtin_amdgcn_readfirstlane((unsigned)obase);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      (void*)obu, (short)0, __builtin_amdgcn_readfirstlane(P * d * 2), 0x00020000);
  char* os = xstage + wv * 32 * FE2_OPITCH;   // this wave's staging; its second buffer FE2_WAVES waves further on
  const f32x16 zero = {};
  for (int c = c_beg; c < c_end; ++c) {
    const int p0 = c * FE2_POS, t2a = p0 / FE_F2;
    __syncthreads();   // the previous chunk's waves are done with im2col and the output staging
    {
      float* xs = reinterpret_cast<float*>(xstage);
#pragma unroll
      for (int i = 0; i < FE2_QPT; ++i) {
        const int q = tid + FE2_NT * i;
        if (q < FE2_NQ) {
          f32x4 x = pv[i];
          if (cm) {   // CMVN after padding (cmvn.py:32-43 on the padded window)
            const int f = 4 * (q % (FE_F0 / 4));
            x = (x - *reinterpret_cast<const f32x4*>(&cmvn[0][f])) * *reinterpret_cast<const f32x4*>(&cmvn[1][f]);
          }
          *reinterpret_cast<f32x4*>(xs + 4 * q) = x;
        }
      }
    }
    __syncthreads();
    // im2col of conv0 rows 2*t2a .. 2*t2a + FE2_T1ROWS - 1; slot (row, parity, i) = column 2i + parity.
    // One thread per (row, i): input columns 4i .. 4i+4 of three rows give both parities' patches.
    for (int idx = tid; idx < FE2_T1ROWS * FE2_SLOTS; idx += FE2_NT) {
      const int tl = idx / FE2_SLOTS, i = idx - tl * FE2_SLOTS;
      const float* xr = reinterpret_cast<const float*>(xstage) + (2 * tl) * FE_F0 + 4 * i;
      f32x4 A[3];
      float Ex[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        A[a] = *reinterpret_cast<const f32x4*>(xr + a * FE_F0);
        Ex[a] = i + 1 < FE2_SLOTS ? xr[a * FE_F0 + 4] : 0.f;   // column 4i+4 (odd parity only)
      }
      const bf16x8 lo0 = pk8<E>(A[0][0], A[0][1], A[0][2], A[1][0], A[1][1], A[1][2], A[2][0], A[2][1]);
      const bf16x8 hi0 = pk8<E>(A[2][2], 1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f);
      const int s0 = fe2_slot(tl, i) * 16, s1 = (FE2_PLANE + fe2_slot(tl, i)) * 16;
      *reinterpret_cast<bf16x8*>(im2col + s0) = lo0;
      *reinterpret_cast<bf16x8*>(im2col + FE2_IMG + s0) = hi0;
      if (2 * i + 1 < FE_F1) {
        const bf16x8 lo1 = pk8<E>(A[0][2], A[0][3], Ex[0], A[1][2], A[1][3], Ex[1], A[2][2], A[2][3]);
        const bf16x8 hi1 = pk8<E>(Ex[2], 1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<bf16x8*>(im2col + s1) = lo1;
        *reinterpret_cast<bf16x8*>(im2col + FE2_IMG + s1) = hi1;
      }
    }
    __syncthreads();
    if (c + 1 < c_end) prefetch(c + 1);   // lands under this chunk's MFMAs
    if (!active) continue;
    const int pend = min(p0 + FE2_POS, P);
    // tile pt's patches: tap (u, v) = conv0 position (2 t2 + u, 2 f2 + v) of the lane's position
    auto patch_base = [&](int pt) {
      const int pos = min(pt + n, P - 1);   // positions past P are computed and dropped at the store
      const int t2 = pos / FE_F2, f2 = pos - t2 * FE_F2;
      return im2col + h * FE2_IMG + (fe2_slot(2 * (t2 - t2a), 0) + f2) * 16;
    };
    // tap (u, v): conv0 row 2 t2 + u (fe2_slot(2 t2 + u, i) - fe2_slot(2 t2, i) = fe2_slot(u, 0)), parity
    // plane v & 1, pair f2 + (v >> 1)
    auto tap_off = [](int s) { return (((s % 3) & 1) * FE2_PLANE + fe2_slot(s / 3, 0) + ((s % 3) >> 1)) * 16; };
    auto ld = [&](const char* xb, int s) { return *reinterpret_cast<const bf16x8*>(xb + tap_off(s)); };
    // the staged outputs of tile pt leave as 64-B row pieces (4 lanes per position)
    auto flush = [&](const char* sb, int pt) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int pl = (lane >> 2) + 16 * k, ch = lane & 3;
        const u32x4 v = *reinterpret_cast<const u32x4*>(sb + pl * FE2_OPITCH + ch * 16);
#ifndef CFM_FE_DIAG_NOSTORE
        __builtin_amdgcn_raw_buffer_store_b128(v, ors, (unsigned)(((pt + pl) * d + ct * 32 + ch * 8) * 2), 0, 0);
#else
        asm volatile("" ::"v"(v));
#endif
      }
    };
    bf16x8 pb[9];
    {
      const char* xb = patch_base(p0);
#pragma unroll
      for (int s = 0; s < 9; ++s) pb[s] = ld(xb, s);
    }
    int it = 0;
    for (int pt = p0; pt < pend; pt += 32, ++it) {
      // the next tile's patches are read into pb as its registers free up (tap t's patch is last
      // used when conv0 of tap t is issued, in loop step t - 1), so they arrive under this tile's
      // MFMAs; the previous tile's staged outputs leave in step 1
      const char* xbn = patch_base(pt + 32 < pend ? pt + 32 : pt);
      char* sb = os + (FE2_STG == 2 ? (it & 1) : 0) * (FE2_WAVES * 32 * FE2_OPITCH);
      f32x16 y = seed;
      f32x16 acc = fe2_mfma<E>(a0, pb[0], zero);
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        f32x16 nxt;
        if (s + 1 < 9) nxt = fe2_mfma<E>(a0, pb[s + 1], zero);
        __builtin_amdgcn_sched_barrier(0);   // conv0 of tap s+1 runs under tap s's VALU work
        u32x4 r0, r1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          r0[q] = fe2_relu_pk<E>(acc[2 * q], acc[2 * q + 1]);
          r1[q] = fe2_relu_pk<E>(acc[8 + 2 * q], acc[9 + 2 * q]);
        }
        y = fe2_mfma<E>(a1[s][0], __builtin_bit_cast(bf16x8, r0), y);
        y = fe2_mfma<E>(a1[s][1], __builtin_bit_cast(bf16x8, r1), y);
        if (FE2_STG == 2 && s == 1 && it > 0) flush(os + ((it - 1) & 1) * (FE2_WAVES * 32 * FE2_OPITCH), pt - 32);
        if (s == 3) {
#pragma unroll
          for (int t = 0; t < 4; ++t) pb[t] = ld(xbn, t);
        }
        if (s == 7) {
#pragma unroll
          for (int t = 4; t < 9; ++t) pb[t] = ld(xbn, t);
        }
        // one tap at a time (left alone, the scheduler hoists all nine conv0 MFMAs and spills)
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < 9) acc = nxt;
      }
      // y: lane (h, position n), register r -> channel (r&3) + 8(r>>2) + 4h; staged [32 pos][32 ch]
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        typedef E e2v __attribute__((ext_vector_type(2)));
        const e2v lo = __builtin_convertvector((f32x2v){y[4 * g], y[4 * g + 1]}, e2v);
        const e2v hi = __builtin_convertvector((f32x2v){y[4 * g + 2], y[4 * g + 3]}, e2v);
        const unsigned long long u = (unsigned long long)__builtin_bit_cast(unsigned, lo) |
                                     ((unsigned long long)__builtin_bit_cast(unsigned, hi) << 32);
        *reinterpret_cast<unsigned long long*>(sb + n * FE2_OPITCH + (8 * g + 4 * h) * 2) = u;
      }
      if (FE2_STG == 1) flush(sb, pt);
    }
    if (FE2_STG == 2 && it > 0)
      flush(os + ((it - 1) & 1) * (FE2_WAVES * 32 * FE2_OPITCH), pend - 1 - ((pend - 1 - p0) % 32));
  }
}

// dw2: [win][T2][19][d] -> [win][T3][9][d], depthwise 3x3 stride 2 + bias (no activation), taps
// tap-major w[9][d].  One thread per (window, f3, 8 channels, row segment) walks down its
// FE_DW2_SEG-th of the window's output rows: input row 2*t3+2 is kept in registers for the next
// output row, so every input byte is read from HBM once, plus one shared row per segment start
// (16-B loads, 64 lanes = one 1-KB channel row).  The segments multiply the waves in flight
// (one walk per thread is latency-bound at ~11 waves per CU).
constexpr int FE_DW2_SEG = 4;
template <typename T>
__global__ __launch_bounds__(256) void fe_dw2_kernel(const T* __restrict__ in, int nwin, int T2, int T3, int d,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     T* __restrict__ out) {
  const int d8 = d >> 3;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)nwin * FE_F3 * d8;
  if (idx >= total) return;
  const int t3a = (int)((long long)blockIdx.y * T3 / gridDim.y), t3b = (int)((long long)(blockIdx.y + 1) * T3 / gridDim.y);
  const int c = (int)(idx % d8) * 8;
  const size_t r = idx / d8;
  const int f3 = r % FE_F3;
  const size_t wn = r / FE_F3;
  if constexpr (sizeof(T) == 2 && DW2_DOT2) {
    // 16-bit activations: channel pairs kept packed, one dw2_dot per channel and tap (cfm_common.h), the same
    // taps in the same order as the fused pw1 + dw2 kernel (gemm_wst_impl.h), so the two agree bit for bit
    constexpr int FMT = std::is_same<T, f16>::value ? 1 : 0;
    typedef unsigned u4_ __attribute__((ext_vector_type(4)));
    unsigned wd[9][8];
    float bias[8];
#pragma unroll
    for (int e = 0; e < 9; ++e)
#pragma unroll
      for (int q = 0; q < 8; ++q) wd[e][q] = dw2_wpack<FMT>(w[(size_t)e * d + c + q], q);
    load8(b + c, bias);
    const T* ib = in + (wn * T2 * FE_F2 + 2 * f3) * d + c;
    T* ob = out + (wn * T3 * FE_F3 + f3) * d + c;
    u4_ top[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) top[v] = *reinterpret_cast<const u4_*>(ib + (size_t)(2 * t3a) * FE_F2 * d + (size_t)v * d);
    for (int t3 = t3a; t3 < t3b; ++t3) {
      u4_ mid[3], bot[3];
      const T* rb = ib + (size_t)(2 * t3 + 1) * FE_F2 * d;
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        mid[v] = *reinterpret_cast<const u4_*>(rb + (size_t)v * d);
        bot[v] = *reinterpret_cast<const u4_*>(rb + (size_t)(FE_F2 + v) * d);
      }
      float a[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = bias[q];
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        const u4_* rows[3] = {&top[v], &mid[v], &bot[v]};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int q = 0; q < 8; ++q) a[q] = dw2_dot<FMT>((*rows[i])[q >> 1], wd[3 * i + v][q], a[q]);
      }
      store8(ob + (size_t)t3 * FE_F3 * d, a);
#pragma unroll
      for (int v = 0; v < 3; ++v) top[v] = bot[v];
    }
    return;
  }
  float wt[9][8], bias[8];
#pragma unroll
  for (int e = 0; e < 9; ++e) load8(w + (size_t)e * d + c, wt[e]);
  load8(b + c, bias);
  const T* ib = in + (wn * T2 * FE_F2 + 2 * f3) * d + c;
  T* ob = out + (wn * T3 * FE_F3 + f3) * d + c;
  // the 16-bit inputs are converted to f32 before the FMAs: pinned, so that hipcc does not fold an f16
  // conversion into v_fma_mix_f32 (measured: its results differ from cvt + fma in the last f32 bit now
  // and then, and the fused pw1 + dw2 kernel, gemm_wst.hip EPI_DW2, converts first)
  auto pin8 = [](float (&x)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(x[q]));
  };
  float top[3][8];   // input row 2*t3 (carried from the previous output row)
#pragma unroll
  for (int v = 0; v < 3; ++v) {
    load8(ib + (size_t)(2 * t3a) * FE_F2 * d + (size_t)v * d, top[v]);
    pin8(top[v]);
  }
  for (int t3 = t3a; t3 < t3b; ++t3) {
    float mid[3][8], bot[3][8];
    const T* rb = ib + (size_t)(2 * t3 + 1) * FE_F2 * d;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      load8(rb + (size_t)v * d, mid[v]);
      load8(rb + (size_t)(FE_F2 + v) * d, bot[v]);
      pin8(mid[v]);
      pin8(bot[v]);
    }
    float a[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float s = bias[q];
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        s = fmaf(wt[v][q], top[v][q], s);
        s = fmaf(wt[3 + v][q], mid[v][q], s);
        s = fmaf(wt[6 + v][q], bot[v][q], s);
      }
      a[q] = s;
    }
    pin8(a);   // the f32 sums are rounded to f32 first (else the last FMA folds into v_fma_mix{lo,hi}_f16)
    store8(ob + (size_t)t3 * FE_F3 * d, a);
#pragma unroll
    for (int v = 0; v < 3; ++v)
#pragma unroll
      for (int q = 0; q < 8; ++q) top[v][q] = bot[v][q];
  }
}

template <typename T>
int frontend_conv0_dw(const float* feats, const float* const* tab, int step, const int32_t* meta, int meta_stride,
                      int nwin, int W,
                      const float* cmvn_mean, const float* cmvn_istd, const float* w0, const float* b0,
                      const float* w1, const float* b1, const float* wpack, const float* wfrag, int d, T* out,
                      hipStream_t st, int var) {
  if (nwin <= 0) return 0;
  const int T1 = (W - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  if (T2 <= 0 || d % FE_CG) return (int)hipErrorInvalidValue;
  const dim3 grid((T2 + FE_T2_TILE - 1) / FE_T2_TILE, nwin);
  if constexpr (sizeof(T) == 2) {
    // one window's dw1 output is addressed by 32-bit byte offsets (buffer stores)
    if (d % 64 || (size_t)T2 * FE_F2 * d * sizeof(T) >= ((size_t)1 << 31)) return (int)hipErrorInvalidValue;
    if (var >= 2 && wfrag) {
      // "fe_conv" 2 + k: about k + 1 chunks of FE2_POS positions per workgroup, balanced per window
      // (bf16: fragments scaled by 2^-24 / 2^24, the ReLU as the conversion's clamp; f16: unscaled
      // fragments, the ReLU as a packed max)
      const int nck = (T2 * FE_F2 + FE2_POS - 1) / FE2_POS, nch = std::max(1, var - 1);
      const int nb = (nck + nch - 1) / nch;
      hipLaunchKernelGGL(fe_conv0_dw_mfma2_kernel<T>, dim3(nb, (d + 32 * FE2_WAVES - 1) / (32 * FE2_WAVES), nwin),
                         dim3(FE2_NT), 0, st, feats, tab, step,
                         meta, meta_stride, W, T2, cmvn_mean, cmvn_istd, wfrag, d, out);
      CFM_CHECK_LAUNCH();
      return 0;
    }
    if (var >= 1 || std::is_same<T, bf16>::value)   // the position-stationary MFMA kernel (bf16: also at 0)
      hipLaunchKernelGGL(fe_conv0_dw_mfma_kernel<T>, dim3((T2 * FE_F2 + FE_POS_BLOCK - 1) / FE_POS_BLOCK, nwin), dim3(256),
                         0, st, feats, tab, step, meta, meta_stride, W, T2, cmvn_mean, cmvn_istd, wpack, d, out);
    else
      hipLaunchKernelGGL((fe_conv0_dw_kernel<T>), grid, dim3(256), 0, st, feats, tab, step, meta, meta_stride, W, T2,
                         cmvn_mean, cmvn_istd, w0, b0, w1, b1, d, out);
  } else {
    hipLaunchKernelGGL((fe_conv0_dw_kernel<T>), grid, dim3(256), 0, st, feats, tab, step, meta, meta_stride, W, T2,
                       cmvn_mean,
                       cmvn_istd, w0, b0, w1, b1, d, out);
  }
  CFM_CHECK_LAUNCH();
  return 0;
}

template <typename T>
int frontend_dw2(const T* in, int nwin, int T2, int d, const float* w, const float* b, T* out, hipStream_t st,
                 int seg) {
  const int T3 = (T2 - 3) / 2 + 1;
  if (d % 8) return (int)hipErrorInvalidValue;
  const size_t total = (size_t)nwin * FE_F3 * (d / 8);
  if (total == 0 || T3 <= 0) return 0;
  seg = std::max(1, seg);   // row segments per walk ("dw2_seg" model option)
  hipLaunchKernelGGL((fe_dw2_kernel<T>), dim3((unsigned)((total + 255) / 256), std::min(seg, T3)), dim3(256), 0, st, in,
                     nwin, T2, T3, d, w, b, out);
  CFM_CHECK_LAUNCH();
  return 0;
}

template int frontend_conv0_dw<float>(const float*, const float* const*, int, const int32_t*, int, int, int, const float*,
                                      const float*,
                                      const float*, const float*, const float*, const float*, const float*, const float*, int, float*, hipStream_t, int);
template int frontend_conv0_dw<bf16>(const float*, const float* const*, int, const int32_t*, int, int, int, const float*,
                                     const float*,
                                     const float*, const float*, const float*, const float*, const float*, const float*, int, bf16*, hipStream_t, int);
template int frontend_conv0_dw<f16>(const float*, const float* const*, int, const int32_t*, int, int, int, const float*,
                                     const float*,
                                     const float*, const float*, const float*, const float*, const float*, const float*, int, f16*, hipStream_t, int);
template int frontend_dw2<float>(const float*, int, int, int, const float*, const float*, float*, hipStream_t, int);
template int frontend_dw2<bf16>(const bf16*, int, int, int, const float*, const float*, bf16*, hipStream_t, int);
template int frontend_dw2<f16>(const f16*, int, int, int, const float*, const float*, f16*, hipStream_t, int);

}  // namespace cfm
