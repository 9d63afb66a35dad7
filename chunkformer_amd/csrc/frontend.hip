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
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

constexpr int FE_T2_TILE = 8;                 // dw1 output rows per block
constexpr int FE_T1_ROWS = 2 * FE_T2_TILE + 1;  // conv0 rows per block
constexpr int FE_IN_ROWS = 2 * FE_T1_ROWS + 1;  // input rows per block
constexpr int FE_F0 = 80, FE_F1 = 39, FE_F2 = 19, FE_F3 = 9;
constexpr int FE_CG = 16;                     // channels per LDS pass

template <typename T>
__global__ __launch_bounds__(256) void fe_conv0_dw_kernel(const float* __restrict__ feats, const int32_t* __restrict__ meta,
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
  const int src = meta[(size_t)win * meta_stride + PM_SRC_ROW];
  const int nvalid = meta[(size_t)win * meta_stride + PM_NVALID];
  const int r0 = 4 * t2_0;   // first input row
  for (int idx = tid; idx < FE_IN_ROWS * FE_F0; idx += 256) {
    const int r = idx / FE_F0, f = idx - r * FE_F0, gr = r0 + r;
    float v = (gr < nvalid && gr < W) ? feats[(size_t)(src + gr) * FE_F0 + f] : 0.f;
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

// dw2: [win][T2][19][d] -> [win][T3][9][d], depthwise 3x3 stride 2 + bias (no activation)
template <typename T>
__global__ __launch_bounds__(256) void fe_dw2_kernel(const T* __restrict__ in, int nwin, int T2, int T3, int d,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     T* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)nwin * T3 * FE_F3 * d;
  if (idx >= total) return;
  const int c = idx % d;
  size_t r = idx / d;
  const int f3 = r % FE_F3; r /= FE_F3;
  const int t3 = r % T3;
  const size_t wn = r / T3;
  const T* ib = in + ((wn * T2 + 2 * t3) * FE_F2 + 2 * f3) * d + c;
  float a = b[c];
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int v = 0; v < 3; ++v) a = fmaf(w[c * 9 + u * 3 + v], to_f32(ib[((size_t)u * FE_F2 + v) * d]), a);
  out[idx] = from_f32<T>(a);
}

template <typename T>
int frontend_conv0_dw(const float* feats, const int32_t* meta, int meta_stride, int nwin, int W,
                      const float* cmvn_mean, const float* cmvn_istd, const float* w0, const float* b0,
                      const float* w1, const float* b1, int d, T* out, hipStream_t st) {
  if (nwin <= 0) return 0;
  const int T1 = (W - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
  if (T2 <= 0 || d % FE_CG) return (int)hipErrorInvalidValue;
  const dim3 grid((T2 + FE_T2_TILE - 1) / FE_T2_TILE, nwin);
  hipLaunchKernelGGL((fe_conv0_dw_kernel<T>), grid, dim3(256), 0, st, feats, meta, meta_stride, W, T2, cmvn_mean,
                     cmvn_istd, w0, b0, w1, b1, d, out);
  CFM_CHECK_LAUNCH();
  return 0;
}

template <typename T>
int frontend_dw2(const T* in, int nwin, int T2, int d, const float* w, const float* b, T* out, hipStream_t st) {
  const int T3 = (T2 - 3) / 2 + 1;
  const size_t total = (size_t)nwin * T3 * FE_F3 * d;
  if (total == 0) return 0;
  hipLaunchKernelGGL((fe_dw2_kernel<T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, nwin, T2, T3, d,
                     w, b, out);
  CFM_CHECK_LAUNCH();
  return 0;
}

template int frontend_conv0_dw<float>(const float*, const int32_t*, int, int, int, const float*, const float*,
                                      const float*, const float*, const float*, const float*, int, float*, hipStream_t);
template int frontend_conv0_dw<bf16>(const float*, const int32_t*, int, int, int, const float*, const float*,
                                     const float*, const float*, const float*, const float*, int, bf16*, hipStream_t);
template int frontend_dw2<float>(const float*, int, int, int, const float*, const float*, float*, hipStream_t);
template int frontend_dw2<bf16>(const bf16*, int, int, int, const float*, const float*, bf16*, hipStream_t);

}  // namespace cfm
