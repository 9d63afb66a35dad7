// LayerNorm kernels (pre-norm of every sub-block, norm_final, after_norm).
//
// Reference: nn.LayerNorm(eps=1e-5) at encoder_layer.py:46-57 and encoder.py:119.
// One wave per row; lane l owns elements [l*VPL, l*VPL + VPL) with VPL = d/64, so
// a row is one coalesced 16/32-B-per-lane load.  Statistics are two-pass in
// registers (mean, then mean of squared deviations = torch's biased variance).
// `layernorm2` fuses norm_final of layer i with the first pre-norm of layer i+1
// (or with after_norm): the row is read once and written twice.  Row stores are non-temporal:
// measured in the full step (one-process A/B) 52.8 -> 52.4 ms, LayerNorms 8.86 -> 8.74 ms, and the
// GEMMs that read h next got faster too (FFN w1 9.28 -> 9.15, QKV 3.13 -> 3.06 ms).
#include "cfm_common.h"
#include "cfm_kernels.h"

#ifndef LN_RPW
#define LN_RPW 1    // A/B: rows per wave of the pre-norm LayerNorm kernel (1 or 2)
#endif
#ifndef LN2_RPW
#define LN2_RPW 2   // rows per wave of the fused norm_final + next LayerNorm kernel: 2 interleaves two rows' loads and
                    // reductions (8.13 -> 8.06 ms/step for the LayerNorm class, profiles/r05_ab_ln2_rpw.txt); 1 = one
#endif
#ifndef LN_Y16
#define LN_Y16 0   // A/B: 16-bit rows (d = 512) as one 16-B load / store per lane instead of two 8-B ones
#endif

namespace cfm {

template <int VPL>
CFM_DEV void ln_row(float (&v)[VPL], int d, const float* w, const float* b, float eps, int lane) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < VPL; ++e) s += v[e];
  const float mean = wave_sum_dpp(s) / d;
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < VPL; ++e) {
    const float t = v[e] - mean;
    q += t * t;
  }
  const float rstd = rsqrtf(wave_sum_dpp(q) / d + eps);
#pragma unroll
  for (int e = 0; e < VPL; ++e) {
    const int c = lane * VPL + e;
    v[e] = (v[e] - mean) * rstd * w[c] + b[c];
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// VPL is 2 (d=128), 4 (d=256) or 8 (d=512): vector width min(VPL, 4) elements
template <int VPL>
CFM_DEV void load_row(const float* p, float (&v)[VPL]) {
  if constexpr (VPL == 2) {
    const f32x2 t = *reinterpret_cast<const f32x2*>(p);
    v[0] = t[0]; v[1] = t[1];
  } else {
#pragma unroll
    for (int e = 0; e < VPL; e += 4) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(p + e);   // (non-temporal here: LayerNorms +0.8 ms)
      v[e] = t[0]; v[e + 1] = t[1]; v[e + 2] = t[2]; v[e + 3] = t[3];
    }
  }
}
template <int VPL>
CFM_DEV void store_row(float* p, const float (&v)[VPL]) {
  if constexpr (VPL == 2) {
    *reinterpret_cast<f32x2*>(p) = (f32x2){v[0], v[1]};
  } else {
#pragma unroll
    for (int e = 0; e < VPL; e += 4) {
      __builtin_nontemporal_store((f32x4){v[e], v[e + 1], v[e + 2], v[e + 3]}, reinterpret_cast<f32x4*>(p + e));
    }
  }
}
template <typename H, int VPL, typename = std::enable_if_t<sizeof(H) == 2>>
CFM_DEV void store_row(H* p, const float (&v)[VPL]) {   // bf16 / f16 rows
  typedef H h2 __attribute__((ext_vector_type(2)));
  typedef H h4 __attribute__((ext_vector_type(4)));
  if constexpr (VPL == 2) {
    *reinterpret_cast<h2*>(p) = (h2){(H)v[0], (H)v[1]};
  } else if constexpr (VPL == 8 && LN_Y16) {   // one 16-B store per lane
    typedef H h8 __attribute__((ext_vector_type(8)));
    __builtin_nontemporal_store((h8){(H)v[0], (H)v[1], (H)v[2], (H)v[3], (H)v[4], (H)v[5], (H)v[6], (H)v[7]},
                                reinterpret_cast<h8*>(p));
  } else {
#pragma unroll
    for (int e = 0; e < VPL; e += 4) {
      __builtin_nontemporal_store((h4){(H)v[e], (H)v[e + 1], (H)v[e + 2], (H)v[e + 3]}, reinterpret_cast<h4*>(p + e));
    }
  }
}

template <typename H, int VPL, typename = std::enable_if_t<sizeof(H) == 2>>
CFM_DEV void load_row(const H* p, float (&v)[VPL]) {
  typedef H h2 __attribute__((ext_vector_type(2)));
  typedef H h4 __attribute__((ext_vector_type(4)));
  if constexpr (VPL == 2) {
    const h2 t = *reinterpret_cast<const h2*>(p);
    v[0] = (float)t[0]; v[1] = (float)t[1];
  } else if constexpr (VPL == 8 && LN_Y16) {   // one 16-B load per lane
    typedef H h8 __attribute__((ext_vector_type(8)));
    const h8 t = __builtin_nontemporal_load(reinterpret_cast<const h8*>(p));
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)t[e];
  } else {
#pragma unroll
    for (int e = 0; e < VPL; e += 4) {
      // the branch outputs y are read once, here: non-temporal (A/B: LayerNorms 8.59 -> 8.14 ms/step)
      const h4 t = __builtin_nontemporal_load(reinterpret_cast<const h4*>(p + e));
      v[e] = (float)t[0]; v[e + 1] = (float)t[1]; v[e + 2] = (float)t[2]; v[e + 3] = (float)t[3];
    }
  }
}

// x += alpha * ymask[row] * y (the sub-block's residual add, encoder_layer.py:196-246), then the
// second branch's term when present; written back unless deferred to the next LayerNorm
template <typename TY, int VPL>
CFM_DEV void resid_terms(float (&v)[VPL], const ResidAdd<TY>& ra, int row, int lane) {
  float yv[VPL];
  load_row(ra.y + (size_t)row * (VPL * 64) + lane * VPL, yv);
  const float a = ra.alpha * (ra.ymask ? (float)ra.ymask[row] : 1.f);
#pragma unroll
  for (int e = 0; e < VPL; ++e) v[e] = fmaf(a, yv[e], v[e]);
  if (ra.y2) {
    load_row(ra.y2 + (size_t)row * (VPL * 64) + lane * VPL, yv);
    const float a2 = ra.alpha2 * (ra.ymask2 ? (float)ra.ymask2[row] : 1.f);
#pragma unroll
    for (int e = 0; e < VPL; ++e) v[e] = fmaf(a2, yv[e], v[e]);
  }
}
template <typename TY, int VPL>
CFM_DEV void resid_add(float (&v)[VPL], float* xp, const ResidAdd<TY>& ra, int row, int lane) {
  if (!ra.y) return;
  resid_terms<TY, VPL>(v, ra, row, lane);
  if (!ra.defer) store_row(xp, v);
}

template <typename T, int VPL>
__global__ __launch_bounds__(256) void ln_kernel(float* __restrict__ x, ResidAdd<T> ra, int M, const float* __restrict__ w,
                                                 const float* __restrict__ b, float eps, T* __restrict__ out,
                                                 const uint8_t* __restrict__ rowmask) {
  const int lane = threadIdx.x & 63;
  constexpr int d = VPL * 64;
  if constexpr (LN_RPW == 2) {   // A/B: two rows per wave (as ln2_kernel)
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2;
    if (row0 >= M) return;
    const int row1 = row0 + 1 < M ? row0 + 1 : row0;
    float v0[VPL], v1[VPL];
    float* xp0 = x + (size_t)row0 * d + lane * VPL;
    float* xp1 = x + (size_t)row1 * d + lane * VPL;
    load_row(xp0, v0);
    load_row(xp1, v1);
    if (ra.y) {
      resid_terms<T, VPL>(v0, ra, row0, lane);
      resid_terms<T, VPL>(v1, ra, row1, lane);
      if (!ra.defer) {
        store_row(xp0, v0);
        if (row1 != row0) store_row(xp1, v1);
      }
    }
    ln_row<VPL>(v0, d, w, b, eps, lane);
    ln_row<VPL>(v1, d, w, b, eps, lane);
    if (rowmask) {
#pragma unroll
      for (int e = 0; e < VPL; ++e) {
        if (!rowmask[row0]) v0[e] = 0.f;
        if (!rowmask[row1]) v1[e] = 0.f;
      }
    }
    store_row(out + (size_t)row0 * d + lane * VPL, v0);
    if (row1 != row0) store_row(out + (size_t)row1 * d + lane * VPL, v1);
    return;
  }
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[VPL];
  float* xp = x + (size_t)row * d + lane * VPL;
  load_row(xp, v);
  resid_add<T, VPL>(v, xp, ra, row, lane);
  ln_row<VPL>(v, d, w, b, eps, lane);
  if (rowmask && !rowmask[row]) {
#pragma unroll
    for (int e = 0; e < VPL; ++e) v[e] = 0.f;
  }
  store_row(out + (size_t)row * d + lane * VPL, v);
}

template <typename TY, typename TO, int VPL>
__global__ __launch_bounds__(256) void ln2_kernel(float* __restrict__ x, ResidAdd<TY> ra, int M,
                                                  const float* __restrict__ w1, const float* __restrict__ b1,
                                                  const float* __restrict__ w2, const float* __restrict__ b2, float eps,
                                                  TO* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  constexpr int d = VPL * 64;
  if constexpr (LN2_RPW == 2) {   // A/B: two rows per wave, their loads and reductions interleaved
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2;
    if (row0 >= M) return;
    const int row1 = row0 + 1 < M ? row0 + 1 : row0;
    float v0[VPL], v1[VPL];
    float* xp0 = x + (size_t)row0 * d + lane * VPL;
    float* xp1 = x + (size_t)row1 * d + lane * VPL;
    load_row(xp0, v0);
    load_row(xp1, v1);
    if (ra.y) {
      resid_terms<TY, VPL>(v0, ra, row0, lane);
      resid_terms<TY, VPL>(v1, ra, row1, lane);
    }
    ln_row<VPL>(v0, d, w1, b1, eps, lane);
    ln_row<VPL>(v1, d, w1, b1, eps, lane);
    store_row(xp0, v0);
    if (row1 != row0) store_row(xp1, v1);
    if (w2) {
      ln_row<VPL>(v0, d, w2, b2, eps, lane);
      ln_row<VPL>(v1, d, w2, b2, eps, lane);
    }
    store_row(out + (size_t)row0 * d + lane * VPL, v0);
    if (row1 != row0) store_row(out + (size_t)row1 * d + lane * VPL, v1);
    return;
  }
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[VPL];
  float* xp = x + (size_t)row * d + lane * VPL;
  load_row(xp, v);
  if (ra.y) resid_terms<TY, VPL>(v, ra, row, lane);
  ln_row<VPL>(v, d, w1, b1, eps, lane);
  store_row(xp, v);
  if (w2) ln_row<VPL>(v, d, w2, b2, eps, lane);
  store_row(out + (size_t)row * d + lane * VPL, v);
}

template <typename T>
int layernorm(float* x, const ResidAdd<T>& ra, int M, int d, const float* w, const float* b, float eps, T* out,
              const uint8_t* rowmask, hipStream_t st) {
  if (M <= 0) return 0;
  const int nblk = (M + 4 * LN_RPW - 1) / (4 * LN_RPW);
  if (d == 128) hipLaunchKernelGGL((ln_kernel<T, 2>), dim3(nblk), dim3(256), 0, st, x, ra, M, w, b, eps, out, rowmask);
  else if (d == 256) hipLaunchKernelGGL((ln_kernel<T, 4>), dim3(nblk), dim3(256), 0, st, x, ra, M, w, b, eps, out, rowmask);
  else if (d == 512) hipLaunchKernelGGL((ln_kernel<T, 8>), dim3(nblk), dim3(256), 0, st, x, ra, M, w, b, eps, out, rowmask);
  else return (int)hipErrorInvalidValue;
  CFM_CHECK_LAUNCH();
  return 0;
}

template <typename TY, typename TO>
static int ln2_launch(float* x, const ResidAdd<TY>& ra, int M, int d, const float* w1, const float* b1, const float* w2,
                      const float* b2, float eps, TO* out, hipStream_t st) {
  if (M <= 0) return 0;
  const int nblk = (M + 4 * LN2_RPW - 1) / (4 * LN2_RPW);
  if (d == 128) hipLaunchKernelGGL((ln2_kernel<TY, TO, 2>), dim3(nblk), dim3(256), 0, st, x, ra, M, w1, b1, w2, b2, eps, out);
  else if (d == 256) hipLaunchKernelGGL((ln2_kernel<TY, TO, 4>), dim3(nblk), dim3(256), 0, st, x, ra, M, w1, b1, w2, b2, eps, out);
  else if (d == 512) hipLaunchKernelGGL((ln2_kernel<TY, TO, 8>), dim3(nblk), dim3(256), 0, st, x, ra, M, w1, b1, w2, b2, eps, out);
  else return (int)hipErrorInvalidValue;
  CFM_CHECK_LAUNCH();
  return 0;
}

template <typename T>
int layernorm2(float* x, const ResidAdd<T>& ra, int M, int d, const float* w1, const float* b1, const float* w2,
               const float* b2, float eps, T* out, hipStream_t st) {
  return ln2_launch<T, T>(x, ra, M, d, w1, b1, w2, b2, eps, out, st);
}
template <typename T>
int layernorm2_f32(float* x, const ResidAdd<T>& ra, int M, int d, const float* w1, const float* b1, const float* w2,
                   const float* b2, float eps, float* out, hipStream_t st) {
  return ln2_launch<T, float>(x, ra, M, d, w1, b1, w2, b2, eps, out, st);
}

template int layernorm<float>(float*, const ResidAdd<float>&, int, int, const float*, const float*, float, float*,
                              const uint8_t*, hipStream_t);
template int layernorm<bf16>(float*, const ResidAdd<bf16>&, int, int, const float*, const float*, float, bf16*,
                             const uint8_t*, hipStream_t);
template int layernorm<f16>(float*, const ResidAdd<f16>&, int, int, const float*, const float*, float, f16*,
                             const uint8_t*, hipStream_t);
template int layernorm2<float>(float*, const ResidAdd<float>&, int, int, const float*, const float*, const float*,
                               const float*, float, float*, hipStream_t);
template int layernorm2<bf16>(float*, const ResidAdd<bf16>&, int, int, const float*, const float*, const float*,
                              const float*, float, bf16*, hipStream_t);
template int layernorm2<f16>(float*, const ResidAdd<f16>&, int, int, const float*, const float*, const float*,
                              const float*, float, f16*, hipStream_t);
template int layernorm2_f32<float>(float*, const ResidAdd<float>&, int, int, const float*, const float*, const float*,
                                   const float*, float, float*, hipStream_t);
template int layernorm2_f32<bf16>(float*, const ResidAdd<bf16>&, int, int, const float*, const float*, const float*,
                                  const float*, float, float*, hipStream_t);
template int layernorm2_f32<f16>(float*, const ResidAdd<f16>&, int, int, const float*, const float*, const float*,
                                  const float*, float, float*, hipStream_t);

}  // namespace cfm
