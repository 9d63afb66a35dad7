// Chunked relative-position multi-head self-attention over the overlapping-chunk
// KV stream (the "OCT" of attention.py:459-473).
//
// Reference: ChunkAttentionWithRelativeRightContext.forward_parallel_chunk
// (attention.py:420-505) with rel_shift (242-266) and forward_attention
// (104-150); the padded `forward` (268-418) uses the same kernel with other
// descriptors.  For block b (<= 64 queries of one head h):
//
//   s(i, j) = ((q_i + u_h) . k_j + (q_i + v_h) . P[P_BASE - i + j]) / sqrt(64)
//   keys j outside [KEY_LO, KEY_HI) are -inf, softmax in f32, out_i = sum_j p_ij v_j,
//   rows i >= Q_VALID are fully masked (reference: NaN -> 0) and written as 0.
//
// The rel_shift is never materialised: per 64-key tile each wave computes the
// 16 x 80 band Qv . P^T that its 16 query rows need (P rows P_BASE-i0-15+j0 ..
// +79), parks it in LDS and reads it back along the skewed diagonal.  Keys run
// in 64-key tiles with an online softmax; tiles entirely outside [KEY_LO,KEY_HI)
// are skipped (their probabilities are exactly 0 in the reference).  V^T tiles
// are staged in LDS (144/272-B pitch: conflict-free 16-row fragment reads).
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

template <typename T> struct AttnLds {
  static constexpr int VT_PITCH = 64 * sizeof(T) + 16;   // bytes per dim row of V^T
  static constexpr int P_PITCH = 64 * sizeof(T) + 16;    // bytes per query row of probabilities
  static constexpr int BD_PITCH = 85;                    // floats per row of the bd band
  static constexpr int VT_BYTES = 64 * VT_PITCH;
  static constexpr int P_BYTES = 16 * P_PITCH;           // per wave
  static constexpr int BD_BYTES = 16 * BD_PITCH * 4;     // per wave
  static constexpr int TOTAL = VT_BYTES + 4 * (P_BYTES + BD_BYTES);
};

template <typename T>
__global__ __launch_bounds__(256) void chunk_attention_kernel(
    const T* __restrict__ Q, const T* __restrict__ KV, int kv_rows, const T* __restrict__ P, int p_rows,
    const float* __restrict__ pos_u, const float* __restrict__ pos_v, const int32_t* __restrict__ desc, int H,
    T* __restrict__ out) {
  using LY = AttnLds<T>;
  using FT = typename Frag<T>::type;
  __shared__ __attribute__((aligned(16))) char smem[LY::TOTAL];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y;
  const int32_t* D = desc + (size_t)blockIdx.x * AD_INTS;
  const int q_row0 = D[AD_Q_ROW0], nq = D[AD_NQ], kv_row0 = D[AD_KV_ROW0];
  const int key_lo = D[AD_KEY_LO], key_hi = D[AD_KEY_HI], p_base = D[AD_P_BASE], q_valid = D[AD_Q_VALID];
  const int d = H * 64;
  const int i0 = w * 16;

  char* vt = smem;
  char* pb = smem + LY::VT_BYTES + w * (LY::P_BYTES + LY::BD_BYTES);
  float* bd = reinterpret_cast<float*>(pb + LY::P_BYTES);

  // ---- query fragments (row i0 + fr), with u / v biases, two 32-deep sub-steps over dk = 64
  FT qu[2], qv[2];
  {
    const int qi = min(i0 + fr, nq - 1);
    const T* qp = Q + (size_t)(q_row0 + qi) * d + h * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const FT raw = ld8<T>(qp + s * 32 + 8 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int dd = s * 32 + 8 * g + e;
        const float qf = to_f32(raw[e]);
        qu[s][e] = from_f32<T>(qf + pos_u[h * 64 + dd]);
        qv[s][e] = from_f32<T>(qf + pos_v[h * 64 + dd]);
      }
    }
  }

  f32x4 O[4];
  float m_r[4], l_r[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) O[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) { m_r[r] = -INFINITY; l_r[r] = 0.f; }

  const float scale = 0.125f;   // 1 / sqrt(64)
  for (int j0 = key_lo; j0 < key_hi; j0 += 64) {
    // ---- stage V^T of keys j0 .. j0+63 (each thread: one key, 16 dims)
    {
      const int key = tid >> 2, dq = (tid & 3) * 16;
      const int row = min(max(kv_row0 + j0 + key, 0), kv_rows - 1);
      const T* vp = KV + (size_t)row * (2 * d) + h * 128 + 64 + dq;
      const FT v0 = ld8<T>(vp), v1 = ld8<T>(vp + 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        *reinterpret_cast<T*>(vt + (dq + e) * LY::VT_PITCH + key * sizeof(T)) = v0[e];
        *reinterpret_cast<T*>(vt + (dq + 8 + e) * LY::VT_PITCH + key * sizeof(T)) = v1[e];
      }
    }
    // ---- ac = (q+u) K^T  (4 key sub-tiles of 16)
    f32x4 S[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = min(max(kv_row0 + j0 + n * 16 + fr, 0), kv_rows - 1);
      const T* kp = KV + (size_t)row * (2 * d) + h * 128;
      f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) a = mma16(qu[s], ld8<T>(kp + s * 32 + 8 * g), a);
      S[n] = a;
    }
    // ---- bd band = (q+v) P^T over rel-pos rows kb .. kb+79
    const int kb = p_base - i0 - 15 + j0;
#pragma unroll
    for (int n = 0; n < 5; ++n) {
      const int prow = min(max(kb + n * 16 + fr, 0), p_rows - 1);
      const T* pp = P + (size_t)prow * d + h * 64;
      f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) a = mma16(qv[s], ld8<T>(pp + s * 32 + 8 * g), a);
#pragma unroll
      for (int r = 0; r < 4; ++r) bd[(4 * g + r) * LY::BD_PITCH + n * 16 + fr] = a[r];
    }
    __syncthreads();
    // ---- scores, mask, online softmax
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g + r;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int jj = n * 16 + fr;
        float sv = (S[n][r] + bd[row * LY::BD_PITCH + jj + 15 - row]) * scale;
        if (j0 + jj >= key_hi) sv = -INFINITY;
        S[n][r] = sv;
        mx = fmaxf(mx, sv);
      }
      mt[r] = group16_max(mx);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m_r[r], mt[r]);
      const float alpha = __expf(m_r[r] - mn);
      m_r[r] = mn;
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = __expf(S[n][r] - mn);
        S[n][r] = p;
        rs += p;
      }
      l_r[r] = l_r[r] * alpha + group16_sum(rs);
#pragma unroll
      for (int n = 0; n < 4; ++n) O[n][r] *= alpha;
    }
    // ---- probabilities -> LDS (row-major [query][key]) -> A fragments
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<T*>(pb + (4 * g + r) * LY::P_PITCH + (n * 16 + fr) * sizeof(T)) = from_f32<T>(S[n][r]);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const FT pa = *reinterpret_cast<const FT*>(pb + fr * LY::P_PITCH + (s * 32 + 8 * g) * sizeof(T));
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const FT vb = *reinterpret_cast<const FT*>(vt + (n * 16 + fr) * LY::VT_PITCH + (s * 32 + 8 * g) * sizeof(T));
        O[n] = mma16(pa, vb, O[n]);
      }
    }
    __syncthreads();
  }

  // ---- normalise and store (head-merged layout [row][h*64 + dim])
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    if (i >= nq) continue;
    const bool live = (i < q_valid) && (l_r[r] > 0.f);
    const float inv = live ? 1.f / l_r[r] : 0.f;
    T* op = out + (size_t)(q_row0 + i) * d + h * 64;
#pragma unroll
    for (int n = 0; n < 4; ++n) op[n * 16 + fr] = from_f32<T>(O[n][r] * inv);
  }
}

template <typename T>
int chunk_attention(const T* q, const T* kv, int kv_rows, const T* P, int p_rows, const float* pos_u,
                    const float* pos_v, const int32_t* desc, int nblk, int H, T* out, hipStream_t st) {
  if (nblk <= 0) return 0;
  hipLaunchKernelGGL((chunk_attention_kernel<T>), dim3(nblk, H), dim3(256), 0, st, q, kv, kv_rows, P, p_rows, pos_u,
                     pos_v, desc, H, out);
  CFM_CHECK_LAUNCH();
  return 0;
}

template int chunk_attention<float>(const float*, const float*, int, const float*, int, const float*, const float*,
                                    const int32_t*, int, int, float*, hipStream_t);
template int chunk_attention<bf16>(const bf16*, const bf16*, int, const bf16*, int, const float*, const float*,
                                   const int32_t*, int, int, bf16*, hipStream_t);

}  // namespace cfm
