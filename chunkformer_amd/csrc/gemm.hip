// MFMA GEMM with fused epilogues for every projection on the encoder path.
//
//   C[M, N] = A[M, K] . W[N, K]^T      (A, W row-major, K contiguous: nn.Linear layout)
//
// Tile 128 x 128 x 128 B of K (64 bf16 / 32 f32), 256 threads = 4 waves in 2x2,
// each wave owns 64x64 = 4x4 MFMA 16x16 tiles.  Operands are staged
// global -> registers -> LDS with one barrier per K-step (issue the next tile's
// loads before the MFMAs, write them to the other LDS buffer after: T14 split).
// LDS rows are 128 B; chunk c of row r lives at chunk c ^ ((r >> 1) & 7), which
// makes the 16-row ds_read_b128 fragment reads conflict-free (two 128-B rows
// share one 256-B bank row, so the XOR key skips the row-parity bit).
// Blocks are remapped so that the column tiles of one row panel run on the
// same XCD (bijective remap, cdna_hip_programming.md T1): the A panel is then
// re-read from that XCD's L2 instead of HBM.
//
// Epilogues (reference ops they replace):
//   EPI_STORE      out_T = act(acc + b)          FFN w_1+SiLU (positionwise_feed_forward.py:59),
//                                                 front-end pointwise conv + ReLU (subsampling.py:94-104)
//   EPI_STORE_F32  out_f32 = alpha (acc + b)     front-end out Linear * sqrt(d) (subsampling.py:164,
//                                                 embedding.py:509), linear_pos (attention.py:482), CTC ctc_lo
//   EPI_RESID      x += alpha (acc + b) [rowmask] FFN w_2 residual x0.5 (encoder_layer.py:190-196, 236-243),
//                                                 linear_out (attention.py:150 + encoder_layer.py:215),
//                                                 pointwise_conv2 + mask (convolution.py:250-253)
//   EPI_QKV        q / K,V stream rows           linear_q/k/v + KV concat (attention.py:450-461)
//   EPI_GLU        a * sigmoid(g) stream rows    pointwise_conv1 + GLU (convolution.py:220-221)
#include "cfm_common.h"
#include "cfm_kernels.h"
#include <cstdlib>

namespace cfm {

template <typename T> struct GemmTraits {
  static constexpr int EPC = 16 / sizeof(T);   // elements per 16-B chunk
  static constexpr int BK = 8 * EPC;           // elements per 128-B LDS row
  static constexpr int KSUB = BK / 32;         // 32-deep MFMA sub-steps per K tile (bf16: 2, f32: 1)
};

CFM_DEV int swz(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

template <typename T, int EPI, int ACT>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const T* __restrict__ A, int lda,
                                                      const T* __restrict__ W, int ldw,
                                                      int M, int N, int K, EpiArgs ep) {
  using Tr = GemmTraits<T>;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 128 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int nbn = (N + 127) >> 7, nbm = (M + 127) >> 7;
  const int nwg = nbn * nbm;
  // XCD-aware bijective remap: blocks b, b+8, b+16 ... (one XCD) get consecutive logical tiles
  const int b = blockIdx.x, xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int tm = L / nbn, tn = L - tm * nbn;
  const int m0 = tm * 128, n0 = tn * 128;

  // staging: 1024 16-B chunks per operand tile, 4 per thread
  const T* asrc[4];
  const T* wsrc[4];
  int soff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qd = tid + 256 * i, row = qd >> 3, ch = qd & 7;
    asrc[i] = A + (size_t)min(m0 + row, M - 1) * lda + ch * Tr::EPC;
    wsrc[i] = W + (size_t)min(n0 + row, N - 1) * ldw + ch * Tr::EPC;
    soff[i] = swz(row, ch);
  }
  u32x4 ra[4], rw[4];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const u32x4*>(asrc[i] + (size_t)kt * Tr::BK);
      rw[i] = *reinterpret_cast<const u32x4*>(wsrc[i] + (size_t)kt * Tr::BK);
    }
  };
  auto sstore = [&](int buf) {
    char* as = smem + buf * 32768;
    char* ws = as + 16384;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<u32x4*>(as + soff[i]) = ra[i];
      *reinterpret_cast<u32x4*>(ws + soff[i]) = rw[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / Tr::BK;
  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15, g = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kt + 1);
    const char* as = smem + (kt & 1) * 32768;
    const char* ws = as + 16384;
#pragma unroll
    for (int s = 0; s < Tr::KSUB; ++s) {
      typename Frag<T>::type af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra_ = wm * 64 + i * 16 + fr, rb_ = wn * 64 + i * 16 + fr;
        if constexpr (sizeof(T) == 2) {
          const int ch = s * 4 + g;
          af[i] = *reinterpret_cast<const typename Frag<T>::type*>(as + swz(ra_, ch));
          bfr[i] = *reinterpret_cast<const typename Frag<T>::type*>(ws + swz(rb_, ch));
        } else {
          f32x4 lo = *reinterpret_cast<const f32x4*>(as + swz(ra_, 2 * g));
          f32x4 hi = *reinterpret_cast<const f32x4*>(as + swz(ra_, 2 * g + 1));
          af[i] = (f32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          lo = *reinterpret_cast<const f32x4*>(ws + swz(rb_, 2 * g));
          hi = *reinterpret_cast<const f32x4*>(ws + swz(rb_, 2 * g + 1));
          bfr[i] = (f32x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore((kt + 1) & 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  const int rbase = m0 + wm * 64 + 4 * g;
  const int cbase = n0 + wn * 64 + fr;
  if constexpr (EPI == EPI_GLU) {
    // weights are interleaved in 16-column blocks: [a(16) | gate(16)] per 32 columns
    T* out = reinterpret_cast<T*>(ep.out);
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      const int col = cbase + j * 16;                    // a-column (even block)
      if (col >= N) continue;
      const int ch = ((col - fr) >> 5) * 16 + fr;
      const float ba = ep.bias[col], bg = ep.bias[col + 16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r;
          if (row < M) {
            const float a = acc[i][j][r] + ba, gt = acc[i][j + 1][r] + bg;
            const float sg = ACT == ACT_SILU_L2E ? 1.f / (1.f + exp2f(gt)) : sigmoid_f(gt);
            out[(size_t)(row + ep.row_off) * ep.ldo + ch] = from_f32<T>(a * sg);
          }
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cbase + j * 16;
      if (col >= N) continue;
      const float bias = ep.bias ? ep.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r;
          if (row >= M) continue;
          float v = acc[i][j][r] + bias;
          if constexpr (EPI == EPI_STORE) {
            if constexpr (ACT == ACT_RELU) v = fmaxf(v, 0.f);
            if constexpr (ACT == ACT_SILU) v = silu_f(v);
            if constexpr (ACT == ACT_SILU_L2E) v = v / (1.f + exp2f(v));
            reinterpret_cast<T*>(ep.out)[(size_t)(row + ep.row_off) * ep.ldo + col] = from_f32<T>(v);
          } else if constexpr (EPI == EPI_STORE_F32) {
            reinterpret_cast<float*>(ep.out)[(size_t)(row + ep.row_off) * ep.ldo + col] = ep.alpha * v;
          } else if constexpr (EPI == EPI_RESID) {
            float* xp = ep.x + (size_t)row * ep.ldx + col;
            const float m = ep.rowmask ? (float)ep.rowmask[row] : 1.f;
            *xp = *xp + ep.alpha * v * m;
          } else if constexpr (EPI == EPI_QKV) {
            const int d = ep.d;
            if (col < d) {
              reinterpret_cast<T*>(ep.out)[(size_t)row * d + col] = from_f32<T>(v);
            } else {
              const int c2 = col - d, which = c2 >= d ? 1 : 0, cc = c2 - which * d;
              reinterpret_cast<T*>(ep.out2)[(size_t)(row + ep.row_off) * (2 * d) + qkv_kv_col(cc, which, ep.dk)] =
                  from_f32<T>(v);
            }
          }
        }
    }
  }
}

template <typename T, int EPI, int ACT>
static int launch(const T* A, int lda, const T* W, int ldw, int M, int N, int K, const EpiArgs& ep,
                  hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (K % GemmTraits<T>::BK) return (int)hipErrorInvalidValue;
  const int nwg = ((M + 127) / 128) * ((N + 127) / 128);
  hipLaunchKernelGGL((gemm_kernel<T, EPI, ACT>), dim3(nwg), dim3(256), 0, st, A, lda, W, ldw, M, N, K, ep);
  CFM_CHECK_LAUNCH();
  return 0;
}

int gemm_bf16_big(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st);

template <typename T>
int gemm(int epi, int act, const T* A, int lda, const T* W, int ldw, int M, int N, int K, const EpiArgs& ep,
         hipStream_t st) {
  if constexpr (sizeof(T) == 2) {   // bf16 / f16: the 256 x 256 and weight-stationary kernels (EpiArgs::f16)
    if (!ep.small_tiles) {
      EpiArgs e = ep;
      e.f16 = std::is_same<T, f16>::value;
      const int r = gemm_bf16_big(epi, act, reinterpret_cast<const bf16*>(A), lda, reinterpret_cast<const bf16*>(W),
                                  ldw, M, N, K, e, st);
      if (r != -1) return r;
    }
  }
  switch (epi) {
    case EPI_STORE:
      if (act == ACT_RELU) return launch<T, EPI_STORE, ACT_RELU>(A, lda, W, ldw, M, N, K, ep, st);
      if (act == ACT_SILU) return launch<T, EPI_STORE, ACT_SILU>(A, lda, W, ldw, M, N, K, ep, st);
      if (act == ACT_SILU_L2E) return launch<T, EPI_STORE, ACT_SILU_L2E>(A, lda, W, ldw, M, N, K, ep, st);
      return launch<T, EPI_STORE, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_STORE_F32: return launch<T, EPI_STORE_F32, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_RESID: return launch<T, EPI_RESID, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_QKV: return launch<T, EPI_QKV, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
    case EPI_GLU:
      if (act == ACT_SILU_L2E) return launch<T, EPI_GLU, ACT_SILU_L2E>(A, lda, W, ldw, M, N, K, ep, st);
      return launch<T, EPI_GLU, ACT_NONE>(A, lda, W, ldw, M, N, K, ep, st);
  }
  return (int)hipErrorInvalidValue;
}

template int gemm<float>(int, int, const float*, int, const float*, int, int, int, int, const EpiArgs&, hipStream_t);
template int gemm<bf16>(int, int, const bf16*, int, const bf16*, int, int, int, int, const EpiArgs&, hipStream_t);
template int gemm<f16>(int, int, const f16*, int, const f16*, int, int, int, int, const EpiArgs&, hipStream_t);

}  // namespace cfm
