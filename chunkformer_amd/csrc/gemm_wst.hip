// Dispatch of the K = 512 weight-stationary GEMM (gemm_wst_impl.h) to its epilogue families, each
// instantiated in its own translation unit (gemm_wst_store / _silu / _qkv / _dw2.hip).
#include "gemm_wst_impl.h"

namespace cfm {

int wst_launch_store(int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep,
                     hipStream_t st);
int wst_launch_silu(int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep,
                    hipStream_t st);
int wst_launch_qkv_glu(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N,
                       const EpiArgs& ep, hipStream_t st);
int wst_launch_dw2(const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep, hipStream_t st);

// -1 = not eligible (caller uses the 256 x 256 kernel)
int gemm_bf16_wst(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st) {
  if (K != WST_K || N % 256 || lda % 8 || ldw % 8 || M <= 0) return -1;
  // enough rows for every CU of an XCD's column tiles to own several tiles
  // enough row tiles for every CU of an XCD's column tiles to own some: 512 for the GLU epilogue,
  // 128 otherwise (measured at endless_decode's 12.7k-row segments: FFN w1 45 -> 41 us, QKV 36 ->
  // 30 us; GLU 20 -> 24 us, so it keeps the 256 x 256 kernel there); ep.wst == 2: any M (A/B)
  const int min_tiles = epi == EPI_GLU ? 512 : 128;
  if (ep.wst < 2 && epi != EPI_DW2 && (M + WST_MT - 1) / WST_MT < min_tiles) return -1;
  if (N / 256 > 32) return -1;
  switch (epi) {
    case EPI_STORE:
      if (act == ACT_SILU || act == ACT_SILU_L2E) return wst_launch_silu(act, A, lda, W, ldw, M, N, ep, st);
      return wst_launch_store(act, A, lda, W, ldw, M, N, ep, st);
    case EPI_QKV: return wst_launch_qkv_glu(EPI_QKV, ACT_NONE, A, lda, W, ldw, M, N, ep, st);
    case EPI_GLU:
      if (ep.bias == nullptr) return -1;
      return wst_launch_qkv_glu(EPI_GLU, act, A, lda, W, ldw, M, N, ep, st);
    case EPI_DW2:   // front-end pw1 + ReLU + dw2 (N = 512, dw2 taps / bias / geometry in ep; bf16 or f16)
      if (act != ACT_RELU || N != 512 || !ep.dw_w || !ep.dw_b || ep.t2n < 3 || ep.ldo % 8) return -1;
      return wst_launch_dw2(A, lda, W, ldw, M, N, ep, st);
  }
  return -1;
}

}  // namespace cfm
