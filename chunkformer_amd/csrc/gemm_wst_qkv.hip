// K = 512 weight-stationary GEMM: the QKV and GLU epilogues (gemm_wst_impl.h)
#include "gemm_wst_impl.h"

namespace cfm {
int wst_launch_qkv_glu(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N,
                       const EpiArgs& ep, hipStream_t st) {
  if (epi == EPI_QKV) return launch_wst<EPI_QKV, ACT_NONE>(A, lda, W, ldw, M, N, ep, st);
  if (act == ACT_SILU_L2E) return launch_wst<EPI_GLU, ACT_SILU_L2E>(A, lda, W, ldw, M, N, ep, st);
  return launch_wst<EPI_GLU, ACT_NONE>(A, lda, W, ldw, M, N, ep, st);
}
}  // namespace cfm
