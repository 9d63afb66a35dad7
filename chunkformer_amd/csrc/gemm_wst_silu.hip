// K = 512 weight-stationary GEMM: SiLU STORE epilogues (FFN w1; gemm_wst_impl.h)
#include "gemm_wst_impl.h"

namespace cfm {
int wst_launch_silu(int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep,
                    hipStream_t st) {
  if (act == ACT_SILU_L2E) return launch_wst<EPI_STORE, ACT_SILU_L2E>(A, lda, W, ldw, M, N, ep, st);
  return launch_wst<EPI_STORE, ACT_SILU>(A, lda, W, ldw, M, N, ep, st);
}
}  // namespace cfm
