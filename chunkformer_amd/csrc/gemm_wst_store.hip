// K = 512 weight-stationary GEMM: plain and ReLU STORE epilogues (gemm_wst_impl.h)
#include "gemm_wst_impl.h"

namespace cfm {
int wst_launch_store(int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep,
                     hipStream_t st) {
  if (act == ACT_RELU) return launch_wst<EPI_STORE, ACT_RELU>(A, lda, W, ldw, M, N, ep, st);
  return launch_wst<EPI_STORE, ACT_NONE>(A, lda, W, ldw, M, N, ep, st);
}
}  // namespace cfm
