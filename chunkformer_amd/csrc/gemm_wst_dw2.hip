// K = 512 weight-stationary GEMM: the front-end pw1 + ReLU + dw2 epilogue (gemm_wst_impl.h)
#include "gemm_wst_impl.h"

namespace cfm {
int wst_launch_dw2(const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep, hipStream_t st) {
  return launch_wst<EPI_DW2, ACT_RELU>(A, lda, W, ldw, M, N, ep, st);
}
}  // namespace cfm
