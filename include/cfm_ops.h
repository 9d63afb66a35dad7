/*
 * cfm_ops.h — operator-level entry points of libcfm.so (tests and integrators).
 *
 * These expose single kernels of the encoder path on caller-owned device
 * buffers, stream-ordered, no allocation.  They are not part of the
 * reference's surface; the parity tests use them to check one kernel at a time
 * against a torch fp32 reference of the same op.
 */
#ifndef CFM_OPS_H
#define CFM_OPS_H
#include "cfm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* epilogue kinds / activations of the projection GEMM C = A . W^T (A [M,K], W [N,K]) */
typedef enum { CFM_EPI_STORE = 0, CFM_EPI_STORE_F32 = 1, CFM_EPI_RESID = 2, CFM_EPI_QKV = 3, CFM_EPI_GLU = 4 } cfm_epi;
typedef enum { CFM_ACT_NONE = 0, CFM_ACT_RELU = 1, CFM_ACT_SILU = 2 } cfm_act;

/* dtype selects the operand type of A / W / T outputs (CFM_DTYPE_F32 or CFM_DTYPE_BF16).
 *   STORE:     out_T[(m+row_off)*ldo + n] = act(acc + bias)
 *   STORE_F32: out_f32[(m+row_off)*ldo + n] = alpha*(acc + bias)
 *   RESID:     x[m*ldx + n] += alpha*(acc + bias)*rowmask[m]
 *   QKV:       n < d -> out_T[m*d + n]; else out2_T[(m+row_off)*2d + head*128 + {0,64} + dim]
 *   GLU:       W rows interleaved [a16 | gate16]: out_T[(m+row_off)*ldo + ch] = a*sigmoid(gate)
 * variant (A/B testing): bit 0 forces the 128x128 kernel; bits 8-15 select a timing diagnostic of
 * the bf16 kernels (1 no MFMA, 2 no DMA in the loop, 3 no epilogue, 5 no stores; 0 = normal; only
 * in a library built with -DCFM_GEMM_DIAG); bits 16-17 the bf16 store policy (2 = nt); bits 18-20 the
 * K = 512 weight-stationary kernel (0 = model default, 1 = on, 2 = on at any M, 7 = off). */
cfm_status cfm_op_gemm(int32_t dtype, int32_t epi, int32_t act, const void* A, int32_t lda, const void* W, int32_t ldw,
                       int32_t M, int32_t N, int32_t K, const float* bias, float alpha, void* out, int32_t ldo,
                       int32_t row_off, void* out2, int32_t d, float* x, int32_t ldx, const uint8_t* rowmask,
                       int32_t variant, cfm_stream stream);

#ifdef __cplusplus
}
#endif
#endif
