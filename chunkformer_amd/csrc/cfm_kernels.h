// Internal launcher declarations (host side) for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;

#define CFM_HD_INLINE __host__ __device__ __forceinline__

namespace cfm {

// compute units of the current device (launch sizing of the persistent kernels), cached per
// device id: correct for a process that drives several GPUs, safe to call from several threads
int cu_count();

enum { EPI_STORE = 0, EPI_STORE_F32 = 1, EPI_RESID = 2, EPI_QKV = 3, EPI_GLU = 4, EPI_DW2 = 5 };
// ACT_SILU_L2E: the accumulator holds a = -log2(e) z (weights and bias pre-scaled at model build), and the
// output is a / (1 + 2^a) = -log2(e) silu(z) (the next GEMM's weights carry the -1 / log2(e)): one multiply per
// value less in the epilogue.  With EPI_GLU it marks the gate half as pre-scaled: out = lin / (1 + 2^gate)
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SILU = 2, ACT_SILU_L2E = 3 };

struct EpiArgs {
  const float* bias = nullptr;   // [N] f32 or null
  float alpha = 1.f;
  void* out = nullptr;           // STORE/STORE_F32/GLU output, QKV: q buffer [M, d]
  void* out2 = nullptr;          // QKV: KV stream [rows, H, 2*dk]
  int ldo = 0;                   // output row stride (elements)
  int row_off = 0;               // STORE*/GLU/QKV(kv): output row offset
  float* x = nullptr;            // RESID: f32 residual stream
  int ldx = 0;
  const uint8_t* rowmask = nullptr;  // RESID: per-row 0/1 multiplier (null = all 1)
  int d = 0;                     // QKV: model dim
  int dk = 64;                   // QKV: head dim (KV stream rows are [H][K dk | V dk])
  int col_group = 0;             // bf16 256-tile walk: column tiles per group (0 = all; tiles ordered group, row, col)
  int store_mode = 0;            // bf16 epilogue stores: 0 = plain, 1 = sc1 (drop the line from L2), 2 = nt
  // kernel selection / diagnostics (per model: cfm_model_set_option, never process-global)
  int diag = 0;                  // timing diagnostics of the bf16 kernels ("gemm_diag"; 0 = normal)
  int wst = 1;                   // K = 512 weight-stationary kernel ("gemm_wst")
  int small_tiles = 0;           // force the 128 x 128 kernel (cfm_op_gemm A/B)
  int big_min_tiles = 0;         // 256 x 256 kernel only from this many tiles (fewer: the 128 x 128 kernel)
  int wsp_small_div = 1;         // weight-stationary kernel below wsp_small_rows rows: grid = CUs / this
                                 // (leaves CUs to the other streams of a pipelined caller)
  int wsp_small_rows = 32768;
  int f16 = 0;                   // 16-bit operands / outputs are f16 (v_mfma_f32_16x16x32_f16), not bf16
  // DW2 (front-end pw1 + ReLU + dw2, K = N = 512 weight-stationary only): dw2 taps tap-major [9][N]
  // f32, bias [N]; the pw1 rows are (window, t2 < t2n, f2 < 19); out = dw2 rows (window, t3 < t3n, f3 < 9)
  const float* dw_w = nullptr;
  const float* dw_b = nullptr;
  int t2n = 0, t3n = 0;
};

int gemm_bf16_wst(int epi, int act, const bf16* A, int lda, const bf16* W, int ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t st);

enum { SITE_QKV = 1, SITE_OPROJ = 2, SITE_PW2 = 4, SITE_FFN2 = 8, SITE_FFN1 = 16, SITE_PW1 = 32, SITE_FE = 64 };

// Per-model kernel tuning (cfm_model_set_option); the defaults are the measured best
struct Tuning {
  int gemm_diag = 0, gemm_wst = 1, store_mode = 0, col_group = 0;
  int attn_reuse = 1;            // ring attention: band subtile carried between key tiles
  int conv_dot2 = 2;             // conv module: bf16 dot2 kernel in half-chunk blocks (1: one block per chunk, 0: per-tap f32)
  int conv_dma = 1;              // conv module: LDS-DMA window staging (0: register staging)
  int dw2_seg = 4;               // front-end dw2: row segments per walk
  int fe_conv = 6;               // bf16 front-end conv0+dw1: 1 = position-stationary (dw1 on VALU), 2 + k = channel-
                                 // stationary with dw1 on MFMA, ~k + 1 chunks per workgroup (2.74 vs 3.10 ms/step);
                                 // its ReLU is a clamp valid for |conv0| < 2^24 (NaN -> 0): models without CMVN
                                 // are created with 1 (build_model)
  int fe_fuse_dw2 = 1;           // front-end: pw1 + ReLU + dw2 in one weight-stationary GEMM (bf16; bench A/B
                                 // 50.85 -> 50.15 ms/step, 3 interleaved pairs; 0 = pw1 GEMM + fe_dw2_kernel)
  int attn128_var = 1;           // head_dim 128 attention kernel variant (A/B)
  // GEMM sites whose bf16 outputs are stored non-temporally ("nt_sites" bit mask, SITE_* below).
  // Default: FFN w2 (its y goes straight to the LayerNorm; bench A/B 52.2 -> 51.4 ms/step); nt on
  // the front-end pointwise outputs (+0.45 ms) or FFN w1's hidden (w1 slower) measured worse.
  int nt_sites = 8;   // SITE_FFN2
  int big_min_tiles = 0;         // 256 x 256 tiles only from this many tiles ("gemm_big_min"; small launches:
                                 // an endless segment's 12.7k rows are 100 tiles of 256 x 256 for 256 CUs)
  int wsp_small_div = 1;         // "wsp_small_div" / "wsp_small_rows" (see EpiArgs)
  int wsp_small_rows = 32768;
  int attn_min_chunks = 2;       // ring attention: chunks per block at least this ("attn_min_chunks")
  void apply(EpiArgs& e, int site = 0) const {
    e.diag = gemm_diag;
    e.big_min_tiles = big_min_tiles;
    e.wsp_small_div = wsp_small_div;
    e.wsp_small_rows = wsp_small_rows;
    e.wst = gemm_wst;
    e.store_mode = (nt_sites & site) ? 2 : store_mode;
    e.col_group = col_group;
  }
};

template <typename T>
int gemm(int epi, int act, const T* A, int lda, const T* W, int ldw, int M, int N, int K, const EpiArgs& ep,
         hipStream_t st);


// LayerNorm over d (eps) of f32 rows -> T rows; optional 0/1 row mask on the output.
// fused residual add of the previous sub-block: x += alpha * ymask[row] * y (y null = none)
// A LayerNorm that defers (defer = true) leaves x unwritten: the next LayerNorm re-applies that
// branch as its FIRST term (y, alpha, ymask) and adds its own as the second (y2, alpha2, ymask2),
// in the same order, so x is bit-identical and one f32 write + read of x is saved per pair.
template <typename T> struct ResidAdd {
  const T* y = nullptr;
  float alpha = 1.f;
  const uint8_t* ymask = nullptr;
  const T* y2 = nullptr;
  float alpha2 = 1.f;
  const uint8_t* ymask2 = nullptr;
  bool defer = false;
};
template <typename T>
int layernorm(float* x, const ResidAdd<T>& ra, int M, int d, const float* w, const float* b, float eps, T* out,
              const uint8_t* rowmask, hipStream_t st);
template <typename T>
int layernorm2(float* x, const ResidAdd<T>& ra, int M, int d, const float* w1, const float* b1, const float* w2,
               const float* b2, float eps, T* out, hipStream_t st);
template <typename T>
int layernorm2_f32(float* x, const ResidAdd<T>& ra, int M, int d, const float* w1, const float* b1, const float* w2,
                   const float* b2, float eps, float* out, hipStream_t st);

// chunk attention (attention.hip)
template <typename T>
int chunk_attention(const T* q, const T* kv, int kv_rows, const T* P, int p_rows, const float* pos_u,
                    const float* pos_v, const int32_t* desc, int nblk, int H, int dk, T* out, hipStream_t st,
                    int p_ld = 0);   // P row stride (elements; 0 = H * dk); dk = 64 or 128

// KV-stream column of K (which = 0) / V (which = 1) column cc (< d) of the QKV projection
CFM_HD_INLINE int qkv_kv_col(int cc, int which, int dk) { return (cc / dk) * 2 * dk + which * dk + (cc & (dk - 1)); }

// masked-batch ring kernel (bf16, head dim 64); -1 = shape not eligible
// full attention (padded plan with chunk_size <= 0), bf16, dk 64, T' <= 384: every key of the utterance
// staged once per block; -1 when not eligible (attention.hip)
int full_attention_bf16(const bf16* q, const bf16* kv, int kv_rows, const bf16* P, int p_rows, const float* pos_u,
                        const float* pos_v, const int32_t* desc, int nutt, int nd, int H, int dk, int t_keys,
                        bf16* out, hipStream_t st, int p_ld);
int chunk_attention_masked_bf16(const bf16* q, const bf16* kv, int kv_rows, const bf16* P, int p_rows,
                                const float* pos_u, const float* pos_v, const int32_t* desc, int n_chunks, int H,
                                int C, int W, bf16* out, hipStream_t st, int diag = 0, int p_ld = 0, int reuse = 1,
                                int min_chunks = 2);
// the same ring kernel on f16 operands (v_mfma_f32_16x16x32_f16; the fp16 compute mode)
int chunk_attention_masked_f16(const f16* q, const f16* kv, int kv_rows, const f16* P, int p_rows,
                               const float* pos_u, const float* pos_v, const int32_t* desc, int n_chunks, int H,
                               int C, int W, f16* out, hipStream_t st, int diag = 0, int p_ld = 0, int reuse = 1,
                               int min_chunks = 2);

// masked-batch attention for head_dim 128 (attention128.hip): V^T copy of the KV stream, then the
// band / score / P.V kernel; -1 when the shape is not eligible (C = 64, W <= 320, W % 64 == 0)
bool attention_a128_eligible(int C, int W, int p_rows, int dk);
int vt_transpose_bf16(const bf16* kv, int kv_rows, int H, bf16* vt, int vt_ld, hipStream_t st);
int chunk_attention_masked_a128(const bf16* q, const bf16* kv, int kv_rows, const bf16* vt, int vt_ld, const bf16* P,
                                int p_rows, int p_ld, const float* pos_u, const float* pos_v, const int32_t* desc,
                                int n_chunks, int H, int C, int W, bf16* out, hipStream_t st, int var = 1);

// conv module: depthwise k=15 + bias + LayerNorm + SiLU (conv_module.hip)
template <typename T>
int conv_dw_ln_silu(const T* glu, const int32_t* desc, int nblk, int d, const float* wdw_t /*[15][d]*/,
                    const float* bdw, const float* lnw, const float* lnb, float eps, T* out, hipStream_t st,
                    int dot2 = 1, int dma = 1);

// front-end (frontend.hip): meta rows give (src_row, nvalid) per window at PM_SRC_ROW / PM_NVALID;
// with `tab` (device array of per-utterance row pointers) window c of utterance u starts at
// tab[u] + c * step rows instead (PM_UTT / PM_CHUNK)
template <typename T>
int frontend_conv0_dw(const float* feats, const float* const* tab, int step, const int32_t* meta, int meta_stride,
                      int nwin, int W,
                      const float* cmvn_mean, const float* cmvn_istd, const float* w0, const float* b0,
                      const float* w1, const float* b1, const float* wpack, const float* wfrag, int d, T* out,
                      hipStream_t st, int var = 1);
// per-channel [w0 taps 0..8 | w1 taps 0..8 | b0 | b1 | pad 2] (FE_WPACK floats) for the bf16 MFMA front-end
constexpr int FE_WPACK = 24;
constexpr int FE2_NFRAG = 23;   // per-lane 16-B fragments of one 32-channel tile (channel-stationary front-end)
template <typename T>
int frontend_dw2(const T* in, int nwin, int T2, int d, const float* w, const float* b, T* out, hipStream_t st,
                 int seg = 4);

// misc (misc.hip)
template <typename T>
int pos_table(int d, int p_rows, int anchor, T* out, hipStream_t st);
template <typename T>
int att_cache_in(const float* cache, int L, int row_elems, T* kv, hipStream_t st);
template <typename T>
int att_cache_out(const T* kv, int start_row, int L, int row_elems, float* cache, hipStream_t st);
template <typename T>
int att_cache_in_hl(const float* cache /*[H][L][2dk]*/, int H, int L, int dk, T* kv, hipStream_t st);
template <typename T>
int att_cache_out_hl(const T* kv, int start_row, int H, int L, int dk, float* cache /*[H][L][2dk]*/, hipStream_t st);
template <typename T>
int cnn_cache_in(const float* cache /*[d][7]*/, int d, int lorder, T* glu, hipStream_t st);
template <typename T>
int cnn_cache_out(const T* glu, int start_row, int d, int lorder, float* cache, hipStream_t st);
// both caches of a layer in one launch (attention: flat rows, or head-major when hl; conv: optional)
template <typename T>
int cache_io(bool in, bool hl, float* acache, int H, int L, int dk, T* kv, float* ccache, int d, int lorder, T* glu,
             hipStream_t st);
int masks_from_plan(const int32_t* meta, int n, int C, int L, int R, uint8_t* att, uint8_t* pad, hipStream_t st);
// CTC head (ctc.hip): ids-only argmax of enc . W^T + b without a logit tensor (bf16 W with rows padded
// to a multiple of 64, d = 512; -1 = not eligible), and the collapse / silence segmentation of ids
bool ctc_argmax_eligible(int V, int d);
int ctc_argmax_bf16(const float* enc, int M, const bf16* W, const float* bias, int V, int d, int32_t* ids,
                    hipStream_t st);
int ctc_argmax_f16(const float* enc, int M, const f16* W, const float* bias, int V, int d, int32_t* ids,
                   hipStream_t st);
int ctc_collapse(const int32_t* ids, const int32_t* row_start, const int32_t* row_len, int B, int blank, int max_sil,
                 int32_t* tok, int32_t* tok_frame, int32_t* n_tok, int32_t* seg, int32_t* n_seg, hipStream_t st);
int log_softmax_rows(float* logits, int M, int V, int write_logp, int32_t* ids, hipStream_t st);

}  // namespace cfm
