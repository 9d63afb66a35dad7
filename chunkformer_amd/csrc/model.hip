// Model handle, weight repacking and the per-call orchestration of the encoder.
//
// ModelT<T>::encode runs, on one stream and without allocation or host sync:
//   front-end (frontend.hip + 3 GEMMs, in window groups) -> x [rows, d] f32
//   P_l = pos_emb . W_pos_l^T for every layer (attention.py:481-483)
//   12 x ChunkFormerEncoderLayer (encoder_layer.py:155-248 masked / 62-153 padded):
//     LN -> FFN_mac (GEMM SiLU, GEMM resid x0.5) -> LN -> QKV GEMM -> chunk attention
//     -> out-proj GEMM (resid) -> LN -> pw1 GEMM + GLU -> dw/LN/SiLU -> pw2 GEMM (masked resid)
//     -> LN -> FFN (x0.5) -> norm_final fused with the next layer's first LN / after_norm
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/cfm.h"
#include "../../include/cfm_ops.h"
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "plan.h"
#include "status.h"

namespace cfm {

static thread_local std::string g_err;
cfm_status set_error(cfm_status s, const std::string& msg) {
  g_err = msg;
  return s;
}

#define HIPC(x)                                                                               \
  do {                                                                                        \
    hipError_t _e = (x);                                                                      \
    if (_e != hipSuccess) return set_error(CFM_ERR_RUNTIME, std::string(#x ": ") + hipGetErrorString(_e)); \
  } while (0)
#define KCHK(x)                                                                               \
  do {                                                                                        \
    int _e = (x);                                                                             \
    if (_e) return set_error(CFM_ERR_RUNTIME, std::string(#x ": ") + hipGetErrorString((hipError_t)_e)); \
  } while (0)

// time one launch (class CLS) with events when that class is enabled in prof_mask
#define PROF(CLS, X)                      \
  do {                                    \
    hipEvent_t _pb;                       \
    prof_begin(CLS, st, &_pb);            \
    KCHK(X);                              \
    prof_end(CLS, st, _pb);               \
  } while (0)

static size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base((char*)b) {}
  template <typename U> U* take(size_t n) {
    U* p = (U*)(base ? base + off : nullptr);
    off += align_up(n * sizeof(U));
    return p;
  }
};

struct LayerW {
  void *ff1m, *ff2m, *ff1, *ff2, *qkv, *pos, *wo, *pw1, *pw2;   // T matrices [N][K]
  float *b_ff1m, *b_ff2m, *b_ff1, *b_ff2, *b_qkv, *b_o, *b_pw1, *b_pw2;
  float *pu, *pv, *dw_t, *b_dw, *cn_w, *cn_b;
  float *ln_ffm_w, *ln_ffm_b, *ln_mha_w, *ln_mha_b, *ln_conv_w, *ln_conv_b, *ln_ff_w, *ln_ff_b, *ln_fin_w, *ln_fin_b;
};

struct FrontW {
  float *cm = nullptr, *ci = nullptr, *w0, *b0, *w1, *b1, *w2, *b2, *b_pw1, *b_pw2, *b_out, *wpack, *wfrag = nullptr;
  void *pw1, *pw2, *wout;
  float *an_w, *an_b;
  void* ctc_w = nullptr;
  float* ctc_b = nullptr;
  void* pos_all = nullptr;   // every layer's linear_pos weight stacked [nb * d, d]: one GEMM per call
};

}  // namespace cfm

// Kernel classes timed by the optional in-stream profiler (HIP events around launches)
enum {
  PC_FE_CONV = 0, PC_FE_GEMM, PC_FE_DW2, PC_POS, PC_LN, PC_FFN1, PC_FFN2, PC_QKV, PC_ATTN, PC_OPROJ, PC_PW1,
  PC_CONV, PC_PW2, PC_CACHE, PC_CTC, PC_N
};
static const char* const PC_NAMES[PC_N] = {
    "frontend_conv0_dw", "frontend_pw_gemm", "frontend_dw2", "pos_gemm", "layernorm", "ffn_w1_gemm", "ffn_w2_gemm",
    "qkv_gemm", "chunk_attention", "out_proj_gemm", "pw1_glu_gemm", "conv_dw_ln_silu", "pw2_gemm", "cache_copy",
    "ctc"};

struct cfm_model {
  cfm_config cfg;
  int device = 0;
  void* dev_mem = nullptr;
  std::vector<cfm::LayerW> layers;
  cfm::FrontW fe;
  int max_layers = -1;
  int fe_group_windows = 0;         // "fe_group_windows": cap on front-end windows per group (0 = by memory)
  bool use_ring_attention = true;
  bool use_fused_ctc = true;        // "ctc_fused": bf16 ids-only CTC head as one argmax kernel (ctc.hip), no [rows, V] logits
  int cache_fuse = 1;               // "cache_fuse": both caches of a layer in one launch at its start / end
  int trim_right = 0;               // "trim_right": this call's rows past `trunc` are dropped by the caller (encode)
  // "fe_carry" / "fe_reuse" / "fe_save_from" (endless_decode's segments): the front-end output rows of the
  // first fe_reuse windows are copied from the f32 buffer fe_carry instead of computed, and those of windows
  // [fe_save_from, nwin) are copied into it after the front-end (a window's rows depend on its own frames
  // only: the next segment's first windows are this segment's last ones)
  float* fe_carry = nullptr;
  int fe_reuse = 0, fe_save_from = -1;
  int attn_diag = 0;                // "attn_diag": 1 = ring kernel without compute (staging only)
  cfm::Tuning tune;                 // per-model kernel selection / diagnostics (cfm_model_set_option)
  // profiler: bitmask of PC_* classes to bracket with events on the launch stream
  uint32_t prof_mask = 0;
  mutable std::vector<hipEvent_t> ev_pool;
  mutable std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_live;
  mutable double prof_ms[PC_N] = {0};
  mutable int64_t prof_n[PC_N] = {0};
  hipEvent_t ev_get() const {
    if (ev_pool.empty()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      return e;
    }
    hipEvent_t e = ev_pool.back();
    ev_pool.pop_back();
    return e;
  }
  void prof_begin(int cls, hipStream_t st, hipEvent_t* b) const {
    *b = nullptr;
    if (!(prof_mask >> cls & 1u)) return;
    *b = ev_get();
    if (*b) (void)hipEventRecord(*b, st);
  }
  void prof_end(int cls, hipStream_t st, hipEvent_t b) const {
    if (!b) return;
    hipEvent_t e = ev_get();
    if (!e) return;
    (void)hipEventRecord(e, st);
    ev_live.push_back({cls, {b, e}});
  }
  void prof_collect() const {   // host-synchronising: only from cfm_profile_read
    for (auto& it : ev_live) {
      float ms = 0.f;
      if (hipEventSynchronize(it.second.second) == hipSuccess &&
          hipEventElapsedTime(&ms, it.second.first, it.second.second) == hipSuccess) {
        prof_ms[it.first] += ms;
        prof_n[it.first] += 1;
      }
      ev_pool.push_back(it.second.first);
      ev_pool.push_back(it.second.second);
    }
    ev_live.clear();
  }
  virtual ~cfm_model() {
    if (dev_mem) { (void)hipSetDevice(device); (void)hipFree(dev_mem); }
    for (auto& it : ev_live) { (void)hipEventDestroy(it.second.first); (void)hipEventDestroy(it.second.second); }
    for (auto e : ev_pool) (void)hipEventDestroy(e);
  }
  // cache_b: batch size of a streaming-chunk call (plan kind 3): its caches are [nb, cache_b, H, L, 2dk] /
  // [nb, cache_b, d, 7] (forward_chunk layout) and `aci` etc. point at this element's [H, L, 2dk] slice
  // stages [stage_lo, stage_hi]: -1 = front-end, relative positions, stream padding and the first
  // LayerNorm; l = encoder layer l (its caches, ending with norm_final fused into the next layer's
  // first LayerNorm or after_norm).  One call with (-1, num_blocks - 1) is the whole encoder; calls
  // over consecutive stage ranges with the same workspace give the same result.
  virtual cfm_status encode(const float* feats, const int32_t* plan_dev, const int32_t* plan_hdr, const float* aci,
                            const float* cci, int trunc, float* aco, float* cco, float* out, void* ws, size_t wsb,
                            hipStream_t st, int cache_b = 1, int stage_lo = -1, int stage_hi = 1 << 30,
                            const float* const* feats_tab = nullptr) const = 0;
  virtual cfm_status ctc(const float* enc, int rows, float* logp, int32_t* ids, void* ws, size_t wsb,
                         hipStream_t st) const = 0;
  virtual size_t ws_bytes(const int32_t* hdr) const = 0;
  virtual size_t ctc_ws_bytes(int rows) const = 0;
  // ids-only CTC (logp == nullptr): 0 bytes on the fused argmax path
  virtual size_t ctc_ids_ws_bytes(int rows) const = 0;
};

namespace cfm {

// 16-bit modes run the FFN SiLU and the conv module's GLU on -log2(e)-prescaled accumulators (ACT_SILU_L2E,
// cfm_kernels.h): the weights are scaled once in build_model
#ifndef CFM_SILU_PRE
#define CFM_SILU_PRE 1   // 0: the plain SiLU / GLU epilogues in the 16-bit modes too (A/B builds)
#endif
template <typename T> constexpr bool kSiluPre = CFM_SILU_PRE && sizeof(T) == 2;
template <typename T> constexpr int kActSilu = kSiluPre<T> ? ACT_SILU_L2E : ACT_SILU;
constexpr float kLog2e = 1.4426950408889634f;

template <typename T>
struct ModelT : public cfm_model {
  // front-end window group size: bounds the [G, T2, 19, d] intermediates to 768 MiB each (measured:
  // 48-192 MiB groups are slower, 1.5-8 GiB equal); the "fe_group_windows" option caps it further
  int fe_group(const int32_t* h) const {
    const int W = h[PH_W];
    const int T1 = (W - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
    const size_t per = (size_t)T2 * 19 * cfg.d_model * sizeof(T);
    int g = (int)std::max<size_t>(1, ((size_t)768 << 20) / per);
    if (fe_group_windows > 0) g = std::min(g, fe_group_windows);
    g = std::min(g, 65535);   // the front-end kernels put a group's windows on gridDim.y / .z
    return std::min(g, h[PH_NWIN]);
  }

  // epilogue args carrying this model's kernel tuning
  EpiArgs E(int site = 0) const {
    EpiArgs e;
    tune.apply(e, site);
    return e;
  }

  struct WS {
    float* x;
    T *h, *hid, *q, *kv, *ao, *glu, *cv, *y, *y2, *P, *pos, *feA, *feB, *feC;
    T* vt = nullptr;   // head_dim 128 masked batch: V^T copy of the KV stream [H][128][vt_ld]
    int vt_ld = 0;
  };
  // the head_dim 128 attention kernel's V^T buffer is needed (bf16 masked batch)
  bool uses_vt(const int32_t* h) const {
    return std::is_same<T, bf16>::value && h[PH_KIND] == 1 && use_ring_attention && cfg.d_model == 128 * cfg.n_heads &&
           attention_a128_eligible(h[PH_C], h[PH_L] + h[PH_C] + h[PH_R], h[PH_PROWS], 128);
  }

  WS carve(void* base, const int32_t* h, size_t* total) const {
    const int d = cfg.d_model, ff = cfg.ffn_dim, nb = cfg.num_blocks;
    const size_t rows = h[PH_ROWS];
    const size_t prow_pad = (h[PH_PROWS] + 127) / 128 * 128;
    const int W = h[PH_W];
    const int T1 = (W - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1;
    const size_t G = fe_group(h);
    Carver c(base);
    WS w;
    w.x = c.take<float>(rows * d);
    w.h = c.take<T>(rows * d);
    w.hid = c.take<T>(rows * ff);
    w.q = c.take<T>(rows * d);
    w.kv = c.take<T>((size_t)h[PH_KVROWS] * 2 * d);
    w.ao = c.take<T>(rows * d);
    w.glu = c.take<T>((size_t)h[PH_GLUROWS] * d);
    w.cv = c.take<T>(rows * d);
    w.y = c.take<T>(rows * d);
    w.y2 = c.take<T>(rows * d);
    w.P = c.take<T>((size_t)nb * prow_pad * d);
    w.pos = c.take<T>(prow_pad * d);
    w.feA = c.take<T>(G * T2 * 19 * d);
    w.feB = c.take<T>(G * T2 * 19 * d);
    // the front-end output Linear's input [nwin * T3, 9d] for every window group: one GEMM over
    // all windows after the group loop (per group it is too small to fill the chip)
    const int T3 = (T2 - 3) / 2 + 1;
    w.feC = c.take<T>((size_t)h[PH_NWIN] * T3 * 9 * d);
    if (uses_vt(h)) {
      w.vt_ld = (h[PH_KVROWS] + 7) / 8 * 8;
      w.vt = c.take<T>((size_t)d * w.vt_ld);
    }
    if (total) *total = c.off;
    return w;
  }

  size_t ws_bytes(const int32_t* hdr) const override {
    size_t t = 0;
    carve(nullptr, hdr, &t);
    return t + 4096;
  }
  size_t ctc_ws_bytes(int rows) const override {
    return align_up((size_t)rows * cfg.vocab * sizeof(float)) + align_up((size_t)rows * cfg.d_model * sizeof(T)) + 4096;
  }
  bool fused_ctc_ok() const { return sizeof(T) == 2 && use_fused_ctc && ctc_argmax_eligible(cfg.vocab, cfg.d_model); }
  size_t ctc_ids_ws_bytes(int rows) const override { return fused_ctc_ok() ? 0 : ctc_ws_bytes(rows); }

  cfm_status encode(const float* feats, const int32_t* plan_dev, const int32_t* hh, const float* aci, const float* cci,
                    int trunc, float* aco, float* cco, float* out, void* ws, size_t wsb,
                    hipStream_t st, int cache_b, int stage_lo, int stage_hi,
                    const float* const* feats_tab) const override {
    const int d = cfg.d_model, ff = cfg.ffn_dim, H = cfg.n_heads, dk = d / H;
    const float eps = cfg.norm_eps;
    const int rows = hh[PH_ROWS], C = hh[PH_C], L = hh[PH_L];
    const int nwin = hh[PH_NWIN], Wn = hh[PH_W], tout = hh[PH_TOUT];
    const int p_rows = hh[PH_PROWS], kv_rows = hh[PH_KVROWS], glu_rows = hh[PH_GLUROWS];
    const int kvoff = hh[PH_KVOFF], gluoff = hh[PH_GLUOFF];
    const bool masked = hh[PH_KIND] == 1;
    const bool stream = hh[PH_KIND] == 3;   // forward_chunk: head-major caches, no row mask
    const size_t att_ls = (size_t)L * 2 * d * (stream ? cache_b : 1);   // cache stride per layer
    const size_t cnn_ls = (size_t)d * 7 * (stream ? cache_b : 1);
    const size_t prow_pad = (p_rows + 127) / 128 * 128;
    if (wsb < ws_bytes(hh)) return set_error(CFM_ERR_VALUE, "workspace too small");
    if (!masked && !stream && (aci || cci))
      return set_error(CFM_ERR_VALUE, "caches are only defined for the masked batch and streaming paths");
    WS w = carve(ws, hh, nullptr);
    const int32_t* meta = plan_dev + plan_meta_off(hh);
    const int32_t* attd = plan_dev + plan_att_off(hh);
    const int32_t* convd = plan_dev + plan_conv_off(hh);
    const uint8_t* rmask = reinterpret_cast<const uint8_t*>(plan_dev + plan_mask_off(hh));
    const int T1 = (Wn - 3) / 2 + 1, T2 = (T1 - 3) / 2 + 1, T3 = (T2 - 3) / 2 + 1;
    if (T3 != tout) return set_error(CFM_ERR_RUNTIME, "plan / front-end geometry mismatch");

    const int nl = (max_layers >= 0 && max_layers < cfg.num_blocks) ? max_layers : cfg.num_blocks;
    const int p_ld = cfg.num_blocks * d;
    const int natt = hh[PH_NATT], nconv = hh[PH_NCONV];
    const int cache_start = std::min(trunc, rows);   // new cache = stream[:trunc + L][-L:] (attention.py:467)
    if (stage_lo < 0) {
    // ---------------- front-end
    const int G = fe_group(hh);
    const int reuse = (fe_carry && masked) ? std::max(0, std::min(fe_reuse, nwin)) : 0;
    for (int g0 = reuse; g0 < nwin; g0 += G) {
      const int ng = std::min(G, nwin - g0);
      PROF(PC_FE_CONV, frontend_conv0_dw<T>(feats, feats_tab, 8 * C, meta + (size_t)g0 * PLAN_REC, PLAN_REC, ng, Wn,
                                fe.cm, fe.ci, fe.w0, fe.b0,
                                fe.w1, fe.b1, fe.wpack, fe.wfrag, d, w.feA, st, tune.fe_conv));
      EpiArgs e1 = E(SITE_FE); e1.bias = fe.b_pw1; e1.out = w.feB; e1.ldo = d;
      T* dw2_rows = w.feA;   // the pw2 GEMM's input
      if constexpr (sizeof(T) == 2) {
        // pw1 + ReLU + dw2 in one weight-stationary kernel (so "gemm_wst" 0 turns it off too): dw2 rows
        // straight into feB (bf16 / f16: the kernel's 16-bit format in ef.f16)
        if (tune.fe_fuse_dw2 && tune.gemm_wst) {
          EpiArgs ef = e1; ef.dw_w = fe.w2; ef.dw_b = fe.b2; ef.t2n = T2; ef.t3n = T3;
          ef.f16 = std::is_same<T, f16>::value;
          int r = -1;
          PROF(PC_FE_GEMM, (r = gemm_bf16_wst(EPI_DW2, ACT_RELU, (const bf16*)w.feA, d, (const bf16*)fe.pw1, d, ng * T2 * 19,
                                              d, d, ef, st),
                            r == -1 ? 0 : r));
          if (r != -1) dw2_rows = w.feB;
        }
      }
      if (dw2_rows == w.feA) {
        PROF(PC_FE_GEMM, gemm<T>(EPI_STORE, ACT_RELU, w.feA, d, (const T*)fe.pw1, d, ng * T2 * 19, d, d, e1, st));
        PROF(PC_FE_DW2, frontend_dw2<T>(w.feB, ng, T2, d, fe.w2, fe.b2, w.feA, st, tune.dw2_seg));
      }
      EpiArgs e2 = E(SITE_FE); e2.bias = fe.b_pw2; e2.out = w.feC + (size_t)g0 * T3 * 9 * d; e2.ldo = d;
      PROF(PC_FE_GEMM, gemm<T>(EPI_STORE, ACT_RELU, dw2_rows, d, (const T*)fe.pw2, d, ng * T3 * 9, d, d, e2, st));
    }
    if (reuse > 0) HIPC(hipMemcpyAsync(w.x, fe_carry, (size_t)reuse * T3 * d * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (reuse < nwin) {
      EpiArgs e3 = E(); e3.bias = fe.b_out; e3.out = w.x; e3.ldo = d; e3.row_off = reuse * T3; e3.alpha = std::sqrt((float)d);
      PROF(PC_FE_GEMM, gemm<T>(EPI_STORE_F32, ACT_NONE, w.feC + (size_t)reuse * T3 * 9 * d, 9 * d, (const T*)fe.wout,
                               9 * d, (nwin - reuse) * T3, d, 9 * d, e3, st));
    }
    if (fe_carry && masked && fe_save_from >= 0 && fe_save_from < nwin)
      HIPC(hipMemcpyAsync(fe_carry, w.x + (size_t)fe_save_from * T3 * d, (size_t)(nwin - fe_save_from) * T3 * d * sizeof(float),
                          hipMemcpyDeviceToDevice, st));
    // ---------------- relative positions: P_l = pos . W_pos_l^T for every layer in ONE GEMM against
    // the stacked weights: P is [p_rows, nb * d], layer l at column l * d (row stride nb * d)
    PROF(PC_POS, pos_table<T>(d, p_rows, hh[PH_PANCHOR], w.pos, st));
    { EpiArgs e = E(); e.out = w.P; e.ldo = p_ld;
      PROF(PC_POS, gemm<T>(EPI_STORE, ACT_NONE, w.pos, d, (const T*)fe.pos_all, d, p_rows, p_ld, d, e, st)); }
    // ---------------- stream padding rows (cache slots and right zero padding)
    if (kvoff > 0) HIPC(hipMemsetAsync(w.kv, 0, (size_t)kvoff * 2 * d * sizeof(T), st));
    if (kv_rows > kvoff + rows)
      HIPC(hipMemsetAsync(w.kv + (size_t)(kvoff + rows) * 2 * d, 0, (size_t)(kv_rows - kvoff - rows) * 2 * d * sizeof(T), st));
    if (gluoff > 0) HIPC(hipMemsetAsync(w.glu, 0, (size_t)gluoff * d * sizeof(T), st));
    if (glu_rows > gluoff + rows)
      HIPC(hipMemsetAsync(w.glu + (size_t)(gluoff + rows) * d, 0, (size_t)(glu_rows - gluoff - rows) * d * sizeof(T), st));

    if (nl == 0) {
      PROF(PC_LN, layernorm2_f32<T>(w.x, ResidAdd<T>(), rows, d, fe.an_w, fe.an_b, nullptr, nullptr, eps, out, st));
      return CFM_OK;
    }
    PROF(PC_LN, layernorm<T>(w.x, ResidAdd<T>(), rows, d, layers[0].ln_ffm_w, layers[0].ln_ffm_b, eps, w.h, nullptr, st));
    }   // stage -1
    // Each residual branch's last GEMM writes y = branch + bias (bf16/T); the residual add
    // x += alpha * y (0.5 for the FFNs, encoder_layer.py:196/246; the conv branch masked by
    // the padded path's row mask) is fused into the LayerNorm that reads x next.
    // Branch outputs alternate between w.y and w.y2, so the LayerNorms after the macaron FFN and
    // after the conv module defer their x write (ResidAdd::defer): the next LayerNorm applies both
    // branches in the same order, x is read and written once per pair (bit-identical x).
    auto resid = [&](const T* y, float alpha, const uint8_t* ym) {
      ResidAdd<T> r; r.y = y; r.alpha = alpha; r.ymask = ym; return r;
    };
    auto resid2 = [&](const T* y, float alpha, const uint8_t* ym, const T* y2, float alpha2, const uint8_t* ym2) {
      ResidAdd<T> r = resid(y, alpha, ym); r.y2 = y2; r.alpha2 = alpha2; r.ymask2 = ym2; return r;
    };
    // y = w2 . SiLU(w1 . h + b1) + b2: two GEMMs through w.hid
    auto ffn = [&](const void* w1, const float* b1, const void* w2, const float* b2, T* yout, int M) -> cfm_status {
      { EpiArgs e = E(SITE_FFN1); e.bias = b1; e.out = w.hid; e.ldo = ff;
        PROF(PC_FFN1, gemm<T>(EPI_STORE, kActSilu<T>, w.h, d, (const T*)w1, d, M, ff, d, e, st)); }
      { EpiArgs e = E(SITE_FFN2); e.bias = b2; e.out = yout; e.ldo = d;
        PROF(PC_FFN2, gemm<T>(EPI_STORE, ACT_NONE, w.hid, ff, (const T*)w2, ff, M, d, ff, e, st)); }
      return CFM_OK;
    };
    // "cache_fuse": the layer's two cache copies in one launch at the layer start (into the KV / GLU stream rows
    // that QKV / pw1 leave alone) and one at the layer end (the KV / GLU rows stay intact after attention / the
    // conv module); 0 = four separate launches next to QKV and pw1
    // (the fused copies ride on the attention cache: a conv cache alone takes the separate launches)
    const bool cfuse_in = cache_fuse && aci, cfuse_out = cache_fuse && aci && aco;
    auto caches_out = [&](int l) -> cfm_status {
      if (cfuse_out)
        PROF(PC_CACHE, cache_io<T>(false, stream, aco + l * att_ls, H, L, dk, w.kv + (size_t)cache_start * 2 * d,
                                   cci && cco ? cco + l * cnn_ls : nullptr, d, 7, w.glu + (size_t)cache_start * d, st));
      return CFM_OK;
    };
    // "trim_right" (endless_decode's segments, whose rows past `trunc` are dropped): layer l computes only the
    // chunks the kept ones depend on.  Kept chunks K = trunc / C; the conv module of a chunk reads 7 rows of
    // the next one (ceil(7 / C) chunks) and attention R keys past a chunk (ceil(R / C)), so layer l's output
    // is needed for n_l = K + (nl - 1 - l)(ceil(7 / C) + ceil(R / C)) chunks: its conv module / pw2 / FFN /
    // norm_final run over n_l, attention / out-proj / pw1 over n_l + ceil(7 / C) and the macaron FFN / LN /
    // QKV over that + ceil(R / C) (= the previous layer's n).  Every row's arithmetic is
    // unchanged (row-wise kernels, per-chunk attention / conv blocks), so the kept rows and the caches are
    // as without it; the rows past them are left unwritten.
    const int n_ch = rows / C, keep_ch = C > 0 ? trunc / C : 0;
    const bool trim = trim_right && masked && aco && trunc > 0 && trunc % C == 0 && trunc < rows &&
                      rows % C == 0 && natt == n_ch && nconv == n_ch && hh[PH_NWIN] == n_ch;
    // chunks of right reach per layer: the conv module's 7 rows, then attention's R keys past those
    const int reach_conv = (7 + C - 1) / C, reach_att = (hh[PH_R] + C - 1) / C;
    for (int l = std::max(0, stage_lo); l < nl && l <= stage_hi; ++l) {
      const LayerW& Lw = layers[l];
      const int n_l = trim ? std::min(n_ch, keep_ch + (reach_conv + reach_att) * (nl - 1 - l)) : n_ch;
      const int cB = trim ? std::min(n_ch, n_l + reach_conv) : n_ch, cA = trim ? std::min(n_ch, cB + reach_att) : n_ch;
      const int rA = trim ? cA * C : rows, rB = trim ? cB * C : rows, rN = trim ? n_l * C : rows;
      const int aB = trim ? cB : natt, vN = trim ? n_l : nconv;   // attention / conv descriptor counts
      if (cfuse_in)
        PROF(PC_CACHE, cache_io<T>(true, stream, const_cast<float*>(aci + l * att_ls), H, L, dk, w.kv,
                                   cci ? const_cast<float*>(cci + l * cnn_ls) : nullptr, d, 7, w.glu, st));
      // macaron FFN (x 0.5)
      { const cfm_status fs = ffn(Lw.ff1m, Lw.b_ff1m, Lw.ff2m, Lw.b_ff2m, w.y, rA); if (fs != CFM_OK) return fs; }
      // MHSA (x + 0.5 y_ffm is not stored: the conv LayerNorm re-applies it)
      { ResidAdd<T> r = resid(w.y, 0.5f, nullptr); r.defer = true;
        PROF(PC_LN, layernorm<T>(w.x, r, rA, d, Lw.ln_mha_w, Lw.ln_mha_b, eps, w.h, nullptr, st)); }
      if (aci && !cfuse_in) {
        if (stream) PROF(PC_CACHE, att_cache_in_hl<T>(aci + l * att_ls, H, L, dk, w.kv, st));
        else PROF(PC_CACHE, att_cache_in<T>(aci + l * att_ls, L, 2 * d, w.kv, st));
      }
      { EpiArgs e = E(SITE_QKV); e.bias = Lw.b_qkv; e.out = w.q; e.out2 = w.kv; e.row_off = kvoff; e.d = d; e.dk = dk;
        PROF(PC_QKV, gemm<T>(EPI_QKV, ACT_NONE, w.h, d, (const T*)Lw.qkv, d, rA, 3 * d, d, e, st)); }
      if (aci && aco && !cfuse_out) {
        if (stream) PROF(PC_CACHE, att_cache_out_hl<T>(w.kv, cache_start, H, L, dk, aco + l * att_ls, st));
        else PROF(PC_CACHE, att_cache_out<T>(w.kv, cache_start, L, 2 * d, aco + l * att_ls, st));
      }
      {
        int r = -1;
        hipEvent_t pb_;
        prof_begin(PC_ATTN, st, &pb_);
        if constexpr (std::is_same<T, bf16>::value) {
          if (masked && use_ring_attention && dk == 64)
            r = chunk_attention_masked_bf16(w.q, w.kv, kv_rows, w.P + (size_t)l * d, p_rows, Lw.pu, Lw.pv,
                                            attd, aB, H, C, hh[PH_L] + C + hh[PH_R], w.ao, st, attn_diag, p_ld,
                                            tune.attn_reuse, tune.attn_min_chunks);
          else if (w.vt) {   // head_dim 128 (4-head d=512): V^T copy, then the band / score / P.V kernel
            KCHK(vt_transpose_bf16(w.kv, kv_rows, H, w.vt, w.vt_ld, st));
            r = chunk_attention_masked_a128(w.q, w.kv, kv_rows, w.vt, w.vt_ld, w.P + (size_t)l * d, p_rows, p_ld,
                                            Lw.pu, Lw.pv, attd, aB, H, C, hh[PH_L] + C + hh[PH_R], w.ao, st,
                                            tune.attn128_var);
          }
          // full attention (padded plan, one chunk of T' per utterance: key window [0, T')) -> dense kernel
          else if (!masked && !stream && hh[PH_L] == 0 && hh[PH_R] == 0 && hh[PH_C] == hh[PH_TOUT] &&
                   use_ring_attention && natt == hh[PH_NWIN] * ((hh[PH_TOUT] + 63) / 64))
            r = full_attention_bf16(w.q, w.kv, kv_rows, w.P + (size_t)l * d, p_rows, Lw.pu, Lw.pv, attd, hh[PH_NWIN],
                                    (hh[PH_TOUT] + 63) / 64, H, dk, hh[PH_TOUT], w.ao, st, p_ld);
        }
        if constexpr (std::is_same<T, f16>::value) {
          if (masked && use_ring_attention && dk == 64)
            r = chunk_attention_masked_f16(w.q, w.kv, kv_rows, w.P + (size_t)l * d, p_rows, Lw.pu, Lw.pv, attd, aB, H, C,
                                           hh[PH_L] + C + hh[PH_R], w.ao, st, attn_diag, p_ld, tune.attn_reuse,
                                           tune.attn_min_chunks);
        }
        if (r == -1)
          r = chunk_attention<T>(w.q, w.kv, kv_rows, w.P + (size_t)l * d, p_rows, Lw.pu, Lw.pv, attd, aB,
                                 H, dk, w.ao, st, p_ld);
        KCHK(r);
        prof_end(PC_ATTN, st, pb_);
      }
      { EpiArgs e = E(SITE_OPROJ); e.bias = Lw.b_o; e.out = w.y2; e.ldo = d;
        PROF(PC_OPROJ, gemm<T>(EPI_STORE, ACT_NONE, w.ao, d, (const T*)Lw.wo, d, rB, d, d, e, st)); }
      // convolution module: x += 0.5 y_ffm + y_attn, stored
      PROF(PC_LN, layernorm<T>(w.x, resid2(w.y, 0.5f, nullptr, w.y2, 1.f, nullptr), rB, d, Lw.ln_conv_w, Lw.ln_conv_b,
                               eps, w.h, (masked || stream) ? nullptr : rmask, st));
      if (cci && !cfuse_in) PROF(PC_CACHE, cnn_cache_in<T>(cci + l * cnn_ls, d, 7, w.glu, st));
      { EpiArgs e = E(SITE_PW1); e.bias = Lw.b_pw1; e.out = w.glu; e.ldo = d; e.row_off = gluoff;
        PROF(PC_PW1, gemm<T>(EPI_GLU, kSiluPre<T> ? ACT_SILU_L2E : ACT_NONE, w.h, d, (const T*)Lw.pw1, d, rB, 2 * d, d, e, st)); }
      if (cci && cco && !cfuse_out) PROF(PC_CACHE, cnn_cache_out<T>(w.glu, cache_start, d, 7, cco + l * cnn_ls, st));
      PROF(PC_CONV, conv_dw_ln_silu<T>(w.glu, convd, vN, d, Lw.dw_t, Lw.b_dw, Lw.cn_w, Lw.cn_b, eps, w.cv, st,
                                        tune.conv_dot2, tune.conv_dma));
      { EpiArgs e = E(SITE_PW2); e.bias = Lw.b_pw2; e.out = w.y; e.ldo = d;
        PROF(PC_PW2, gemm<T>(EPI_STORE, ACT_NONE, w.cv, d, (const T*)Lw.pw2, d, rN, d, d, e, st)); }
      // FFN (x 0.5); x + y_conv is not stored: norm_final re-applies it
      { ResidAdd<T> r = resid(w.y, 1.f, rmask); r.defer = true;
        PROF(PC_LN, layernorm<T>(w.x, r, rN, d, Lw.ln_ff_w, Lw.ln_ff_b, eps, w.h, nullptr, st)); }
      { const cfm_status fs = ffn(Lw.ff1, Lw.b_ff1, Lw.ff2, Lw.b_ff2, w.y2, rN); if (fs != CFM_OK) return fs; }
      // norm_final over x + y_conv + 0.5 y_ffn (+ next layer's macaron LN, or after_norm)
      const ResidAdd<T> rf = resid2(w.y, 1.f, rmask, w.y2, 0.5f, nullptr);
      if (l + 1 < nl)
        PROF(PC_LN, layernorm2<T>(w.x, rf, rN, d, Lw.ln_fin_w, Lw.ln_fin_b, layers[l + 1].ln_ffm_w,
                                  layers[l + 1].ln_ffm_b, eps, w.h, st));
      else
        PROF(PC_LN, layernorm2_f32<T>(w.x, rf, rN, d, Lw.ln_fin_w, Lw.ln_fin_b, fe.an_w, fe.an_b, eps, out, st));
      { const cfm_status cs = caches_out(l); if (cs != CFM_OK) return cs; }
    }
    return CFM_OK;
  }

  cfm_status ctc(const float* enc, int rows, float* logp, int32_t* ids, void* ws, size_t wsb,
                 hipStream_t st) const override {
    if (!fe.ctc_w) return set_error(CFM_ERR_ASSERT, "model has no CTC head (vocab == 0)");
    const int d = cfg.d_model, V = cfg.vocab;
    if constexpr (sizeof(T) == 2) {
      // ids only: the fused argmax head (ctc.hip) keeps every logit in registers
      if (!logp && ids && fused_ctc_ok()) {
        int r;
        if constexpr (std::is_same<T, bf16>::value)
          PROF(PC_CTC, (r = ctc_argmax_bf16(enc, rows, (const bf16*)fe.ctc_w, fe.ctc_b, V, d, ids, st)) < 0 ? 0 : r);
        else
          PROF(PC_CTC, (r = ctc_argmax_f16(enc, rows, (const f16*)fe.ctc_w, fe.ctc_b, V, d, ids, st)) < 0 ? 0 : r);
        if (r == 0) return CFM_OK;
      }
    }
    if (wsb < ctc_ws_bytes(rows)) return set_error(CFM_ERR_VALUE, "ctc workspace too small");
    Carver c(ws);
    float* logits = c.take<float>((size_t)rows * V);
    T* a = c.take<T>((size_t)rows * d);
    const T* A;
    if constexpr (sizeof(T) == 4) {
      A = reinterpret_cast<const T*>(enc);
    } else {
      KCHK(att_cache_in<T>(enc, rows, d, a, st));   // f32 -> T row copy
      A = a;
    }
    float* dst = logp ? logp : logits;
    // the vocabulary splits into a 256-multiple part (256 x 256 MFMA tiles) and a remainder (128 x 128
    // tiles); f32x4 epilogue stores need the row pitch V % 4 == 0
    const int V1 = (sizeof(T) == 2 && V % 4 == 0) ? V / 256 * 256 : 0;
    if (V1 > 0) {
      EpiArgs e = E(); e.bias = fe.ctc_b; e.out = dst; e.ldo = V;
      PROF(PC_CTC, gemm<T>(EPI_STORE_F32, ACT_NONE, A, d, (const T*)fe.ctc_w, d, rows, V1, d, e, st));
    }
    if (V1 < V) {
      EpiArgs e = E(); e.bias = fe.ctc_b + V1; e.out = dst + V1; e.ldo = V;
      PROF(PC_CTC, gemm<T>(EPI_STORE_F32, ACT_NONE, A, d, (const T*)fe.ctc_w + (size_t)V1 * d, d, rows, V - V1, d, e, st));
    }
    PROF(PC_CTC, log_softmax_rows(dst, rows, V, logp ? 1 : 0, ids, st));
    return CFM_OK;
  }
};

// ----------------------------------------------------------------------------- weight packing
struct HostW {
  std::map<std::string, std::pair<const float*, int64_t>> m;
  const float* get(const std::string& k, int64_t numel) const {
    auto it = m.find(k);
    if (it == m.end()) throw std::string("missing weight " + k);
    if (it->second.second != numel)
      throw std::string("weight " + k + ": numel " + std::to_string(it->second.second) + " != " + std::to_string(numel));
    return it->second.first;
  }
  bool has(const std::string& k) const { return m.count(k) > 0; }
};

static uint16_t bf16_bits_rne(float f) {   // round-to-nearest-even f32 -> bf16 bits (host)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <typename T>
static cfm_status build_model(const cfm_config& cfg, const HostW& hw, int device, cfm_model** out) {
  auto* M = new ModelT<T>();
  std::unique_ptr<cfm_model> guard(M);
  M->cfg = cfg;
  M->device = device;
  const int d = cfg.d_model, ff = cfg.ffn_dim, H = cfg.n_heads, nb = cfg.num_blocks, V = cfg.vocab;
  // host staging image of the whole device block
  struct Item { size_t off; size_t bytes; };
  std::vector<char> img;
  auto reserve = [&](size_t bytes) {
    size_t off = align_up(img.size());
    img.resize(off + align_up(bytes));
    return off;
  };
  std::vector<std::pair<size_t, void**>> fix;   // (offset, pointer slot) patched after allocation
  auto put_f32 = [&](const float* src, size_t n, float** slot) {
    size_t off = reserve(n * 4);
    std::memcpy(img.data() + off, src, n * 4);
    fix.push_back({off, (void**)slot});
  };
  auto put_T = [&](const std::vector<float>& src, void** slot) {
    size_t off = reserve(src.size() * sizeof(T));
    T* p = reinterpret_cast<T*>(img.data() + off);
    for (size_t i = 0; i < src.size(); ++i) {
      if constexpr (sizeof(T) == 4) p[i] = src[i];
      else if constexpr (std::is_same<T, f16>::value) p[i] = (f16)src[i];   // round-to-nearest-even (host)
      else {   // round-to-nearest-even f32 -> bf16 (host)
        uint32_t u;
        std::memcpy(&u, &src[i], 4);
        uint16_t r;
        if ((u & 0x7f800000u) == 0x7f800000u) r = (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
        else r = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
        std::memcpy(&p[i], &r, 2);
      }
    }
    fix.push_back({off, slot});
  };
  auto vec = [&](const std::string& k, int64_t n) { const float* s = hw.get(k, n); return std::vector<float>(s, s + n); };
  try {
    const std::string E = "encoder.";
    FrontW& F = M->fe;
    if (cfg.has_cmvn) {
      put_f32(hw.get(E + "global_cmvn.mean", cfg.input_dim), cfg.input_dim, &F.cm);
      put_f32(hw.get(E + "global_cmvn.istd", cfg.input_dim), cfg.input_dim, &F.ci);
    }
    put_f32(hw.get(E + "embed.conv.0.weight", (int64_t)d * 9), (size_t)d * 9, &F.w0);
    put_f32(hw.get(E + "embed.conv.0.bias", d), d, &F.b0);
    put_f32(hw.get(E + "embed.conv.2.weight", (int64_t)d * 9), (size_t)d * 9, &F.w1);
    put_f32(hw.get(E + "embed.conv.2.bias", d), d, &F.b1);
    {   // conv0 + dw1 weights packed per channel for the MFMA front-end
      const float *a = hw.get(E + "embed.conv.0.weight", (int64_t)d * 9), *ab = hw.get(E + "embed.conv.0.bias", d);
      const float *b = hw.get(E + "embed.conv.2.weight", (int64_t)d * 9), *bb = hw.get(E + "embed.conv.2.bias", d);
      std::vector<float> w((size_t)d * FE_WPACK, 0.f);
      for (int c = 0; c < d; ++c) {
        for (int e = 0; e < 9; ++e) {
          w[(size_t)c * FE_WPACK + e] = a[c * 9 + e];
          w[(size_t)c * FE_WPACK + 9 + e] = b[c * 9 + e];
        }
        w[(size_t)c * FE_WPACK + 18] = ab[c];
        w[(size_t)c * FE_WPACK + 19] = bb[c];
      }
      put_f32(w.data(), w.size(), &F.wpack);
      // the channel-stationary kernel's per-lane MFMA fragments ("fe_conv" >= 2), [tile][FE2_NFRAG][64 lanes]
      // x 16 B: W0 rows + b0 (bf16), the diagonal dw1 fragments of the 9 taps x 2 k-steps (bf16), the b1
      // seed in accumulator order (f32).  W0 and b0 are scaled by 2^-24 and w1 by 2^24 (exact), so conv0's
      // accumulator carries 2^-24 x its value: the ReLU can then be a clamp to [0, 1] (frontend.hip FE2_CLAMP)
      if (d % 32 == 0) {
        std::vector<uint32_t> fr((size_t)(d / 32) * FE2_NFRAG * 64 * 4, 0u);
        // fp16 model: f16 fragments, unscaled (f16 has no exponent range for 2^-24; its kernel takes the
        // ReLU as a packed max instead of the clamp)
        constexpr bool H16 = std::is_same<T, f16>::value;
        auto bf = [](float x) -> uint32_t {
          if constexpr (H16) {
            const f16 h = (f16)x;
            uint16_t u;
            std::memcpy(&u, &h, 2);
            return u;
          } else {
            return (uint32_t)bf16_bits_rne(x);
          }
        };
        const int sc0 = H16 ? 0 : -24, sc1 = H16 ? 0 : 24;
        for (int ct = 0; ct < d / 32; ++ct)
          for (int lane = 0; lane < 64; ++lane) {
            const int h = lane >> 5, n = lane & 31, c = ct * 32 + n;
            auto slot = [&](int q) { return &fr[(((size_t)ct * FE2_NFRAG + q) * 64 + lane) * 4]; };
            uint16_t a0[8];
            for (int j = 0; j < 8; ++j) {
              const int k = 8 * h + j;
              a0[j] = (uint16_t)bf(std::ldexp(k < 9 ? a[c * 9 + k] : k == 9 ? ab[c] : 0.f, sc0));
            }
            std::memcpy(slot(0), a0, 16);
            const bool own = h == ((n >> 2) & 1);
            const int town = n >> 4, j0 = (n & 3) + 4 * ((n >> 3) & 1);
            for (int sp = 0; sp < 9; ++sp)
              for (int t = 0; t < 2; ++t) {
                uint16_t a1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                if (own && t == town) a1[j0] = (uint16_t)bf(std::ldexp(b[c * 9 + sp], sc1));
                std::memcpy(slot(1 + 2 * sp + t), a1, 16);
              }
            for (int r = 0; r < 16; ++r) {
              const float v = bb[ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * h];
              std::memcpy(slot(19 + r / 4) + (r & 3), &v, 4);
            }
          }
        put_f32(reinterpret_cast<const float*>(fr.data()), fr.size(), &F.wfrag);
      }
    }
    put_T(vec(E + "embed.conv.3.weight", (int64_t)d * d), &F.pw1);
    put_f32(hw.get(E + "embed.conv.3.bias", d), d, &F.b_pw1);
    {   // dw2 taps tap-major [9][d] (16-B channel vectors per tap for fe_dw2_kernel)
      const float* s = hw.get(E + "embed.conv.5.weight", (int64_t)d * 9);
      std::vector<float> w((size_t)d * 9);
      for (int c = 0; c < d; ++c)
        for (int e = 0; e < 9; ++e) w[(size_t)e * d + c] = s[(size_t)c * 9 + e];
      put_f32(w.data(), w.size(), &F.w2);
    }
    put_f32(hw.get(E + "embed.conv.5.bias", d), d, &F.b2);
    put_T(vec(E + "embed.conv.6.weight", (int64_t)d * d), &F.pw2);
    put_f32(hw.get(E + "embed.conv.6.bias", d), d, &F.b_pw2);
    {   // out Linear columns (c*9 + f) -> channels-last (f*d + c)
      const float* s = hw.get(E + "embed.out.weight", (int64_t)d * 9 * d);
      std::vector<float> w((size_t)d * 9 * d);
      for (int o = 0; o < d; ++o)
        for (int c = 0; c < d; ++c)
          for (int f = 0; f < 9; ++f) w[(size_t)o * 9 * d + f * d + c] = s[(size_t)o * 9 * d + c * 9 + f];
      put_T(w, &F.wout);
    }
    put_f32(hw.get(E + "embed.out.bias", d), d, &F.b_out);
    put_f32(hw.get(E + "after_norm.weight", d), d, &F.an_w);
    put_f32(hw.get(E + "after_norm.bias", d), d, &F.an_b);
    if (V > 0) {
      // rows padded with zeros to a multiple of 64 (the fused argmax head streams 64-row tiles)
      std::vector<float> w = vec("ctc.ctc_lo.weight", (int64_t)V * d);
      w.resize((size_t)(V + 63) / 64 * 64 * d, 0.f);
      put_T(w, &F.ctc_w);
      put_f32(hw.get("ctc.ctc_lo.bias", V), V, &F.ctc_b);
    }
    M->layers.resize(nb);
    for (int l = 0; l < nb; ++l) {
      LayerW& Lw = M->layers[l];
      const std::string p = E + "encoders." + std::to_string(l) + ".";
      // 16-bit modes (ACT_SILU_L2E): w_1 and its bias x -log2(e), w_2 x -1/log2(e), so the SiLU epilogue
      // skips its input multiply; the product w_2 . silu(w_1 h + b_1) is unchanged
      auto scaled = [](std::vector<float> v, float f) { for (float& x : v) x *= f; return v; };
      const float s1 = kSiluPre<T> ? -kLog2e : 1.f, s2 = kSiluPre<T> ? -1.f / kLog2e : 1.f;
      put_T(scaled(vec(p + "feed_forward_macaron.w_1.weight", (int64_t)ff * d), s1), &Lw.ff1m);
      { const auto b = scaled(vec(p + "feed_forward_macaron.w_1.bias", ff), s1); put_f32(b.data(), b.size(), &Lw.b_ff1m); }
      put_T(scaled(vec(p + "feed_forward_macaron.w_2.weight", (int64_t)d * ff), s2), &Lw.ff2m);
      put_f32(hw.get(p + "feed_forward_macaron.w_2.bias", d), d, &Lw.b_ff2m);
      put_T(scaled(vec(p + "feed_forward.w_1.weight", (int64_t)ff * d), s1), &Lw.ff1);
      { const auto b = scaled(vec(p + "feed_forward.w_1.bias", ff), s1); put_f32(b.data(), b.size(), &Lw.b_ff1); }
      put_T(scaled(vec(p + "feed_forward.w_2.weight", (int64_t)d * ff), s2), &Lw.ff2);
      put_f32(hw.get(p + "feed_forward.w_2.bias", d), d, &Lw.b_ff2);
      {
        std::vector<float> w, b;
        for (const char* nm : {"linear_q", "linear_k", "linear_v"}) {
          auto wv = vec(p + "self_attn." + nm + ".weight", (int64_t)d * d);
          auto bv = vec(p + "self_attn." + nm + ".bias", d);
          w.insert(w.end(), wv.begin(), wv.end());
          b.insert(b.end(), bv.begin(), bv.end());
        }
        put_T(w, &Lw.qkv);
        put_f32(b.data(), b.size(), &Lw.b_qkv);
      }
      put_T(vec(p + "self_attn.linear_pos.weight", (int64_t)d * d), &Lw.pos);
      put_T(vec(p + "self_attn.linear_out.weight", (int64_t)d * d), &Lw.wo);
      put_f32(hw.get(p + "self_attn.linear_out.bias", d), d, &Lw.b_o);
      put_f32(hw.get(p + "self_attn.pos_bias_u", (int64_t)d), (size_t)d, &Lw.pu);   // [H, dk]
      put_f32(hw.get(p + "self_attn.pos_bias_v", (int64_t)d), (size_t)d, &Lw.pv);
      {   // pointwise_conv1 rows interleaved per 16: [a(16t..16t+15) | gate(d+16t..)] for the fused GLU
        const float* s = hw.get(p + "conv_module.pointwise_conv1.weight", (int64_t)2 * d * d);
        const float* sb = hw.get(p + "conv_module.pointwise_conv1.bias", 2 * d);
        std::vector<float> w((size_t)2 * d * d), b(2 * d);
        // 16-bit modes: the gate rows and bias x -log2(e) (EPI_GLU with ACT_SILU_L2E)
        const float sg = kSiluPre<T> ? -kLog2e : 1.f;
        for (int t = 0; t < d / 16; ++t)
          for (int r = 0; r < 16; ++r) {
            const int ra = 16 * t + r, rg = d + 16 * t + r;
            std::memcpy(&w[(size_t)(32 * t + r) * d], s + (size_t)ra * d, 4 * d);
            for (int k = 0; k < d; ++k) w[(size_t)(32 * t + 16 + r) * d + k] = sg * s[(size_t)rg * d + k];
            b[32 * t + r] = sb[ra];
            b[32 * t + 16 + r] = sg * sb[rg];
          }
        put_T(w, &Lw.pw1);
        put_f32(b.data(), b.size(), &Lw.b_pw1);
      }
      {   // depthwise [d][1][15] -> tap-major [15][d]
        const float* s = hw.get(p + "conv_module.depthwise_conv.weight", (int64_t)d * 15);
        std::vector<float> w((size_t)15 * d);
        for (int c = 0; c < d; ++c)
          for (int t = 0; t < 15; ++t) w[(size_t)t * d + c] = s[c * 15 + t];
        put_f32(w.data(), w.size(), &Lw.dw_t);
      }
      put_f32(hw.get(p + "conv_module.depthwise_conv.bias", d), d, &Lw.b_dw);
      put_f32(hw.get(p + "conv_module.norm.weight", d), d, &Lw.cn_w);
      put_f32(hw.get(p + "conv_module.norm.bias", d), d, &Lw.cn_b);
      put_T(vec(p + "conv_module.pointwise_conv2.weight", (int64_t)d * d), &Lw.pw2);
      put_f32(hw.get(p + "conv_module.pointwise_conv2.bias", d), d, &Lw.b_pw2);
      const std::pair<const char*, float**> lns[] = {
          {"norm_ff_macaron.weight", &Lw.ln_ffm_w}, {"norm_ff_macaron.bias", &Lw.ln_ffm_b},
          {"norm_mha.weight", &Lw.ln_mha_w},        {"norm_mha.bias", &Lw.ln_mha_b},
          {"norm_conv.weight", &Lw.ln_conv_w},      {"norm_conv.bias", &Lw.ln_conv_b},
          {"norm_ff.weight", &Lw.ln_ff_w},          {"norm_ff.bias", &Lw.ln_ff_b},
          {"norm_final.weight", &Lw.ln_fin_w},      {"norm_final.bias", &Lw.ln_fin_b}};
      for (auto& kv : lns) put_f32(hw.get(p + kv.first, d), d, kv.second);
    }
    {   // every layer's linear_pos weight stacked [nb * d, d] (ModelT::encode: one P GEMM per call)
      std::vector<float> all((size_t)nb * d * d);
      for (int l = 0; l < nb; ++l) {
        const std::string p = E + "encoders." + std::to_string(l) + ".";
        std::memcpy(all.data() + (size_t)l * d * d, hw.get(p + "self_attn.linear_pos.weight", (int64_t)d * d),
                    (size_t)d * d * sizeof(float));
      }
      put_T(all, &F.pos_all);
    }
  } catch (const std::string& e) {
    return set_error(CFM_ERR_VALUE, e);
  }
  // the channel-stationary front-end (fe_conv >= 2) applies conv0's ReLU as the bf16 conversion's clamp on
  // values scaled by 2^-24: exact while |conv0| < 2^24, which CMVN-normalised features keep by orders of
  // magnitude; without CMVN the raw features are not bounded by construction, so such a model keeps the
  // position-stationary kernel (fe_conv 1: an f32 max, no saturation).  Neither propagates a NaN input.
  if (!cfg.has_cmvn) M->tune.fe_conv = 1;
  HIPC(hipSetDevice(device));
  HIPC(hipMalloc(&M->dev_mem, img.size()));
  HIPC(hipMemcpy(M->dev_mem, img.data(), img.size(), hipMemcpyHostToDevice));
  for (auto& f : fix) *f.second = (char*)M->dev_mem + f.first;
  *out = guard.release();
  return CFM_OK;
}

}  // namespace cfm

using namespace cfm;

extern "C" {

const char* cfm_version(void) { return "chunkformer_amd 0.1 (gfx950)"; }
const char* cfm_last_error(void) { return g_err.c_str(); }

cfm_status cfm_model_create(const cfm_config* cfg, const cfm_tensor_view* weights, int32_t n, int32_t device,
                            cfm_model** out) {
  if (!cfg || !out) return set_error(CFM_ERR_VALUE, "null argument");
  *out = nullptr;
  if (cfg->input_dim != 80) return set_error(CFM_ERR_ASSERT, "front-end kernel supports input_dim == 80");
  if (cfg->d_model != 128 && cfg->d_model != 256 && cfg->d_model != 512)
    return set_error(CFM_ERR_ASSERT, "d_model must be 128, 256 or 512");
  if (cfg->n_heads <= 0 || (cfg->d_model != 64 * cfg->n_heads && cfg->d_model != 128 * cfg->n_heads))
    return set_error(CFM_ERR_ASSERT, "head_dim (d_model / attention_heads) must be 64 or 128");
  if (cfg->ffn_dim % 128) return set_error(CFM_ERR_ASSERT, "ffn_dim must be a multiple of 128");
  if (cfg->kernel_size != 15) return set_error(CFM_ERR_ASSERT, "cnn_module_kernel must be 15");
  if (cfg->num_blocks <= 0 || cfg->vocab < 0) return set_error(CFM_ERR_VALUE, "bad num_blocks / vocab");
  HostW hw;
  for (int i = 0; i < n; ++i) hw.m[weights[i].name] = {weights[i].data, weights[i].numel};
  if (cfg->compute_dtype == CFM_DTYPE_F32) return build_model<float>(*cfg, hw, device, out);
  if (cfg->compute_dtype == CFM_DTYPE_BF16) return build_model<bf16>(*cfg, hw, device, out);
  if (cfg->compute_dtype == CFM_DTYPE_F16) return build_model<f16>(*cfg, hw, device, out);
  return set_error(CFM_ERR_VALUE, "unknown compute dtype");
}

void cfm_model_destroy(cfm_model* m) { delete m; }

cfm_status cfm_model_set_option(cfm_model* m, const char* key, int64_t value) {
  if (!m || !key) return set_error(CFM_ERR_VALUE, "null argument");
  if (!std::strcmp(key, "max_layers")) { m->max_layers = (int)value; return CFM_OK; }
  if (!std::strcmp(key, "fe_group_windows")) { m->fe_group_windows = (int)std::max<int64_t>(0, value); return CFM_OK; }
  if (!std::strcmp(key, "profile")) { m->prof_mask = (uint32_t)value; return CFM_OK; }
  if (!std::strcmp(key, "ring_attention")) { m->use_ring_attention = value != 0; return CFM_OK; }
  if (!std::strcmp(key, "ctc_fused")) { m->use_fused_ctc = value != 0; return CFM_OK; }
  {   // per-model kernel tuning / diagnostics; defaults are the measured best
    const std::pair<const char*, int*> knobs[] = {
        {"gemm_diag", &m->tune.gemm_diag}, {"gemm_wst", &m->tune.gemm_wst},   {"store_mode", &m->tune.store_mode},
        {"col_group", &m->tune.col_group}, {"attn_reuse", &m->tune.attn_reuse}, {"conv_dot2", &m->tune.conv_dot2},
        {"conv_dma", &m->tune.conv_dma},   {"dw2_seg", &m->tune.dw2_seg},   {"nt_sites", &m->tune.nt_sites},
        {"fe_fuse_dw2", &m->tune.fe_fuse_dw2}, {"fe_conv", &m->tune.fe_conv},
        {"attn128_var", &m->tune.attn128_var},
        {"gemm_big_min", &m->tune.big_min_tiles}, {"wsp_small_div", &m->tune.wsp_small_div},
        {"wsp_small_rows", &m->tune.wsp_small_rows},
        {"attn_min_chunks", &m->tune.attn_min_chunks}};
    for (auto& k : knobs)
      if (!std::strcmp(key, k.first)) { *k.second = (int)value; return CFM_OK; }
  }
  if (!std::strcmp(key, "attn_diag")) { m->attn_diag = (int)value; return CFM_OK; }
  if (!std::strcmp(key, "cache_fuse")) { m->cache_fuse = (int)(value != 0); return CFM_OK; }
  if (!std::strcmp(key, "trim_right")) { m->trim_right = (int)(value != 0); return CFM_OK; }
  if (!std::strcmp(key, "fe_carry")) { m->fe_carry = reinterpret_cast<float*>((intptr_t)value); return CFM_OK; }
  if (!std::strcmp(key, "fe_reuse")) { m->fe_reuse = (int)std::max<int64_t>(0, value); return CFM_OK; }
  if (!std::strcmp(key, "fe_save_from")) { m->fe_save_from = (int)value; return CFM_OK; }
  if (!std::strcmp(key, "profile_reset")) {
    m->prof_collect();
    for (int i = 0; i < PC_N; ++i) { m->prof_ms[i] = 0; m->prof_n[i] = 0; }
    return CFM_OK;
  }
  return set_error(CFM_ERR_VALUE, std::string("unknown option ") + key);
}

size_t cfm_workspace_bytes_masked(const cfm_model* m, int32_t N, int32_t C, int32_t L, int32_t R) {
  if (!m || N <= 0 || C <= 0) return 0;
  int32_t h[PH_HEADER] = {0};
  const int rows = N * C;
  h[PH_KIND] = 1; h[PH_NWIN] = N; h[PH_ROWS] = rows; h[PH_C] = C; h[PH_L] = L; h[PH_R] = R;
  h[PH_W] = (C - 1) * 8 + 15; h[PH_TOUT] = C; h[PH_PROWS] = L + 2 * C + R - 1;
  h[PH_KVROWS] = L + rows + R; h[PH_GLUROWS] = rows + 14;
  return m->ws_bytes(h);
}

size_t cfm_workspace_bytes_padded(const cfm_model* m, int32_t B, int32_t T, int32_t C, int32_t L, int32_t R) {
  if (!m || B <= 0) return 0;
  const int Tp = calc_length(T);
  if (Tp <= 0) return 0;
  if (C <= 0) { C = Tp; L = 0; R = 0; }
  int32_t h[PH_HEADER] = {0};
  const int rows = B * Tp;
  h[PH_KIND] = 2; h[PH_NWIN] = B; h[PH_ROWS] = rows; h[PH_C] = C; h[PH_L] = L; h[PH_R] = R;
  h[PH_W] = T; h[PH_TOUT] = Tp; h[PH_PROWS] = L + 2 * C + R - 1; h[PH_KVROWS] = rows; h[PH_GLUROWS] = rows;
  return m->ws_bytes(h);
}

cfm_status cfm_encode_masked(const cfm_model* m, const float* feats, const int32_t* h, const int32_t* plan_dev,
                             const float* aci, const float* cci, int32_t trunc, float* aco, float* cco, float* out,
                             void* ws, size_t wsb, cfm_stream stream) {
  if (!m || !feats || !h || !plan_dev || !out) return set_error(CFM_ERR_VALUE, "null argument");
  if (h[PH_KIND] != 1) return set_error(CFM_ERR_VALUE, "not a masked-batch plan");
  if ((aci == nullptr) != (cci == nullptr)) return set_error(CFM_ERR_VALUE, "att_cache and cnn_cache must be given together");
  HIPC(hipSetDevice(m->device));
  return m->encode(feats, plan_dev, h, aci, cci, trunc, aco, cco, out, ws, wsb, (hipStream_t)stream);
}

cfm_status cfm_encode_masked_utts(const cfm_model* m, const float* const* utt_feats, const int32_t* h,
                                  const int32_t* plan_dev, const float* aci, const float* cci, int32_t trunc, float* aco,
                                  float* cco, float* out, void* ws, size_t wsb, cfm_stream stream) {
  if (!m || !utt_feats || !h || !plan_dev || !out) return set_error(CFM_ERR_VALUE, "null argument");
  if (h[PH_KIND] != 1) return set_error(CFM_ERR_VALUE, "not a masked-batch plan");
  if ((aci == nullptr) != (cci == nullptr)) return set_error(CFM_ERR_VALUE, "att_cache and cnn_cache must be given together");
  HIPC(hipSetDevice(m->device));
  return m->encode(nullptr, plan_dev, h, aci, cci, trunc, aco, cco, out, ws, wsb, (hipStream_t)stream, 1, -1, 1 << 30,
                   utt_feats);
}

cfm_status cfm_encode_masked_stages(const cfm_model* m, const float* feats, const int32_t* h, const int32_t* plan_dev,
                                    const float* aci, const float* cci, int32_t trunc, float* aco, float* cco, float* out,
                                    void* ws, size_t wsb, int32_t stage_lo, int32_t stage_hi, cfm_stream stream) {
  if (!m || !feats || !h || !plan_dev || !out) return set_error(CFM_ERR_VALUE, "null argument");
  if (h[PH_KIND] != 1) return set_error(CFM_ERR_VALUE, "not a masked-batch plan");
  if ((aci == nullptr) != (cci == nullptr)) return set_error(CFM_ERR_VALUE, "att_cache and cnn_cache must be given together");
  if (stage_lo < -1 || stage_hi < stage_lo) return set_error(CFM_ERR_VALUE, "bad stage range");
  HIPC(hipSetDevice(m->device));
  return m->encode(feats, plan_dev, h, aci, cci, trunc, aco, cco, out, ws, wsb, (hipStream_t)stream, 1, stage_lo,
                   stage_hi);
}

cfm_status cfm_encode_padded(const cfm_model* m, const float* xs, const int32_t* h, const int32_t* plan_dev, float* out,
                             void* ws, size_t wsb, cfm_stream stream) {
  if (!m || !xs || !h || !plan_dev || !out) return set_error(CFM_ERR_VALUE, "null argument");
  if (h[PH_KIND] != 2) return set_error(CFM_ERR_VALUE, "not a padded-batch plan");
  HIPC(hipSetDevice(m->device));
  return m->encode(xs, plan_dev, h, nullptr, nullptr, 0, nullptr, nullptr, out, ws, wsb, (hipStream_t)stream);
}

size_t cfm_workspace_bytes_stream(const cfm_model* m, int32_t T, int32_t C, int32_t L, int32_t R) {
  if (!m || C <= 0) return 0;
  const int Tp = calc_length(T);
  if (Tp <= 0) return 0;
  int32_t h[PH_HEADER] = {0};
  h[PH_KIND] = 3; h[PH_NWIN] = 1; h[PH_ROWS] = Tp; h[PH_C] = C; h[PH_L] = L; h[PH_R] = R;
  h[PH_W] = T; h[PH_TOUT] = Tp; h[PH_PROWS] = L + 2 * (C + R) - 1; h[PH_KVROWS] = L + Tp; h[PH_GLUROWS] = 7 + Tp;
  return m->ws_bytes(h);
}

cfm_status cfm_encode_stream(const cfm_model* m, const float* xs, int32_t B, const int32_t* h, const int32_t* plan_dev,
                             const float* aci, const float* cci, float* aco, float* cco, float* out, void* ws,
                             size_t wsb, cfm_stream stream) {
  if (!m || !xs || !h || !plan_dev || !out) return set_error(CFM_ERR_VALUE, "null argument");
  if (h[PH_KIND] != 3) return set_error(CFM_ERR_VALUE, "not a streaming-chunk plan");
  if (B <= 0) return set_error(CFM_ERR_VALUE, "batch must be >= 1");
  if (!aci || !cci) return set_error(CFM_ERR_ASSERT, "forward_chunk needs att_cache [nb, B, H, L, 2dk] and cnn_cache [nb, B, d, 7]");
  if ((aco == nullptr) != (cco == nullptr)) return set_error(CFM_ERR_VALUE, "att_cache_out and cnn_cache_out go together");
  HIPC(hipSetDevice(m->device));
  const int T = h[PH_W], Tp = h[PH_TOUT], L = h[PH_L], R = h[PH_R], d = m->cfg.d_model;
  const size_t att_b = (size_t)L * 2 * d, cnn_b = (size_t)d * 7;
  for (int b = 0; b < B; ++b) {
    const cfm_status r = m->encode(xs + (size_t)b * T * m->cfg.input_dim, plan_dev, h, aci + b * att_b, cci + b * cnn_b,
                                   Tp - R, aco ? aco + b * att_b : nullptr, cco ? cco + b * cnn_b : nullptr,
                                   out + (size_t)b * Tp * d, ws, wsb, (hipStream_t)stream, B);
    if (r != CFM_OK) return r;
  }
  return CFM_OK;
}

cfm_status cfm_masks_from_plan(const int32_t* h, const int32_t* plan_dev, uint8_t* att, uint8_t* pad,
                               cfm_stream stream) {
  if (!h || !plan_dev || !att || !pad) return set_error(CFM_ERR_VALUE, "null argument");
  if (h[PH_KIND] != 1) return set_error(CFM_ERR_VALUE, "not a masked-batch plan");
  KCHK(masks_from_plan(plan_dev + PH_HEADER, h[PH_NWIN], h[PH_C], h[PH_L], h[PH_R], att, pad, (hipStream_t)stream));
  return CFM_OK;
}

int32_t cfm_profile_read(const cfm_model* m, const char** names, double* total_ms, int64_t* launches, int32_t cap) {
  if (!m) return 0;
  m->prof_collect();
  const int n = std::min<int>(cap, PC_N);
  for (int i = 0; i < n; ++i) {
    if (names) names[i] = PC_NAMES[i];
    if (total_ms) total_ms[i] = m->prof_ms[i];
    if (launches) launches[i] = m->prof_n[i];
  }
  return PC_N;
}

cfm_status cfm_op_gemm(int32_t dtype, int32_t epi, int32_t act, const void* A, int32_t lda, const void* W, int32_t ldw,
                       int32_t M, int32_t N, int32_t K, const float* bias, float alpha, void* out, int32_t ldo,
                       int32_t row_off, void* out2, int32_t d, float* x, int32_t ldx, const uint8_t* rowmask,
                       int32_t variant, cfm_stream stream) {
  EpiArgs e;
  e.bias = bias; e.alpha = alpha; e.out = out; e.out2 = out2; e.ldo = ldo; e.row_off = row_off; e.x = x; e.ldx = ldx;
  e.rowmask = rowmask; e.d = d; e.small_tiles = variant & 1; e.diag = (variant >> 8) & 0xff;
  e.store_mode = (variant >> 16) & 3;
  if ((variant >> 18) & 7) e.wst = ((variant >> 18) & 7) == 7 ? 0 : (variant >> 18) & 7;
  int r;
  if (dtype == CFM_DTYPE_F32)
    r = gemm<float>(epi, act, (const float*)A, lda, (const float*)W, ldw, M, N, K, e, (hipStream_t)stream);
  else if (dtype == CFM_DTYPE_F16)
    r = gemm<f16>(epi, act, (const f16*)A, lda, (const f16*)W, ldw, M, N, K, e, (hipStream_t)stream);
  else
    r = gemm<bf16>(epi, act, (const bf16*)A, lda, (const bf16*)W, ldw, M, N, K, e, (hipStream_t)stream);
  if (r) return set_error(CFM_ERR_RUNTIME, std::string("gemm: ") + hipGetErrorString((hipError_t)r));
  return CFM_OK;
}

size_t cfm_ctc_workspace_bytes(const cfm_model* m, int32_t rows) { return m ? m->ctc_ws_bytes(rows) : 0; }

cfm_status cfm_ctc_logprobs(const cfm_model* m, const float* enc, int32_t rows, float* logp, int32_t* ids, void* ws,
                            size_t wsb, cfm_stream stream) {
  if (!m || !enc) return set_error(CFM_ERR_VALUE, "null argument");
  if (rows <= 0) return CFM_OK;
  HIPC(hipSetDevice(m->device));
  return m->ctc(enc, rows, logp, ids, ws, wsb, (hipStream_t)stream);
}

size_t cfm_ctc_ids_workspace_bytes(const cfm_model* m, int32_t rows) { return m ? m->ctc_ids_ws_bytes(rows) : 0; }

cfm_status cfm_ctc_ids(const cfm_model* m, const float* enc, int32_t rows, int32_t* ids, void* ws, size_t wsb,
                       cfm_stream stream) {
  if (!m || !enc || !ids) return set_error(CFM_ERR_VALUE, "null argument");
  if (rows <= 0) return CFM_OK;
  HIPC(hipSetDevice(m->device));
  return m->ctc(enc, rows, nullptr, ids, ws, wsb, (hipStream_t)stream);
}

cfm_status cfm_ctc_collapse(const int32_t* ids, const int32_t* row_start, const int32_t* row_len, int32_t B,
                            int32_t blank_id, int32_t max_silence, int32_t* tokens, int32_t* token_frames,
                            int32_t* n_tokens, int32_t* segments, int32_t* n_segments, cfm_stream stream) {
  if (B < 0) return set_error(CFM_ERR_VALUE, "B < 0");
  if (B == 0) return CFM_OK;
  if (!ids || !row_start || !row_len || !tokens || !token_frames || !n_tokens)
    return set_error(CFM_ERR_VALUE, "null argument");
  if (max_silence >= 0 && (!segments || !n_segments))
    return set_error(CFM_ERR_VALUE, "segmentation needs segments and n_segments");
  KCHK(ctc_collapse(ids, row_start, row_len, B, blank_id, max_silence, tokens, token_frames, n_tokens, segments,
                    n_segments, (hipStream_t)stream));
  return CFM_OK;
}

}  // extern "C"
