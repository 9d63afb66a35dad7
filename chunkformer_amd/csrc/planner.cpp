// Host planner: the integer part of the reference's packer, computed in C++.
//
// cfm_plan_masked restates ChunkFormerEncoder.forward_parallel_chunk's packer
// (encoder.py:534-604) and mask build (625-645) in closed form:
//   size = (C-1)*8 + 15, step = 8C,
//   n_pad = (step - ((T-size) % step)) % step if T >= size else size - T,
//   n_chunk = (T + n_pad - size) / step + 1, max_len = 1 + floor((T-15)/8),
//   attention key j of chunk c: g = C*c - L + j, valid iff -o <= g < max_len,
//   conv column j:             g = C*c - 7 + j, valid iff -o <= g < max_len and j-7 <= C+R-1.
// Both valid sets are contiguous, so masks travel as [lo, hi) ranges.
// cfm_plan_padded restates forward_encoder's geometry (attention.py:334-386,
// convolution.py:133-167).  cfm_plan_stream restates forward_chunk's (encoder.py:310-385): one
// window of T frames -> T' rows; keys = [L cached | T' current], valid from L - offset
// (encoder.py:351-357); rel-pos table of a C+R chunk read at row T'-1-i+j (attention.py:256-266);
// conv chunks of C over [7 cached | T'] with the right edge zero-padded (convolution.py:148-180).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cfm.h"
#include "cfm_common.h"
#include "plan.h"
#include "status.h"

namespace cfm {

static inline int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
static inline int64_t floormod(int64_t a, int64_t b) { return a - floordiv(a, b) * b; }

// subsampling.py:270-288 (three times floor((L-3)/2 + 1)); equals 1 + floor((T-15)/8)
int calc_length(int T) {
  int64_t L = T;
  for (int i = 0; i < 3; ++i) L = floordiv(L - 3, 2) + 1;
  return (int)L;
}

}  // namespace cfm

using namespace cfm;

// rows[b]: feature rows of utterance b (x.size(0): padding, unfold and window validity,
// encoder.py:556-564, 598); mask_lens[b] (NULL = rows): xs_origin_lens[b], which bounds the masks
// and gives the output length (encoder.py:567-596, 673).  The reference builds one bound per
// arange(0, 1 + (len + n_pad - 15) // 8, C) entry; a count different from the window count is its
// shape-mismatch RuntimeError.
extern "C" cfm_status cfm_plan_masked_ex(const int32_t* lens, const int32_t* mask_lens, const int32_t* offsets,
                                         int32_t B, int32_t C, int32_t L, int32_t R, int32_t* n_chunks_out,
                                         int32_t* out_lens, int32_t* total_chunks, int32_t* plan, int64_t* plan_n) {
  if (B <= 0 || !lens) return set_error(CFM_ERR_VALUE, "plan_masked: empty batch");
  if (C <= 0 || L < 0 || R < 0) return set_error(CFM_ERR_VALUE, "plan_masked: chunk_size must be > 0, contexts >= 0");
  const int size = (C - 1) * 8 + 15, step = 8 * C;
  const int nsub = (C + 63) / 64;   // attention / conv blocks per chunk (<= 64 rows each)
  int64_t N = 0;
  std::vector<int> nch(B);
  for (int b = 0; b < B; ++b) {
    const int T = lens[b];
    if (T < 0) return set_error(CFM_ERR_VALUE, "plan_masked: negative length");
    const int n_pad = (T >= size) ? (int)floormod((int64_t)step - floormod(T - size, step), step) : size - T;
    nch[b] = (T + n_pad - size) / step + 1;
    const int Tm = mask_lens ? mask_lens[b] : T;
    if (mask_lens) {
      const int64_t stop = 1 + floordiv((int64_t)Tm + n_pad - 15, 8);
      const int64_t nb = stop > 0 ? (stop + C - 1) / C : 0;
      if (nb != nch[b])
        return set_error(CFM_ERR_RUNTIME, "plan_masked: utterance " + std::to_string(b) + ": " + std::to_string(T) +
                                              " feature rows make " + std::to_string(nch[b]) +
                                              " chunks but xs_origin_lens " + std::to_string(Tm) + " bounds " +
                                              std::to_string(nb) + " (shape mismatch, encoder.py:567-612)");
    }
    N += nch[b];
    if (n_chunks_out) n_chunks_out[b] = nch[b];
    if (out_lens) out_lens[b] = calc_length(Tm);
  }
  if (N * C >= (int64_t)1 << 31) return set_error(CFM_ERR_VALUE, "plan_masked: batch too large");
  const int rows = (int)(N * C);
  const int64_t need = plan_ints((int)N, (int)N * nsub, (int)N * nsub, rows);
  if (total_chunks) *total_chunks = (int32_t)N;
  if (plan_n && !plan) { *plan_n = need; return CFM_OK; }
  if (!plan) return CFM_OK;
  if (plan_n && *plan_n < need) return set_error(CFM_ERR_VALUE, "plan_masked: plan buffer too small");
  std::memset(plan, 0, sizeof(int32_t) * need);
  int32_t* h = plan;
  h[PH_KIND] = 1; h[PH_NWIN] = (int)N; h[PH_NATT] = (int)N * nsub; h[PH_NCONV] = (int)N * nsub;
  h[PH_ROWS] = rows; h[PH_C] = C; h[PH_L] = L; h[PH_R] = R; h[PH_W] = size; h[PH_TOUT] = C;
  h[PH_PROWS] = L + 2 * C + R - 1; h[PH_PANCHOR] = C + L - 1;
  h[PH_KVROWS] = L + rows + R; h[PH_GLUROWS] = 7 + rows + 7; h[PH_KVOFF] = L; h[PH_GLUOFF] = 7;
  int32_t* meta = plan + plan_meta_off(h);
  int32_t* att = plan + plan_att_off(h);
  int32_t* conv = plan + plan_conv_off(h);
  uint8_t* rmask = reinterpret_cast<uint8_t*>(plan + plan_mask_off(h));
  const int W = L + C + R, WC = C + 14;
  int64_t n = 0, src = 0;
  for (int b = 0; b < B; ++b) {
    const int T = lens[b];
    const int o = offsets ? offsets[b] : 0;
    const int max_len = 1 + (int)floordiv((mask_lens ? mask_lens[b] : T) - 15, 8);
    for (int c = 0; c < nch[b]; ++c, ++n) {
      int32_t* m = meta + n * PLAN_REC;
      const int base = C * c;
      // attention: -o <= base - L + j < max_len
      const int alo = std::max(0, L - o - base), ahi = std::min(W, max_len - base + L);
      // conv: -o <= base - 7 + j < max_len, j <= C + R + 6
      const int clo = std::max(0, 7 - o - base), chi = std::min(std::min(WC, C + R + 7), max_len - base + 7);
      m[PM_SRC_ROW] = (int32_t)(src + (int64_t)c * step);
      m[PM_NVALID] = std::max(0, std::min(size, T - c * step));
      m[PM_ATT_LO] = alo; m[PM_ATT_HI] = std::max(alo, ahi);
      m[PM_CONV_LO] = clo; m[PM_CONV_HI] = std::max(clo, chi);
      m[PM_UTT] = b; m[PM_CHUNK] = c;
      for (int s = 0; s < nsub; ++s) {
        const int q0 = 64 * s, nq = std::min(64, C - q0);
        int32_t* a = att + (n * nsub + s) * PLAN_REC;
        a[AD_Q_ROW0] = (int32_t)(n * C + q0); a[AD_NQ] = nq; a[AD_KV_ROW0] = (int32_t)(n * C);
        a[AD_KEY_LO] = m[PM_ATT_LO]; a[AD_KEY_HI] = m[PM_ATT_HI]; a[AD_P_BASE] = C - 1 - q0; a[AD_Q_VALID] = nq;
        int32_t* cd = conv + (n * nsub + s) * PLAN_REC;
        cd[CD_OUT_ROW0] = (int32_t)(n * C + q0); cd[CD_NOUT] = nq; cd[CD_SRC_ROW0] = (int32_t)(n * C + q0);
        cd[CD_J_LO] = m[PM_CONV_LO] - q0; cd[CD_J_HI] = m[PM_CONV_HI] - q0;
      }
      for (int i = 0; i < C; ++i) rmask[n * C + i] = (i + 7 >= m[PM_CONV_LO] && i + 7 < m[PM_CONV_HI]) ? 1 : 0;
    }
    src += T;
  }
  return CFM_OK;
}

extern "C" cfm_status cfm_plan_masked(const int32_t* lens, const int32_t* offsets, int32_t B, int32_t C, int32_t L,
                                      int32_t R, int32_t* n_chunks_out, int32_t* out_lens, int32_t* total_chunks,
                                      int32_t* plan, int64_t* plan_n) {
  return cfm_plan_masked_ex(lens, nullptr, offsets, B, C, L, R, n_chunks_out, out_lens, total_chunks, plan, plan_n);
}

extern "C" cfm_status cfm_plan_padded(const int32_t* lens, int32_t B, int32_t T, int32_t C, int32_t L, int32_t R,
                                      int32_t* t_out, int32_t* plan, int64_t* plan_n) {
  if (B <= 0 || !lens) return set_error(CFM_ERR_VALUE, "plan_padded: empty batch");
  const int Tp = calc_length(T);
  if (Tp <= 0) return set_error(CFM_ERR_VALUE, "plan_padded: input too short for 8x subsampling");
  if (t_out) *t_out = Tp;
  const bool full = C <= 0;
  if (full) { L = 0; R = 0; }
  if (L < 0 || R < 0) return set_error(CFM_ERR_VALUE, "plan_padded: negative context");
  const int Ce = full ? Tp : C;
  if (Ce + L >= 5000) return set_error(CFM_ERR_ASSERT, "relative PE table: left_context + chunk_size >= 5000 (embedding.py:163)");
  const int nch = (Tp + Ce - 1) / Ce;
  const int nsub = (Ce + 63) / 64;
  // blocks per utterance: every chunk k, every 64-row piece that holds rows < T'
  int per_utt = 0;
  for (int k = 0; k < nch; ++k) {
    const int rk = std::min(Ce, Tp - k * Ce);
    per_utt += (rk + 63) / 64;
  }
  (void)nsub;
  const int nblk = per_utt * B;
  const int64_t rows64 = (int64_t)B * Tp;
  if (rows64 >= (int64_t)1 << 31) return set_error(CFM_ERR_VALUE, "plan_padded: batch too large");
  const int rows = (int)rows64;
  const int64_t need = plan_ints(B, nblk, nblk, rows);
  if (plan_n && !plan) { *plan_n = need; return CFM_OK; }
  if (!plan) return CFM_OK;
  if (plan_n && *plan_n < need) return set_error(CFM_ERR_VALUE, "plan_padded: plan buffer too small");
  std::memset(plan, 0, sizeof(int32_t) * need);
  int32_t* h = plan;
  h[PH_KIND] = 2; h[PH_NWIN] = B; h[PH_NATT] = nblk; h[PH_NCONV] = nblk; h[PH_ROWS] = rows;
  h[PH_C] = Ce; h[PH_L] = L; h[PH_R] = R; h[PH_W] = T; h[PH_TOUT] = Tp;
  h[PH_PROWS] = L + 2 * Ce + R - 1; h[PH_PANCHOR] = Ce + L - 1;
  h[PH_KVROWS] = rows; h[PH_GLUROWS] = rows; h[PH_KVOFF] = 0; h[PH_GLUOFF] = 0;
  int32_t* meta = plan + plan_meta_off(h);
  int32_t* att = plan + plan_att_off(h);
  int32_t* conv = plan + plan_conv_off(h);
  uint8_t* rmask = reinterpret_cast<uint8_t*>(plan + plan_mask_off(h));
  int64_t blk = 0;
  for (int b = 0; b < B; ++b) {
    const int lb = std::min(calc_length(lens[b]), Tp);   // valid subsampled frames (may be <= 0)
    int32_t* m = meta + (int64_t)b * PLAN_REC;
    m[PM_SRC_ROW] = b * T; m[PM_NVALID] = T; m[PM_UTT] = b;
    for (int t = 0; t < Tp; ++t) rmask[(int64_t)b * Tp + t] = t < lb ? 1 : 0;
    for (int k = 0; k < nch; ++k) {
      const int kc = k * Ce, rk = std::min(Ce, Tp - kc);
      for (int q0 = 0; q0 < rk; q0 += 64, ++blk) {
        const int nq = std::min(64, rk - q0);
        int32_t* a = att + blk * PLAN_REC;
        a[AD_Q_ROW0] = b * Tp + kc + q0; a[AD_NQ] = nq;
        a[AD_P_BASE] = Ce - 1 - q0;
        if (full) {   // key padding mask only (attention.py:129-136 with mask [B,1,T])
          a[AD_KV_ROW0] = b * Tp; a[AD_KEY_LO] = 0; a[AD_KEY_HI] = std::max(0, lb); a[AD_Q_VALID] = nq;
        } else {      // chunk window [kc-L, kc+C+R) of the zero-padded utterance; mask_q & mask_kv
          a[AD_KV_ROW0] = b * Tp + kc - L;
          const int lo = std::max(0, L - kc), hi = std::min(L + Ce + R, lb - kc + L);
          a[AD_KEY_LO] = lo; a[AD_KEY_HI] = std::max(lo, hi);
          a[AD_Q_VALID] = std::max(0, std::min(nq, lb - kc - q0));
        }
        // conv: output position p = kc+q0+i reads p-7 .. p+7 within [max(0,kc-7), min(kc+Ce, T'))
        int32_t* cd = conv + blk * PLAN_REC;
        const int p0 = kc + q0 - 7;   // position of window column 0
        cd[CD_OUT_ROW0] = b * Tp + kc + q0; cd[CD_NOUT] = nq; cd[CD_SRC_ROW0] = b * Tp + p0;
        cd[CD_J_LO] = std::max(0, kc - 7) - p0;
        cd[CD_J_HI] = std::min(kc + Ce, Tp) - p0;
      }
    }
  }
  return CFM_OK;
}

extern "C" cfm_status cfm_plan_stream(int32_t T, int32_t C, int32_t L, int32_t R, int32_t offset, int32_t* t_out,
                                      int32_t* plan, int64_t* plan_n) {
  if (C <= 0 || L < 0 || R < 0 || offset < 0)
    return set_error(CFM_ERR_VALUE, "plan_stream: chunk_size must be > 0, contexts and offset >= 0");
  const int Tp = calc_length(T);
  if (Tp <= 0) return set_error(CFM_ERR_VALUE, "plan_stream: input too short for 8x subsampling");
  if (Tp < R) return set_error(CFM_ERR_VALUE, "plan_stream: the chunk must have at least right_context_size frames");
  if (Tp > C + R) return set_error(CFM_ERR_VALUE, "plan_stream: more than chunk_size + right_context_size frames");
  if (C + R + L >= 5000) return set_error(CFM_ERR_ASSERT, "relative PE table: left_context + chunk_size >= 5000 (embedding.py:163)");
  if (t_out) *t_out = Tp;
  const int natt = (Tp + 63) / 64;
  int nconv = 0;
  for (int j0 = 0; j0 < Tp; j0 += C) nconv += (std::min(C, Tp - j0) + 63) / 64;
  const int64_t need = plan_ints(1, natt, nconv, Tp);
  if (plan_n && !plan) { *plan_n = need; return CFM_OK; }
  if (!plan) return CFM_OK;
  if (plan_n && *plan_n < need) return set_error(CFM_ERR_VALUE, "plan_stream: plan buffer too small");
  std::memset(plan, 0, sizeof(int32_t) * need);
  int32_t* h = plan;
  h[PH_KIND] = 3; h[PH_NWIN] = 1; h[PH_NATT] = natt; h[PH_NCONV] = nconv; h[PH_ROWS] = Tp;
  h[PH_C] = C; h[PH_L] = L; h[PH_R] = R; h[PH_W] = T; h[PH_TOUT] = Tp;
  h[PH_PROWS] = L + 2 * (C + R) - 1; h[PH_PANCHOR] = C + R + L - 1;
  h[PH_KVROWS] = L + Tp; h[PH_GLUROWS] = 7 + Tp; h[PH_KVOFF] = L; h[PH_GLUOFF] = 7;
  int32_t* meta = plan + plan_meta_off(h);
  int32_t* att = plan + plan_att_off(h);
  int32_t* conv = plan + plan_conv_off(h);
  uint8_t* rmask = reinterpret_cast<uint8_t*>(plan + plan_mask_off(h));
  meta[PM_SRC_ROW] = 0; meta[PM_NVALID] = T;
  const int klo = std::min(std::max(0, L - offset), L + Tp);
  for (int s = 0; s < natt; ++s) {
    const int q0 = 64 * s, nq = std::min(64, Tp - q0);
    int32_t* a = att + (int64_t)s * PLAN_REC;
    a[AD_Q_ROW0] = q0; a[AD_NQ] = nq; a[AD_KV_ROW0] = 0;
    a[AD_KEY_LO] = klo; a[AD_KEY_HI] = L + Tp; a[AD_P_BASE] = Tp - 1 - q0; a[AD_Q_VALID] = nq;
  }
  int blk = 0;
  for (int j0 = 0; j0 < Tp; j0 += C) {
    const int rj = std::min(C, Tp - j0);
    const int lim = std::min(j0 + C + 7, 7 + Tp);   // chunk end (+ its 7 zero pads) / sequence end
    for (int q0 = 0; q0 < rj; q0 += 64, ++blk) {
      const int t0 = j0 + q0;
      int32_t* cd = conv + (int64_t)blk * PLAN_REC;
      cd[CD_OUT_ROW0] = t0; cd[CD_NOUT] = std::min(64, rj - q0); cd[CD_SRC_ROW0] = t0;
      cd[CD_J_LO] = 0; cd[CD_J_HI] = lim - t0;
    }
  }
  for (int t = 0; t < Tp; ++t) rmask[t] = 1;
  return CFM_OK;
}
