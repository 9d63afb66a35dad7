// CTC head on the encoder tail.
//
// ctc_argmax_kernel: ids[m] = argmax_v (enc[m] . W[v] + b[v])  -- the argmax of CTC.log_softmax
//   (ctc.py:73-81; chunkformer_model.py:437-438, 526-527: log_softmax is monotone per row, so its
//   argmax is the logits' argmax) with NO [rows, V] logit tensor: every logit lives only in
//   registers.  bf16 (or, for the fp16 model, f16) MFMA, f32 accumulate, the same operands as the
//   two-pass path (enc rounded to the 16-bit format RNE, W in it); ties resolve to the lowest index
//   like torch.argmax.
//     * block = 4 waves, 256 rows (64 per wave); the wave's rows stay in AGPRs for the whole
//       launch as MFMA B fragments (enc is read from HBM once, f32 -> bf16 in registers);
//     * the vocabulary streams through a 2 x 64 KiB LDS ring in 64-column tiles (LDS-DMA, one
//       1-KiB row per instruction, 16-B chunks XOR-swizzled by row so the fragment reads are
//       conflict-free); every CU walks W in the same order, so the tiles come from L2;
//     * the accumulators are seeded with the bias from an LDS image of b padded with -inf
//       (columns >= V can never win, and a dummy tile past the end contributes nothing);
//     * per 64-column tile a wave issues 16 K-steps x 16 v_mfma_f32_16x16x32_bf16; the previous
//       tile's running (max, argmax) update (3 VALU per logit) rides in the MFMA gaps of K-steps
//       1..11 (double-buffered accumulators), the next tile's bias seeds in steps 12..13.
//
// ctc_collapse_kernel: per utterance, on the argmax ids
//   mode < 0  : remove_duplicates_and_blank (model_utils.py:23-32) + CTC peak frames
//               (gen_ctc_peak_time, model_utils.py:49-58);
//   mode >= 0 : get_output_with_timestamps' sentence split at `mode` = max_silence blank frames
//               (model_utils.py:174-221): per segment the de-duplicated non-blank tokens and the
//               start / end frames (80 ms units).
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "gemm_bf16_epi.h"
#include <type_traits>

namespace cfm {

namespace {
constexpr int CT_K = 512;                  // d_model of the fused head
constexpr int CT_ROWS = 256;               // rows per block (4 waves x 64)
constexpr int CT_NT = 64;                  // vocabulary columns per tile
constexpr int CT_TILE = CT_NT * CT_K * 2;  // 64 KiB of bf16 W per tile
constexpr int CT_BIAS = 7936;              // f32 bias image (V padded by >= 2 tiles of -inf): 31 KiB

template <int B, int E, class F>
CFM_DEV void cfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    cfor<B + 1, E>(f);
  }
}
}  // namespace

// acc += W fragment (VGPR, MFMA A: 16 vocabulary columns) x enc fragment (AGPR, MFMA B: 16 rows):
// lane (fr, g) of acc holds logit[row 16 mb + fr][column 16 nb + 4 g + r]
// (FMT 1: f16 operands, v_mfma_f32_16x16x32_f16, the fp16 model's head)
template <int FMT>
CFM_DEV void ctc_mfma(f32x4& acc, const bf16x8& w, const bf16x8& a) {
  if constexpr (FMT == 1)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "a"(a));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "a"(a));
}
// running argmax, 3 VALU per logit: if (x > best) { best = x; slot = SLOT; } with the tile-local
// column SLOT (< 64) as an inline constant (VOP2 v_cndmask reads VCC, so an SGPR column would not
// fit the constant bus); ctc_argmax_fix turns a slot set in this tile into an absolute column
template <int SLOT>
CFM_DEV void ctc_argmax_step(float x, float& best, int& slot) {
  asm volatile(
      "v_cmp_ngt_f32 vcc, %2, %0\n\t"
      "v_cndmask_b32 %1, %3, %1, vcc\n\t"
      "v_cndmask_b32 %0, %2, %0, vcc"
      : "+v"(best), "+v"(slot)
      : "v"(x), "i"(SLOT)
      : "vcc");
}
// if (slot >= 0) col = tile_col0 + slot; slot = -1
CFM_DEV void ctc_argmax_fix(int& col, int& slot, int tile_col0) {
  int t;
  asm volatile(
      "v_add_u32 %2, %3, %1\n\t"
      "v_cmp_le_i32 vcc, 0, %1\n\t"
      "v_cndmask_b32 %0, %0, %2, vcc\n\t"
      "v_mov_b32 %1, -1"
      : "+v"(col), "+v"(slot), "=&v"(t)
      : "s"(tile_col0)
      : "vcc");
}
template <int OFF>
CFM_DEV void ctc_lds_read(f32x4& v, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(v) : "v"(addr), "i"(OFF));
}
template <int OFF>
CFM_DEV void ctc_lds_read(bf16x8& v, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(v) : "v"(addr), "i"(OFF));
}

template <int FMT>
__global__ __launch_bounds__(256, 1) void ctc_argmax_kernel(const float* __restrict__ enc, int M,
                                                            const bf16* __restrict__ W /*[nt*64, 512]*/,
                                                            const float* __restrict__ bias, int V,
                                                            int32_t* __restrict__ ids) {
  __shared__ __attribute__((aligned(16))) char smem[2 * CT_TILE + CT_BIAS * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int nt = (V + CT_NT - 1) / CT_NT;
  const int row0 = blockIdx.x * CT_ROWS + wv * 64;
  float* bl = reinterpret_cast<float*>(smem + 2 * CT_TILE);
  for (int i = tid; i < CT_BIAS; i += 256) bl[i] = i < V ? bias[i] : -INFINITY;

  // W tile t -> buffer b: wave wv DMAs rows n = 16 wv + p (p = 0..15), one 1-KiB row per
  // instruction; lane l of row n writes LDS chunk l, which holds W chunk l ^ (n & 15)
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, nt * CT_TILE, 0x00020000);
  auto issue_tile = [&](int t, int b) {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const int n = 16 * wv + p;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wrs, (__attribute__((address_space(3))) void*)(smem + b * CT_TILE + n * 1024), 16,
          (unsigned)((lane ^ p) * 16), t * CT_TILE + n * 1024, 0, 0);
    }
  };
  issue_tile(0, 0);

  // the wave's 64 rows as bf16 B fragments: lane (fr, g) holds row 16 mb + fr, k = 32 s + 8 g .. +7
  // (rows past M repeat row M-1; their argmax is never stored)
  bf16x8 af[4][16];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = min(row0 + 16 * mb + fr, M - 1);
    const float* ap = enc + (size_t)m * CT_K + 8 * g;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const f32x4 lo = *reinterpret_cast<const f32x4*>(ap + 32 * s);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(ap + 32 * s + 4);
      if constexpr (FMT == 1)   // the 16-bit format's raw lanes in the bf16x8 fragment type
        af[mb][s] = __builtin_bit_cast(bf16x8, (f16x8){(f16)lo[0], (f16)lo[1], (f16)lo[2], (f16)lo[3],
                                                       (f16)hi[0], (f16)hi[1], (f16)hi[2], (f16)hi[3]});
      else
        af[mb][s] = (bf16x8){(bf16)lo[0], (bf16)lo[1], (bf16)lo[2], (bf16)lo[3],
                             (bf16)hi[0], (bf16)hi[1], (bf16)hi[2], (bf16)hi[3]};
    }
  }

  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  // fragment read of K-step s, n-block nb: row n = 16 nb + fr, chunk (4 s + g) ^ fr
  //   = 4 (s ^ (fr >> 2)) + ((g ^ fr) & 3): one lane base per (buffer, s & 3), s & ~3 and nb in the
  //   immediate offset
  unsigned rb[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
      rb[b][s4] = lds0 + b * CT_TILE + fr * 1024 + (unsigned)((4 * (s4 ^ (fr >> 2)) + ((g ^ fr) & 3)) * 16);
  // bias seeds: acc[nb][*] of tile t <- bl[64 t + 16 nb + 4 g .. +3]
  const unsigned sb0 = lds0 + 2 * CT_TILE + (unsigned)(4 * g) * 4;

  f32x4 acc[2][4][4];
  bf16x8 wf[2][4];
  float bv[4];
  int bi[4], bs[4];   // running best logit, its column, and its slot if set in the tile being scanned
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    bv[mb] = -INFINITY;
    bi[mb] = 0;
    bs[mb] = -1;
  }

  __syncthreads();   // bias image (plain LDS stores) before the asm reads
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");   // tile 0 landed for every wave
  // seeds: acc[0] <- tile 0, acc[1] <- the -inf pad (a "previous tile" that never wins)
  const int pad_t = nt + 1;   // bl[64 (nt + 1) ..] is -inf (CT_BIAS >= 64 (nt + 2))
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      acc[0][nb][mb] = (f32x4){0.f, 0.f, 0.f, 0.f};
      acc[1][nb][mb] = (f32x4){0.f, 0.f, 0.f, 0.f};
      ctc_lds_read<0>(acc[0][nb][mb], sb0 + nb * 64);
      ctc_lds_read<0>(acc[1][nb][mb], sb0 + pad_t * 256 + nb * 64);
    }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    wf[0][nb] = (bf16x8){};
    wf[1][nb] = (bf16x8){};
    ctc_lds_read<0>(wf[0][nb], rb[0][0] + nb * 16384);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // + AGPR writes -> MFMA reads

  // one 64-column tile t into acc[A]; its gaps update the running argmax from acc[1 - A]
  // (tile tp = t - 1, or the -inf pad) and seed acc[1 - A] for tile t + 1
  auto tile = [&](auto Ac, int t, int tp) {
    constexpr int A = decltype(Ac)::value;
    const int b = t & 1;
    const unsigned rbase[4] = {rb[b][0], rb[b][1], rb[b][2], rb[b][3]};
    const unsigned rnext = rb[b ^ 1][0];
    const unsigned seed = sb0 + (unsigned)(t + 1) * 256;
    const bool more = t + 1 < nt;
    cfor<0, 16>([&](auto Sc) {
      constexpr int s = decltype(Sc)::value;
      bf16x8(&cur)[4] = wf[s & 1];
      bf16x8(&nxt)[4] = wf[(s + 1) & 1];
      cfor<0, 16>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        constexpr int nb = i >> 2, mb = i & 3;
        ctc_mfma<FMT>(acc[A][nb][mb], cur[nb], af[mb][s]);
        // next K-step's W fragments (the next tile's K-step 0 from the other buffer at s = 15)
        if constexpr ((i & 3) == 1) {
          constexpr int rn = i >> 2;
          if constexpr (s < 15)
            ctc_lds_read<((s + 1) & ~3) * 64 + rn * 16384>(nxt[rn], rbase[(s + 1) & 3]);
          else
            ctc_lds_read<rn * 16384>(nxt[rn], rnext);
        }
        // the DMA of tile t + 1 into the other buffer (free: every wave passed the barrier that
        // followed its last reads of it)
        if constexpr (s == 0) {
          if (more) {
            const int n = 16 * wv + i;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                wrs, (__attribute__((address_space(3))) void*)(smem + (b ^ 1) * CT_TILE + n * 1024), 16,
                (unsigned)((lane ^ i) * 16), (t + 1) * CT_TILE + n * 1024, 0, 0);
          }
        }
        // running argmax over the previous tile: logit v = 16 (s - 1) / 3 .. in the gaps
        // (i = 0, 3, 6, 9, 12, 15) of K-steps 1..11 -> 66 slots for 64 logits in column order
        if constexpr (s >= 1 && s <= 11 && i % 3 == 0) {
          constexpr int v = (s - 1) * 6 + i / 3;
          if constexpr (v < 64) {
            constexpr int pmb = v >> 4, pnb = (v >> 2) & 3, r = v & 3;
            ctc_argmax_step<16 * pnb + r>(acc[1 - A][pnb][pmb][r], bv[pmb], bs[pmb]);
          }
        }
        if constexpr (s == 12 && (i & 3) == 1) ctc_argmax_fix(bi[i >> 2], bs[i >> 2], tp * CT_NT);
        // bias seeds of tile t + 1 into acc[1 - A] (after its last VALU read in step 11)
        if constexpr ((s == 12 || s == 13) && (i & 1) == 0) {
          constexpr int q = (s - 12) * 8 + (i >> 1), snb = q >> 2, smb = q & 3;
          ctc_lds_read<snb * 64>(acc[1 - A][snb][smb], seed);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if constexpr (s == 14)   // tile t + 1 landed for every wave before K-step 15 reads its K-step 0
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    });
  };

  // tiles in pairs (acc[0], acc[1]); an odd count runs one dummy tile t = nt (seeded -inf, its
  // stale W reads add finite products to -inf), so the final drain is always acc[1]
  const int npair = (nt + 1) >> 1;
  for (int it = 0; it < npair; ++it) {
    const int t = 2 * it;
    tile(std::integral_constant<int, 0>{}, t, it > 0 ? t - 1 : pad_t);
    tile(std::integral_constant<int, 1>{}, t + 1, t);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // last MFMA writes -> VALU reads
  const int tl = 2 * npair - 1;
  cfor<0, 64>([&](auto Vc) {
    constexpr int v = decltype(Vc)::value;
    constexpr int pmb = v >> 4, pnb = (v >> 2) & 3, r = v & 3;
    ctc_argmax_step<16 * pnb + r>(acc[1][pnb][pmb][r], bv[pmb], bs[pmb]);
  });
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) ctc_argmax_fix(bi[mb], bs[mb], tl * CT_NT);
  // lane-relative columns -> absolute (+4 g), then the 4 lanes of a row (xor 16, 32) merge:
  // larger logit wins, equal logits keep the lower column
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    float x = bv[mb];
    int c = bi[mb] + 4 * g;
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ox = __shfl_xor(x, o, 64);
      const int oc = __shfl_xor(c, o, 64);
      if (ox > x || (ox == x && oc < c)) {
        x = ox;
        c = oc;
      }
    }
    const int m = row0 + 16 * mb + fr;
    if (g == 0 && m < M) ids[m] = c;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

bool ctc_argmax_eligible(int V, int d) { return d == CT_K && V > 0 && CT_NT * ((V + CT_NT - 1) / CT_NT + 2) <= CT_BIAS; }

int ctc_argmax_bf16(const float* enc, int M, const bf16* W, const float* bias, int V, int d, int32_t* ids,
                    hipStream_t st) {
  if (!ctc_argmax_eligible(V, d)) return -1;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(ctc_argmax_kernel<0>, dim3((M + CT_ROWS - 1) / CT_ROWS), dim3(256), 0, st, enc, M, W, bias, V, ids);
  CFM_CHECK_LAUNCH();
  return 0;
}
int ctc_argmax_f16(const float* enc, int M, const f16* W, const float* bias, int V, int d, int32_t* ids,
                   hipStream_t st) {
  if (!ctc_argmax_eligible(V, d)) return -1;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(ctc_argmax_kernel<1>, dim3((M + CT_ROWS - 1) / CT_ROWS), dim3(256), 0, st, enc, M,
                     reinterpret_cast<const bf16*>(W), bias, V, ids);
  CFM_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------ collapse
// One block per utterance b: frames [row_start[b], row_start[b] + row_len[b]) of ids.  Each of the
// 512 threads walks a contiguous span twice (count, then write); a serial scan over the 512
// per-thread summaries in between carries the counts and the last non-blank frame.
namespace {
constexpr int CL_THREADS = 512;
struct SpanSum {
  int keeps, segs;     // kept tokens / segment starts inside the span (first non-blank: resolved by the scan)
  int tf, idf;         // first non-blank frame of the span (-1: none) and its id
  int tl, idl;         // last non-blank frame of the span and its id
};
}  // namespace

__global__ __launch_bounds__(CL_THREADS) void ctc_collapse_kernel(const int32_t* __restrict__ ids,
                                                                  const int32_t* __restrict__ row_start,
                                                                  const int32_t* __restrict__ row_len, int blank,
                                                                  int max_sil, int32_t* __restrict__ tok,
                                                                  int32_t* __restrict__ tok_frame,
                                                                  int32_t* __restrict__ n_tok, int32_t* __restrict__ seg,
                                                                  int32_t* __restrict__ n_seg) {
  __shared__ SpanSum ss[CL_THREADS];
  __shared__ int carry_keep[CL_THREADS], carry_seg[CL_THREADS], carry_t[CL_THREADS], carry_id[CL_THREADS];
  __shared__ int tot_keep, tot_seg, last_t;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int base = row_start[b], T = row_len[b];
  const int span = (T + CL_THREADS - 1) / CL_THREADS;
  const int a0 = min(T, tid * span), a1 = min(T, a0 + span);
  const int32_t* x = ids + base;
  const bool segm = max_sil >= 0;

  // pass 1: span summary
  SpanSum s = {0, 0, -1, 0, -1, 0};
  {
    int prev = a0 > 0 ? x[a0 - 1] : -1;   // plain collapse: the previous FRAME decides
    int tp = -1, idp = 0;                 // segment mode: the previous non-blank frame inside the span
    for (int t = a0; t < a1; ++t) {
      const int v = x[t];
      if (!segm) {
        if (v != blank && v != prev) s.keeps++;
        prev = v;
      } else if (v != blank) {
        if (tp < 0) {
          s.tf = t;
          s.idf = v;
        } else {
          const bool start = t - tp - 1 >= max_sil;
          s.segs += start;
          s.keeps += start || v != idp;
        }
        tp = t;
        idp = v;
      }
    }
    s.tl = tp;
    s.idl = idp;
  }
  ss[tid] = s;
  __syncthreads();
  if (tid == 0) {   // exclusive scan: counts and the last non-blank frame before each span
    int k = 0, sg = 0, lt = -1, lid = 0;
    for (int i = 0; i < CL_THREADS; ++i) {
      const SpanSum& q = ss[i];
      carry_keep[i] = k;
      carry_seg[i] = sg;
      carry_t[i] = lt;
      carry_id[i] = lid;
      k += q.keeps;
      sg += q.segs;
      if (segm && q.tf >= 0) {
        const bool start = lt < 0 || q.tf - lt - 1 >= max_sil;
        sg += start;
        k += start || q.idf != lid;
        lt = q.tl;
        lid = q.idl;
      }
    }
    tot_keep = k;
    tot_seg = sg;
    last_t = lt;
  }
  __syncthreads();

  // pass 2: write
  {
    int k = carry_keep[tid], sg = carry_seg[tid];
    int prev = a0 > 0 ? x[a0 - 1] : -1;
    int tp = carry_t[tid], idp = carry_id[tid];
    for (int t = a0; t < a1; ++t) {
      const int v = x[t];
      if (!segm) {
        if (v != blank && v != prev) {
          tok[base + k] = v;
          tok_frame[base + k] = t;
          ++k;
        }
        prev = v;
      } else if (v != blank) {
        const bool start = tp < 0 || t - tp - 1 >= max_sil;
        if (start) {
          // segment sg: [token k, start frame, end frame]; the previous segment closed at tp + max_sil
          int32_t* r = seg + (size_t)(base + sg) * 3;
          r[0] = k;
          r[1] = tp < 0 ? max(t - 2, 0) : max((t + tp + max_sil + 1) / 2, t - 2);
          if (sg > 0) seg[(size_t)(base + sg - 1) * 3 + 2] = tp + max_sil;
          ++sg;
        }
        if (start || v != idp) {
          tok[base + k] = v;
          tok_frame[base + k] = t;
          ++k;
        }
        tp = t;
        idp = v;
      }
    }
  }
  if (tid == 0) {
    n_tok[b] = tot_keep;
    if (segm) {
      n_seg[b] = tot_seg;
      // the last segment closes after max_sil blank frames, or at the utterance's last frame
      if (tot_seg > 0) seg[(size_t)(base + tot_seg - 1) * 3 + 2] = last_t + max_sil <= T - 1 ? last_t + max_sil : T - 1;
    }
  }
}

int ctc_collapse(const int32_t* ids, const int32_t* row_start, const int32_t* row_len, int B, int blank, int max_sil,
                 int32_t* tok, int32_t* tok_frame, int32_t* n_tok, int32_t* seg, int32_t* n_seg, hipStream_t st) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ctc_collapse_kernel, dim3(B), dim3(CL_THREADS), 0, st, ids, row_start, row_len, blank, max_sil,
                     tok, tok_frame, n_tok, seg, n_seg);
  CFM_CHECK_LAUNCH();
  return 0;
}

}  // namespace cfm
