// Masked-batch chunk attention for head_dim 128 (bf16): the 4-head d=512 recipes
// (examples/asr/rnnt/conf/chunkformer-rnnt-large-vie.yaml:5-6, classification single_task.yaml:7-8).
//
// Reference: ChunkAttentionWithRelativeRightContext.forward_parallel_chunk (attention.py:420-505):
//   s(i, j) = ((q_i + u) . k_j + (q_i + v) . P[C - 1 - i + j]) / sqrt(128),  keys outside [lo, hi) -inf,
//   softmax over the L + C + R window, out_i = sum_j p_ij v_j.
//
// The dk = 64 ring kernel keeps K, V^T and P of a head in LDS (158 KiB); at dk = 128 those are
// 290 KiB, so this kernel re-partitions the work instead of the data.  One 512-thread block = one
// head x a run of consecutive chunks (C = 64 queries each), chunk by chunk:
//   LDS: the K ring (W rows x 256 B, 16-B chunks XOR-swizzled by row: the next chunk's 64 new rows
//        replace the current chunk's first 64), the chunk's (q+u) / (q+v) (bf16, swizzled), and one
//        buffer that holds the skewed band and then the probabilities;
//   band:   every wave owns 48 relative-position rows (their MFMA fragments stay in registers for the
//           whole block: P rows do not depend on the chunk) and computes band^T = P . (q+v)^T for all
//           64 queries, written skewed (query i, key j at column j + 4, the rel_shift) into the buffer;
//   scores: wave (query group, key parity) computes S^T = K . (q+u)^T over 10 of the 20 key subtiles
//           with the skewed band as the MFMA C operand; exact softmax with the partner wave's max /
//           sum exchanged through LDS; probabilities (bf16, as p_attn under autocast) into the buffer;
//   P.V:    wave w computes O^T for head dims 16w .. 16w+15 and all 64 queries, V^T fragments read
//           straight from a transposed V copy in global memory (vt_transpose_kernel after the QKV
//           GEMM: 16-B fragment loads, issued a chunk ahead) -- V never needs LDS.
// Per chunk every KV row, P row and query is read from L2 / LDS once per block, not once per wave.
#include <algorithm>

#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

namespace {
constexpr int A8_RING_MAX = 320;                  // ring rows = W (<= 320, multiple of 64)
constexpr int A8_KROW = 256;                      // bytes per K row (128 dims bf16)
constexpr int A8_BAND_PITCH = 336;                // band buffer columns per query (bf16)
constexpr int A8_PROB_PITCH = 328;                // probability columns per query (bf16)
constexpr int A8_K_BYTES = A8_RING_MAX * A8_KROW;                 // 80 KiB
constexpr int A8_B_BYTES = 64 * A8_BAND_PITCH * 2;                // 42 KiB (>= 64 * A8_PROB_PITCH * 2)
constexpr int A8_Q_BYTES = 64 * 256;                              // (q+u) or (q+v): 16 KiB each
constexpr int A8_LDS = A8_K_BYTES + A8_B_BYTES + 2 * A8_Q_BYTES + 2048;
static_assert(64 * A8_PROB_PITCH * 2 <= A8_B_BYTES, "probabilities alias the band buffer");
static_assert(A8_LDS <= 160 * 1024, "LDS");

typedef bf16 bf16x4_ __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));

CFM_DEV int sw256(int row, int ch) { return row * 256 + ((ch ^ (row & 15)) << 4); }
CFM_DEV unsigned pk2(float a, float b) {
  typedef bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, (b2){(bf16)a, (bf16)b});
}
}  // namespace

// V of the KV stream ([rows][H][K dk | V dk], dk = 128) -> V^T [H][128][vt_ld].  Each thread
// transposes an 8-row x 8-dim bf16 block in registers (8 x 16-B loads, 32 v_perm_b32, 8 x 16-B
// stores): a wave's loads cover 2 full 256-B V rows per load slot, its stores 64-B runs per dim.
// Rows past kv_rows are not written (never read).
__global__ __launch_bounds__(256) void vt_transpose_kernel(const bf16* __restrict__ kv, int kv_rows, int H,
                                                           bf16* __restrict__ vt, int vt_ld) {
  const int tid = threadIdx.x, h = blockIdx.y;
  const int dg = tid & 15, rg = tid >> 4;             // 16 dim groups x 16 row groups (128 rows per block)
  const int r0 = blockIdx.x * 128 + rg * 8, d0 = dg * 8;
  if (r0 >= kv_rows) return;
  const int d = H * 128;
  u32x4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    v[i] = *reinterpret_cast<const u32x4*>(kv + (size_t)min(r0 + i, kv_rows - 1) * 2 * d + h * 256 + 128 + d0);
#pragma unroll
  for (int k = 0; k < 8; ++k) {   // output dim d0 + k: rows r0 .. r0 + 7
    u32x4 o;
    // word j = (row 2j, row 2j+1) of dim k: the low / high halves of word k/2 of both rows
    const unsigned sel = (k & 1) ? 0x07060302u : 0x05040100u;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_perm(v[2 * j + 1][k >> 1], v[2 * j][k >> 1], sel);
    *reinterpret_cast<u32x4*>(vt + ((size_t)h * 128 + d0 + k) * vt_ld + r0) = o;
  }
}

// NT = W / 64 key tiles per window (W = L + C + R; 5 at C = 64, L = R = 128)
template <int NT, int VAR>
__global__ __launch_bounds__(512, 1) void chunk_attention_a128_kernel(
    const bf16* __restrict__ Q, const bf16* __restrict__ KV, int kv_rows, const bf16* __restrict__ VT, int vt_ld,
    const bf16* __restrict__ P, int p_rows, int p_ld, const float* __restrict__ pos_u, const float* __restrict__ pos_v,
    const int32_t* __restrict__ desc, int n_chunks, int H, int nch, bf16* __restrict__ out) {
  constexpr int W = 64 * NT, NSUB = 2 * NT;   // key subtiles per score wave (of 4 * NT)
  __shared__ __attribute__((aligned(16))) char smem[A8_LDS];
  char* kr = smem;
  char* bb = smem + A8_K_BYTES;                       // band, then probabilities
  char* qu_s = bb + A8_B_BYTES;
  char* qv_s = qu_s + A8_Q_BYTES;
  float* xch = reinterpret_cast<float*>(qv_s + A8_Q_BYTES);   // [max | sum][2 key halves][64 queries]
  float* uv = xch + 256;                                        // pos_bias_u / v of head h [2][128]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y;
  const int d = H * 128;
  const int c0 = blockIdx.x * nch, c1 = min(c0 + nch, n_chunks);
  if (c0 >= c1) return;
  const int RING = W;
  const float scale = 0.08838834764831845f;   // 1 / sqrt(128)
  const float L2E = 1.4426950408889634f;

  // ---- the wave's relative-position rows 48w .. 48w+47 (fragments for the whole block)
  bf16x8 pf[3][4];
#pragma unroll
  for (int rs = 0; rs < 3; ++rs) {
    const int prow = 48 * w + 16 * rs + fr;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      pf[rs][s] = prow < p_rows ? *reinterpret_cast<const bf16x8*>(P + (size_t)prow * p_ld + h * 128 + 32 * s + 8 * g)
                                : (bf16x8){};
  }
  // ---- staging helpers: 16-B pieces; a thread owns pieces tid and tid + 512 of a 64-row block
  const int kvb = desc[(size_t)c0 * AD_INTS + AD_KV_ROW0];
  auto load_k = [&](int frow, int ch) {
    return *reinterpret_cast<const u32x4*>(KV + (size_t)min(max(frow, 0), kv_rows - 1) * (2 * d) + h * 256 + ch * 8);
  };
  // q pieces: chunk c's query r, 16-B chunk ch -> (q+u), (q+v) bf16 (bias added in f32)
  auto load_q = [&](int c, int idx) {
    const int r = idx >> 4, ch = idx & 15;
    return *reinterpret_cast<const u32x4*>(Q + ((size_t)c * 64 + r) * d + h * 128 + ch * 8);
  };
  auto store_q = [&](int idx, const u32x4& raw) {
    const int r = idx >> 4, ch = idx & 15;
    const bf16x8 q = __builtin_bit_cast(bf16x8, raw);
    bf16x8 a, b;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float qf = (float)q[e];
      a[e] = (bf16)(qf + uv[ch * 8 + e]);
      b[e] = (bf16)(qf + uv[128 + ch * 8 + e]);
    }
    *reinterpret_cast<bf16x8*>(qu_s + sw256(r, ch)) = a;
    *reinterpret_cast<bf16x8*>(qv_s + sw256(r, ch)) = b;
  };
  // ---- prologue: the biases, the first window's K rows, the first chunk's queries
  if (tid < 256) uv[tid] = (tid < 128 ? pos_u : pos_v)[h * 128 + (tid & 127)];
  __syncthreads();
  for (int idx = tid; idx < RING * 16; idx += 512) {
    const int r = idx >> 4, ch = idx & 15;
    *reinterpret_cast<u32x4*>(kr + sw256(r, ch)) = load_k(kvb + r, ch);
  }
  for (int idx = tid; idx < 64 * 16; idx += 512) store_q(idx, load_q(c0, idx));

  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  const unsigned bb_lds = lds0 + A8_K_BYTES;
  const int qg = w & 3, kh = w >> 2;        // score phase: query group, key parity
  // V^T fragments of one chunk: dims 16w + fr, keys 32ks + 8g .. +7 (16 B each)
  bf16x8 vf[2 * NT];
  auto load_vt = [&](int c) {
    const bf16* vp = VT + ((size_t)h * 128 + 16 * w + fr) * vt_ld + (size_t)(kvb + (c - c0) * 64) + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 2 * NT; ++ks) {
      if constexpr (VAR == 13) vf[ks] = (bf16x8){};   // timing only: no V^T loads
      else vf[ks] = *reinterpret_cast<const bf16x8*>(vp + 32 * ks);
    }
  };
  __syncthreads();

  for (int c = c0; c < c1; ++c) {
    const int key_lo = desc[(size_t)c * AD_INTS + AD_KEY_LO], key_hi = desc[(size_t)c * AD_INTS + AD_KEY_HI];
    const int rb = ((c - c0) * 64) % RING;   // ring slot of window key 0
    // prefetch the next chunk's 64 new K rows and its queries into registers
    const bool more = c + 1 < c1;
    u32x4 nk[2], nq[2];
    if (more) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int idx = tid + 512 * k;
        nk[k] = load_k(kvb + (c + 1 - c0) * 64 + W - 64 + (idx >> 4), idx & 15);
        nq[k] = load_q(c + 1, idx);
      }
    }
    // ---- band^T[r][i] = P[r] . (q_i + v) for the wave's rows, all 64 queries, written skewed:
    // query i's value for P row r lands at column r + i - 59 (key j = r - 63 + i reads column j + 4)
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      bf16x8 qvf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) qvf[s] = *reinterpret_cast<const bf16x8*>(qv_s + sw256(16 * qs + fr, 4 * s + g));
#pragma unroll
      for (int rs = 0; rs < 3; ++rs) {
        f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (VAR != 10) {
#pragma unroll
          for (int s = 0; s < 4; ++s) a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[rs][s], qvf[s], a, 0, 0, 0);
        }
        const int i = 16 * qs + fr;
        const int col = 48 * w + 16 * rs + 4 * g + i - 59;
        if (col >= 1 && col <= W + 3) {   // groups that reach a read column j + 4, j in [0, W)
          const unsigned addr = bb_lds + 2u * (unsigned)(i * A8_BAND_PITCH + col);   // 2-B aligned
          if constexpr (VAR == 3)   // A/B: one unaligned ds_write_b64 (replayed by the LDS)
            asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"((u32x2_){pk2(a[0], a[1]), pk2(a[2], a[3])}) : "memory");
          else
            lds_store_4bf16_a2(addr, pk2(a[0], a[1]), pk2(a[2], a[3]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the asm band writes (opaque to the compiler)
    __syncthreads();
    // ---- scores S^T[key][query] for query group qg, key subtiles kh, kh + 2, ..., (+ band as C)
    bf16x8 quf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) quf[s] = *reinterpret_cast<const bf16x8*>(qu_s + sw256(16 * qg + fr, 4 * s + g));
    const int qi = 16 * qg + fr;
    // interior chunks see the whole window: no per-score mask (wave-uniform)
    const bool need_mask = __builtin_amdgcn_readfirstlane(key_lo != 0 || key_hi != W) != 0;
    f32x4 S[NSUB];
    float mx = -INFINITY;
    // subtiles in pairs: two independent MFMA chains interleaved, the pair's fragments loaded together
    // (VAR 0: one subtile at a time)
    constexpr int PAIR = VAR == 0 ? 1 : 2;
#pragma unroll
    for (int t0 = 0; t0 < NSUB; t0 += PAIR) {
      bf16x8 kf[PAIR][4];
      f32x4 a[PAIR];
#pragma unroll
      for (int u = 0; u < PAIR; ++u) {
        const int j0 = 16 * (kh + 2 * (t0 + u));
        const bf16x4_ bv = *reinterpret_cast<const bf16x4_*>(bb + 2 * (qi * A8_BAND_PITCH + j0 + 4 * g + 4));
        int slot = rb + j0;
        if (slot >= RING) slot -= RING;
#pragma unroll
        for (int s = 0; s < 4; ++s) kf[u][s] = *reinterpret_cast<const bf16x8*>(kr + sw256(slot + fr, 4 * s + g));
        a[u] = (f32x4){(float)bv[0], (float)bv[1], (float)bv[2], (float)bv[3]};
      }
      if constexpr (VAR != 11) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int u = 0; u < PAIR; ++u) a[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[u][s], quf[s], a[u], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < PAIR; ++u) S[t0 + u] = a[u] * scale;
      __builtin_amdgcn_sched_barrier(0);   // keep each group's fragment loads next to its MFMAs
    }
    if (need_mask) {
#pragma unroll
      for (int t = 0; t < NSUB; ++t)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int j = 16 * (kh + 2 * t) + 4 * g + rr;
          if (j < key_lo || j >= key_hi) S[t][rr] = -INFINITY;
        }
    }
#pragma unroll
    for (int t = 0; t < NSUB; ++t) mx = fmaxf(mx, fmaxf(fmaxf(S[t][0], S[t][1]), fmaxf(S[t][2], S[t][3])));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    if (g == 0) xch[kh * 64 + qi] = mx;
    load_vt(c);   // V^T fragments of this chunk: in flight during the softmax
    __syncthreads();
    // ---- exact softmax: the partner wave's max, probabilities into the (now free) band buffer
    float m = fmaxf(xch[qi], xch[64 + qi]);
    if (m == -INFINITY) m = 0.f;   // fully masked query: every p = 0, output 0 (reference: NaN -> 0)
    const float ml = m * L2E;
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < NSUB; ++t) {
      const int j0 = 16 * (kh + 2 * t);
      float p[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        p[rr] = __builtin_amdgcn_exp2f(fmaf(S[t][rr], L2E, -ml));
        sum += p[rr];
      }
      *reinterpret_cast<u32x2_*>(bb + 2 * (qi * A8_PROB_PITCH + j0 + 4 * g)) = (u32x2_){pk2(p[0], p[1]), pk2(p[2], p[3])};
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    // (xch reads above happen before any wave passes the next barrier; sums go to a second slot)
    if (g == 0) xch[128 + kh * 64 + qi] = sum;
    // the next chunk's K rows replace this chunk's keys 0..63 (read by every wave before the last
    // barrier) and its queries replace this chunk's (q+u) / (q+v)
    if (more) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int idx = tid + 512 * k;
        int slot = rb + (idx >> 4);
        if (slot >= RING) slot -= RING;
        *reinterpret_cast<u32x4*>(kr + sw256(slot, idx & 15)) = nk[k];
        store_q(idx, nq[k]);
      }
    }
    __syncthreads();
    // ---- O^T[dim 16w + 4g + rr][query 16qs + fr] = sum_keys V^T . P^T
    f32x4 O[4];
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) O[qs] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2 * NT; ++ks) {
#pragma unroll
      for (int qs = 0; qs < 4; ++qs) {
        const bf16x8 pb = *reinterpret_cast<const bf16x8*>(bb + ((16 * qs + fr) * A8_PROB_PITCH + 32 * ks + 8 * g) * 2);
        if constexpr (VAR != 12) O[qs] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[ks], pb, O[qs], 0, 0, 0);
        else O[qs][0] += (float)pb[0];
      }
    }
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      const int i = 16 * qs + fr;
      const float l = xch[128 + i] + xch[192 + i];
      const float inv = l > 0.f ? 1.f / l : 0.f;
      bf16* op = out + ((size_t)c * 64 + i) * d + h * 128 + 16 * w + 4 * g;
      *reinterpret_cast<bf16x4_*>(op) = (bf16x4_){(bf16)(O[qs][0] * inv), (bf16)(O[qs][1] * inv),
                                                  (bf16)(O[qs][2] * inv), (bf16)(O[qs][3] * inv)};
    }
    __syncthreads();   // the probabilities and sums are dead: the next chunk's band may overwrite them
  }
}

int vt_transpose_bf16(const bf16* kv, int kv_rows, int H, bf16* vt, int vt_ld, hipStream_t st) {
  if (kv_rows <= 0) return 0;
  if (kv_rows % 8) return (int)hipErrorInvalidValue;   // whole 8-row groups (masked plans: L + 64N + R)
  hipLaunchKernelGGL(vt_transpose_kernel, dim3((kv_rows + 127) / 128, H), dim3(256), 0, st, kv, kv_rows, H, vt, vt_ld);
  CFM_CHECK_LAUNCH();
  return 0;
}

bool attention_a128_eligible(int C, int W, int p_rows, int dk) {
  return dk == 128 && C == 64 && W >= 64 && W <= A8_RING_MAX && W % 64 == 0 && p_rows <= 384;
}

int chunk_attention_masked_a128(const bf16* q, const bf16* kv, int kv_rows, const bf16* vt, int vt_ld, const bf16* P,
                                int p_rows, int p_ld, const float* pos_u, const float* pos_v, const int32_t* desc,
                                int n_chunks, int H, int C, int W, bf16* out, hipStream_t st, int var) {
  if (!attention_a128_eligible(C, W, p_rows, 128) || n_chunks <= 0) return -1;
  const int n_cu = cu_count();
  // one block per CU sweeping consecutive chunks of one head (one K-ring prologue per block)
  int nch = (int)(((long long)n_chunks * H + n_cu - 1) / n_cu);
  nch = std::max(4, nch);
  const dim3 grid((n_chunks + nch - 1) / nch, H);
#define A128(NT_, V_)                                                                                                \
  hipLaunchKernelGGL((chunk_attention_a128_kernel<NT_, V_>), grid, dim3(512), 0, st, q, kv, kv_rows, vt, vt_ld, P,   \
                     p_rows, p_ld, pos_u, pos_v, desc, n_chunks, H, nch, out)
  // var ("attn128_var" model option, A/B): 1 = paired score subtiles (default), 0 = one at a time
  switch (W / 64) {
    case 1: A128(1, 1); break;
    case 2: A128(2, 1); break;
    case 3: A128(3, 1); break;
    case 4: A128(4, 1); break;
    default:
      switch (var) {   // 10-13: timing-only diagnostics (no band / score / P.V MFMAs, no V^T loads)
        case 0: A128(5, 0); break;
        case 3: A128(5, 3); break;
        case 10: A128(5, 10); break;
        case 11: A128(5, 11); break;
        case 12: A128(5, 12); break;
        case 13: A128(5, 13); break;
        default: A128(5, 1); break;
      }
      break;
  }
#undef A128
  CFM_CHECK_LAUNCH();
  return 0;
}

}  // namespace cfm
