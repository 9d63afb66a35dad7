// Masked-batch chunk attention, head_dim 64, bf16, C = 64: 32 queries per wave, one wave per SIMD.
//
// Reference: ChunkAttentionWithRelativeRightContext.forward_parallel_chunk (attention.py:420-505) with
// rel_shift (242-266) and forward_attention (104-150): for chunk n, head h, query i, window key j,
//   s(i, j) = ((q_i + u_h) . k_j + (q_i + v_h) . P[C - 1 - i + j]) / sqrt(64),
//   keys outside [lo, hi) -> -inf, softmax over the L + C + R window, out_i = sum_j p_ij v_j.
//
// Why a second dk = 64 kernel: the 8-wave ring kernel (attention.hip) gives each wave 16 queries, so
// every K, V and P fragment is read from LDS by 4 waves per chunk and the LDS pipe, not the MFMA pipe,
// sets its pace (SQ_LDS_IDX_ACTIVE ~85% of the kernel's cycles).  Here one 256-thread block (4 waves,
// one per SIMD, 512 registers each) sweeps a run of consecutive chunks of one head, two chunks per
// iteration, and each wave owns 32 queries (two 16-query groups q = 0, 1):
//   * P rows stay in AGPRs for the whole block: a wave's queries need the same 22 relative-position
//     tiles of 16 rows in every chunk (P does not depend on the chunk), so P never touches LDS;
//   * every K fragment (scores) and V^T fragment (P.V) read from LDS feeds both query groups;
//   * K and V rows live in LDS rings in their natural [key][dim] layout (16-B chunks XOR-swizzled by
//     row: conflict-free for the b128 K reads and the ds_read_b64_tr_b16 V^T reads), filled by
//     LDS-DMA (global_load_lds) one pair of chunks ahead, with no register staging;
//   * the rel_shift: each band tile band^T = P . (q+v)^T (16 P rows x 16 queries, f32) is written to a
//     per-wave scratch at pitch 57 and read back at pitch 56 (the reshape trick of attention.py:242-266),
//     as the f32 C operand of the score MFMAs S^T = K . (q+u)^T (so S = ac + bd costs no VALU add);
//   * softmax online per 32-key half (running max over the query's 4 lanes by permlane swaps, O
//     rescaled only when a maximum grows), probabilities as bf16 B operands straight from the score
//     registers, the denominator as one more MFMA against a ones row.
// 1/sqrt(64) = 2^-3 is folded into q+u and q+v (exact in bf16 and f32).
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

namespace {
typedef short s16x4_q __attribute__((ext_vector_type(4)));
typedef bf16 bf16x4_q __attribute__((ext_vector_type(4)));
constexpr int Q32_PR = 56;                              // band scratch read pitch (floats; conflict-free b128 reads)
constexpr int Q32_PW = Q32_PR + 1;                      // write pitch: the rel_shift reshape
constexpr int Q32_BQ = 912;                             // floats per query group (max write index 903; 16-B multiple)
constexpr int Q32_BW = 2 * Q32_BQ;                      // per wave

CFM_DEV int q32_swz(int row) { return ((row >> 1) & 3) << 1; }   // 16-B chunk XOR of ring row `row`
CFM_DEV unsigned q32_pk(float a, float b) {
  typedef bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, (b2){(bf16)a, (bf16)b});
}
// D = A (AGPR) x B + C, 16x16x32 bf16: the P fragments live in the AGPR half of the register file
// a bf16 fragment moved into the AGPR half of the register file (MFMA A/B operands may be AGPRs):
// keeps the query operands out of the VGPRs the scores and the P.V accumulators need
CFM_DEV bf16x8 to_agpr(const bf16x8& v) {
  const u32x4 x = __builtin_bit_cast(u32x4, v);
  unsigned a0, a1, a2, a3;
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a0) : "v"(x[0]));
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a1) : "v"(x[1]));
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a2) : "v"(x[2]));
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a3) : "v"(x[3]));
  return __builtin_bit_cast(bf16x8, (u32x4){a0, a1, a2, a3});
}
// (not volatile: a pure function of its operands, so hipcc may schedule it like any other instruction)
CFM_DEV f32x4 mfma_pa(const bf16x8& a, const bf16x8& b, f32x4 c) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "a"(a), "v"(b));
  return c;
}
CFM_DEV f32x4 mfma_pa0(const bf16x8& a, const bf16x8& b) {   // C = 0 (inline constant)
  f32x4 c;
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=v"(c) : "a"(a), "v"(b));
  return c;
}
// the running maximum is raised only when a half's maximum exceeds it by more than this (natural
// units; 2^8 in probability): exp(s - m) <= 256 stays exact enough in bf16 / f32, and the O rescale
// (40 multiplies) runs for few halves instead of nearly every one (cdna_hip_programming.md T13)
constexpr float Q32_DEFER = 5.545177444479562f;   // 8 / log2(e)
}  // namespace

// NH = W / 32 key halves per window (2..10; W = L + 64 + R); PIPE bit 0: software-pipelined by one
// half (else one half after the other), bit 1: branch-free O rescale (alpha = 1 when no maximum grew:
// one basic block per half for the scheduler); DG: the timing-only `diag` hooks are compiled in (the
// production instantiation has no diag branch inside the half loop)
template <int NH, int PIPE, bool DG>
__global__ __launch_bounds__(256, 1) void chunk_attention_q32_kernel(
    const bf16* __restrict__ Q, const bf16* __restrict__ KV, int kv_rows, const bf16* __restrict__ P, int p_rows,
    int p_ld, const float* __restrict__ pos_u, const float* __restrict__ pos_v, const int32_t* __restrict__ desc,
    int n_chunks, int H, int nch, bf16* __restrict__ out, int diag_arg) {
  const int diag = DG ? diag_arg : 0;
  // diag (timing only, model option "attn_diag" >= 64): bit 0 no band MFMAs / writes, bit 1 no exp +
  // P.V, bit 2 no score MFMAs, bit 3 no LDS-DMA of the next pair (stale rows)
  constexpr int W = 32 * NH;
  constexpr int RING = W + 192;          // ring rows: a pair's windows (W + 64) + the next pair's 128 new rows
  constexpr int NPT = 2 * NH + 2;        // P tiles per wave
  __shared__ __attribute__((aligned(16))) char smem[2 * RING * 128 + 4 * Q32_BW * 4];
  char* kr = smem;
  char* vr = smem + RING * 128;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  float* bs = reinterpret_cast<float*>(smem + 2 * RING * 128) + w * Q32_BW;
  const int h = blockIdx.y, d = H * 64;
  const int c0 = blockIdx.x * nch, c1 = min(c0 + nch, n_chunks);
  if (c0 >= c1) return;
  const int i0 = 32 * (w & 1);            // the wave's first query in its chunk
  const int kvb = desc[(size_t)c0 * AD_INTS + AD_KV_ROW0];

  // ---- LDS-DMA of 8 KV rows (kind 0 = K, 1 = V): flat rows frow0.. -> ring rows rr0.. (rr0 % 8 == 0);
  // lane l writes LDS bytes 16 l of the piece: row l >> 3, 16-B slot l & 7 holding chunk slot ^ swz(row)
  auto dma8 = [&](int kind, int frow0, int rr0) {
    const int r = lane >> 3;
    const int ch = (lane & 7) ^ q32_swz(rr0 + r);
    const int frow = min(frow0 + r, kv_rows - 1);
    const bf16* src = KV + (size_t)frow * (2 * d) + h * 128 + kind * 64 + ch * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)((kind ? vr : kr) + rr0 * 128), 16, 0, 0);
  };
  // rows [x0, x1) of the window sequence starting at chunk c0 (flat row kvb + x), 8-row pieces over the waves
  auto dma_rows = [&](int x0, int x1) {
    const int np = (x1 - x0) >> 3;
    for (int p = w; p < 2 * np; p += 4) {
      const int kind = p >= np, x = x0 + 8 * (p - kind * np);
      dma8(kind, kvb + x, x % RING);
    }
  };
  // first pair's windows
  dma_rows(0, W + (c0 + 1 < c1 ? 64 : 0));

  // ---- P tiles of this wave's queries (rows 32 - i0 + 16 n + fr), for the whole block, in AGPRs
  // (loaded straight into AGPRs; rows past the table are clamped: P row 63 - i + j never exceeds
  // W + 62 for a valid (query, key) pair, so a clamped row only reaches skew slots nobody reads)
  bf16x8 pf[NPT][2];
#pragma unroll
  for (int n = 0; n < NPT; ++n) {
    const int prow = min(32 - i0 + 16 * n + fr, p_rows - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
      asm volatile("global_load_dwordx4 %0, %1, off"
                   : "=a"(pf[n][s])
                   : "v"(P + (size_t)prow * p_ld + h * 64 + 32 * s + 8 * g));
  }
  // ---- raw q of the wave's first chunk, and its key range
  // (the next chunk's q waits in AGPRs: asm loads, covered by the s_waitcnt vmcnt(0) that ends every
  // iteration)
  bf16x8 qn[2][2];
  auto load_q = [&](int c) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        asm volatile("global_load_dwordx4 %0, %1, off"
                     : "=a"(qn[q][s])
                     : "v"(Q + ((size_t)c * 64 + i0 + 16 * q + fr) * d + h * 64 + 32 * s + 8 * g));
  };
  int klo_n = 0, khi_n = W;
  {
    const int c = min(c0 + (w >> 1), c1 - 1);
    load_q(c);
    klo_n = desc[(size_t)c * AD_INTS + AD_KEY_LO];
    khi_n = desc[(size_t)c * AD_INTS + AD_KEY_HI];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane LDS addresses (bytes)
  const int bw_lane = fr * Q32_PW + 4 * g + 1;     // band write base (floats): + 16 pt + rr
  const int br_lane = fr * Q32_PR + 4 * g + 16;    // band read base (floats): + 16 st2
  // K fragments (A operands): row (subtile base, a multiple of 16) + fr, 16-B chunk 4s + g, swizzled
  int k_lane[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) k_lane[s] = fr * 128 + 16 * ((4 * s + g) ^ q32_swz(fr));
  // V^T fragments (ds_read_b64_tr_b16): lane i of 16-lane group g supplies row 4g + (i >> 2), dims
  // 16 dt + 4 (i & 3) .. +3, i.e. 16-B chunk 2 dt + ((i & 3) >> 1) at byte 8 (i & 1) of it
  int v_lane[4];
  {
    const int tr_row = 4 * g + ((lane & 15) >> 2);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      v_lane[dt] = tr_row * 128 + 16 * ((2 * dt + ((lane & 3) >> 1)) ^ q32_swz(tr_row)) + 8 * (lane & 1);
  }
  // max over the 4 lanes of a query (fr, fr + 16, fr + 32, fr + 48) by two permlane swaps
  auto qmax4 = [](float x) {
    const auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x),
                                                    false, false);
    x = fmaxf(__builtin_bit_cast(float, (unsigned)a[0]), __builtin_bit_cast(float, (unsigned)a[1]));
    const auto b = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x),
                                                    false, false);
    return fmaxf(__builtin_bit_cast(float, (unsigned)b[0]), __builtin_bit_cast(float, (unsigned)b[1]));
  };
  const bf16 one_or_zero = (bf16)(fr == 0 ? 1.f : 0.f);
  const bf16x8 ones = (bf16x8){one_or_zero, one_or_zero, one_or_zero, one_or_zero,
                               one_or_zero, one_or_zero, one_or_zero, one_or_zero};

  for (int cp = c0; cp < c1; cp += 2) {
    const int c = cp + (w >> 1);
    const bool act = c < c1;
    const int key_lo = klo_n, key_hi = khi_n;
    // ---- the next pair's 128 new rows by LDS-DMA (they replace the rows the previous pair dropped)
    if (cp + 2 < c1 && !(diag & 8)) {
      const int x0 = (cp - c0) * 64 + W + 64;
      dma_rows(x0, x0 + (cp + 3 < c1 ? 128 : 64));
    }
    bf16x8 qr[2][2];
#pragma unroll
    for (int q = 0; q < 2; ++q) { qr[q][0] = qn[q][0]; qr[q][1] = qn[q][1]; }
    {
      const int cn = c + 2;
      if (cn < c1) load_q(cn);
      const int cc = min(cn, c1 - 1);
      klo_n = desc[(size_t)cc * AD_INTS + AD_KEY_LO];
      khi_n = desc[(size_t)cc * AD_INTS + AD_KEY_HI];
    }
    if (act) {
      const int rb = (c - c0) * 64 % RING;   // ring row of window key 0 (a multiple of 32)
      auto ring32 = [&](int j) { const int r = rb + j; return r >= RING ? r - RING : r; };   // j % 32 == 0
      // ---- (q+u)/8 and (q+v)/8 as bf16 B fragments
      bf16x8 qu[2][2], qv[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f32x4 u0 = *reinterpret_cast<const f32x4*>(pos_u + h * 64 + 32 * s + 8 * g);
        const f32x4 u1 = *reinterpret_cast<const f32x4*>(pos_u + h * 64 + 32 * s + 8 * g + 4);
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(pos_v + h * 64 + 32 * s + 8 * g);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(pos_v + h * 64 + 32 * s + 8 * g + 4);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            // q / 8 + u / 8 in one fma = (q + u) / 8 rounded once (a power-of-two scale commutes with
            // the rounding), the value the two-step form gives
            const float qf = (float)qr[q][s][e];
            qu[q][s][e] = (bf16)fmaf(qf, 0.125f, (e < 4 ? u0[e] : u1[e - 4]) * 0.125f);
            qv[q][s][e] = (bf16)fmaf(qf, 0.125f, (e < 4 ? v0[e] : v1[e - 4]) * 0.125f);
          }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          qu[q][s] = to_agpr(qu[q][s]);
          qv[q][s] = to_agpr(qv[q][s]);
        }
      // interior chunks see the whole window: the masking code exists only in the edge-chunk copy
      const bool need_mask = __builtin_amdgcn_readfirstlane(key_lo != 0 || key_hi != W) != 0;
      auto body = [&](auto MASKc) {
      constexpr bool MASK = decltype(MASKc)::value;

      // band tiles of half hf: q = 0 uses P tiles 2hf+1 .. 2hf+3, q = 1 tiles 2hf .. 2hf+2 (pt = 0..2);
      // tile pt = 0 equals the previous half's pt = 2 (carried in registers)
      f32x4 bnd[2][3];
      auto band = [&](auto HFc, bool carry) {
        constexpr int hf = decltype(HFc)::value;
        if (diag & 1) return;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int pt = 0; pt < 3; ++pt) {
            if (pt == 0 && carry) { bnd[q][0] = bnd[q][2]; continue; }
            const int n = 2 * hf + pt + (q == 0 ? 1 : 0);
            bnd[q][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                pf[n][1], qv[q][1], __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[n][0], qv[q][0], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0),
                0, 0, 0);
          }
        // skewed write (pitch 57; read back at pitch 56 by scores())
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int pt = 0; pt < 3; ++pt)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) bs[q * Q32_BQ + bw_lane + 16 * pt + rr] = bnd[q][pt][rr];
      };

      // online softmax state per query group: running max m (all 4 lanes of a query hold it), O^T
      // accumulators (dims 16 dt + 4g + rr of query fr) and the denominator row (ones-row MFMA)
      float m[2] = {-INFINITY, -INFINITY};
      f32x4 O[2][4], Ol[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        Ol[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) O[q][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      // the LDS operands of half hf (K fragments, skewed band C operands), read one half ahead
      struct HalfOps { bf16x8 kf[2][2]; f32x4 bc[2][2]; };
      auto load_ops = [&](int hf) {
        HalfOps o;
        const int kb = ring32(32 * hf);
#pragma unroll
        for (int st2 = 0; st2 < 2; ++st2)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            o.kf[st2][s] = *reinterpret_cast<const bf16x8*>(kr + (kb + 16 * st2) * 128 + k_lane[s]);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int st2 = 0; st2 < 2; ++st2)
            o.bc[q][st2] = *reinterpret_cast<const f32x4*>(bs + q * Q32_BQ + br_lane + 16 * st2);
        return o;
      };
      band(std::integral_constant<int, 0>{}, false);
      // V^T fragments of half hf's P.V: two transposed reads per 16-dim tile (rows kb + 4g + ..,
      // kb + 16 + 4g + ..)
      auto load_va = [&](int hf, bf16x8 (&va)[4]) {
        const char* vb = vr + ring32(32 * hf) * 128;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const s16x4_q lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_q*)(vb + v_lane[dt]));
          const s16x4_q hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4_q*)(vb + v_lane[dt] + 16 * 128));
          const bf16x4_q l4 = __builtin_bit_cast(bf16x4_q, lo), h4 = __builtin_bit_cast(bf16x4_q, hi);
          va[dt] = (bf16x8){l4[0], l4[1], l4[2], l4[3], h4[0], h4[1], h4[2], h4[3]};
        }
      };
      // scores S^T = K . (q+u)^T + skewed band (keys 32hf + 16 st2 + 4g + rr, query i0 + 16q + fr)
      auto scores = [&](const HalfOps& o, f32x4 (&S)[2][2]) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int st2 = 0; st2 < 2; ++st2) {
            if (diag & 4) { S[st2][q] = o.bc[q][st2] + (float)o.kf[st2][0][0]; continue; }
            f32x4 a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o.kf[st2][0], qu[q][0], o.bc[q][st2], 0, 0, 0);
            S[st2][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(o.kf[st2][1], qu[q][1], a, 0, 0, 0);
          }
      };
      auto mask = [&](int hf, f32x4 (&S)[2][2]) {
        if constexpr (MASK) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int st2 = 0; st2 < 2; ++st2)
#pragma unroll
              for (int rr = 0; rr < 4; ++rr) {
                const int j = 32 * hf + 16 * st2 + 4 * g + rr;
                S[st2][q][rr] = (j < key_lo || j >= key_hi) ? -INFINITY : S[st2][q][rr];
              }
        }
      };
      // running max over the query's 4 lanes (permlane swaps, no LDS); O rescaled when it is raised;
      // returns m * log2(e) for the exps
      auto softmax_max = [&](bool first, const f32x4 (&S)[2][2], float (&ml)[2]) {
        bool grew = false;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float x = S[0][q][0];
#pragma unroll
          for (int st2 = 0; st2 < 2; ++st2)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) x = fmaxf(x, S[st2][q][rr]);
          x = qmax4(x);
          // raise the maximum only past the deferral margin (and always from -inf)
          const bool up = x > m[q] + Q32_DEFER;
          grew |= up;
          ml[q] = up ? x : m[q];
        }
        if constexpr (PIPE & 2) {
          if (!first) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              // 1 where the maximum stayed (exp2(0)), 0 while no key of the query was unmasked
              const float alpha = m[q] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m[q] - ml[q]) * 1.4426950408889634f);
              Ol[q] *= alpha;
#pragma unroll
              for (int dt = 0; dt < 4; ++dt) O[q][dt] *= alpha;
            }
          }
        } else if (!first && __builtin_amdgcn_ballot_w64(grew)) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            // pass-through terms at the old maximum, rescaled (0 while no key of the query was unmasked)
            const float alpha = m[q] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f((m[q] - ml[q]) * 1.4426950408889634f);
            Ol[q] *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) O[q][dt] *= alpha;
          }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          m[q] = ml[q];
          ml[q] = (ml[q] == -INFINITY ? 0.f : ml[q]) * 1.4426950408889634f;   // fully masked so far: p = 0
        }
      };
      // probabilities (bf16, keys in the score registers' order) as B fragments
      auto probs = [&](const f32x4 (&S)[2][2], const float (&ml)[2], bf16x8 (&pb)[2]) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int st2 = 0; st2 < 2; ++st2)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
              pb[q][4 * st2 + rr] = (bf16)__builtin_amdgcn_exp2f(fmaf(S[st2][q][rr], 1.4426950408889634f, -ml[q]));
      };
      auto pv = [&](const bf16x8 (&va)[4], const bf16x8 (&pb)[2]) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int q = 0; q < 2; ++q) O[q][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[dt], pb[q], O[q][dt], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 2; ++q) Ol[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[q], Ol[q], 0, 0, 0);
      };

      HalfOps cur = load_ops(0);
      if constexpr ((PIPE & 1) == 0) {
        // one half after the other: V^T reads, scores, the next half's band and operands, softmax, P.V
        sfor<0, NH>([&](auto HFc) {
          constexpr int hf = decltype(HFc)::value;
          bf16x8 va[4];
          load_va(hf, va);
          f32x4 S[2][2];
          scores(cur, S);
          // the next half's band, then its operands (its scratch writes follow this half's band reads
          // and precede the next reads in program order: the LDS serves one wave in order)
          if constexpr (hf + 1 < NH) {
            band(std::integral_constant<int, hf + 1>{}, true);
            cur = load_ops(hf + 1);
          }
          mask(hf, S);
          if (diag & 2) {   // timing only: keep the scores alive, skip the softmax and P.V
#pragma unroll
            for (int q = 0; q < 2; ++q) O[q][0] += S[0][q] + S[1][q] + (float)va[0][0];
            return;
          }
          float ml[2];
          softmax_max(hf == 0, S, ml);
          bf16x8 pb[2];
          probs(S, ml, pb);
          pv(va, pb);
        });
      } else {
        // software-pipelined by one half: iteration hf runs half hf + 1's score MFMAs beside half hf's
        // max, then half hf's exps beside half hf + 2's band MFMAs and half hf's P.V
        f32x4 Sn[2][2];
        scores(cur, Sn);
        if constexpr (NH > 1) {
          band(std::integral_constant<int, 1>{}, true);
          cur = load_ops(1);
        }
        bf16x8 va[4];
        load_va(0, va);
        sfor<0, NH>([&](auto HFc) {
          constexpr int hf = decltype(HFc)::value;
          f32x4 S[2][2];
#pragma unroll
          for (int q = 0; q < 2; ++q) { S[0][q] = Sn[0][q]; S[1][q] = Sn[1][q]; }
          if constexpr (hf + 1 < NH) scores(cur, Sn);
          mask(hf, S);
          float ml[2];
          softmax_max(hf == 0, S, ml);
          bf16x8 pb[2];
          if (!(diag & 2)) probs(S, ml, pb);
          if constexpr (hf + 2 < NH) {
            band(std::integral_constant<int, hf + 2>{}, true);
            cur = load_ops(hf + 2);
          }
          if (!(diag & 2)) pv(va, pb);
          if constexpr (hf + 1 < NH) load_va(hf + 1, va);
        });
      }
      // ---- normalise and store: lane (query fr, g) holds dims 16 dt + 4g .. +3; permlane16 swaps give
      // each lane 8 contiguous dims, so a query row leaves as 16-B pieces
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float l = __shfl(Ol[q][0], fr, 64);
        const float inv = l > 0.f ? __builtin_amdgcn_rcpf(l) : 0.f;
        bf16* op = out + ((size_t)c * 64 + i0 + 16 * q + fr) * d + h * 64;
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const unsigned x0 = q32_pk(O[q][2 * pr][0] * inv, O[q][2 * pr][1] * inv),
                         x1 = q32_pk(O[q][2 * pr][2] * inv, O[q][2 * pr][3] * inv);
          const unsigned y0 = q32_pk(O[q][2 * pr + 1][0] * inv, O[q][2 * pr + 1][1] * inv),
                         y1 = q32_pk(O[q][2 * pr + 1][2] * inv, O[q][2 * pr + 1][3] * inv);
          const auto r0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
          *reinterpret_cast<u32x4*>(op + 32 * pr + 16 * (g & 1) + 8 * (g >> 1)) = (u32x4){r0[0], r1[0], r0[1], r1[1]};
        }
      }
      };
      if (need_mask) body(std::true_type{});
      else body(std::false_type{});
    }
    // the next pair's rows have landed (every wave's DMA) and every wave is done with this pair
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

bool attention_q32_eligible(int C, int W, int p_rows) {
  return C == 64 && W >= 64 && W <= 320 && W % 32 == 0 && p_rows <= W + 63;
}

int chunk_attention_masked_q32(const bf16* q, const bf16* kv, int kv_rows, const bf16* P, int p_rows, int p_ld,
                               const float* pos_u, const float* pos_v, const int32_t* desc, int n_chunks, int H, int C,
                               int W, bf16* out, hipStream_t st, int diag, int pipe) {
  if (!attention_q32_eligible(C, W, p_rows) || n_chunks <= 0) return -1;
  if (p_ld <= 0) p_ld = H * 64;
  // one block per CU (LDS-bound), a run of consecutive chunks of one head (even: two per iteration)
  int nch = (int)(((long long)n_chunks * H + cu_count() - 1) / cu_count());
  nch = max(4, (nch + 1) & ~1);
  const dim3 grid((n_chunks + nch - 1) / nch, H);
#define Q32L(NH_, PP_, DG_)                                                                                          \
  hipLaunchKernelGGL((chunk_attention_q32_kernel<NH_, PP_, DG_>), grid, dim3(256), 0, st, q, kv, kv_rows, P, p_rows, \
                     p_ld, pos_u, pos_v, desc, n_chunks, H, nch, out, diag)
  // the production shape (W = 320) also has the pipelining variants and the diag build; the others
  // only the default
#define Q32(NH_)                                                                                                     \
  if (NH_ != 10 || (pipe == 3 && !diag)) Q32L(NH_, 3, false);                                                        \
  else if (diag) Q32L(NH_, 3, true);                                                                                 \
  else if (pipe == 2) Q32L(NH_, 1, false);                                                                           \
  else Q32L(NH_, 0, false)
  switch (W / 32) {
    case 2: Q32(2); break;
    case 3: Q32(3); break;
    case 4: Q32(4); break;
    case 5: Q32(5); break;
    case 6: Q32(6); break;
    case 7: Q32(7); break;
    case 8: Q32(8); break;
    case 9: Q32(9); break;
    default: Q32(10); break;
  }
#undef Q32
#undef Q32L
  CFM_CHECK_LAUNCH();
  return 0;
}

}  // namespace cfm
