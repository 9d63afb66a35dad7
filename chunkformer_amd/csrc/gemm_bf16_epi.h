// Shared device helpers of the bf16 MFMA GEMM kernels (gemm_bf16.hip, gemm_wst.hip): LDS fragment
// reads, fast activations, the swapped-operand tile epilogue (bias-seeded accumulators, fused
// activation / QKV split / GLU, 16-B bf16 row stores).
#pragma once
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));

// ds_read_b128 as inline asm: hipcc's waitcnt pass cannot tell these reads from the in-flight
// LDS-DMA destinations and would insert s_waitcnt vmcnt(0) in front of them; the kernel orders
// them itself (explicit lgkmcnt(0) + barrier before the MFMA segment that consumes them).
template <int OFF>
CFM_DEV bf16x8 lds_read_b128(unsigned addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

// fast activations for the bf16 epilogue: v_exp_f32 + v_rcp_f32 (the results are rounded to bf16)
CFM_DEV float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x)); }
CFM_DEV float fast_silu(float x) { return x * fast_sigmoid(x); }

// Tile epilogue of one wave (128 x 64 of C).  With swapped operands acc[i][j] (n-block i of 16
// columns, m-block j of 16 rows) holds, in lane (fr, g), C[m = 16j + fr][n = 16i + 4g .. 4g+3];
// the bias is already in the accumulator (it seeds the tile).  bf16 outputs: n-blocks are
// paired (2p, 2p+1) and packed, then one v_permlane16_swap per dword leaves every lane with
// 8 contiguous columns, so each row segment of 32 columns is ONE 16-B store per lane
// (16 stores per tile instead of 32 8-B ones; the store tail is issue-bound).
//   after the swap lane g holds columns 16*(2p) + 16*(g & 1) + 8*(g >> 1) .. +7
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
CFM_DEV unsigned pack_bf16x2(float a, float b) {
  typedef bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, (b2){(bf16)a, (bf16)b});
}
// FMT: the 16-bit format of operands and outputs, 0 = bf16, 1 = f16 (the kernels move both as raw
// 16-bit lanes; only the MFMA and the output conversion differ)
template <int FMT>
CFM_DEV unsigned pack_h2(float a, float b) {
  if constexpr (FMT == 1) {
    typedef f16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, (h2){(f16)a, (f16)b});
  } else {
    return pack_bf16x2(a, b);
  }
}
template <int FMT>
CFM_DEV f32x4 mfma16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (FMT == 1)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int ACT>
CFM_DEV f32x4 act4(f32x4 v) {
  if constexpr (ACT == ACT_RELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
  }
  if constexpr (ACT == ACT_SILU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fast_silu(v[r]);
  }
  if constexpr (ACT == ACT_SILU_L2E) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = v[r] * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v[r]));
  }
  return v;
}
// store two packed 16-column blocks (x = block 0, y = block 1) of row `row` after the swap
template <bool NOST = false>
CFM_DEV void store_pair16(bf16* base, size_t ld, int row, int g, u32x2_t x, u32x2_t y, int sm = 0) {
  const auto r0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
  const int col = 16 * (g & 1) + 8 * (g >> 1);
  const u32x4 v = (u32x4){r0[0], r1[0], r0[1], r1[1]};
  u32x4* p = reinterpret_cast<u32x4*>(base + (size_t)row * ld + col);
  if constexpr (NOST) {   // timing experiment: values computed, not stored
    asm volatile("" ::"v"(r0[0]), "v"(r1[0]), "v"(r0[1]), "v"(r1[1]));
  } else {
    if (sm == 1)
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if (sm == 2)
      __builtin_nontemporal_store(v, p);
    else
      *p = v;
  }
}

// One wave's 16*MB x 64 piece of C: m0 = row of m-block 0 for this lane (row base + fr), nw = first
// column of the wave.
template <int EPI, int ACT, int MB, bool NOST = false, int FMT = 0>
CFM_DEV void wave_epilogue(f32x4 (&acc)[4][MB], int m0, int nw, int g, int M, const EpiArgs& ep) {
  if constexpr (EPI == EPI_STORE_F32 || EPI == EPI_RESID) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = nw + i * 16 + 4 * g;
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const int m = m0 + 16 * j;
        if (m >= M) continue;
        if constexpr (EPI == EPI_STORE_F32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(ep.out) + (size_t)(m + ep.row_off) * ep.ldo + n) =
              ep.alpha * acc[i][j];
        } else {
          const float mk = ep.rowmask ? (float)ep.rowmask[m] : 1.f;
          f32x4* xp = reinterpret_cast<f32x4*>(ep.x + (size_t)m * ep.ldx + n);
          *xp = *xp + (ep.alpha * mk) * acc[i][j];
        }
      }
    }
  } else if constexpr (EPI == EPI_GLU) {
    // n-blocks (0,1) = (a, gate) of output channels c0 .. c0+15, (2,3) of c0+16 .. c0+31
    bf16* base = reinterpret_cast<bf16*>(ep.out) + (size_t)ep.row_off * ep.ldo + nw / 2;
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const int m = m0 + 16 * j;
      u32x2_t o[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const f32x4 a = acc[2 * p][j], gt = acc[2 * p + 1][j];
        auto sg = [](float x) {   // sigmoid of the gate (pre-scaled by -log2(e) with ACT_SILU_L2E)
          if constexpr (ACT == ACT_SILU_L2E) return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x));
          else return fast_sigmoid(x);
        };
        o[p] = (u32x2_t){pack_h2<FMT>(a[0] * sg(gt[0]), a[1] * sg(gt[1])),
                         pack_h2<FMT>(a[2] * sg(gt[2]), a[3] * sg(gt[3]))};
      }
      if (m < M) store_pair16<NOST>(base, ep.ldo, m, g, o[0], o[1], ep.store_mode);
    }
  } else {   // EPI_STORE / EPI_QKV: bf16 out, pairs (0,1) and (2,3)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nw + 32 * p;   // a 32-column span never crosses a head group (dk = 64 or 128)
      bf16* base;
      size_t ld;
      if constexpr (EPI == EPI_QKV) {
        const int d = ep.d;
        if (n < d) {
          base = reinterpret_cast<bf16*>(ep.out) + n;
          ld = d;
        } else {
          const int c2 = n - d, which = c2 >= d ? 1 : 0, cc = c2 - which * d;
          base = reinterpret_cast<bf16*>(ep.out2) + (size_t)ep.row_off * 2 * d + qkv_kv_col(cc, which, ep.dk);
          ld = 2 * (size_t)d;
        }
      } else {
        base = reinterpret_cast<bf16*>(ep.out) + (size_t)ep.row_off * ep.ldo + n;
        ld = ep.ldo;
      }
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const int m = m0 + 16 * j;
        const f32x4 v0 = act4<ACT>(acc[2 * p][j]), v1 = act4<ACT>(acc[2 * p + 1][j]);
        const u32x2_t x = (u32x2_t){pack_h2<FMT>(v0[0], v0[1]), pack_h2<FMT>(v0[2], v0[3])};
        const u32x2_t y = (u32x2_t){pack_h2<FMT>(v1[0], v1[1]), pack_h2<FMT>(v1[2], v1[3])};
        if (m < M) store_pair16<NOST>(base, ld, m, g, x, y, ep.store_mode);
      }
    }
  }
}

// EPI_STORE through an LDS staging tile (per wave 16 rows x 144 B): each m-block's four 4-column
// pieces per lane are written with ds_write_b64, read back as full 128-B row pieces (8 rows per
// read) and stored as whole lines, instead of 16-row x 64-B pieces after permlane swaps.
template <int ACT, int FMT = 0>
CFM_DEV void wave_epilogue_fullrow(f32x4 (&acc)[4][8], int row0, int nw, int fr, int g, int lane, int M,
                                   const EpiArgs& ep, unsigned stg) {
  constexpr int PITCH = 144;
  bf16* base = reinterpret_cast<bf16*>(ep.out) + (size_t)ep.row_off * ep.ldo + nw;
  const unsigned wr = stg + (unsigned)(fr * PITCH + 8 * g);
  const unsigned rd = stg + (unsigned)((lane >> 3) * PITCH + 16 * (lane & 7));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 v = act4<ACT>(acc[i][j]);
      asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(wr), "v"((u32x2_t){pack_h2<FMT>(v[0], v[1]), pack_h2<FMT>(v[2], v[3])}),
                   "i"(32 * i) : "memory");
    }
    u32x4 r[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[b]) : "v"(rd), "i"(8 * PITCH * b) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int m = row0 + 16 * j + (lane >> 3) + 8 * b;
      if (m >= M) continue;
      u32x4* p = reinterpret_cast<u32x4*>(base + (size_t)m * ep.ldo + 8 * (lane & 7));
      if (ep.store_mode == 2) __builtin_nontemporal_store(r[b], p);
      else *p = r[b];
    }
  }
}

template <int EPI, int ACT, bool NOST = false, int FMT = 0>
CFM_DEV void tile_epilogue(f32x4 (&acc)[4][8], int tm, int tn, int wm, int wn, int fr, int g, int M,
                           const EpiArgs& ep) {
  wave_epilogue<EPI, ACT, 8, NOST, FMT>(acc, tm * 256 + wm * 128 + fr, tn * 256 + wn * 64, g, M, ep);
}

// seed the accumulators of tile (tm, tn) with the bias (every m-block of an n-block gets the same 4 values)
CFM_DEV void seed_bias(f32x4 (&acc)[4][8], const float* bias, int tn, int wn, int g) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 b = bias ? *reinterpret_cast<const f32x4*>(bias + tn * 256 + wn * 64 + i * 16 + 4 * g)
                         : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = b;
  }
}

}  // namespace cfm
