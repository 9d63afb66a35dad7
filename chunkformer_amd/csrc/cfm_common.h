// Common device/host helpers for the gfx950 (CDNA4) ChunkFormer kernels.
//
// Element type T of every activation/weight stream is `float` (parity
// mode: exact-f32 MFMA v_mfma_f32_16x16x4_f32), `bf16` (fast mode:
// v_mfma_f32_16x16x32_bf16) or `f16` (the reference's --autocast_dtype fp16:
// v_mfma_f32_16x16x32_f16 on the generic kernels).  Accumulation, softmax and
// LayerNorm statistics are always f32.  Both operand types share ONE fragment abstraction: a lane
// holds 8 consecutive K elements of its row (A) / column (B); for bf16 that is
// one 16x16x32 MFMA, for f32 eight 16x16x4 MFMAs (instruction e consumes
// element e of every lane: k = 8*(lane>>4) + e).  Any consistent K permutation
// is a valid contraction, so LDS images and address math are identical for
// both types and only the byte width of a fragment differs (16 B vs 32 B).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CFM_DEV __device__ __forceinline__

// compile-time loop: f(std::integral_constant<int, i>) for i = B .. E-1
template <int B, int E, class F>
CFM_DEV void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

template <typename T> struct Frag;
template <> struct Frag<float> { typedef f32x8 type; };
template <> struct Frag<bf16> { typedef bf16x8 type; };
template <> struct Frag<f16> { typedef f16x8 type; };

CFM_DEV float to_f32(float x) { return x; }
CFM_DEV float to_f32(bf16 x) { return (float)x; }
CFM_DEV float to_f32(f16 x) { return (float)x; }
template <typename T> CFM_DEV T from_f32(float x);
template <> CFM_DEV float from_f32<float>(float x) { return x; }
template <> CFM_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }
template <> CFM_DEV f16 from_f32<f16>(float x) { return (f16)x; }

// 16x16 output tile += A(16 x 32) * B(32 x 16) expressed on 8-element fragments
CFM_DEV f32x4 mma16(const f32x8& a, const f32x8& b, f32x4 acc) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], acc, 0, 0, 0);
  return acc;
}
CFM_DEV f32x4 mma16(const bf16x8& a, const bf16x8& b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}
CFM_DEV f32x4 mma16(const f16x8& a, const f16x8& b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
}

// load 8 consecutive elements (16 B for bf16, 32 B for f32)
template <typename T> CFM_DEV typename Frag<T>::type ld8(const T* p) {
  return *reinterpret_cast<const typename Frag<T>::type*>(p);
}
template <typename T> CFM_DEV void st8(T* p, const typename Frag<T>::type& v) {
  *reinterpret_cast<typename Frag<T>::type*>(p) = v;
}
// 8 consecutive elements <-> f32[8]
CFM_DEV void load8(const float* p, float* x) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) { x[q] = a[q]; x[q + 4] = b[q]; }
}
CFM_DEV void load8(const bf16* p, float* x) {
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = (float)a[q];
}
CFM_DEV void load8(const f16* p, float* x) {
  const f16x8 a = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
  for (int q = 0; q < 8; ++q) x[q] = (float)a[q];
}
CFM_DEV void store8(float* p, const float* x) {
  *reinterpret_cast<f32x4*>(p) = (f32x4){x[0], x[1], x[2], x[3]};
  *reinterpret_cast<f32x4*>(p + 4) = (f32x4){x[4], x[5], x[6], x[7]};
}
CFM_DEV void store8(bf16* p, const float* x) {
  bf16x8 v;
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = (bf16)x[q];
  *reinterpret_cast<bf16x8*>(p) = v;
}
CFM_DEV void store8(f16* p, const float* x) {
  f16x8 v;
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = (f16)x[q];
  *reinterpret_cast<f16x8*>(p) = v;
}

// front-end dw2 (depthwise 3x3 stride 2) on 16-bit activations, shared by fe_dw2_kernel and the fused pw1 + dw2
// GEMM epilogue so that both compute bit-identical sums: a channel pair's activations stay one packed dword and each
// channel's tap is ONE dot2 against a weight dword holding (w, 0) or (0, w) in the same 16-bit format -- the weights
// rounded to that format, as the reference's autocast conv2d casts them (FMT 0 = bf16, 1 = f16)
#ifndef DW2_DOT2
#define DW2_DOT2 1
#endif
template <int FMT> CFM_DEV float dw2_dot(unsigned x, unsigned wd, float c) {
  typedef __bf16 bf2_ __attribute__((ext_vector_type(2)));
  typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
  if constexpr (FMT == 1)
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_, x), __builtin_bit_cast(h2_, wd), c, false);
  else
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_, x), __builtin_bit_cast(bf2_, wd), c, false);
}
// the weight dword of channel c: w in the 16-bit half that holds channel c's activation (c & 1), zero in the other
template <int FMT> CFM_DEV unsigned dw2_wpack(float w, int c) {
  unsigned short b;
  if constexpr (FMT == 1) b = __builtin_bit_cast(unsigned short, (f16)w);
  else b = __builtin_bit_cast(unsigned short, (bf16)w);
  return (unsigned)b << (16 * (c & 1));
}
template <typename T> CFM_DEV typename Frag<T>::type zero8() {
  typename Frag<T>::type z;
#pragma unroll
  for (int e = 0; e < 8; ++e) z[e] = (T)0.0f;
  return z;
}

CFM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
CFM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reductions inside aligned groups of 16 lanes (one MFMA 16x16 output row group)
CFM_DEV float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
CFM_DEV float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// wave-wide sum with no LDS round trip: DPP quad / half-row / row mirrors leave every lane of a
// 16-lane row with the row total, row_bcast:15 / row_bcast:31 fold the rows into lane 63, and a
// readlane returns that one value to every lane (bit-identical, wave-uniform)
template <int CTRL, int ROWS = 0xF>
CFM_DEV float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xF, false));
}
CFM_DEV float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(v);          // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);          // quad_perm [2,3,0,1]
  v += dpp_f32<0x141>(v);         // row_half_mirror
  v += dpp_f32<0x140>(v);         // row_mirror
  v += dpp_f32<0x142, 0xA>(v);    // row_bcast:15 into rows 1, 3
  v += dpp_f32<0x143, 0xC>(v);    // row_bcast:31 into rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// Four bf16 (two packed dwords) to a 2-B-aligned LDS address as four aligned 16-bit stores: a
// _b64 store off its 8-B alignment is replayed by the LDS at ~64 cycles per wave-instruction
// (MI355X_MICROARCH.md §LDS / cdna_hip_programming.md G17), four ds_write_b16 cost ~2 LDS cycles each.
CFM_DEV void lds_store_4bf16_a2(unsigned addr, unsigned lo, unsigned hi) {
  asm volatile(
      "ds_write_b16 %0, %1\n\tds_write_b16_d16_hi %0, %1 offset:2\n\t"
      "ds_write_b16 %0, %2 offset:4\n\tds_write_b16_d16_hi %0, %2 offset:6" ::"v"(addr),
      "v"(lo), "v"(hi)
      : "memory");
}

CFM_DEV float silu_f(float x) { return x / (1.0f + __expf(-x)); }
CFM_DEV float sigmoid_f(float x) { return 1.0f / (1.0f + __expf(-x)); }

// ----------------------------------------------------------------------------- plan records
// Per packed chunk (masked batch), produced by the host planner (planner.cpp):
enum {
  PM_SRC_ROW = 0,   // first feature row of the chunk's window in the packed [sum T, 80] feats
  PM_NVALID = 1,    // real feature rows in the window (rest is zero padding)
  PM_ATT_LO = 2,    // attention window keys j in [lo, hi) are unmasked
  PM_ATT_HI = 3,
  PM_CONV_LO = 4,   // conv window columns j in [lo, hi) are unmasked (mask_pad)
  PM_CONV_HI = 5,
  PM_UTT = 6,
  PM_CHUNK = 7,
  PM_INTS = 8
};

// Attention block descriptor (one block of <=64 query rows x one head):
enum {
  AD_Q_ROW0 = 0,    // first query row in the Q / output buffers
  AD_NQ = 1,        // query rows in this block (<= 64)
  AD_KV_ROW0 = 2,   // KV stream row of window key j = 0 (may be negative: only keys in [lo,hi) are read)
  AD_KEY_LO = 3,    // window keys j in [lo, hi) are unmasked, all others are -inf
  AD_KEY_HI = 4,
  AD_P_BASE = 5,    // rel-pos row of (query i, key j) is P_BASE - i + j
  AD_Q_VALID = 6,   // query rows i >= Q_VALID are fully masked (output 0)
  AD_PAD = 7,
  AD_INTS = 8
};

// Depthwise-conv block descriptor (<= 64 output rows of one chunk / one padded segment)
enum {
  CD_OUT_ROW0 = 0,  // first output row
  CD_NOUT = 1,      // output rows
  CD_SRC_ROW0 = 2,  // input (GLU stream) row of window column j = 0; column j feeds output i = j - 7 .. j + 7
  CD_J_LO = 3,      // window columns j in [lo, hi) are real, others are 0
  CD_J_HI = 4,
  CD_SEG_LO = 5,    // padded path: extra per-row segment bound (see conv_module.hip)
  CD_SEG = 6,       // padded path: chunk length for per-row segments (0 = none)
  CD_PAD = 7,
  CD_INTS = 8
};

#define CFM_CHECK_LAUNCH() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
