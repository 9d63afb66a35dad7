// bf16 MFMA GEMM for K = 512 with the weight tile held in registers ("W-stationary").
//
//   C[M, N] = A[M, K] . W[N, K]^T   (bf16 in, f32 accumulate), K == 512, N % 256 == 0
//
// Why: the 256 x 256 LDS-DMA kernel (gemm_bf16.hip) streams BOTH operands through LDS, 128 FLOP per
// byte filled, and its per-CU L2 -> LDS fill rate caps it well below the MFMA rate.  With K = 512 a
// 256-column weight tile is 256 KiB of bf16: spread over the 4 waves of a CU (one wave per SIMD,
// 512 registers each) it fits in registers, 256 AGPRs per lane.  Only A is streamed, 64 rows x 512
// per 64 x 256 output tile: 256 FLOP per byte filled, and a 16-slot LDS ring keeps 14 K-steps
// (112 KiB) of A in flight per CU.
//
//   * block = 4 waves (256 threads), one per CU; wave w owns output columns 64w .. 64w+63 of the
//     block's column tile: W fragments wf[n-block 0..3][k32 0..15] (bf16x8), loaded once;
//   * a tile = 64 rows x 256 columns, 8 K-steps of 64; per K-step each wave reads 4 x 2 A
//     fragments (ds_read_b128, swizzled conflict-free image) and issues 32
//     v_mfma_f32_16x16x32_bf16 (MFMA A operand = W fragment, B = A fragment: the accumulator holds
//     C^T, the swapped-operand layout of gemm_bf16_epi.h, stored as 16-B bf16 row pieces);
//   * A staging: buffer LDS-DMA, 2 x 1 KiB per wave per step, lane-linear LDS destination with the
//     16-B chunk swizzle applied on the source offset; one barrier per step;
//   * placement: the row tiles are cut into 8 XCD ranges; on one XCD the column tiles of a row
//     range run on different CUs at the same pace, so each A tile comes from HBM once and is
//     re-read from that XCD's L2 by the other column tiles (blockIdx % 8 = XCD is a speed
//     assumption only, never a correctness one).
#pragma once
// The weight-stationary GEMM kernel and its launcher, included by the gemm_wst*.hip translation units
// (one per epilogue family, compiled in parallel: the kernel is heavily unrolled).
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "gemm_bf16_epi.h"
#include <cstdlib>
#include <type_traits>

namespace cfm {

namespace {
constexpr int WST_K = 512;
constexpr int WST_MT = 64;              // rows per tile
constexpr int WST_KS = 64;              // K per step
constexpr int WST_NK = WST_K / WST_KS;  // 8 steps per tile
constexpr int WST_SLOT = WST_MT * WST_KS * 2;   // 8 KiB
constexpr int WST_NSLOT = 16;
#ifndef WSP_BARP
#define WSP_BARP 2   // K-steps per barrier (1, 2 or 4): the DMA runs 16 - WSP_BARP steps ahead and refills
                     // the slot of step y - WSP_BARP, so only every WSP_BARP-th step needs the barrier
#endif
constexpr int WST_DEPTH = WST_NSLOT - WSP_BARP;   // steps in flight ahead of the one being read
static_assert(WSP_BARP == 1 || WSP_BARP == 2 || WSP_BARP == 4, "barrier period");
// DW2 (front-end pw1 + ReLU + dw2): an 8-slot A ring leaves LDS for the pw1 output ring
template <int EPI> constexpr int wst_nslot() { return EPI == EPI_DW2 ? 8 : WST_NSLOT; }
#ifndef DW2_BARP
#define DW2_BARP 2   // DW2's barrier period (its 8-slot ring keeps DEPTH - 1 - BARP steps in flight past the wait)
#endif
template <int EPI> constexpr int wst_barp() { return EPI == EPI_DW2 ? DW2_BARP : WSP_BARP; }
template <int EPI> constexpr int wst_depth() { return wst_nslot<EPI>() - wst_barp<EPI>(); }
// dw2 phase: positions per lane, tap-loop unroll, timing diagnostics (1 = no stores, 2 = no phase)
#ifndef DW2_PPL
#define DW2_PPL 1
#endif
#ifndef DW2_VUNROLL
#define DW2_VUNROLL 1
#endif
#ifndef DW2_DIAG
#define DW2_DIAG 0
#endif
#ifndef DW2_NT
#define DW2_NT 0     // dw2 output stores non-temporal (A/B)
#endif
#ifndef DW2_PIPE
#define DW2_PIPE 2   // dw2 taps software-pipelined two deep (explicit LDS reads and waits; 2: rank + bias in one
                     // round trip). Bench A/B, 3 interleaved runs: front-end GEMMs 5.88 -> 5.58 ms/step
#endif
#ifndef DW2_UNPK_SCALAR
#define DW2_UNPK_SCALAR 0
#endif
#ifndef DW2_OFFTAB
#define DW2_OFFTAB 1  // the rank table also holds each output's element offset (computed once, where `last` is decided:
                      // no integer division per pass)
#endif
constexpr int DW2_TABW = DW2_OFFTAB ? 512 : 256;   // rank table bytes per wave
#ifndef DW2_DEFER
#define DW2_DEFER 0  // dw2 outputs staged in LDS and stored at the start of the next phase (A/B)
#endif
constexpr int DW2_STG = 3 * (64 * 16 + 64 * 4);   // per wave: 3 passes x (64 lanes x 16 B + a u32 offset)
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int DW2_RP = 528;                 // pw1 ring row pitch (256 bf16 + 16 B): conflict-free ds_write_b64
constexpr int DW2_RING = 128 * DW2_RP;      // two 64-row tiles
constexpr int DW2_WB = (9 + 1) * 256 * 4;   // dw2 taps [9][256] + bias [256], f32
template <int N> CFM_DEV void wst_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
// a packed pair of 16-bit pw1 outputs (bf16 or f16) -> f32 (exact either way)
template <int FMT> CFM_DEV f32x2 dw2_unpk2(unsigned x) {
  if constexpr (FMT == 1) {
#if DW2_UNPK_SCALAR
    const f16 lo = __builtin_bit_cast(f16, (unsigned short)(x & 0xffffu)), hi = __builtin_bit_cast(f16, (unsigned short)(x >> 16));
    return (f32x2){(float)lo, (float)hi};
#else
    typedef f16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_convertvector(__builtin_bit_cast(h2, x), f32x2);
#endif
  } else {
    return (f32x2){__builtin_bit_cast(float, x << 16), __builtin_bit_cast(float, x & 0xffff0000u)};
  }
}
}  // namespace

#ifndef WSP_LGKM
#define WSP_LGKM 1   // 0: every K-step closes with lgkmcnt(0) (re-seed reads waited at once)
#endif
#ifndef WSP_FULLROW
#define WSP_FULLROW 1   // 0: permlane-swapped 64-B row pieces stored per step (A/B)
#endif
#ifndef WSP_FULLROW_ACT
#define WSP_FULLROW_ACT 1   // also the SiLU / ReLU epilogues (0: permlane-swapped 64-B pieces there; A/B)
#endif
#define WST_VMCNT(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

// acc += W-fragment (AGPR, "a") x A-fragment (VGPR): the 256 weight registers per lane live in the
// AGPR half of the register file and feed the MFMA directly (with the builtin, hipcc keeps them in
// AGPRs but copies each one to VGPRs before use).  asm volatile keeps program order with the
// explicit LDS waits; the VALU <-> MFMA hazards around it are padded by hand (s_nop) where the
// accumulators are seeded (VALU write -> MFMA srcC) and read back (MFMA write -> VALU read).
template <int FMT>
CFM_DEV void mfma_wa(f32x4& acc, const bf16x8& w, const bf16x8& a) {
  if constexpr (FMT == 1)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(a));
}

// ------------------------------------------------------------------------------------------------
// Software pipelining ("wsp"): with ONE wave per SIMD nothing else hides the non-MFMA work, so
// every K-step is laid out by hand as 32 MFMA gaps:
//   * the 8 ds_read_b128 of the NEXT step's A fragments sit in gaps 0, 2, .., 14;
//   * the 2 LDS-DMA pieces of step y + 14 in gaps 6 and 22 (one barrier per two steps);
//   * the PREVIOUS tile's epilogue (bias-seeded accumulators double-buffered: the tile computes
//     into acc[BUF] while acc[1 - BUF] is drained) is cut into micro-ops (scale, exp2, +1, rcp,
//     mul, pack, permlane16 swap, one 16-B store, re-seed) spread evenly over the gaps, one
//     epilogue group (a 32-column x 16-row piece) per K-step;
//   * __builtin_amdgcn_sched_barrier(0) after every gap keeps hipcc from regrouping them.
// An MFMA (16x16x32 bf16) occupies 16 cycles of which it holds vector issue for 8, so one or two
// VALU micro-ops per gap ride for free; the MFMA asm is opaque to the compiler's hazard
// recognizer, which is fine here: every VALU access to an accumulator buffer is at least 11
// MFMAs away from the last MFMA that wrote it (or an explicit s_nop pads the gap).
// in-place LDS reads ("+v": the destination keeps its register, so hipcc does not rename the
// fragment / accumulator buffers between steps and pay for it in copies and pressure)
template <int OFF>
CFM_DEV void lds_read_into(f32x4& v, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(v) : "v"(addr), "i"(OFF));
}
template <int OFF>
CFM_DEV void lds_read_into(bf16x8& v, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(v) : "v"(addr), "i"(OFF));
}

namespace {
// micro-ops of epilogue group s (0..7).  STORE/QKV: two halves (one 16-column n-block each) of
// [activation ops on 4 values, 2 packs], then 2 permlane swaps, 1 store, 2 re-seeds.
// GLU: group s = (m-block s/2, channel half s%1): 20 sigmoid-gate ops + 2 packs (+ swaps and the
// store on odd s), 2 re-seeds.
template <int ACT>
constexpr int wsp_half() { return (ACT == ACT_SILU ? 20 : ACT == ACT_SILU_L2E ? 16 : ACT == ACT_RELU ? 4 : 0) + 2; }
// GLU: gate-chain ops per group (4 values x 5 steps, or x 4 with the gate pre-scaled by -log2(e)); then
// 2 packs, 2 re-seeds, 2 swaps and (odd groups) the store
template <int ACT>
constexpr int glu_chain() { return ACT == ACT_SILU_L2E ? 16 : 20; }
// Full-row stores (non-GLU, WSP_FULLROW): per half q the activation ops, 2 packs, one ds_write_b64
// of the 4 packed columns into the wave's 16 x 64 staging tile, the re-seed; an odd group then
// reads the tile back as full 128-B rows (2 x ds_read_b128: rows 0-7, 8-15) and the next (even)
// group stores them first thing (its step opened with lgkmcnt(0)).  2H + 4 ops either way.
// Used everywhere: one-process A/B (tools/gemm_bench.py) QKV 285 -> 251 us, out-proj / pw2 91 -> 89 us.
// On random-data microbenchmarks (power-limited clocks) the SiLU / ReLU epilogues measured 2-6% slower
// with it, but in the bench step (real activations, 2.3 GHz) FFN w1 9.1 -> 8.3 ms/step and the
// front-end pointwise GEMMs 5.2 -> 4.8 ms/step (3 interleaved runs each), so it is on there too.
template <int EPI, int ACT>
constexpr bool wsp_fullrow() {
  return WSP_FULLROW && (EPI == EPI_QKV || (EPI == EPI_STORE && (ACT == ACT_NONE || WSP_FULLROW_ACT)));
}
// DW2 groups: per half q the activation ops, 2 packs, the ds_write_b64 into the pw1 ring, the re-seed
template <int EPI, int ACT>
constexpr int wsp_nops(int s) {
  return EPI == EPI_DW2 ? 2 * (wsp_half<ACT>() + 2)
         : EPI == EPI_GLU ? glu_chain<ACT>() + ((s & 1) ? 7 : 4)
         : wsp_fullrow<EPI, ACT>() ? 2 * wsp_half<ACT>() + 6 : 2 * wsp_half<ACT>() + 5;
}
constexpr int wsp_lo(int i, int n) { return (i * n + 31) / 32; }   // first op of gap i
constexpr int wsp_gap(int o, int n) {                                  // gap that carries op o
  int i = 0;
  while (i < 31 && wsp_lo(i + 1, n) <= o) ++i;
  return i;
}
// re-seed reads (LDS) issued after the step's last A-fragment read (gap 14): the step's closing
// wait leaves exactly these in flight (they land before the next tile's first MFMA on that buffer,
// which the last step of a tile waits for in full)
template <int EPI, int ACT>
constexpr int wsp_late_seeds(int s) {
  const int n = wsp_nops<EPI, ACT>(s), H = wsp_half<ACT>() + 1;
  // full-row: even groups open with the 2 deferred stores (seeds at 2 + H, 2H + 3); odd groups
  // end with the 2 row reads and then both seeds (2H + 2, 2H + 3)
  const bool fr = wsp_fullrow<EPI, ACT>();
  const int G = glu_chain<ACT>();
  const int o0 = EPI == EPI_DW2 ? H : EPI == EPI_GLU ? G + 2 : fr ? ((s & 1) ? 2 * H + 2 : H + 2) : H - 1;
  const int o1 = EPI == EPI_DW2 ? 2 * H + 1 : EPI == EPI_GLU ? G + 3 : fr ? 2 * H + 3 : 2 * H - 1;
  return (wsp_gap(o0, n) >= 14) + (wsp_gap(o1, n) >= 14);
}
}  // namespace

template <int EPI, int ACT, int DIAG = 0, int FMT = 0>
__global__ __launch_bounds__(256, 1) void gemm_wsp_kernel(const bf16* __restrict__ A, int lda,
                                                          const bf16* __restrict__ W, int ldw, int M, int N,
                                                          EpiArgs ep) {
  // A ring + the block's 256 bias values (the re-seed reads them straight into the accumulators)
  // + per wave a 16-row x 64-column bf16 output staging tile (144-B rows) for full-row stores
  constexpr int STG_PITCH = 144, STG_BYTES = 16 * STG_PITCH;
  constexpr int NS = wst_nslot<EPI>(), DP = wst_depth<EPI>();
  constexpr int TAIL = EPI == EPI_DW2 ? DW2_RING + DW2_WB + 4 * DW2_TABW + (DW2_DEFER ? 4 * DW2_STG : 0) : 4 * STG_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[NS * WST_SLOT + 1024 + TAIL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;

  const int nbn = N >> 8, nbm = (M + WST_MT - 1) / WST_MT;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per = gridDim.x >> 3;
  const int cpx = per / nbn;
  if (cpx == 0 || j >= cpx * nbn) return;
  const int ct = j % nbn, sub = j / nbn;
  const int xr0 = (int)((long long)xcd * nbm / 8), xr1 = (int)((long long)(xcd + 1) * nbm / 8);
  const int r0 = xr0 + (int)((long long)sub * (xr1 - xr0) / cpx);
  const int r1 = xr0 + (int)((long long)(sub + 1) * (xr1 - xr0) / cpx);
  if (r0 >= r1) return;
  // DW2: a dw2 output needs the pw1 rows up to 40 before its last row, so the block also computes the
  // tile before its range (halo; its outputs belong to the previous block) and emits the outputs whose
  // last row lies in [64 r0, 64 r1)
  const int r0c = (EPI == EPI_DW2 && r0 > 0) ? r0 - 1 : r0;

  // ---- A stream: buffer LDS-DMA, descriptor = the 64-row tile (rows past M read as 0, so the
  // pieces issued past the block's end need no clamp), lane offset (row, swizzled 16-B chunk)
  unsigned voffA[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (2 * wv + i) * 8 + (lane >> 3);
    voffA[i] = (unsigned)(row * lda + ((lane & 7) ^ ((row >> 1) & 7)) * 8) * 2;
  }
  // descriptor of row tile rt (built once per tile, not per piece: the SALU work would sit in the
  // MFMA gaps).  readfirstlane: min/max of uniform ints select v_med3 (VALU only), and a VGPR
  // descriptor would wrap every buffer op in a waterfall loop
  auto tile_rsrc = [&](int rt) {
    const int rows = __builtin_amdgcn_readfirstlane(max(0, min(WST_MT, M - rt * WST_MT)));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)rt * WST_MT * lda), (short)0, rows * lda * 2,
                                             0x00020000);
  };
  auto issue_piece = [&](__amdgpu_buffer_rsrc_t rs, auto Ic, auto KSc, auto SLc) {
    constexpr int i = decltype(Ic)::value, ks = decltype(KSc)::value, slot = decltype(SLc)::value;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(smem + slot * WST_SLOT + (2 * wv + i) * 1024), 16, voffA[i],
        ks * WST_KS * 2, 0, 0);   // K slice in soffset: the immediate offset would move the LDS side too
  };
  {
    const __amdgpu_buffer_rsrc_t d0 = tile_rsrc(r0c), d1 = tile_rsrc(r0c + 1);
    sfor<0, DP>([&](auto Pc) {
      constexpr int P = decltype(Pc)::value;
      issue_piece(P < WST_NK ? d0 : d1, std::integral_constant<int, 0>{}, std::integral_constant<int, P % WST_NK>{}, Pc);
      issue_piece(P < WST_NK ? d0 : d1, std::integral_constant<int, 1>{}, std::integral_constant<int, P % WST_NK>{}, Pc);
    });
  }

  const int col0 = ct * 256 + wv * 64;
  bf16x8 wf[4][16];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const bf16* wp = W + (size_t)(col0 + 16 * nb + fr) * ldw + 8 * g;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) wf[nb][kk] = *reinterpret_cast<const bf16x8*>(wp + 32 * kk);
  }
  if constexpr (EPI == EPI_DW2) {
    float* dwl = reinterpret_cast<float*>(smem + NS * WST_SLOT + 1024 + DW2_RING);
    for (int idx = tid; idx < 10 * 256; idx += 256) {
      const int e = idx >> 8, j = idx & 255;
      if (DW2_DOT2 && e < 9)   // tap weights as dw2_dot dwords (cfm_common.h); the bias stays f32
        reinterpret_cast<unsigned*>(dwl)[idx] = dw2_wpack<FMT>(ep.dw_w[(size_t)e * N + ct * 256 + j], j);
      else
        dwl[idx] = e < 9 ? ep.dw_w[(size_t)e * N + ct * 256 + j] : ep.dw_b[ct * 256 + j];
    }
  }
  if (tid < 64)
    reinterpret_cast<f32x4*>(smem + NS * WST_SLOT)[tid] =
        ep.bias ? *reinterpret_cast<const f32x4*>(ep.bias + ct * 256 + 4 * tid) : (f32x4){0.f, 0.f, 0.f, 0.f};
  // output of the wave's two 32-column spans: wave-uniform base + row stride, lane offset
  // (row fr, 8 columns after the permlane swap)
  bf16* obase[2];
  int old[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if constexpr (EPI == EPI_QKV) {
      const int d = ep.d, n = col0 + 32 * p;
      if (n < d) {
        obase[p] = reinterpret_cast<bf16*>(ep.out) + n;
        old[p] = d;
      } else {
        const int c2 = n - d, which = c2 >= d ? 1 : 0, cc = c2 - which * d;
        obase[p] = reinterpret_cast<bf16*>(ep.out2) + (size_t)ep.row_off * 2 * d + qkv_kv_col(cc, which, ep.dk);
        old[p] = 2 * d;
      }
    } else if constexpr (EPI == EPI_GLU) {
      obase[p] = reinterpret_cast<bf16*>(ep.out) + (size_t)ep.row_off * ep.ldo + col0 / 2;
      old[p] = ep.ldo;
    } else {
      obase[p] = reinterpret_cast<bf16*>(ep.out) + (size_t)ep.row_off * ep.ldo + col0 + 32 * p;
      old[p] = ep.ldo;
    }
  }
  const int lcol = 16 * (g & 1) + 8 * (g >> 1);
  unsigned voffS[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) voffS[p] = (unsigned)(fr * old[p] + lcol) * 2;
  // full-row stores: lane -> row (lane >> 3) (+ 8), 16-B chunk (lane & 7) of the wave's 64 columns
  // (contiguous in the output: obase[1] = obase[0] + 32 for STORE and for QKV with dk % 64 == 0)
  unsigned voffF[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) voffF[b] = (unsigned)(((lane >> 3) + 8 * b) * old[0] + 8 * (lane & 7)) * 2;
  if constexpr (DIAG == 7) {   // timing only (wrong layout): every store 8 full 128-B rows
#pragma unroll
    for (int p = 0; p < 2; ++p) voffS[p] = (unsigned)(((fr & 7) + 8 * p) * old[p] - 32 * p + ((fr >> 3) * 4 + g) * 8) * 2;
  }

  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)smem;
  const int key = (fr >> 1) & 7;
  // read bases [slot half][kh]; the slot's offset inside its half and the m-block go in the immediate
  unsigned rdb[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    rdb[h][0] = lds_base + h * 8 * WST_SLOT + (unsigned)(fr * 128 + ((g ^ key) << 4));
    rdb[h][1] = lds_base + h * 8 * WST_SLOT + (unsigned)(fr * 128 + (((4 + g) ^ key) << 4));
  }

  // lane's bias f32x4 of n-block nb at bias_lds + 64 nb
  const unsigned bias_lds = lds_base + NS * WST_SLOT + (unsigned)(wv * 64 + 4 * g) * 4;
  // staging tile: write (row fr, columns 32p + 16q + 4g ..), read (row lane >> 3 (+ 8), chunk lane & 7)
  const unsigned stg = lds_base + NS * WST_SLOT + 1024 + (unsigned)wv * STG_BYTES;
  const unsigned stg_w = stg + (unsigned)(fr * STG_PITCH + 8 * g);
  const unsigned stg_r = stg + (unsigned)((lane >> 3) * STG_PITCH + 16 * (lane & 7));
  u32x4 rowv[2] = {(u32x4){0u, 0u, 0u, 0u}, (u32x4){0u, 0u, 0u, 0u}};   // full rows read back, stored next group
  // DW2: pw1 ring (2 tiles x 64 rows x 256 columns, pitch DW2_RP), the block's dw2 taps + bias (f32),
  // a 64-entry rank table per wave
  const unsigned ring_base = lds_base + NS * WST_SLOT + 1024;
  const unsigned dww = ring_base + DW2_RING;
  const unsigned ring_w = ring_base + (unsigned)(fr * DW2_RP + 128 * wv + 8 * g);
  f32x4 acc[2][4][4];
  bf16x8 afr[2][4][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) afr[u][mb][kh] = (bf16x8){};
  float et[4];
  unsigned epk[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) acc[1][nb][mb] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    et[i] = 0.f;
    epk[i] = 0u;
  }

  // Epilogue micro-op O of group S on accumulator buffer a (rows of tile rtp; rows >= lim are not
  // stored: they fall outside the store descriptor's range, so no branch splits the MFMA stream).
  // Every result is pinned where it is produced (empty asm volatile): without that, LLVM sinks the
  // pure arithmetic next to its use and the gaps run dry.
  auto pin = [](auto& v) { asm volatile("" : "+v"(v)); };
  // RESEED = false (the final drain): no re-seed reads -- an async ds_read into an accumulator that
  // is dead afterwards would land in whatever hipcc reuses that register for
  // store descriptors of tile rtp's rows below lim (one per 32-column span, built once per tile)
  struct StoreD { __amdgpu_buffer_rsrc_t d[2]; };
  auto store_rsrc = [&](int rtp, int lim) {
    StoreD sd;
    const int rows = __builtin_amdgcn_readfirstlane(max(0, min(WST_MT, lim - rtp * WST_MT)));
#pragma unroll
    for (int p = 0; p < 2; ++p)
      sd.d[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(obase[p] + (size_t)rtp * WST_MT * old[p]), (short)0,
                                                  rows * old[p] * 2, 0x00020000);
    return sd;
  };
  auto epi_op = [&](auto Sc, auto Oc, f32x4(&a)[4][4], const StoreD& sd, const StoreD& sdp, auto RSc, auto SLc) {
    (void)ring_w;
    (void)stg_w;   // named outside the if-constexpr branches: clang's implicit capture in generic lambdas
    (void)stg_r;
    (void)voffF;
    (void)rowv;
    (void)sdp;
    constexpr int S = decltype(Sc)::value, O = decltype(Oc)::value;
    constexpr bool RESEED = decltype(RSc)::value;
    constexpr float NL2E = -1.4426950408889634f;
    auto store = [&](int p, int jj) {
      constexpr int aux = DIAG == 8 ? 2 : DIAG == 9 ? 16 : 0;   // gfx950 cache policy: nt / sc1
      if constexpr (DIAG != 5)
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){epk[0], epk[1], epk[2], epk[3]}, sd.d[p],
                                               voffS[p] + (unsigned)(16 * jj * old[p] * 2), 0, aux);
    };
    // q = 0: pk0 <-> pk2, q = 1: pk1 <-> pk3 (in place); after both, lane g holds 8 contiguous
    // columns {pk0, pk1, pk2, pk3} (gemm_bf16_epi.h store_pair16)
    auto swap = [&](int q) {
      const auto r = __builtin_amdgcn_permlane16_swap(epk[q], epk[q + 2], false, false);
      epk[q] = r[0];
      epk[q + 2] = r[1];
      pin(epk[q]);
      pin(epk[q + 2]);
    };
    // re-seed with the bias: one ds_read_b128 into the accumulator (waited by the step's
    // closing lgkmcnt(0); the first MFMA on it is a tile later)
    auto seed = [&](auto NBc, int jj) {
      constexpr int nb = decltype(NBc)::value;
      if constexpr (RESEED) lds_read_into<nb * 64>(a[nb][jj], bias_lds);
    };
    // sigmoid-style chain on 4 values: t = x * -log2e; t = 2^t; t += 1; t = 1 / t; t = y * t
    // (ACT_SILU_L2E: x arrives pre-scaled by -log2e, the first step is t = 2^x)
    auto chain = [&](int o, auto xf, auto yf) {
      const int i = o & 3;
      if constexpr (ACT == ACT_SILU_L2E) {
        if (o < 4) et[i] = __builtin_amdgcn_exp2f(xf(i));
        else if (o < 8) et[i] = et[i] + 1.f;
        else if (o < 12) et[i] = __builtin_amdgcn_rcpf(et[i]);
        else et[i] = yf(i) * et[i];
      } else {
        if (o < 4) et[i] = xf(i) * NL2E;
        else if (o < 8) et[i] = __builtin_amdgcn_exp2f(et[i]);
        else if (o < 12) et[i] = et[i] + 1.f;
        else if (o < 16) et[i] = __builtin_amdgcn_rcpf(et[i]);
        else et[i] = yf(i) * et[i];
      }
      pin(et[i]);
    };
    if constexpr (EPI == EPI_DW2) {
      // per half q (n-block 2p + q): the activation ops, 2 packs, ONE ds_write_b64 of the 4 columns into
      // the pw1 ring (row 64 * slot + 16 jj + fr of the drained tile), the re-seed
      constexpr int p = S & 1, jj = S >> 1, SL = decltype(SLc)::value;
      constexpr int H = wsp_half<ACT>() + 2;   // ops per half
      constexpr int q = O / H, o = O % H;
      auto val = [&](int i) -> float { return a[2 * p + q][jj][i]; };
      if constexpr (o == H - 1) {
        seed(std::integral_constant<int, 2 * p + q>{}, jj);
      } else if constexpr (o < H - 4) {
        et[o] = fmaxf(val(o), 0.f);
        pin(et[o]);
      } else if constexpr (o < H - 2) {
        constexpr int k = o - (H - 4);
        epk[2 * q + k] = pack_h2<FMT>(et[2 * k], et[2 * k + 1]);
        pin(epk[2 * q + k]);
      } else {
        typedef unsigned u32x2_w __attribute__((ext_vector_type(2)));
        asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(ring_w), "v"((u32x2_w){epk[2 * q], epk[2 * q + 1]}),
                     "i"(SL * 64 * DW2_RP + jj * 16 * DW2_RP + 64 * p + 32 * q) : "memory");
      }
    } else if constexpr (EPI == EPI_GLU) {
      // ops 0 .. G-1 gate chain, G, G+1 packs, G+2, G+3 re-seeds (both accumulators are dead after
      // op G-1), then on odd S the 2 swaps and the store
      constexpr int jj = S >> 1, h = S & 1, G = glu_chain<ACT>();
      auto gate = [&](int i) -> float { return a[2 * h + 1][jj][i]; };
      auto lin = [&](int i) -> float { return a[2 * h][jj][i]; };
      if constexpr (O == G + 2 || O == G + 3) {
        seed(std::integral_constant<int, 2 * h + (O - G - 2)>{}, jj);
      } else if constexpr (DIAG == 3) {
      } else if constexpr (O < G) {
        chain(O, gate, lin);
      } else if constexpr (O < G + 2) {
        epk[2 * h + O - G] = pack_h2<FMT>(et[2 * (O - G)], et[2 * (O - G) + 1]);
        pin(epk[2 * h + O - G]);
      } else if constexpr (O < G + 6) {
        swap(O - G - 4);
      } else {   // O == G + 6
        store(0, jj);
      }
    } else if constexpr (!wsp_fullrow<EPI, ACT>()) {
      // ops: per half q (one 16-column n-block) H - 2 activation ops, 2 packs and the re-seed of
      // that n-block's accumulator (dead after the packs), then 2 swaps and the store
      constexpr int p = S & 1, jj = S >> 1;   // the two 64-B halves of a 128-B row piece in consecutive steps
      constexpr int H = wsp_half<ACT>() + 1;
      if constexpr (O < 2 * H && O % H == H - 1) {
        seed(std::integral_constant<int, 2 * p + O / H>{}, jj);
      } else if constexpr (DIAG == 3) {
      } else if constexpr (O < 2 * H) {
        constexpr int q = O / H, o = O % H;
        auto val = [&](int i) -> float { return a[2 * p + q][jj][i]; };
        if constexpr (o < H - 3) {
          if constexpr (ACT == ACT_SILU || ACT == ACT_SILU_L2E) {
            chain(o, val, val);
          } else {
            et[o] = fmaxf(val(o), 0.f);
            pin(et[o]);
          }
        } else {
          constexpr int k = o - (H - 3);   // pack k of this half: values 2k, 2k+1
          if constexpr (ACT == ACT_NONE) epk[2 * q + k] = pack_h2<FMT>(val(2 * k), val(2 * k + 1));
          else epk[2 * q + k] = pack_h2<FMT>(et[2 * k], et[2 * k + 1]);
          pin(epk[2 * q + k]);
        }
      } else if constexpr (O < 2 * H + 2) {
        swap(O - 2 * H);
      } else {   // O == 2H + 2
        store(p, jj);
      }
    } else {
      // full rows.  even S: the 2 stores of the previous (odd) group's rows, then per half q
      // (n-block 2p + q) the activation ops, 2 packs, the ds_write_b64 into the staging tile and
      // the re-seed.  odd S: per half the activation ops, packs and write, then the 2 full-row
      // reads, then both re-seeds -- the reads are older than any re-seed, so the step's closing
      // lgkmcnt(late) (re-seeds left in flight) covers them
      constexpr int p = S & 1, jj = S >> 1;
      constexpr int H = wsp_half<ACT>() + 1;
      constexpr int base = p ? 0 : 2, per = p ? H : H + 1;   // ops per half
      if constexpr (p == 0 && O < 2) {
        constexpr int jp = (S + 7) % 8 >> 1;   // rows of group S - 1 (S = 0: the previous tile's last)
        if constexpr (!RESEED) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // drain: no step waits
        constexpr int aux = DIAG == 8 ? 2 : DIAG == 9 ? 16 : 0;   // store policy as in `store`
        if constexpr (DIAG != 5)
          __builtin_amdgcn_raw_buffer_store_b128(rowv[O], (S == 0 ? sdp : sd).d[0],
                                                 voffF[O] + (unsigned)(16 * jp * old[0] * 2), 0, aux);
      } else if constexpr (O >= base && O < base + 2 * per) {
        constexpr int q = (O - base) / per, o = (O - base) % per;
        auto val = [&](int i) -> float { return a[2 * p + q][jj][i]; };
        if constexpr (o == H) {   // even S only
          seed(std::integral_constant<int, 2 * p + q>{}, jj);
        } else if constexpr (DIAG == 3) {
        } else if constexpr (o < H - 3) {
          if constexpr (ACT == ACT_SILU || ACT == ACT_SILU_L2E) {
            chain(o, val, val);
          } else {
            et[o] = fmaxf(val(o), 0.f);
            pin(et[o]);
          }
        } else if constexpr (o < H - 1) {
          constexpr int k = o - (H - 3);   // pack k of this half: values 2k, 2k+1
          if constexpr (ACT == ACT_NONE) epk[2 * q + k] = pack_h2<FMT>(val(2 * k), val(2 * k + 1));
          else epk[2 * q + k] = pack_h2<FMT>(et[2 * k], et[2 * k + 1]);
          pin(epk[2 * q + k]);
        } else {   // o == H - 1: 4 packed columns -> staging tile
          typedef unsigned u32x2_w __attribute__((ext_vector_type(2)));
          asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(stg_w), "v"((u32x2_w){epk[2 * q], epk[2 * q + 1]}),
                       "i"(64 * p + 32 * q) : "memory");
        }
      } else if constexpr (p == 1 && O < 2 * H + 2) {
        constexpr int b = O - 2 * H;   // rows 8b .. 8b + 7 as full 128-B rows
        if constexpr (DIAG != 3)
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "+v"(rowv[b]) : "v"(stg_r), "i"(b * 8 * STG_PITCH) : "memory");
      } else if constexpr (p == 1) {   // O = 2H + 2, 2H + 3: re-seeds of both halves
        seed(std::integral_constant<int, 2 * p + (O - (2 * H + 2))>{}, jj);
      }
    }
  };

  // one 64-row tile into acc[BUF]; the gaps drain acc[1 - BUF] (store descriptor sd: tile rtp's
  // rows below lim; sdp: the previously drained tile, whose last rows the full-row path stores here)
  auto tile = [&](auto BUFc, int rt, const StoreD& sd, const StoreD& sdp) {
    constexpr int BUF = decltype(BUFc)::value;
    const __amdgpu_buffer_rsrc_t dA0 = tile_rsrc(rt), dA1 = tile_rsrc(rt + 1), dA2 = tile_rsrc(rt + 2);
    sfor<0, WST_NK>([&](auto KSc) {
      constexpr int KS = decltype(KSc)::value;
      constexpr int slot_n = (8 * BUF + KS + 1) % NS;     // next step's slot (read)
      constexpr int slot_d = (8 * BUF + KS + DP) % NS;    // step y + DEPTH's slot (DMA)
      constexpr int n_ops = wsp_nops<EPI, ACT>(KS);
      // step y+1 landed (2 pieces per step, issued unconditionally -- past the block's end they
      // land in dead slots -- so exactly 28 loads are younger-or-equal here) and, after the
      // barrier, every wave's pieces of it; every wave is also past its reads of slot y-1, which
      // the DMA below refills
      // every WSP_BARP-th step: steps y+1 .. y+WSP_BARP landed (the younger DMA steps y+WSP_BARP+1 ..
      // y+DEPTH-1 may be in flight, 2 pieces each), then one barrier for all of them
      if constexpr (KS % wst_barp<EPI>() == 0) {
        if constexpr (DIAG != 2 && DIAG != 4) wst_vmcnt<2 * (DP - 1 - wst_barp<EPI>())>();
        if constexpr (DIAG != 10) asm volatile("s_barrier" ::: "memory");
      }
      bf16x8(&cur)[4][2] = afr[KS & 1];
      bf16x8(&nxt)[4][2] = afr[(KS + 1) & 1];
      sfor<0, 32>([&](auto Ic) {
        constexpr int i = decltype(Ic)::value;
        constexpr int kh = i >> 4, nb = (i >> 2) & 3, mb = i & 3;
        if constexpr (DIAG != 1) mfma_wa<FMT>(acc[BUF][nb][mb], wf[nb][2 * KS + kh], cur[mb][kh]);
        if constexpr (i < 16 && (i & 1) == 0) {
          constexpr int rmb = (i >> 1) & 3, rkh = i >> 3;
          lds_read_into<(slot_n & 7) * WST_SLOT + rmb * 2048>(nxt[rmb][rkh], rdb[slot_n >> 3][rkh]);
        }
        if constexpr ((i == 6 || i == 22) && DIAG != 4) {
          constexpr int toff = (KS + DP) / WST_NK;   // tile of step y + DEPTH: this one, the next or the one after
          issue_piece(toff == 0 ? dA0 : toff == 1 ? dA1 : dA2, std::integral_constant<int, i == 22 ? 1 : 0>{},
                      std::integral_constant<int, (KS + DP) % WST_NK>{}, std::integral_constant<int, slot_d>{});
        }
        sfor<wsp_lo(i, n_ops), wsp_lo(i + 1, n_ops)>([&](auto Oc) {
          epi_op(KSc, Oc, acc[1 - BUF], sd, sdp, std::true_type{}, std::integral_constant<int, 1 - BUF>{});
        });
        __builtin_amdgcn_sched_barrier(0);
      });
      constexpr int late = wsp_late_seeds<EPI, ACT>(KS);
      if constexpr (KS == WST_NK - 1 || late == 0 || !WSP_LGKM)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else if constexpr (late == 1)
        asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
    });
  };
  auto drain = [&](f32x4(&a)[4][4], int rt, const StoreD& sdp) {
    const StoreD sd = store_rsrc(rt, M);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");   // last MFMA writes -> VALU reads
    sfor<0, 8>([&](auto Sc) {
      constexpr int S = decltype(Sc)::value;
      sfor<0, wsp_nops<EPI, ACT>(S)>([&](auto Oc) { epi_op(Sc, Oc, a, sd, sdp, std::false_type{}, std::integral_constant<int, 1>{}); });
    });
    return sd;
  };
  // the full-row path's last pending rows (group 7 of the last drained tile, descriptor sd)
  auto flush_rows = [&](const StoreD& sd) {
    if constexpr (wsp_fullrow<EPI, ACT>() && DIAG != 5) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int b = 0; b < 2; ++b)
        __builtin_amdgcn_raw_buffer_store_b128(rowv[b], sd.d[0], voffF[b] + (unsigned)(16 * 3 * old[0] * 2), 0,
                                               DIAG == 8 ? 2 : DIAG == 9 ? 16 : 0);
    }
  };

  // DW2: the dw2 outputs whose last pw1 row lies in tile rtp (drained into ring slot `slot`; tile
  // rtp - 1 sits in the other slot).  Wave-local: a wave reads only its own 64 ring columns.  Lane =
  // (position k of 8 in flight, 8 channels); the same f32 taps and FMA order as fe_dw2_kernel.
  // DW2_DEFER: the previous phase's outputs (npend passes) leave from the LDS staging area here, so
  // their store acknowledgements overlap this phase's arithmetic instead of the next DMA waits
  const unsigned dstg = dww + DW2_WB + 4 * DW2_TABW + (unsigned)wv * DW2_STG;
  int npend = 0;
  auto dw2_flush = [&]() {
    if constexpr (EPI == EPI_DW2 && DW2_DEFER) {
      for (int p = 0; p < npend; ++p) {
        u32x4 v;
        unsigned off;
        asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(v) : "v"(dstg + (unsigned)p * 1280 + 16u * lane) : "memory");
        asm volatile("ds_read_b32 %0, %1 offset:1024" : "=v"(off) : "v"(dstg + (unsigned)p * 1280 + 4u * lane) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (off != 0xffffffffu) {
          u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<bf16*>(ep.out) + off);
          if constexpr (DW2_NT) __builtin_nontemporal_store(v, dst);
          else *dst = v;
        }
      }
      npend = 0;
    }
  };
  auto dw2_phase = [&](int rtp, int slot) {
    (void)dww;
    (void)dstg;
    dw2_flush();
    if constexpr (EPI == EPI_DW2 && DW2_DIAG != 2) {
      const int wrows = ep.t2n * 19;
      const int R = rtp * WST_MT + lane;
      bool last = false;
      unsigned ooff = 0;   // DW2_OFFTAB: the output's element offset (without the lane's channels)
      if (R < M) {
        const int w_ = R / wrows, rem = R - w_ * wrows, t2 = rem / 19, f2 = rem - t2 * 19;
        last = t2 >= 2 && !(t2 & 1) && f2 >= 2 && !(f2 & 1);
        ooff = (unsigned)(((w_ * ep.t3n + ((t2 - 2) >> 1)) * 9 + ((f2 - 2) >> 1)) * ep.ldo + ct * 256);
      }
      const unsigned long long mask = __builtin_amdgcn_ballot_w64(last);
      const int n = __builtin_popcountll(mask);
      const unsigned tab = dww + DW2_WB + (unsigned)wv * DW2_TABW;
      if (last) {
        const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
        if constexpr (DW2_OFFTAB) {
          typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
          asm volatile("ds_write_b64 %0, %1" ::"v"(tab + 8u * rank), "v"((u32x2_t){(unsigned)lane, ooff}) : "memory");
        } else {
          asm volatile("ds_write_b32 %0, %1" ::"v"(tab + 4u * rank), "v"(lane) : "memory");
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (DW2_DIAG == 3) return;   // timing only: the phase's setup (output rows, rank table) alone
      const int cl = wv * 64 + 8 * (lane & 7);   // the lane's 8 channels within the block's 256
      const float* dwl = reinterpret_cast<const float*>(smem + NS * WST_SLOT + 1024 + DW2_RING);
      const char* ring = smem + NS * WST_SLOT + 1024 + 128 * wv + 16 * (lane & 7);
      // DW2_PPL positions per lane (k, k + 8, ..): each tap's 8 f32 weights are read from LDS once for
      // all of them; packed f32 FMAs (v_pk_fma_f32: per-element fma, the same rounding as fmaf)
      constexpr int P = DW2_PPL;
      static_assert(!DW2_DOT2 || (DW2_PIPE >= 2 && DW2_PPL == 1), "DW2_DOT2 weights serve the pipelined P = 1 path only");
      const bool defer = DW2_DEFER && P == 1 && n <= 24;
      for (int base = 0; base < n; base += 8 * P) {
        const int k0 = base + (lane >> 3);
        if (defer)   // marker first: lanes without a position store nothing at the flush
          asm volatile("ds_write_b32 %0, %1 offset:1024" ::"v"(dstg + (unsigned)(base >> 3) * 1280 + 4u * lane), "v"(0xffffffffu) : "memory");
        if (k0 >= n) continue;
        int Rl[P];
        unsigned Ol = 0;   // DW2_OFFTAB, P == 1: the output offset from the table
        f32x4 b0, b1;
        if constexpr (DW2_PIPE >= 2 && P == 1 && DW2_OFFTAB) {
          // the rank, the output offset and the bias seeds in one LDS round trip
          typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
          const unsigned bl = dww + 4u * (unsigned)(9 * 256 + cl);
          u32x2_t ro;
          asm volatile("ds_read_b64 %0, %1" : "=v"(ro) : "v"(tab + 8u * min(k0, n - 1)) : "memory");
          asm volatile("ds_read_b128 %0, %1" : "=v"(b0) : "v"(bl) : "memory");
          asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(b1) : "v"(bl) : "memory");
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ro), "+v"(b0), "+v"(b1)::"memory");
          Rl[0] = (int)ro[0];
          Ol = ro[1];
        } else if constexpr (DW2_PIPE >= 2 && P == 1) {
          // the rank and the bias seeds in one LDS round trip
          const unsigned bl = dww + 4u * (unsigned)(9 * 256 + cl);
          asm volatile("ds_read_b32 %0, %1" : "=v"(Rl[0]) : "v"(tab + 4u * min(k0, n - 1)) : "memory");
          asm volatile("ds_read_b128 %0, %1" : "=v"(b0) : "v"(bl) : "memory");
          asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(b1) : "v"(bl) : "memory");
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(Rl[0]), "+v"(b0), "+v"(b1)::"memory");
        } else {
#pragma unroll
          for (int u = 0; u < P; ++u) {
            const int ku = min(k0 + 8 * u, n - 1);
            int rr;
            asm volatile("ds_read_b32 %0, %1" : "=v"(rr) : "v"(tab + (DW2_OFFTAB ? 8u : 4u) * ku) : "memory");
            Rl[u] = rr;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          b0 = *reinterpret_cast<const f32x4*>(dwl + 9 * 256 + cl);
          b1 = *reinterpret_cast<const f32x4*>(dwl + 9 * 256 + cl + 4);
        }
        f32x2 a[P][4];
        {
#pragma unroll
          for (int u = 0; u < P; ++u) {
            a[u][0] = (f32x2){b0[0], b0[1]};
            a[u][1] = (f32x2){b0[2], b0[3]};
            a[u][2] = (f32x2){b1[0], b1[1]};
            a[u][3] = (f32x2){b1[2], b1[3]};
          }
        }
        // ring row of pw1 row `row` (tile t sits in slot (t - r0c) & 1): (row - 64 r0c) mod 128
        int rb[P];
#pragma unroll
        for (int u = 0; u < P; ++u) rb[u] = Rl[u] + rtp * WST_MT - WST_MT * r0c + 128;
        if constexpr (DW2_PIPE && P == 1) {
          // the 9 taps (t = 3v + i, the order below) software-pipelined two deep: tap t + 2's ring row and
          // weights are read while tap t computes (the compiler issued each tap's reads only after the
          // previous tap's FMAs: one LDS round trip per tap with one wave per SIMD)
          const unsigned rl = ring_base + 128u * (unsigned)wv + 16u * (unsigned)(lane & 7);
          const unsigned wl = dww + 4u * (unsigned)cl;
          u32x4 xs[2];
          f32x4 ws[2][2];
          // the bias seeds landed before the first asm read (the compiler's own lgkmcnt wait for them
          // would otherwise come after those reads and drain them)
          asm volatile("" : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[0][2]), "+v"(a[0][3]));
          auto issue = [&xs, &ws, &rb, rl, wl](auto Tc) {
            constexpr int t = decltype(Tc)::value, v = t / 3, i = t % 3, sl = t & 1;
            constexpr int off = (2 - i) * 19 + (2 - v);
            const unsigned xa = rl + (unsigned)(((rb[0] - off) & 127) * DW2_RP);
            asm volatile("ds_read_b128 %0, %1" : "=v"(xs[sl]) : "v"(xa) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ws[sl][0]) : "v"(wl), "i"((3 * i + v) * 1024) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ws[sl][1]) : "v"(wl), "i"((3 * i + v) * 1024 + 16) : "memory");
          };
          issue(std::integral_constant<int, 0>{});
          issue(std::integral_constant<int, 1>{});
          sfor<0, 9>([&xs, &ws, &a, &issue](auto Tc) {
            constexpr int t = decltype(Tc)::value, sl = t & 1;
            if constexpr (t < 8)
              asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(xs[sl]), "+v"(ws[sl][0]), "+v"(ws[sl][1])::"memory");
            else
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xs[sl]), "+v"(ws[sl][0]), "+v"(ws[sl][1])::"memory");
            const f32x4 w0 = ws[sl][0], w1 = ws[sl][1];
            const u32x4 x = xs[sl];
            if constexpr (DW2_DOT2) {
              // channel pair h: one dot2 per channel against its (w, 0) / (0, w) weight dword
              const u32x4 d0 = __builtin_bit_cast(u32x4, w0), d1 = __builtin_bit_cast(u32x4, w1);
              const unsigned wd[8] = {d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
#pragma unroll
              for (int h = 0; h < 4; ++h) {
                a[0][h][0] = dw2_dot<FMT>(x[h], wd[2 * h], a[0][h][0]);
                a[0][h][1] = dw2_dot<FMT>(x[h], wd[2 * h + 1], a[0][h][1]);
              }
            } else {
              const f32x2 wq[4] = {(f32x2){w0[0], w0[1]}, (f32x2){w0[2], w0[3]}, (f32x2){w1[0], w1[1]}, (f32x2){w1[2], w1[3]}};
#pragma unroll
              for (int h = 0; h < 4; ++h) {
                const f32x2 xv = dw2_unpk2<FMT>(x[h]);
                a[0][h] = __builtin_elementwise_fma(wq[h], xv, a[0][h]);
              }
            }
            if constexpr (t + 2 < 9) issue(std::integral_constant<int, t + 2>{});
          });
        } else
#pragma unroll DW2_VUNROLL
        for (int v = 0; v < 3; ++v)
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const int off = (2 - i) * 19 + (2 - v);
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(dwl + (3 * i + v) * 256 + cl);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(dwl + (3 * i + v) * 256 + cl + 4);
            const f32x2 wq[4] = {(f32x2){w0[0], w0[1]}, (f32x2){w0[2], w0[3]}, (f32x2){w1[0], w1[1]}, (f32x2){w1[2], w1[3]}};
#pragma unroll
            for (int u = 0; u < P; ++u) {
              const u32x4 x = *reinterpret_cast<const u32x4*>(ring + ((rb[u] - off) & 127) * DW2_RP);
#pragma unroll
              for (int h = 0; h < 4; ++h) {
                const f32x2 xv = dw2_unpk2<FMT>(x[h]);
                a[u][h] = __builtin_elementwise_fma(wq[h], xv, a[u][h]);
              }
            }
          }
#pragma unroll
        for (int u = 0; u < P; ++u) {
          if (k0 + 8 * u >= n) break;
          u32x4 o8;   // the same conversion as fe_dw2_kernel's store8 (round to nearest even)
#pragma unroll
          for (int h = 0; h < 4; ++h) o8[h] = pack_h2<FMT>(a[u][h][0], a[u][h][1]);
          size_t oel;
          if constexpr (DW2_OFFTAB && DW2_PIPE >= 2 && P == 1) {
            oel = (size_t)Ol + cl;
          } else {
            const int R = rtp * WST_MT + Rl[u];
            const int w_ = R / wrows, rem = R - w_ * wrows, t2 = rem / 19, f2 = rem - t2 * 19;
            const int t3 = (t2 - 2) >> 1, f3 = (f2 - 2) >> 1;
            oel = ((size_t)(w_ * ep.t3n + t3) * 9 + f3) * ep.ldo + ct * 256 + cl;
          }
          u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<bf16*>(ep.out) + oel);
          if constexpr (DW2_DIAG != 1) {
            if (defer) {
              const unsigned sb = dstg + (unsigned)(base >> 3) * 1280;
              asm volatile("ds_write_b128 %0, %1 offset:0" ::"v"(sb + 16u * lane), "v"(o8) : "memory");
              asm volatile("ds_write_b32 %0, %1 offset:1024" ::"v"(sb + 4u * lane),
                           "v"((unsigned)oel) : "memory");
            } else if constexpr (DW2_NT) {
              __builtin_nontemporal_store(o8, dst);
            } else {
              *dst = o8;
            }
          }
        }
      }
      if (defer) npend = (n + 7) >> 3;
    }
  };

  // prologue: weights in AGPRs (s_nop: AGPR writes -> MFMA reads), step 0 landed, its fragments read
  asm volatile("s_nop 7" ::: "memory");
  wst_vmcnt<2 * (DP - 1)>();   // step 0 landed: DEPTH - 1 younger steps in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // + the bias in LDS
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      acc[0][nb][mb] = (f32x4){0.f, 0.f, 0.f, 0.f};
      lds_read_into<0>(acc[0][nb][mb], bias_lds + nb * 64);
    }
  sfor<0, 8>([&](auto Rc) {
    constexpr int r = decltype(Rc)::value;
    lds_read_into<(r & 3) * 2048>(afr[0][r & 3][r >> 2], rdb[0][r >> 2]);
  });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // tiles in pairs (acc[0], acc[1]); an odd count runs one dummy tile past the block's range whose
  // results are never stored (lim = 0 in the drain), which keeps one straight loop body
  const int npair = (r1 - r0c + 1) >> 1;
  // the first tile's gaps drain a fake previous tile: rows of a REAL tile (never negative, so the
  // store descriptors' row bases stay inside the output) with lim = 0, i.e. zero-record stores
  StoreD sd_prev = store_rsrc(r0c, 0);
  for (int it = 0; it < npair; ++it) {
    const int rt = r0c + 2 * it;
    const StoreD sd0 = store_rsrc(it > 0 ? rt - 1 : rt, it > 0 ? M : 0);
    tile(std::integral_constant<int, 0>{}, rt, sd0, sd_prev);
    if (EPI == EPI_DW2 && it > 0 && rt - 1 >= r0) dw2_phase(rt - 1, 1);   // drained into ring slot 1
    const StoreD sd1 = store_rsrc(rt, M);
    tile(std::integral_constant<int, 1>{}, rt + 1, sd1, sd0);
    if (EPI == EPI_DW2 && rt >= r0 && rt < r1) dw2_phase(rt, 0);
    sd_prev = sd1;
  }
  if (((r1 - r0c) & 1) == 0) {
    flush_rows(drain(acc[1], r1 - 1, sd_prev));
    if (EPI == EPI_DW2 && r1 - 1 >= r0) dw2_phase(r1 - 1, 1);
  } else {
    flush_rows(sd_prev);   // odd count: the last tile call drained the last real tile
  }
  dw2_flush();
  // the pieces issued past the end land (and the drain's seed reads return) before the
  // workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

template <int EPI, int ACT>
static int launch_wst(const bf16* A, int lda, const bf16* W, int ldw, int M, int N, const EpiArgs& ep,
                      hipStream_t st) {
  int n_cu = cu_count() / 8 * 8;
  // small launches in a pipelined caller (endless_decode's segments): fewer workgroups, each taking
  // more row tiles per weight-tile fill, and CUs left to the other streams' kernels
  if (ep.wsp_small_div > 1 && M < ep.wsp_small_rows) n_cu = max(8 * (N >> 8), n_cu / ep.wsp_small_div / 8 * 8);
  // buffer descriptors are built per 64-row tile on 64-bit bases (offsets inside one tile stay
  // below 64 rows x ld), so outputs past 2 GiB (a 980-minute batch's FFN hidden: 3 GB) stay here
#define WSP_LAUNCH(D)                                                                                         \
  do {                                                                                                        \
    if (ep.f16) {                                                                                             \
      hipLaunchKernelGGL((gemm_wsp_kernel<EPI, ACT, D, 1>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep); \
      break;                                                                                                  \
    }                                                                                                         \
    hipLaunchKernelGGL((gemm_wsp_kernel<EPI, ACT, D, 0>), dim3(n_cu), dim3(256), 0, st, A, lda, W, ldw, M, N, ep); \
  } while (0)
#ifdef CFM_GEMM_DIAG
  // DIAG (timing experiments only, diagnostic builds, model option "gemm_diag"): 1 = no MFMAs,
  // 2 = no DMA wait (stale LDS), 3 = no epilogue (re-seeds only), 4 = no DMA in the loop (stale LDS),
  // 5 = no stores, 7 = full-line stores (wrong layout), 10 = no per-step barrier (wrong results)
  switch (ep.diag) {
    case 1: WSP_LAUNCH(1); break;
    case 2: WSP_LAUNCH(2); break;
    case 3: WSP_LAUNCH(3); break;
    case 4: WSP_LAUNCH(4); break;
    case 5: WSP_LAUNCH(5); break;
    case 7: WSP_LAUNCH(7); break;
    case 10: WSP_LAUNCH(10); break;
    default: break;
  }
  if ((ep.diag >= 1 && ep.diag <= 7 && ep.diag != 6) || ep.diag == 10) {
    CFM_CHECK_LAUNCH();
    return 0;
  }
#endif
  // store policy (per GEMM site, EpiArgs::store_mode): 2 = nt
  if (ep.store_mode == 2) WSP_LAUNCH(8);
  else WSP_LAUNCH(0);
#undef WSP_LAUNCH
  CFM_CHECK_LAUNCH();
  return 0;
}

}  // namespace cfm
