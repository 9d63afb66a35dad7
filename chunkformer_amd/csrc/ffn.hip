// Fused position-wise feed-forward block (bf16, d = 512):
//
//   y = W2 . SiLU(W1 . x + b1) + b2        (positionwise_feed_forward.py:21-60, activation = SiLU)
//
// The two-GEMM path writes the [rows, ff] hidden activation to HBM and reads it back
// (4 x 186 MB per FFN at the bench size); FFN w1 sits on the HBM/MFMA ridge because of that
// write.  Here the hidden activation never leaves the CU:
//
//   * a block owns 128 rows; wave w (of 4, one per SIMD, 512-register budget) owns 32 rows:
//     its x fragments (32 rows x 512, 128 VGPRs) stay in registers for the whole block and its
//     output accumulators out^T[512][32] (256 VGPRs) too;
//   * the hidden dimension runs in chunks of 64: h^T = W1_f . x^T (MFMA A = W1 rows, B = x
//     rows), bias + SiLU + bf16 in registers, and the C-layout of h^T is used directly as the
//     B operand of out^T += W2_f . h^T: lane (row, g) holds hidden 4g..4g+3 of two 16-row
//     blocks, i.e. a fixed permutation of the 32-deep K fragment, which the repacked W2 slab
//     matches (cfm_ffn_pack below) -- no LDS round trip, no transpose;
//   * the only operand stream is the weights (4 MiB per layer FFN, L2 / Infinity-Cache
//     resident, identical for every block): repacked at model load into 512 contiguous 8-KiB
//     slabs in consumption order (per hidden chunk: 8 W1 K-slabs, 8 W2 output slabs), each the
//     exact LDS image of 8 MFMA fragments (lane-linear, conflict-free ds_read_b128), streamed
//     by `buffer_load_dwordx4 ... lds` into a 20-slot (160 KiB) ring in batches of 4 slabs;
//     three batches stay in flight, one wait + barrier per batch (64 MFMAs per wave);
//   * fragment reads run one 4-fragment group ahead of the MFMAs (also across batch
//     boundaries: a batch is waited for one batch early), so the MFMA issue stream only waits
//     on LDS latency at row-block boundaries.
// HBM traffic per row: x 1 KiB in, y 1 KiB out.
#include "cfm_common.h"
#include "cfm_kernels.h"
#include <cstdlib>

namespace cfm {

namespace {
constexpr int FD = 512;            // model dim (register-resident x fragments / accumulators)
constexpr int FROWS = 128;         // rows per block, 32 per wave
constexpr int SLAB = 8192;         // bytes per weight slab (8 MFMA fragments)
constexpr int RSLOTS = 20;         // ring slots (160 KiB)
constexpr int BATCH = 4;           // slabs per wait + barrier
constexpr int RB = RSLOTS / BATCH; // ring batches (5)
constexpr int KQ = FD / 64;        // W1 K-slabs per hidden chunk (8)
constexpr int OQ = FD / 64;        // W2 output slabs per hidden chunk (8)
constexpr int SPF = KQ + OQ;       // slabs per hidden chunk (16 = 4 batches)
}  // namespace

typedef int i32x4_f __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_f __attribute__((ext_vector_type(2)));

template <int OFF>
CFM_DEV bf16x8 ffn_lds_read(unsigned addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
#define FFN_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define FFN_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

// 4 consecutive f32 of a wave-uniform array selected by lane group g: bias[base + 4g .. +3]
CFM_DEV f32x4 smem_bias4(const float* p /*uniform, 16 floats*/, int g) {
  i32x4_f s0, s1, s2, s3;
  asm volatile("s_load_dwordx4 %0, %4, 0x0\n\ts_load_dwordx4 %1, %4, 0x10\n\t"
               "s_load_dwordx4 %2, %4, 0x20\n\ts_load_dwordx4 %3, %4, 0x30\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&s"(s3)
               : "s"(p)
               : "memory");
  const i32x4_f lo = (g & 1) ? s1 : s0, hi = (g & 1) ? s3 : s2;
  return __builtin_bit_cast(f32x4, (g & 2) ? hi : lo);
}

// h^T accumulation in VGPRs (inline asm pins the VGPR form): the 256 out^T accumulators take
// every AGPR, and the allocator otherwise spills trying to fit h^T beside them.  Hazards the
// compiler cannot see: the seeds (VALU writes) are >= a batch before the first use as SrcC and
// the SiLU reads follow >= 8 MFMAs after the last write plus an explicit s_nop pad.
CFM_DEV void mfma_v(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

CFM_DEV float ffn_silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
CFM_DEV unsigned ffn_pack2(float a, float b) {
  typedef bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, (b2){(bf16)a, (bf16)b});
}

// DIAG (timing experiments, wrong results): 1 = no SiLU, 2 = no bias seeding, 3 = no batch waits /
// barriers after the first, 4 = no LDS fragment reads in the loop
template <int DIAG, bool NT>
__global__ __launch_bounds__(256, 1) void ffn_fused_kernel(const bf16* __restrict__ X, int M,
                                                           const bf16* __restrict__ Ws, const float* __restrict__ b1,
                                                           const float* __restrict__ b2, bf16* __restrict__ Y, int ff) {
  __shared__ __attribute__((aligned(16))) char ring[RSLOTS * SLAB];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int fr = lane & 15, g = lane >> 4;
  const int nF = ff >> 6;
  const int bpb = nF * (SPF / BATCH);                      // batches per row block (4 per hidden chunk)
  const int nblk = (M + FROWS - 1) / FROWS;
  if ((int)blockIdx.x >= nblk) return;
  const int my_blocks = (nblk - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int ZT = my_blocks * bpb;                          // batches this block streams

  // ---- weight stream: batch z = slabs 4(z mod bpb) .. +3 of the per-row-block sequence, ring slot z mod 5
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)Ws, (short)0, nF * SPF * SLAB, 0x00020000);
  const int voff = wid * 2048 + lane * 16;                 // this wave's 2 KiB of every slab
  const unsigned ring_base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)ring;
  int iz = 0, iz_rel = 0, iz_slot = 0;                     // next batch to issue
  auto issue = [&]() {
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int slab_off = (iz_rel * BATCH + i) * SLAB;
      char* dst = ring + (iz_slot * BATCH + i) * SLAB + wid * 2048;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)dst, 16, voff, slab_off, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(dst + 1024), 16, voff,
                                               slab_off + 1024, 0, 0);
    }
    ++iz;
    iz_rel = iz_rel + 1 == bpb ? 0 : iz_rel + 1;
    iz_slot = iz_slot + 1 == RB ? 0 : iz_slot + 1;
  };

  bf16x8 xf[2][16];        // x fragments: rows 16rb + fr, k 32kk + 8g .. +7
  f32x4 oacc[32][2];       // out^T: outputs 16ob + 4g .. +3 of row 16rb + fr
  f32x4 hacc[4][2];        // h^T chunk: hidden 16hb + 4g .. +3 of row 16rb + fr (bias-seeded)
  bf16x8 hf[2][2];         // SiLU(h) as the B operand of the W2 MFMAs: [K-half s][rb]
  bf16x8 wq[2][4];         // W fragment groups (double buffer)

  // group reads.  W1 slab (K 128): fragments [hb' 2][kk 4] -> group u = kk 2u, 2u+1 of both hb';
  // W2 slab (128 outputs): fragments [ob' 8] -> group u = ob' 4u .. 4u+3.
  auto read_w1 = [&](bf16x8 (&w)[4], unsigned slab_addr, int u) {
    if (DIAG == 4) return;
    const unsigned a = slab_addr + (unsigned)(u * 2048 + lane * 16);
    w[0] = ffn_lds_read<0>(a);      // hb' 0, kk 2u
    w[1] = ffn_lds_read<1024>(a);   // hb' 0, kk 2u+1
    w[2] = ffn_lds_read<4096>(a);   // hb' 1, kk 2u
    w[3] = ffn_lds_read<5120>(a);   // hb' 1, kk 2u+1
  };
  auto read_w2 = [&](bf16x8 (&w)[4], unsigned slab_addr, int u) {
    if (DIAG == 4) return;
    const unsigned a = slab_addr + (unsigned)(u * 4096 + lane * 16);
    w[0] = ffn_lds_read<0>(a);
    w[1] = ffn_lds_read<1024>(a);
    w[2] = ffn_lds_read<2048>(a);
    w[3] = ffn_lds_read<3072>(a);
  };
  // hidden-chunk-F bias seeds of hacc[2s], hacc[2s+1] (scalar loads; lgkmcnt(0) inside)
  auto seed = [&](int F, int s) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x4 b = DIAG == 2 ? (f32x4){0.f, 0.f, 0.f, 0.f} : smem_bias4(b1 + 64 * F + 16 * (2 * s + t), g);
      hacc[2 * s + t][0] = b;
      hacc[2 * s + t][1] = b;
    }
  };
  // SiLU of the 2 values (index p = 2q, 2q+1 of the 16 of half s) in place; pack at q == 7
  auto silu_part = [&](int s, int q) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int p = 2 * q + e, t = p >> 3, rb = (p >> 2) & 1, v = p & 3;
      if (DIAG != 1) hacc[2 * s + t][rb][v] = ffn_silu(hacc[2 * s + t][rb][v]);
    }
    if (q == 7) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const f32x4 a = hacc[2 * s][rb], c = hacc[2 * s + 1][rb];
        hf[s][rb] = __builtin_bit_cast(bf16x8, (u32x4){ffn_pack2(a[0], a[1]), ffn_pack2(a[2], a[3]),
                                                      ffn_pack2(c[0], c[1]), ffn_pack2(c[2], c[3])});
      }
    }
  };

  // prologue: batches RB .. RB+PF_AHEAD-1 warmed, batches 0..4 in flight, 0 and 1 landed and visible
  for (int p = 0; p < RB && iz < ZT; ++p) issue();
  if (ZT >= RB) FFN_VM(24); else FFN_VM(0);   // younger than batch 1's DMA: batches 2..4
  seed(0, 0);
  seed(0, 1);
  asm volatile("s_barrier" ::: "memory");

  int z = 0;               // batch being consumed
  int zslot = 0;
  read_w1(wq[0], ring_base, 0);
  for (int bi = 0; bi < my_blocks; ++bi) {
    const int row0 = ((int)blockIdx.x + bi * (int)gridDim.x) * FROWS + wid * 32;
    // ---- x fragments of the wave's 32 rows (clamped: rows >= M are computed, never stored)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const bf16* xp = X + (size_t)min(row0 + 16 * rb + fr, M - 1) * FD + 8 * g;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        xf[rb][kk] = NT ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(xp + 32 * kk))
                        : *reinterpret_cast<const bf16x8*>(xp + 32 * kk);
    }
    FFN_VM(0);   // x landed (also lands the weight batches in flight: once per row block)
#pragma unroll
    for (int ob = 0; ob < 32; ++ob) {
      oacc[ob][0] = (f32x4){0.f, 0.f, 0.f, 0.f};
      oacc[ob][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    unsigned sbase = ring_base + (unsigned)zslot * (BATCH * SLAB);

    for (int F = 0; F < nF; ++F) {
      const int Fn = F + 1 == nF ? 0 : F + 1;   // the chunk the next seeds are for
      // 4 batches x 4 slabs x 2 groups; group n = 8b + 2i + u (batch b, slab i, half u) uses wq[n & 1]
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int n = 8 * b + 2 * i + u;
            const bool last = (i == 3 && u == 1);
            // ---- prefetch the next group (next batch: landed and visible since the previous boundary)
            const bool more = !(last && b == 3 && F + 1 == nF && bi + 1 == my_blocks);
            if (more) {
              const int nb = last ? (b + 1) & 3 : b, ni = last ? 0 : (u ? i + 1 : i), nu = last ? 0 : (u ^ 1);
              const unsigned na = (last ? ring_base + (unsigned)(zslot == RB - 1 ? 0 : zslot + 1) * (BATCH * SLAB) : sbase) +
                                  (unsigned)(ni * SLAB);
              if (nb < 2) read_w1(wq[(n + 1) & 1], na, nu); else read_w2(wq[(n + 1) & 1], na, nu);
              FFN_LGKM(4);
            } else {
              FFN_LGKM(0);
            }
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8(&w)[4] = wq[n & 1];
            if (b < 2) {
              // h^T[2b + hb'][.] += W1[.][128 i + 32 kk + .] . x[.][128 i + 32 kk + .],  kk = 2u + t
#pragma unroll
              for (int hb = 0; hb < 2; ++hb)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                  for (int rb = 0; rb < 2; ++rb)
                    mfma_v(hacc[2 * b + hb][rb], w[2 * hb + t], xf[rb][4 * i + 2 * u + t]);
            } else {
              // out^T[128 i + 16 ob' + .][.] += W2[.][64F + 32 s + perm] . SiLU(h)^T, s = b - 2
#pragma unroll
              for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int rb = 0; rb < 2; ++rb)
                  oacc[8 * i + 4 * u + k][rb] =
                      __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[k], hf[b - 2][rb], oacc[8 * i + 4 * u + k][rb], 0, 0, 0);
            }
            // ---- VALU work beside the MFMAs: SiLU of half 0 during W1 half 1, of half 1 during
            // W2 half 0; bias seeds of the next chunk once their hacc are free
            const int q = 2 * i + u;
            if ((b == 1 || b == 2) && q == 0) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            if (b == 1) silu_part(0, q);
            if (b == 2) silu_part(1, q);
            if (b == 2 && q == 7) seed(Fn, 0);
            if (b == 3 && q == 7) seed(Fn, 1);
            // ---- batch boundary: batch z+2 landed (own DMA) and, after the barrier, visible; every
            // wave is done with batch z, whose slot takes batch z+5
            if (last) {
              if (DIAG != 3) {
                if (z + 4 < ZT) FFN_VM(16); else FFN_VM(0);   // younger than z+2's DMA: batches z+3, z+4
                asm volatile("s_barrier" ::: "memory");
                if (iz < ZT) issue();
              }
              ++z;
              zslot = zslot == RB - 1 ? 0 : zslot + 1;
              sbase = ring_base + (unsigned)zslot * (BATCH * SLAB);
            }
            __builtin_amdgcn_sched_barrier(0);   // one group at a time (bounded live ranges)
          }
    }
    // ---- epilogue: y[row][col] = out + b2 (bf16); pairs of 16-column blocks -> one 16-B store per lane and row
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int m = row0 + 16 * rb + fr;
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        // b2 added here (plain loads: the weight stream is landed at the next row block anyway)
        const f32x4 ba = *reinterpret_cast<const f32x4*>(b2 + 32 * p + 4 * g);
        const f32x4 bc = *reinterpret_cast<const f32x4*>(b2 + 32 * p + 16 + 4 * g);
        const f32x4 a = oacc[2 * p][rb] + ba, c = oacc[2 * p + 1][rb] + bc;
        const auto r0 = __builtin_amdgcn_permlane16_swap(ffn_pack2(a[0], a[1]), ffn_pack2(c[0], c[1]), false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(ffn_pack2(a[2], a[3]), ffn_pack2(c[2], c[3]), false, false);
        if (m < M) {
          u32x4* yp = reinterpret_cast<u32x4*>(Y + (size_t)m * FD + 32 * p + 16 * (g & 1) + 8 * (g >> 1));
          if (NT)   // sc1 (write-through) store: the line leaves the XCD L2, which stays with the weight stream
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(yp), "v"((u32x4){r0[0], r1[0], r0[1], r1[1]})
                         : "memory");
          else
            *yp = (u32x4){r0[0], r1[0], r0[1], r1[1]};
        }
      }
    }
  }
  FFN_VM(0);
}

static int g_ffn_variant = 0;   // A/B switch ("ffn_variant" model option): 1 = nt x loads + sc1 y stores
void ffn_set_variant(int v) { g_ffn_variant = v; }

int ffn_fused(const bf16* x, int M, const bf16* wstream, const float* b1, const float* b2, bf16* y, int d, int ff,
              hipStream_t st) {
  if (M <= 0) return 0;
  if (d != FD || ff % 64 || ff <= 0) return -1;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
  }
  const int nblk = (M + FROWS - 1) / FROWS;
  const int grid = nblk < n_cu ? nblk : n_cu;
  static int diag = -1;
  if (diag < 0) { const char* e = getenv("CFM_FFN_DIAG"); diag = e ? atoi(e) : 0; }
#define FFN_LAUNCH(D, N) hipLaunchKernelGGL((ffn_fused_kernel<D, N>), dim3(grid), dim3(256), 0, st, x, M, wstream, b1, b2, y, ff)
  if (g_ffn_variant == 1) {
    FFN_LAUNCH(0, true);
  } else {
    switch (diag) {
      case 1: FFN_LAUNCH(1, false); break;
      case 2: FFN_LAUNCH(2, false); break;
      case 3: FFN_LAUNCH(3, false); break;
      case 4: FFN_LAUNCH(4, false); break;
      default: FFN_LAUNCH(0, false);
    }
  }
#undef FFN_LAUNCH
  CFM_CHECK_LAUNCH();
  return 0;
}

// Host repack of W1 [ff][d], W2 [d][ff] (f32, reference layout) into the slab stream (bf16 bits).
// Per hidden chunk F (64 units = K-halves s 0/1 of 32) the 16 slabs are, in consumption order:
//   W1 half s, K-slab i (s = 0, 1; i = 0..3):  [hb' 2][kk 4][g 4][fr 16][e 8]
//       = W1[64F + 32s + 16hb' + fr][128i + 32kk + 8g + e]
//   W2 half s, output slab i (s = 0, 1; i = 0..3):  [ob' 8][g 4][fr 16][e 8]
//       = W2[128i + 16ob' + fr][64F + 32s + perm(g, e)]
//   perm(g, e) = e < 4 ? 4g + e : 16 + 4g + e - 4   (the C-layout rows of h^T a lane holds)
void ffn_pack_stream(const float* w1, const float* w2, int d, int ff, uint16_t* out,
                     uint16_t (*to_bf16)(float)) {
  const int nF = ff / 64;
  size_t idx = 0;
  for (int F = 0; F < nF; ++F) {
    for (int s = 0; s < 2; ++s)
      for (int i = 0; i < d / 128; ++i)
        for (int hb = 0; hb < 2; ++hb)
          for (int kk = 0; kk < 4; ++kk)
            for (int g = 0; g < 4; ++g)
              for (int fr = 0; fr < 16; ++fr)
                for (int e = 0; e < 8; ++e)
                  out[idx++] = to_bf16(w1[(size_t)(64 * F + 32 * s + 16 * hb + fr) * d + 128 * i + 32 * kk + 8 * g + e]);
    for (int s = 0; s < 2; ++s)
      for (int i = 0; i < d / 128; ++i)
        for (int ob = 0; ob < 8; ++ob)
          for (int g = 0; g < 4; ++g)
            for (int fr = 0; fr < 16; ++fr)
              for (int e = 0; e < 8; ++e) {
                const int h = 64 * F + 32 * s + (e < 4 ? 4 * g + e : 16 + 4 * g + e - 4);
                out[idx++] = to_bf16(w2[(size_t)(128 * i + 16 * ob + fr) * ff + h]);
              }
  }
}

}  // namespace cfm
