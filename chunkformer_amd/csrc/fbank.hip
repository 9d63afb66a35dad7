// Kaldi log-mel filterbank on the GPU: the feature front of the reference's decode paths
// (chunkformer_model.py:276-318 and dataset/processor.py:210-239 call
// torchaudio.compliance.kaldi.fbank with dither 0, energy_floor 0, povey window, snip_edges).
//
// The published algorithm (torchaudio >= 2.5.1, compliance/kaldi.py: fbank, _get_window,
// get_mel_banks; torchaudio is pinned by the reference's pyproject.toml:28 and is not vendored),
// per frame of `win` samples every `shift` samples (snip_edges: 1 + (n - win) / shift frames):
//   remove the frame mean; pre-emphasis y[i] = x[i] - 0.97 x[i-1] (x[-1] = x[0]); window;
//   zero-pad to N = 2^ceil(log2 win); power spectrum |rfft|^2 (N/2 + 1 bins); triangular mel
//   filters (mel = 1127 ln(1 + f/700), low 20 Hz, high = Nyquist); log(max(e, FLT_EPSILON)).
//
// Layout and kernel: the waveform is a flat f32 device array (int16 scale, as the reference feeds
// pydub samples); one 256-thread block takes FB = 16 consecutive frames, 16 threads per frame; each
// wave stages the samples of its 4 frames once in LDS (3 * shift + win: frames overlap) and works
// without block barriers (every exchange is among the 16 lanes of one frame).  The N-point real FFT
// runs as an N/2-point complex FFT of z[n] = y[2n] + i y[2n+1] plus the real-split post-pass: for
// N = 512 (the reference's 25 ms at 16 kHz) a four-step 16 x 16 FFT, two 16-point DFTs in
// registers around one LDS transpose; other sizes a radix-2 FFT in LDS (input written in
// bit-reversed order).  Mel filters are sparse ranges (each FFT bin feeds at most two filters).  Bytes per frame: 4 * shift in (the overlap is re-read from LDS, not
// HBM) + 4 * bins out = 960 B at 16 kHz / 80 bins: the kernel is LDS-bound, far below HBM.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "cfm_common.h"
#include "status.h"

#ifndef CFM_FBANK_DIAG
#define CFM_FBANK_DIAG 0   // timing-only builds (tools/build_variant.py): 1 no mel sums, 2 no DFTs
#endif

namespace cfm {

namespace {
constexpr int FB = 16;    // frames per block (one group)
constexpr int TPF = 16;   // threads per frame
constexpr int FBW = 4;    // frames per wave (64 / TPF)
constexpr int FBK_WSAMPLES = 2048;   // samples staged per wave and group (3 shift + win)

// Every LDS exchange after the constants is between the 16 lanes of one frame, i.e. inside one
// wave: LDS operations of a wave complete in order, so waiting for them (and fencing the
// compiler) replaces the block barriers.
CFM_DEV void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

CFM_DEV int brev(int v, int bits) { return (int)(__builtin_bitreverse32((unsigned)v) >> (32 - bits)); }
CFM_DEV float2 cmul(float2 a, float2 w) { return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x); }

// in-register 16-point DFT, a[k] = sum_m a[m] e^{-2 pi i m k / 16} (radix-2 DIT, natural-order output)
CFM_DEV void fft16(float2 (&a)[16]) {
  constexpr int br[16] = {0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15};
  constexpr float C[8] = {1.f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
                          0.f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f};
  constexpr float S[8] = {0.f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f,
                          1.f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f};
  float2 b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = a[br[i]];
#pragma unroll
  for (int st = 1; st <= 4; ++st) {
    const int half = 1 << (st - 1);
#pragma unroll
    for (int i0 = 0; i0 < 16; ++i0) {
      const int k = i0 & (2 * half - 1);
      if (k >= half) continue;
      const int i1 = i0 + half, e = k << (4 - st);   // W_{2 half}^k = W16^(k 16 / 2 half)
      const float2 t = cmul(b[i1], make_float2(C[e], -S[e]));
      b[i1] = make_float2(b[i0].x - t.x, b[i0].y - t.y);
      b[i0] = make_float2(b[i0].x + t.x, b[i0].y + t.y);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = b[i];
}
}  // namespace

template <int LOGM>
__global__ __launch_bounds__(256) void fbank_kernel(const float* __restrict__ wave, long long n_samples,
                                                    long long n_frames, int shift, int win,
                                                    const float* __restrict__ window, const float2* __restrict__ tw,
                                                    const float2* __restrict__ tw2, const int* __restrict__ mel_lo,
                                                    const int* __restrict__ mel_off, const float* __restrict__ mel_w,
                                                    int nbins, float preemph, int remove_dc, int use_log,
                                                    float* __restrict__ out) {
  constexpr int M = 1 << LOGM;   // complex points; N = 2M real points
  constexpr int ZS = M + 2, PS = M + 5;   // per-frame strides, padded so the 4 frames of a wave use different LDS banks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* cz = reinterpret_cast<float2*>(smem);               // [FB][ZS]
  float* pw = reinterpret_cast<float*>(cz + FB * ZS);         // [FB][PS] power spectrum
  float2* ltw = reinterpret_cast<float2*>(pw + FB * PS);      // [M/2] FFT twiddles
  float2* ltw2 = ltw + M / 2;                                 // [M/2 + 1] real-split twiddles
  float* lwin = reinterpret_cast<float*>(ltw2 + M / 2 + 1);   // [win]
  const int nw = mel_off[nbins];
  float* lmw = lwin + win;                                    // [nw] mel weights
  int* lmi = reinterpret_cast<int*>(lmw + nw);                // [nbins] lo, [nbins + 1] offsets
  const int wspan = (FBW - 1) * shift + win;
  const int tid = threadIdx.x, f = tid / TPF, j = tid % TPF, wv = tid >> 6, lane = tid & 63;
  float* sx = reinterpret_cast<float*>(lmi + 2 * nbins + 1) + wv * wspan;   // this wave's samples
  // constants in LDS once per (persistent) block: every stage and filter reads them at LDS latency
  for (int i = tid; i < M / 2; i += 256) ltw[i] = tw[i];
  for (int i = tid; i <= M / 2; i += 256) ltw2[i] = tw2[i];
  for (int i = tid; i < win; i += 256) lwin[i] = window[i];
  for (int i = tid; i < nw; i += 256) lmw[i] = mel_w[i];
  for (int i = tid; i < 2 * nbins + 1; i += 256) lmi[i] = i < nbins ? mel_lo[i] : mel_off[i - nbins];
  __syncthreads();   // constants staged; from here on the waves run independently
  // samples of the wave's 4 frames (3 shift + win <= FBK_WSAMPLES), prefetched into registers one
  // group ahead
  float pre[FBK_WSAMPLES / 64];
  const long long ngroups = (n_frames + FB - 1) / FB;
  auto fetch = [&](long long grp) {
    const long long base = (grp * FB + wv * FBW) * shift;
#pragma unroll
    for (int q = 0; q < FBK_WSAMPLES / 64; ++q) {
      const int i = lane + 64 * q;
      pre[q] = (grp < ngroups && i < wspan && base + i < n_samples) ? wave[base + i] : 0.f;
    }
  };
  fetch(blockIdx.x);
  for (long long grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    wave_lds_sync();   // the previous group's reads of sx / cz / pw are done
#pragma unroll
    for (int q = 0; q < FBK_WSAMPLES / 64; ++q)
      if (lane + 64 * q < wspan) sx[lane + 64 * q] = pre[q];
    wave_lds_sync();
    fetch(grp + gridDim.x);

    const long long F = grp * FB + f;
    const bool live = F < n_frames;
    const float* x = sx + (f - wv * FBW) * shift;
    float2* z = cz + f * ZS;
    // ---- frame mean over the 16 threads of the frame (lanes 16f .. 16f+15 of one wave)
    float s = 0.f;
    if (live)
      for (int n = j; n < win; n += TPF) s += x[n];
#pragma unroll
    for (int o = TPF / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, TPF);
    const float mean = remove_dc ? s / (float)win : 0.f;
    // ---- DC removal, pre-emphasis, window, zero pad; z[n] = y[2n] + i y[2n+1] at bit-reversed n
    for (int n = j; n < 2 * M; n += TPF) {
      float y = 0.f;
      if (live && n < win) {
        const float cur = x[n] - mean, prev = x[n > 0 ? n - 1 : 0] - mean;
        y = (cur - preemph * prev) * lwin[n];
      }
      float* zp = reinterpret_cast<float*>(&z[brev(n >> 1, LOGM)]);
      zp[n & 1] = y;
    }
    wave_lds_sync();
    // ---- radix-2 DIT, M/2 butterflies per stage, 16 threads per frame
#pragma unroll 1
    for (int st = 1; st <= LOGM; ++st) {
      const int half = 1 << (st - 1);
      for (int b = j; b < M / 2; b += TPF) {
        const int k = b & (half - 1), i0 = ((b >> (st - 1)) << st) + k, i1 = i0 + half;
        const float2 w = ltw[k << (LOGM - st)];
        const float2 av = z[i0], c = z[i1];
        const float2 t = make_float2(w.x * c.x - w.y * c.y, w.x * c.y + w.y * c.x);
        z[i0] = make_float2(av.x + t.x, av.y + t.y);
        z[i1] = make_float2(av.x - t.x, av.y - t.y);
      }
      wave_lds_sync();
    }
    // ---- real split: X[k] = (Z[k] + conj Z[M-k]) / 2 - i W^k (Z[k] - conj Z[M-k]) / 2, W = e^{-2 pi i / N};
    // power = |X|^2
    float* p = pw + f * PS;
    for (int k = j; k <= M / 2; k += TPF) {
      const float2 zk = z[k & (M - 1)], zm = z[(M - k) & (M - 1)];
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        if (side == 1 && (k == 0 || 2 * k == M)) {   // k = 0 also yields bin M; k = M/2 is its own mirror
          if (k == 0) {
            const float a = zk.x - zk.y;
            p[M] = a * a;
          }
          continue;
        }
        const int kk = side ? M - k : k;
        const float2 A = side ? zm : zk, B = side ? zk : zm;   // Z[kk], Z[M - kk]
        const float er = 0.5f * (A.x + B.x), ei = 0.5f * (A.y - B.y);     // (Z[kk] + conj Z[M-kk]) / 2
        const float orr = 0.5f * (A.y + B.y), oi = -0.5f * (A.x - B.x);   // (Z[kk] - conj Z[M-kk]) / (2i)
        // W^kk; past M/2 (side 1): W^(M-k) = -conj(W^k)
        const float2 w = side ? make_float2(-ltw2[k].x, ltw2[k].y) : ltw2[k];
        const float xr = er + (w.x * orr - w.y * oi), xi = ei + (w.x * oi + w.y * orr);
        p[kk] = fmaf(xr, xr, xi * xi);   // |X|^2 (torch: abs, then squared; equal to an ulp)
      }
    }
    wave_lds_sync();
    // ---- mel filters (sparse ranges) and log
    if (live)
      for (int m = j; m < nbins; m += TPF) {
        const int lo = lmi[m], o0 = lmi[nbins + m], o1 = lmi[nbins + m + 1];
        float e = 0.f;
        for (int q = o0; q < o1; ++q) e = fmaf(lmw[q], p[lo + q - o0], e);
        if (use_log) e = __logf(fmaxf(e, 1.1920928955078125e-07f));   // v_log_f32 x ln 2
        out[F * nbins + m] = e;
      }
  }   // group loop
}


// N = 512 (the reference's 25 ms / 10 ms at 16 kHz; win <= 512): the samples go straight from
// global memory into registers -- lane j of a frame holds samples 2(j + 16m), 2(j + 16m) + 1,
// m = 0..15, which are exactly its inputs of the four-step FFT -- the pre-emphasis neighbour of
// an even sample comes from lane j - 1 by a DPP row rotate, and the power spectrum is written over
// the frame's own FFT buffer.  LDS: 34 KiB of FFT buffers + 8 KiB of constants per 16 frames ->
// 3 blocks per CU (143 VGPRs), and no sample staging.  Persistent blocks, samples of the next
// group in flight while the current one is transformed.
__global__ __launch_bounds__(256, 3) void fbank512_kernel(const float* __restrict__ wave, long long n_samples,
                                                          long long n_frames, int shift, int win,
                                                          const float* __restrict__ window,
                                                          const float2* __restrict__ tw, const float2* __restrict__ tw2,
                                                          const int* __restrict__ mel_lo, const int* __restrict__ mel_off,
                                                          const float* __restrict__ mel_w, int nbins, float preemph,
                                                          int remove_dc, int use_log, float* __restrict__ out,
                                                          int vec2) {
  // (transpose rows of pitch 17 or 18 against bank conflicts measured equal or slower: the row
  // reads are ds_read_b128 at pitch 16)
  constexpr int M = 256, ZP = 16, ZS = M + 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* cz = reinterpret_cast<float2*>(smem);               // [FB][ZS]: FFT buffer, then |X|^2
  float2* ltw = cz + FB * ZS;                                 // [16 k1][16 j] W256^(j k1)
  float2* ltw2 = ltw + M;                                     // [M/2 + 1] real-split twiddles
  float* lwin = reinterpret_cast<float*>(ltw2 + M / 2 + 1);   // [2M] window, zero past win
  const int nw = mel_off[nbins];
  float* lmw = lwin + 2 * M;                                  // [nw] mel weights
  int* lmi = reinterpret_cast<int*>(lmw + nw);                // [nbins] lo, [nbins + 1] offsets
  const int tid = threadIdx.x, f = tid / TPF, j = tid % TPF;
  for (int i = tid; i < M; i += 256) {   // lane j reads row k1 at column j: conflict-free
    const int e = (i >> 4) * (i & 15);     // < 256: W256^e = -W256^(e - 128) past 128
    const float2 w = tw[e & 127];
    ltw[i] = (e & 128) ? make_float2(-w.x, -w.y) : w;
  }
  for (int i = tid; i <= M / 2; i += 256) ltw2[i] = tw2[i];
  for (int i = tid; i < 2 * M; i += 256) lwin[i] = i < win ? window[i] : 0.f;
  for (int i = tid; i < nw; i += 256) lmw[i] = mel_w[i];
  for (int i = tid; i < 2 * nbins + 1; i += 256) lmi[i] = i < nbins ? mel_lo[i] : mel_off[i - nbins];
  __syncthreads();   // constants staged; from here on the waves run independently
  const long long ngroups = (n_frames + FB - 1) / FB;
  float2 pre[16];
  auto fetch = [&](long long grp) {
    const long long F = grp * FB + f;
    const bool ok = grp < ngroups && F < n_frames;   // a live frame's samples are all in range
    const float* xs = wave + (ok ? F * shift : 0);
    if (vec2) {   // frames start 8-B aligned: one dwordx2 per sample pair
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int n0 = 2 * (j + 16 * m);
        pre[m] = ok && n0 + 1 < win ? *reinterpret_cast<const float2*>(xs + n0)
                                    : make_float2(ok && n0 < win ? xs[n0] : 0.f, 0.f);
      }
    } else {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int n0 = 2 * (j + 16 * m);
        pre[m].x = ok && n0 < win ? xs[n0] : 0.f;
        pre[m].y = ok && n0 + 1 < win ? xs[n0 + 1] : 0.f;
      }
    }
  };
  fetch(blockIdx.x);
  for (long long grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const long long F = grp * FB + f;
    const bool live = F < n_frames;
    float2* z = cz + f * ZS;
    // ---- frame mean over the 16 lanes of the frame (samples past win are zero)
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 16; ++m) s += pre[m].x + pre[m].y;
#pragma unroll
    for (int o = TPF / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, TPF);
    const float mean = remove_dc ? s / (float)win : 0.f;
    // ---- DC removal, pre-emphasis (x[-1] = x[0]), window, zero pad: a[m] = (y[n0], y[n0 + 1]).
    // x[n0 - 1] is lane j-1's odd sample of the same m (row_ror:1 within the 16 lanes), for j = 0
    // lane 15's odd sample of m - 1 (the previous m's rotate)
    float2 a[16];
    float up_prev = 0.f;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const float up = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, pre[m].y),
                                                                          0x121, 0xf, 0xf, false));
      const float prev = j > 0 ? up : (m > 0 ? up_prev : pre[0].x);
      up_prev = up;
      const float c0 = pre[m].x - mean, c1 = pre[m].y - mean;
      const float2 w = reinterpret_cast<const float2*>(lwin)[j + 16 * m];
      a[m] = make_float2((c0 - preemph * (prev - mean)) * w.x, (c1 - preemph * c0) * w.y);
    }
    // ---- four-step 256 = 16 x 16 FFT: a 16-point DFT in registers, the W256^(j k1) twiddle, one
    // transpose through LDS, a second 16-point DFT
#if CFM_FBANK_DIAG != 2
    fft16(a);
#endif
    wave_lds_sync();   // the previous group's mel reads of z are done
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) z[ZP * k1 + j] = cmul(a[k1], ltw[16 * k1 + j]);
    wave_lds_sync();
#pragma unroll
    for (int t = 0; t < 16; ++t) a[t] = z[ZP * j + t];
#if CFM_FBANK_DIAG != 2
    fft16(a);   // a[k2] = Z[j + 16 k2]
#endif
    wave_lds_sync();
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) z[j + 16 * k2] = a[k2];
    fetch(grp + gridDim.x);   // the next group's samples load under the real split and mel filters
    wave_lds_sync();
    // ---- real split and |X|^2 into registers (k = j + 16 i <= M/2, both mirrors), then over z
    float q0[9], q1[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int k = j + 16 * i;
      q0[i] = q1[i] = 0.f;
      if (k > M / 2) continue;
      const float2 zk = z[k & (M - 1)], zm = z[(M - k) & (M - 1)];
      const float2 w2 = ltw2[k];
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const float2 A = side ? zm : zk, B = side ? zk : zm;   // Z[kk], Z[M - kk]
        const float er = 0.5f * (A.x + B.x), ei = 0.5f * (A.y - B.y);
        const float orr = 0.5f * (A.y + B.y), oi = -0.5f * (A.x - B.x);
        const float2 w = side ? make_float2(-w2.x, w2.y) : w2;   // W^(M-k) = -conj(W^k)
        const float xr = er + (w.x * orr - w.y * oi), xi = ei + (w.x * oi + w.y * orr);
        (side ? q1[i] : q0[i]) = fmaf(xr, xr, xi * xi);
      }
      if (k == 0) q1[i] = (zk.x - zk.y) * (zk.x - zk.y);   // bin M
    }
    wave_lds_sync();   // every lane's reads of z are done before z is overwritten
    float* p = reinterpret_cast<float*>(z);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int k = j + 16 * i;
      if (k > M / 2) continue;
      p[k] = q0[i];
      if (k != M / 2) p[k == 0 ? M : M - k] = q1[i];
    }
    wave_lds_sync();
    // ---- mel filters (sparse ranges) and log
    if (live)
      for (int m = j; m < nbins; m += TPF) {
        const int lo = lmi[m], o0 = lmi[nbins + m], o1 = lmi[nbins + m + 1];
        float e = 0.f;
#if CFM_FBANK_DIAG == 1
        e = p[lo] + (float)(o1 - o0);
#else
        for (int q = o0; q < o1; ++q) e = fmaf(lmw[q], p[lo + q - o0], e);
#endif
        if (use_log) e = __logf(fmaxf(e, 1.1920928955078125e-07f));
        out[F * nbins + m] = e;
      }
  }   // group loop
}

}  // namespace cfm

struct cfm_fbank {
  cfm_fbank_config cfg;
  int win = 0, shift = 0, logm = 0, nbins = 0, n_mel_w = 0;
  float* window = nullptr;
  float2 *tw = nullptr, *tw2 = nullptr;
  int *mel_lo = nullptr, *mel_off = nullptr;
  float* mel_w = nullptr;
  int device = 0;
  int n_cu = 256;   // compute units of `device` (launch sizing)
};

namespace {
using cfm::set_error;

// dynamic LDS of fbank_kernel: spectra [FB][M + 2] float2, power [FB][M + 5], the block's samples
size_t fbank512_lds(int nbins, int nw) {
  return (size_t)cfm::FB * 258 * 8 + (size_t)(256 + 129) * 8 + (size_t)(512 + nw + 2 * nbins + 1) * 4;
}

size_t fbank_lds(int M, int shift, int win, int nbins, int nw) {
  return (size_t)cfm::FB * (M + 2) * 8 + (size_t)cfm::FB * (M + 5) * 4 + (size_t)(M + 1) * 8 +
         (size_t)(win + nw + 2 * nbins + 1) * 4 + (size_t)(cfm::FB / cfm::FBW) * ((cfm::FBW - 1) * shift + win) * 4;
}

// torch.hann_window(N, periodic=False) (and the other kaldi window types) as torchaudio builds it in
// float32: alpha - beta * cos(2 pi n / (N - 1)); povey = hann ** 0.85 (compliance/kaldi.py _get_window)
std::vector<float> make_window(int type, int n) {
  std::vector<float> w(n);
  const float step = (float)(2.0 * M_PI / (n - 1));
  for (int i = 0; i < n; ++i) {
    const float a = (float)i * step;
    switch (type) {
      case CFM_WINDOW_HAMMING: w[i] = 0.54f - 0.46f * std::cos(a); break;
      case CFM_WINDOW_HANNING: w[i] = 0.5f - 0.5f * std::cos(a); break;
      case CFM_WINDOW_RECTANGULAR: w[i] = 1.f; break;
      case CFM_WINDOW_BLACKMAN: {
        const float b = (float)(2.0 * M_PI / (n - 1));
        w[i] = 0.42f - 0.5f * std::cos((float)i * b) + 0.08f * std::cos(2.f * (float)i * b);
        break;
      }
      default: w[i] = std::pow(0.5f - 0.5f * std::cos(a), 0.85f); break;   // povey
    }
  }
  return w;
}

// get_mel_banks (vtln_warp = 1): bins[m][k] = max(0, min(up, down)) over the N/2 FFT bins, the
// Nyquist column appended as 0 (fbank pads it) -> sparse [lo, hi) ranges per filter
void make_mel(int nbins, int N, float fs, float low, float high, std::vector<int>& lo, std::vector<int>& off,
              std::vector<float>& w) {
  const int nfft = N / 2;
  const float nyq = 0.5f * fs;
  if (high <= 0.f) high += nyq;
  const float bin_w = fs / (float)N;
  auto mel_d = [](double f) { return 1127.0 * std::log(1.0 + f / 700.0); };
  const double mlo = mel_d(low), mhi = mel_d(high), delta = (mhi - mlo) / (nbins + 1);
  lo.assign(nbins, 0);
  off.assign(nbins + 1, 0);
  w.clear();
  for (int m = 0; m < nbins; ++m) {
    const float left = (float)(mlo + m * delta), center = (float)(mlo + (m + 1.0) * delta),
                right = (float)(mlo + (m + 2.0) * delta);
    int first = -1, last = -1;
    std::vector<float> vals(nfft + 1, 0.f);
    for (int k = 0; k < nfft; ++k) {
      const float mel = 1127.0f * std::log(1.0f + (bin_w * (float)k) / 700.0f);
      const float up = (mel - left) / (center - left), down = (right - mel) / (right - center);
      const float v = std::max(0.f, std::min(up, down));
      vals[k] = v;
      if (v > 0.f) {
        if (first < 0) first = k;
        last = k;
      }
    }
    if (first < 0) first = last = 0;
    lo[m] = first;
    off[m] = (int)w.size();
    for (int k = first; k <= last; ++k) w.push_back(vals[k]);
  }
  off[nbins] = (int)w.size();
}
}  // namespace

extern "C" {

cfm_status cfm_fbank_create(const cfm_fbank_config* cfg, int32_t device, cfm_fbank** out) {
  if (!cfg || !out) return set_error(CFM_ERR_VALUE, "fbank: null argument");
  *out = nullptr;
  if (cfg->dither != 0.f) return set_error(CFM_ERR_ASSERT, "fbank: dither must be 0 (the reference decodes with dither 0.0)");
  if (!cfg->snip_edges) return set_error(CFM_ERR_ASSERT, "fbank: only snip_edges=True is supported");
  if (cfg->use_energy) return set_error(CFM_ERR_ASSERT, "fbank: use_energy is not supported");
  const int win = (int)((double)cfg->sample_frequency * cfg->frame_length_ms * 0.001);
  const int shift = (int)((double)cfg->sample_frequency * cfg->frame_shift_ms * 0.001);
  if (win < 2 || shift < 1) return set_error(CFM_ERR_VALUE, "fbank: frame length / shift too small");
  int N = 1;
  while (N < win) N <<= 1;
  if (!cfg->round_to_power_of_two && N != win)
    return set_error(CFM_ERR_ASSERT, "fbank: round_to_power_of_two=False needs a power-of-two frame");
  const int logm = __builtin_ctz(N) - 1;
  if (logm < 6 || logm > 9) return set_error(CFM_ERR_ASSERT, "fbank: padded frame must be 128 .. 1024 samples");
  if (cfg->num_mel_bins < 1 || cfg->num_mel_bins > 512) return set_error(CFM_ERR_VALUE, "fbank: num_mel_bins");
  if (logm != 8 && (size_t)(cfm::FBW - 1) * shift + win > (size_t)cfm::FBK_WSAMPLES)
    return set_error(CFM_ERR_ASSERT, "fbank: frame length / shift too large (3 shift + length > 2048 samples)");
  if (hipSetDevice(device) != hipSuccess) return set_error(CFM_ERR_RUNTIME, "fbank: hipSetDevice");
  auto* h = new cfm_fbank();
  h->cfg = *cfg;
  h->win = win;
  h->shift = shift;
  h->logm = logm;
  h->nbins = cfg->num_mel_bins;
  h->device = device;
  if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || h->n_cu <= 0)
    h->n_cu = 256;
  const int M = 1 << logm;
  std::vector<float> w = make_window(cfg->window_type, win);
  std::vector<float2> tw(M / 2), tw2(M / 2 + 1);
  for (int k = 0; k < M / 2; ++k) {
    const double a = -2.0 * M_PI * k / M;
    tw[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  for (int k = 0; k <= M / 2; ++k) {
    const double a = -2.0 * M_PI * k / (2 * M);
    tw2[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  std::vector<int> lo, off;
  std::vector<float> mw;
  make_mel(h->nbins, 2 * M, cfg->sample_frequency, cfg->low_freq, cfg->high_freq, lo, off, mw);
  h->n_mel_w = off[h->nbins];
  if (mw.empty()) mw.push_back(0.f);
  bool ok = hipMalloc(&h->window, w.size() * 4) == hipSuccess && hipMalloc(&h->tw, tw.size() * 8) == hipSuccess &&
            hipMalloc(&h->tw2, tw2.size() * 8) == hipSuccess && hipMalloc(&h->mel_lo, lo.size() * 4) == hipSuccess &&
            hipMalloc(&h->mel_off, off.size() * 4) == hipSuccess && hipMalloc(&h->mel_w, mw.size() * 4) == hipSuccess;
  ok = ok && hipMemcpy(h->window, w.data(), w.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(h->tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(h->tw2, tw2.data(), tw2.size() * 8, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(h->mel_lo, lo.data(), lo.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(h->mel_off, off.data(), off.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(h->mel_w, mw.data(), mw.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
  if (!ok) {
    cfm_fbank_destroy(h);
    return set_error(CFM_ERR_RUNTIME, "fbank: device allocation / upload failed");
  }
  // LDS beyond the default 64 KiB (N = 1024 frames; the N = 512 kernel needs < 40 KiB)
  const size_t lds = fbank_lds(M, shift, win, h->nbins, (int)mw.size());
  if (logm != 8 && lds > 65536) {
    const void* fn = logm == 9   ? (const void*)cfm::fbank_kernel<9>
                     : logm == 7 ? (const void*)cfm::fbank_kernel<7>
                                 : (const void*)cfm::fbank_kernel<6>;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
      cfm_fbank_destroy(h);
      return set_error(CFM_ERR_RUNTIME, "fbank: LDS size attribute");
    }
  }
  *out = h;
  return CFM_OK;
}

void cfm_fbank_destroy(cfm_fbank* h) {
  if (!h) return;
  (void)hipFree(h->window);
  (void)hipFree(h->tw);
  (void)hipFree(h->tw2);
  (void)hipFree(h->mel_lo);
  (void)hipFree(h->mel_off);
  (void)hipFree(h->mel_w);
  delete h;
}

int64_t cfm_fbank_num_frames(const cfm_fbank* h, int64_t num_samples) {
  if (!h || num_samples < h->win) return 0;
  return 1 + (num_samples - h->win) / h->shift;
}

cfm_status cfm_fbank_compute(const cfm_fbank* h, const float* wave_dev, int64_t num_samples, float* out_dev,
                             cfm_stream stream) {
  if (!h) return set_error(CFM_ERR_VALUE, "fbank: null handle");
  if (num_samples < 0) return set_error(CFM_ERR_VALUE, "fbank: negative sample count");
  const int64_t nf = cfm_fbank_num_frames(h, num_samples);
  if (nf == 0) return CFM_OK;
  if (!wave_dev || !out_dev) return set_error(CFM_ERR_VALUE, "fbank: null buffer");
  const int M = 1 << h->logm;
  const size_t lds = h->logm == 8 ? fbank512_lds(h->nbins, h->n_mel_w) : fbank_lds(M, h->shift, h->win, h->nbins, h->n_mel_w);
  // the handle's device (its constants live there), whatever the caller's current device
  if (hipSetDevice(h->device) != hipSuccess) return set_error(CFM_ERR_RUNTIME, "fbank: hipSetDevice");
  // persistent blocks (constants staged once each): three resident per CU for N = 512, else two
  const int n_cu = h->n_cu;
  const long long groups = (nf + cfm::FB - 1) / cfm::FB;
  const dim3 grid((unsigned)std::min<long long>(groups, (h->logm == 8 ? 3LL : 2LL) * n_cu));
  const hipStream_t st = (hipStream_t)stream;
#define FBK(L)                                                                                                      \
  hipLaunchKernelGGL(cfm::fbank_kernel<L>, grid, dim3(256), lds, st, wave_dev, (long long)num_samples, (long long)nf, \
                     h->shift, h->win, h->window, h->tw, h->tw2, h->mel_lo, h->mel_off, h->mel_w, h->nbins,           \
                     h->cfg.preemphasis_coefficient, h->cfg.remove_dc_offset, h->cfg.use_log_fbank, out_dev)
  switch (h->logm) {
    case 6: FBK(6); break;
    case 7: FBK(7); break;
    case 8:
      hipLaunchKernelGGL(cfm::fbank512_kernel, grid, dim3(256), lds, st, wave_dev, (long long)num_samples, (long long)nf,
                         h->shift, h->win, h->window, h->tw, h->tw2, h->mel_lo, h->mel_off, h->mel_w, h->nbins,
                         h->cfg.preemphasis_coefficient, h->cfg.remove_dc_offset, h->cfg.use_log_fbank, out_dev,
                         (int)(h->shift % 2 == 0 && reinterpret_cast<uintptr_t>(wave_dev) % 8 == 0));
      break;
    default: FBK(9); break;
  }
#undef FBK
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(CFM_ERR_RUNTIME, std::string("fbank launch: ") + hipGetErrorString(e));
  return CFM_OK;
}

}  // extern "C"
