// RNN-T greedy search (the encoder's transducer consumer), gfx950.
//
// Replaces transducer/search/greedy_search.py:6-92 (optimized_search / batch_greedy_search) as the
// reference calls it from endless_decode / batch_decode (chunkformer_model.py:439-448, 533-543),
// with the shipped predictor / joint (RNNPredictor lstm, predictor.py:66-208; TransducerJoint
// prejoin + add + tanh + ffn_out, joint.py:74-111).  Blank id 0.
//
//   1. enc_proj = enc . enc_ffn^T + b for every frame: one f32 MFMA GEMM (gemm<float>);
//   2. rnnt_greedy_kernel: ONE persistent workgroup per utterance runs the whole search, with the
//      utterance's state (last token, LSTM h / c, predictor output) in LDS:
//        - the predictor (embedding -> LSTM layers -> projection -> pred_ffn) is evaluated once per
//          emitted token: optimized_search recomputes predictor.forward_step at every step, but its
//          input (last non-blank token, committed LSTM state) only changes on an emission;
//        - the joint (tanh(enc_proj[t] + pred) . ffn_out^T + b, argmax) is evaluated for a block of
//          RF consecutive frames at once, reading ffn_out once per block; the frames before the
//          block's first non-blank decision are blank under the same predictor state, exactly as
//          the sequential loop decides them, and the search resumes at that frame.
//      Every loop iteration either advances the frame or counts an emission against the frame's
//      n_steps budget, so the kernel ends after at most T * (n_steps + 1) iterations.
//   Matrix-vector products read transposed f32 weights [K][M] with one float4 of outputs per
//   thread (coalesced rows, the input vector broadcast from LDS); argmax ties go to the lower id
//   like torch.argmax.  Everything is f32 (log_softmax is monotone: argmax of the logits).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/cfm.h"
#include "cfm_common.h"
#include "cfm_kernels.h"
#include "status.h"

namespace cfm {

constexpr int RNNT_NT = 512;   // threads per workgroup (8 waves)
constexpr int RNNT_RF = 8;     // frames per joint block
constexpr int RNNT_MAXL = 4;   // LSTM layers

struct RnntDev {
  const float* embed;                     // [V, E]
  const float* wg[RNNT_MAXL];             // [(in_l + H), 4H]: W_ih^T rows then W_hh^T rows
  const float* bg[RNNT_MAXL];             // [4H] b_ih + b_hh
  const float *wp, *bp;                   // [H, P], [P]
  const float *wpj, *bpj;                 // [P, J], [J]
  const float *wo, *bo;                   // [J, Vp] (zero-padded columns), [Vp] (padding -inf)
  int V, Vp, E, H, nl, P, J, blank;
};

// y[0:M) = WT^T x + bias (WT [K][M] row-major, M % 4 == 0); x, y, red in LDS.  Outputs are split
// into float4 groups; when there are fewer groups than threads the K range is split too and the
// partial sums reduced through `red` ([ks][M] floats).
CFM_DEV void matvec(const float* __restrict__ WT, int K, int M, const float* x, const float* __restrict__ bias,
                    float* y, float* red, int tid) {
  const int groups = M >> 2;
  int ks = RNNT_NT / groups;
  ks = ks < 1 ? 1 : (ks > 8 ? 8 : ks);
  const int kc = (K + ks - 1) / ks;
  const float4* W4 = reinterpret_cast<const float4*>(WT);
  for (int w = tid; w < groups * ks; w += RNNT_NT) {
    const int g = w % groups, s = w / groups;
    const int k0 = s * kc, k1 = min(K, k0 + kc);
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    const float4* col = W4 + g;
#pragma unroll 8
    for (int k = k0; k < k1; ++k) {
      const float4 wv = col[(size_t)k * groups];
      const float xv = x[k];
      acc.x = fmaf(wv.x, xv, acc.x);
      acc.y = fmaf(wv.y, xv, acc.y);
      acc.z = fmaf(wv.z, xv, acc.z);
      acc.w = fmaf(wv.w, xv, acc.w);
    }
    if (ks == 1) {
      const float4 b = reinterpret_cast<const float4*>(bias)[g];
      reinterpret_cast<float4*>(y)[g] = make_float4(acc.x + b.x, acc.y + b.y, acc.z + b.z, acc.w + b.w);
    } else {
      reinterpret_cast<float4*>(red + (size_t)s * M)[g] = acc;
    }
  }
  if (ks > 1) {
    __syncthreads();
    for (int m = tid; m < M; m += RNNT_NT) {
      float v = 0.f;
      for (int s = 0; s < ks; ++s) v += red[(size_t)s * M + m];
      y[m] = v + bias[m];
    }
  }
  __syncthreads();
}

CFM_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// the predictor for input token `tok` and committed state (h, c): new state (hn, cn) and
// pj = pred_ffn(projection(h_top)) (joint.py:87-88 pre-projection of the predictor output)
CFM_DEV void predictor(const RnntDev& w, int tok, const float* h, const float* c, float* hn, float* cn, float* xin,
                       float* gates, float* pvec, float* pj, float* red, int tid) {
  const int H = w.H;
  for (int e = tid; e < w.E; e += RNNT_NT) xin[e] = w.embed[(size_t)tok * w.E + e];
  int in = w.E;
  for (int l = 0; l < w.nl; ++l) {
    for (int e = tid; e < H; e += RNNT_NT) xin[in + e] = h[l * H + e];
    __syncthreads();
    matvec(w.wg[l], in + H, 4 * H, xin, w.bg[l], gates, red, tid);
    for (int e = tid; e < H; e += RNNT_NT) {   // torch LSTM gate order i, f, g, o
      const float ig = sigm(gates[e]), fg = sigm(gates[H + e]), gg = tanhf(gates[2 * H + e]),
                  og = sigm(gates[3 * H + e]);
      const float cv = fg * c[l * H + e] + ig * gg;
      cn[l * H + e] = cv;
      const float hv = og * tanhf(cv);
      hn[l * H + e] = hv;
      xin[e] = hv;   // the next layer's input
    }
    __syncthreads();
    in = H;
  }
  matvec(w.wp, H, w.P, xin, w.bp, pvec, red, tid);
  matvec(w.wpj, w.P, w.J, pvec, w.bpj, pj, red, tid);
}

__global__ __launch_bounds__(RNNT_NT) void rnnt_greedy_kernel(RnntDev w, const float* __restrict__ enc_proj,
                                                              const int32_t* __restrict__ row_start,
                                                              const int32_t* __restrict__ row_len, int n_steps,
                                                              int32_t* __restrict__ out) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int H = w.H, J = w.J, nl = w.nl;
  const int b = blockIdx.x;
  const int r0 = row_start[b], T = row_len[b];
  // LDS carve (floats)
  float* h = lds;                        // [nl][H] committed state
  float* c = h + nl * H;
  float* hn = c + nl * H;                // [nl][H] state after the last predictor evaluation
  float* cn = hn + nl * H;
  float* xin = cn + nl * H;              // [max(E, H) + H]
  float* gates = xin + (max(w.E, H) + H);   // [4H]
  float* pvec = gates + 4 * H;           // [P]
  float* pj = pvec + w.P;                // [J]
  float* z = pj + J;                     // [RF][J] joint inputs of the block
  float* red = z + RNNT_RF * J;          // [4 * NT] split-K partials (ks * M <= 4 * NT)
  float* wbest = red + 4 * RNNT_NT;      // [8 waves][RF] best value
  int* wbidx = reinterpret_cast<int*>(wbest + 8 * RNNT_RF);  // [8][RF] its id
  int* ctl = wbidx + 8 * RNNT_RF;        // [RF] decisions of the block

  for (int e = tid; e < nl * H; e += RNNT_NT) { h[e] = 0.f; c[e] = 0.f; }
  __syncthreads();
  int tok = w.blank;
  predictor(w, tok, h, c, hn, cn, xin, gates, pvec, pj, red, tid);

  int t = 0, step = 0;
  while (t < T) {
    const int nf = min(RNNT_RF, T - t);
    // joint inputs z[f] = tanh(enc_proj[t + f] + pj)
    for (int e = tid; e < nf * J; e += RNNT_NT) {
      const int f = e / J, j = e - f * J;
      z[e] = tanhf(enc_proj[(size_t)(r0 + t + f) * J + j] + pj[j]);
    }
    __syncthreads();
    // logits of the block: threads over float4 groups of the (padded) vocabulary, all frames
    float bv[RNNT_RF];
    int bi[RNNT_RF];
#pragma unroll
    for (int f = 0; f < RNNT_RF; ++f) { bv[f] = -INFINITY; bi[f] = 0x7fffffff; }
    const int vg = w.Vp >> 2;
    const float4* W4 = reinterpret_cast<const float4*>(w.wo);
    for (int g = tid; g < vg; g += RNNT_NT) {
      float4 acc[RNNT_RF];
#pragma unroll
      for (int f = 0; f < RNNT_RF; ++f) acc[f] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
      for (int j = 0; j < J; ++j) {
        const float4 wv = W4[(size_t)j * vg + g];
#pragma unroll
        for (int f = 0; f < RNNT_RF; ++f) {
          const float zv = z[f * J + j];
          acc[f].x = fmaf(wv.x, zv, acc[f].x);
          acc[f].y = fmaf(wv.y, zv, acc[f].y);
          acc[f].z = fmaf(wv.z, zv, acc[f].z);
          acc[f].w = fmaf(wv.w, zv, acc[f].w);
        }
      }
      const float4 bb = reinterpret_cast<const float4*>(w.bo)[g];
#pragma unroll
      for (int f = 0; f < RNNT_RF; ++f) {
        const float v4[4] = {acc[f].x + bb.x, acc[f].y + bb.y, acc[f].z + bb.z, acc[f].w + bb.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)   // ascending ids: strict > keeps the lowest id of a tie
          if (v4[q] > bv[f]) { bv[f] = v4[q]; bi[f] = 4 * g + q; }
      }
    }
    // argmax per frame: wave (value, lowest id), then across the 8 waves
#pragma unroll
    for (int f = 0; f < RNNT_RF; ++f) {
      float v = bv[f];
      int i = bi[f];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
      }
      if (lane == 0) { wbest[wid * RNNT_RF + f] = v; wbidx[wid * RNNT_RF + f] = i; }
    }
    __syncthreads();
    if (tid < RNNT_RF) {
      float v = wbest[tid];
      int i = wbidx[tid];
      for (int q = 1; q < RNNT_NT / 64; ++q) {
        const float ov = wbest[q * RNNT_RF + tid];
        const int oi = wbidx[q * RNNT_RF + tid];
        if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
      }
      ctl[tid] = i;
    }
    __syncthreads();
    int f = 0;
    while (f < nf && ctl[f] == w.blank) ++f;   // uniform: every thread reads the same LDS words
    __syncthreads();
    if (f == nf) {   // the whole block is blank under this predictor state
      t += nf;
      step = 0;
      continue;
    }
    if (f > 0) { t += f; step = 0; }
    const int k = ctl[f];
    if (tid == 0) out[(size_t)(r0 + t) * n_steps + step] = k;
    ++step;
    // commit the emission: the predictor's new state becomes the state, k the next input
    for (int e = tid; e < nl * H; e += RNNT_NT) { h[e] = hn[e]; c[e] = cn[e]; }
    __syncthreads();
    tok = k;
    predictor(w, tok, h, c, hn, cn, xin, gates, pvec, pj, red, tid);
    if (step == n_steps) { ++t; step = 0; }
  }
}

size_t rnnt_lds_bytes(const RnntDev& w) {
  const size_t H = w.H, J = w.J, P = w.P;
  size_t f = 4 * w.nl * H + (std::max<size_t>(w.E, H) + H) + 4 * H + P + J + RNNT_RF * J + 4 * RNNT_NT +
             8 * RNNT_RF;
  return f * 4 + 8 * RNNT_RF * 4 + RNNT_RF * 4;
}

}  // namespace cfm

struct cfm_rnnt {
  cfm_rnnt_config cfg;
  int device = 0;
  void* dev_mem = nullptr;
  cfm::RnntDev w{};
  const float *we = nullptr, *be = nullptr;   // enc_ffn [J, Eenc] (torch layout), [J]
  ~cfm_rnnt() {
    if (dev_mem) { (void)hipSetDevice(device); (void)hipFree(dev_mem); }
  }
};

using namespace cfm;

namespace {

struct Img {
  std::vector<char> bytes;
  std::vector<std::pair<size_t, const float**>> fix;
  void put(const std::vector<float>& v, const float** slot) {
    size_t off = (bytes.size() + 255) / 256 * 256;
    bytes.resize(off + (v.size() * 4 + 255) / 256 * 256);
    std::memcpy(bytes.data() + off, v.data(), v.size() * 4);
    fix.push_back({off, slot});
  }
};

}  // namespace

extern "C" {

cfm_status cfm_rnnt_create(const cfm_rnnt_config* cfg, const cfm_tensor_view* weights, int32_t n, int32_t device,
                           cfm_rnnt** out) {
  if (!cfg || !out || (!weights && n > 0)) return set_error(CFM_ERR_VALUE, "null argument");
  *out = nullptr;
  const int V = cfg->vocab, E = cfg->embed_size, H = cfg->hidden, nl = cfg->num_layers, P = cfg->pred_out,
            J = cfg->join_dim, Ee = cfg->enc_dim;
  if (V < 2 || nl < 1 || nl > RNNT_MAXL) return set_error(CFM_ERR_ASSERT, "vocab >= 2 and 1 <= num_layers <= 4");
  for (int v : {E, H, P, J, Ee})
    if (v <= 0 || v % 4 || v > 1024) return set_error(CFM_ERR_ASSERT, "predictor / joint widths: multiples of 4, <= 1024");
  if (Ee % 32) return set_error(CFM_ERR_ASSERT, "enc_output_size must be a multiple of 32");
  if (cfg->blank < 0 || cfg->blank >= V) return set_error(CFM_ERR_VALUE, "blank id out of range");
  std::map<std::string, std::pair<const float*, int64_t>> m;
  for (int i = 0; i < n; ++i) m[weights[i].name] = {weights[i].data, weights[i].numel};
  auto get = [&](const std::string& k, int64_t numel) -> const float* {
    auto it = m.find(k);
    if (it == m.end()) throw std::string("missing weight " + k);
    if (it->second.second != numel) throw std::string("weight " + k + ": wrong numel");
    return it->second.first;
  };
  auto transpose = [](const float* s, int rows, int cols, int cols_pad) {   // [rows][cols] -> [cols][pad rows]
    std::vector<float> t((size_t)cols * cols_pad, 0.f);
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) t[(size_t)c * cols_pad + r] = s[(size_t)r * cols + c];
    return t;
  };
  auto h = std::make_unique<cfm_rnnt>();
  h->cfg = *cfg;
  h->device = device;
  Img img;
  RnntDev& w = h->w;
  w.V = V; w.Vp = (V + 3) / 4 * 4; w.E = E; w.H = H; w.nl = nl; w.P = P; w.J = J; w.blank = cfg->blank;
  try {
    const float* emb = get("predictor.embed.weight", (int64_t)V * E);
    img.put(std::vector<float>(emb, emb + (size_t)V * E), &w.embed);
    for (int l = 0; l < nl; ++l) {
      const int in = l == 0 ? E : H;
      const std::string s = std::to_string(l);
      const float* wih = get("predictor.rnn.weight_ih_l" + s, (int64_t)4 * H * in);
      const float* whh = get("predictor.rnn.weight_hh_l" + s, (int64_t)4 * H * H);
      const float* bih = get("predictor.rnn.bias_ih_l" + s, 4 * H);
      const float* bhh = get("predictor.rnn.bias_hh_l" + s, 4 * H);
      std::vector<float> a = transpose(wih, 4 * H, in, 4 * H), bm = transpose(whh, 4 * H, H, 4 * H);
      a.insert(a.end(), bm.begin(), bm.end());   // [(in + H)][4H]
      img.put(a, &w.wg[l]);
      std::vector<float> bias(4 * H);
      for (int i = 0; i < 4 * H; ++i) bias[i] = bih[i] + bhh[i];
      img.put(bias, &w.bg[l]);
    }
    img.put(transpose(get("predictor.projection.weight", (int64_t)P * H), P, H, P), &w.wp);
    const float* bp = get("predictor.projection.bias", P);
    img.put(std::vector<float>(bp, bp + P), &w.bp);
    img.put(transpose(get("joint.pred_ffn.weight", (int64_t)J * P), J, P, J), &w.wpj);
    const float* bpj = get("joint.pred_ffn.bias", J);
    img.put(std::vector<float>(bpj, bpj + J), &w.bpj);
    img.put(transpose(get("joint.ffn_out.weight", (int64_t)V * J), V, J, w.Vp), &w.wo);
    const float* bo = get("joint.ffn_out.bias", V);
    std::vector<float> bov(w.Vp, -std::numeric_limits<float>::infinity());
    std::copy(bo, bo + V, bov.begin());
    img.put(bov, &w.bo);
    const float* we = get("joint.enc_ffn.weight", (int64_t)J * Ee);
    img.put(std::vector<float>(we, we + (size_t)J * Ee), &h->we);
    const float* be = get("joint.enc_ffn.bias", J);
    img.put(std::vector<float>(be, be + J), &h->be);
  } catch (const std::string& e) {
    return set_error(CFM_ERR_VALUE, e);
  }
  if (rnnt_lds_bytes(w) > 160 * 1024) return set_error(CFM_ERR_ASSERT, "predictor / joint too wide for one workgroup's LDS");
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&h->dev_mem, img.bytes.size()) != hipSuccess ||
      hipMemcpy(h->dev_mem, img.bytes.data(), img.bytes.size(), hipMemcpyHostToDevice) != hipSuccess)
    return set_error(CFM_ERR_RUNTIME, std::string("rnnt weights upload: ") + hipGetErrorString(hipGetLastError()));
  for (auto& f : img.fix) *f.second = reinterpret_cast<const float*>((char*)h->dev_mem + f.first);
  *out = h.release();
  return CFM_OK;
}

void cfm_rnnt_destroy(cfm_rnnt* h) { delete h; }

size_t cfm_rnnt_workspace_bytes(const cfm_rnnt* h, int32_t rows) {
  return h && rows > 0 ? (size_t)rows * h->cfg.join_dim * sizeof(float) + 256 : 0;
}

cfm_status cfm_rnnt_greedy(const cfm_rnnt* h, const float* enc, int32_t rows, const int32_t* row_start,
                           const int32_t* row_len, int32_t B, int32_t n_steps, int32_t* out, void* ws, size_t wsb,
                           cfm_stream stream) {
  if (!h) return set_error(CFM_ERR_VALUE, "null handle");
  if (B < 0 || rows < 0 || n_steps < 1) return set_error(CFM_ERR_VALUE, "bad B / rows / n_steps");
  if (B == 0 || rows == 0) return CFM_OK;
  if (!enc || !row_start || !row_len || !out || !ws) return set_error(CFM_ERR_VALUE, "null argument");
  if (wsb < cfm_rnnt_workspace_bytes(h, rows)) return set_error(CFM_ERR_VALUE, "rnnt workspace too small");
  if (hipSetDevice(h->device) != hipSuccess) return set_error(CFM_ERR_RUNTIME, "hipSetDevice");
  const hipStream_t st = (hipStream_t)stream;
  float* proj = (float*)ws;
  EpiArgs e;
  e.bias = h->be; e.out = proj; e.ldo = h->cfg.join_dim;
  int r = gemm<float>(EPI_STORE, ACT_NONE, enc, h->cfg.enc_dim, h->we, h->cfg.enc_dim, rows, h->cfg.join_dim,
                      h->cfg.enc_dim, e, st);
  if (r) return set_error(CFM_ERR_RUNTIME, std::string("rnnt enc_ffn gemm: ") + hipGetErrorString((hipError_t)r));
  const size_t lds = rnnt_lds_bytes(h->w);
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)rnnt_greedy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return set_error(CFM_ERR_RUNTIME, "rnnt: dynamic LDS attribute");
  hipLaunchKernelGGL(rnnt_greedy_kernel, dim3(B), dim3(RNNT_NT), lds, st, h->w, proj, row_start, row_len, n_steps,
                     out);
  const hipError_t le = hipGetLastError();
  if (le != hipSuccess) return set_error(CFM_ERR_RUNTIME, std::string("rnnt_greedy_kernel: ") + hipGetErrorString(le));
  return CFM_OK;
}

}  // extern "C"
