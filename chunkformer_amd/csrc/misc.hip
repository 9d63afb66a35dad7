// Small kernels: relative PE table, cache carry, mask materialisation, CTC log-softmax.
#include <atomic>
#include "cfm_common.h"
#include "cfm_kernels.h"

namespace cfm {

int cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if (dev >= 64) dev = 63;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}


// Relative PE rows (embedding.py:119-142 / 144-174): row k <-> distance p = anchor - k,
// [2i] = sin(p * div_i), [2i+1] = cos(p * div_i), div_i = exp(2i * -(ln 1e4 / d)); f32 math.
template <typename T>
__global__ void pos_table_kernel(int d, int p_rows, int anchor, T* out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= p_rows * (d / 2)) return;
  const int k = idx / (d / 2), i = idx - k * (d / 2);
  const int p = anchor - k;
  const float div = expf((float)(2 * i) * (float)(-(9.210340371976184 / (double)d)));
  const float a = (float)(p < 0 ? -p : p) * div;
  const float sv = sinf(a), cv = cosf(a);
  out[(size_t)k * d + 2 * i] = from_f32<T>(p < 0 ? -sv : sv);
  out[(size_t)k * d + 2 * i + 1] = from_f32<T>(cv);
}
template <typename T>
int pos_table(int d, int p_rows, int anchor, T* out, hipStream_t st) {
  const int n = p_rows * (d / 2);
  if (n <= 0) return 0;
  hipLaunchKernelGGL((pos_table_kernel<T>), dim3((n + 255) / 256), dim3(256), 0, st, d, p_rows, anchor, out);
  CFM_CHECK_LAUNCH();
  return 0;
}

template <typename TI, typename TO>
__global__ void copy_rows_kernel(const TI* in, size_t n, TO* out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = from_f32<TO>(to_f32(in[i]));
}
template <typename T>
int att_cache_in(const float* cache, int L, int row_elems, T* kv, hipStream_t st) {
  const size_t n = (size_t)L * row_elems;
  if (!n) return 0;
  hipLaunchKernelGGL((copy_rows_kernel<float, T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cache, n, kv);
  CFM_CHECK_LAUNCH();
  return 0;
}
template <typename T>
int att_cache_out(const T* kv, int start_row, int L, int row_elems, float* cache, hipStream_t st) {
  const size_t n = (size_t)L * row_elems;
  if (!n) return 0;
  hipLaunchKernelGGL((copy_rows_kernel<T, float>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     kv + (size_t)start_row * row_elems, n, cache);
  CFM_CHECK_LAUNCH();
  return 0;
}

// forward_chunk attention cache [H][L][2dk] (head-major, encoder.py:310-385 layout
// [n_layers, batch, head, cache_t, 2dk]) <-> KV stream rows [t][H][2dk]
template <typename T, bool IN>
__global__ void att_cache_hl_kernel(float* cache, int H, int L, int dk2, T* kv) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t n = (size_t)H * L * dk2;
  if (i >= n) return;
  const int e = (int)(i % dk2);
  const int t = (int)((i / dk2) % L);
  const int h = (int)(i / ((size_t)dk2 * L));
  T* r = kv + ((size_t)t * H + h) * dk2 + e;
  if (IN) *r = from_f32<T>(cache[i]);
  else cache[i] = to_f32(*r);
}
template <typename T>
int att_cache_in_hl(const float* cache, int H, int L, int dk, T* kv, hipStream_t st) {
  const size_t n = (size_t)H * L * 2 * dk;
  if (!n) return 0;
  hipLaunchKernelGGL((att_cache_hl_kernel<T, true>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     const_cast<float*>(cache), H, L, 2 * dk, kv);
  CFM_CHECK_LAUNCH();
  return 0;
}
template <typename T>
int att_cache_out_hl(const T* kv, int start_row, int H, int L, int dk, float* cache, hipStream_t st) {
  const size_t n = (size_t)H * L * 2 * dk;
  if (!n) return 0;
  hipLaunchKernelGGL((att_cache_hl_kernel<T, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, cache,
                     H, L, 2 * dk, const_cast<T*>(kv) + (size_t)start_row * H * 2 * dk);
  CFM_CHECK_LAUNCH();
  return 0;
}

// conv cache [d][lorder] (channel-major, convolution.py:216-231) <-> GLU stream rows [t][d]
template <typename T, bool IN>
__global__ void cnn_cache_kernel(float* cache, int d, int lorder, T* glu) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= d * lorder) return;
  const int t = i / d, c = i - t * d;
  if (IN) glu[(size_t)t * d + c] = from_f32<T>(cache[c * lorder + t]);
  else cache[c * lorder + t] = to_f32(glu[(size_t)t * d + c]);
}
template <typename T>
int cnn_cache_in(const float* cache, int d, int lorder, T* glu, hipStream_t st) {
  hipLaunchKernelGGL((cnn_cache_kernel<T, true>), dim3((d * lorder + 255) / 256), dim3(256), 0, st,
                     const_cast<float*>(cache), d, lorder, glu);
  CFM_CHECK_LAUNCH();
  return 0;
}
template <typename T>
int cnn_cache_out(const T* glu, int start_row, int d, int lorder, float* cache, hipStream_t st) {
  hipLaunchKernelGGL((cnn_cache_kernel<T, false>), dim3((d * lorder + 255) / 256), dim3(256), 0, st, cache, d, lorder,
                     const_cast<T*>(glu) + (size_t)start_row * d);
  CFM_CHECK_LAUNCH();
  return 0;
}

// Both caches of one layer in ONE launch (endless_decode's / forward_chunk's per-layer cache traffic: four
// 5-us launches per layer on the segment pipeline's critical path otherwise).  Blocks [0, na) copy the
// attention cache (flat [L][2d] rows, or head-major [H][L][2dk] when HL), the rest the conv cache
// ([d][lorder] channel-major <-> GLU rows [t][d]); IN: f32 caches -> T stream rows, else the reverse.
template <typename T, bool IN, bool HL>
__global__ void cache_io_kernel(float* acache, int H, int L, int dk2, T* kv, float* ccache, int d, int lorder, T* glu,
                                int na) {
  if ((int)blockIdx.x < na) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t n = (size_t)H * L * dk2;
    if (i >= n) return;
    T* r = kv + i;   // flat: cache row t = stream row t, same [H][2dk] order
    if constexpr (HL) {
      const int e = (int)(i % dk2), t = (int)((i / dk2) % L), h = (int)(i / ((size_t)dk2 * L));
      r = kv + ((size_t)t * H + h) * dk2 + e;
    }
    if (IN) *r = from_f32<T>(acache[i]);
    else acache[i] = to_f32(*r);
    return;
  }
  const int i = ((int)blockIdx.x - na) * 256 + threadIdx.x;
  if (i >= d * lorder) return;
  const int t = i / d, c = i - t * d;
  if (IN) glu[(size_t)t * d + c] = from_f32<T>(ccache[c * lorder + t]);
  else ccache[c * lorder + t] = to_f32(glu[(size_t)t * d + c]);
}
// kv / glu point at the first stream row of the copied range (start row already applied)
template <typename T>
int cache_io(bool in, bool hl, float* acache, int H, int L, int dk, T* kv, float* ccache, int d, int lorder, T* glu,
             hipStream_t st) {
  const int na = (int)(((size_t)H * L * 2 * dk + 255) / 256), nc = ccache ? (d * lorder + 255) / 256 : 0;
  if (!acache) return (int)hipErrorInvalidValue;
  if (na + nc == 0) return 0;
#define CIO(I_, H_) hipLaunchKernelGGL((cache_io_kernel<T, I_, H_>), dim3(na + nc), dim3(256), 0, st, acache, H, L, 2 * dk, \
                                       kv, ccache, d, lorder, glu, na)
  if (in) { if (hl) CIO(true, true); else CIO(true, false); }
  else { if (hl) CIO(false, true); else CIO(false, false); }
#undef CIO
  CFM_CHECK_LAUNCH();
  return 0;
}

// att_mask [n][L+C+R] / mask_pad [n][C+14] from the plan (encoder.py:625-645 closed form)
__global__ void masks_kernel(const int32_t* meta, int n, int wa, int wp, uint8_t* att, uint8_t* pad) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int per = wa + wp;
  if (i >= n * per) return;
  const int c = i / per, j = i - c * per;
  const int32_t* m = meta + (size_t)c * PM_INTS;
  if (j < wa) att[(size_t)c * wa + j] = (j >= m[PM_ATT_LO] && j < m[PM_ATT_HI]) ? 1 : 0;
  else pad[(size_t)c * wp + (j - wa)] = (j - wa >= m[PM_CONV_LO] && j - wa < m[PM_CONV_HI]) ? 1 : 0;
}
int masks_from_plan(const int32_t* meta, int n, int C, int L, int R, uint8_t* att, uint8_t* pad, hipStream_t st) {
  const int wa = L + C + R, wp = C + 14, tot = n * (wa + wp);
  if (tot <= 0) return 0;
  hipLaunchKernelGGL(masks_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, meta, n, wa, wp, att, pad);
  CFM_CHECK_LAUNCH();
  return 0;
}

// CTC log_softmax (ctc.py:81) + argmax (chunkformer_model.py:437, 527), one wave per row, in place
__global__ __launch_bounds__(256) void log_softmax_kernel(float* x, int M, int V, int write_logp, int32_t* ids) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float* p = x + (size_t)row * V;
  float mx = -INFINITY;
  int am = 0x7fffffff;
  for (int v = lane; v < V; v += 64) {
    const float t = p[v];
    if (t > mx) { mx = t; am = v; }
  }
  // reduce (max, first index)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oi = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oi < am)) { mx = om; am = oi; }
  }
  if (ids && lane == 0) ids[row] = am;
  if (!write_logp) return;
  float s = 0.f;
  for (int v = lane; v < V; v += 64) s += __expf(p[v] - mx);
  const float lse = mx + __logf(wave_sum(s));
  for (int v = lane; v < V; v += 64) p[v] = p[v] - lse;
}
int log_softmax_rows(float* logits, int M, int V, int write_logp, int32_t* ids, hipStream_t st) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(log_softmax_kernel, dim3((M + 3) / 4), dim3(256), 0, st, logits, M, V, write_logp, ids);
  CFM_CHECK_LAUNCH();
  return 0;
}

template int pos_table<float>(int, int, int, float*, hipStream_t);
template int pos_table<bf16>(int, int, int, bf16*, hipStream_t);
template int pos_table<f16>(int, int, int, f16*, hipStream_t);
template int att_cache_in<float>(const float*, int, int, float*, hipStream_t);
template int att_cache_in<bf16>(const float*, int, int, bf16*, hipStream_t);
template int att_cache_in<f16>(const float*, int, int, f16*, hipStream_t);
template int att_cache_out<float>(const float*, int, int, int, float*, hipStream_t);
template int att_cache_out<bf16>(const bf16*, int, int, int, float*, hipStream_t);
template int att_cache_out<f16>(const f16*, int, int, int, float*, hipStream_t);
template int att_cache_in_hl<float>(const float*, int, int, int, float*, hipStream_t);
template int att_cache_in_hl<bf16>(const float*, int, int, int, bf16*, hipStream_t);
template int att_cache_in_hl<f16>(const float*, int, int, int, f16*, hipStream_t);
template int att_cache_out_hl<float>(const float*, int, int, int, int, float*, hipStream_t);
template int att_cache_out_hl<bf16>(const bf16*, int, int, int, int, float*, hipStream_t);
template int att_cache_out_hl<f16>(const f16*, int, int, int, int, float*, hipStream_t);
template int cnn_cache_in<float>(const float*, int, int, float*, hipStream_t);
template int cnn_cache_in<bf16>(const float*, int, int, bf16*, hipStream_t);
template int cnn_cache_in<f16>(const float*, int, int, f16*, hipStream_t);
template int cnn_cache_out<float>(const float*, int, int, int, float*, hipStream_t);
template int cnn_cache_out<bf16>(const bf16*, int, int, int, float*, hipStream_t);
template int cnn_cache_out<f16>(const f16*, int, int, int, float*, hipStream_t);

template int cache_io<float>(bool, bool, float*, int, int, int, float*, float*, int, int, float*, hipStream_t);
template int cache_io<bf16>(bool, bool, float*, int, int, int, bf16*, float*, int, int, bf16*, hipStream_t);
template int cache_io<f16>(bool, bool, float*, int, int, int, f16*, float*, int, int, f16*, hipStream_t);

}  // namespace cfm
