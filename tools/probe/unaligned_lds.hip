// probe: does ds_write_b64 / ds_read_b64 at a 2-byte-aligned LDS address work on this GPU?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long* out, int off) {
  __shared__ __attribute__((aligned(16))) unsigned short s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = 0;
  __syncthreads();
  unsigned long long v = 0x0004000300020001ull + 0x0001000100010001ull * (unsigned long long)(threadIdx.x * 4);
  unsigned addr = (unsigned)(size_t)(__attribute__((address_space(3))) char*)s + (threadIdx.x * 8 + off) * 2;
  asm volatile("ds_write_b64 %0, %1\n s_waitcnt lgkmcnt(0)" :: "v"(addr), "v"(v) : "memory");
  __syncthreads();
  unsigned long long r;
  asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
  out[threadIdx.x] = r;
  if (threadIdx.x == 0) out[64] = ((unsigned long long)s[off + 1] << 16) | s[off];
}
int main() {
  unsigned long long* d; hipMalloc(&d, 65 * 8);
  for (int off = 0; off < 4; ++off) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, off);
    unsigned long long h[65]; hipMemcpy(h, d, 65 * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 64; ++t) {
      unsigned long long e = 0x0004000300020001ull + 0x0001000100010001ull * (unsigned long long)(t * 4);
      if (h[t] != e) bad++;
    }
    printf("off=%d (byte misalign %d): %d lanes wrong, s[off..off+1]=%llx, hipErr=%s\n", off, (off * 2) % 8, bad, h[64],
           hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
