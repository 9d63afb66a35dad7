// Probe: what the clamp modifier does on v_cvt_pk_bf16_f32 (gfx950).  If it saturates to [0, 1],
// relu(x) = 2^16 * clamp(x * 2^-16) for |x| < 2^16 (exact: power-of-two scaling), which would fold the
// front-end's ReLU into the f32 -> bf16 conversion.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
__global__ void k(const float* a, unsigned* o, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  unsigned r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a[2 * i]), "v"(a[2 * i + 1]));
  o[i] = r;
}
static float bf(unsigned short b) { unsigned u = (unsigned)b << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
  const float nan = __builtin_nanf("");
  float h[] = {-3.5f, -0.0f, 0.0f, 0.5f, 1.0f, 1.5f, 2.0e-5f, -2.0e-5f, 65504.f, nan, 1e-30f, -1e-30f,
               0.999f, 1.001f, 3.0e-5f, -7.0f};
  const int n = sizeof(h) / sizeof(h[0]) / 2;
  float* da; unsigned* dout;
  hipMalloc(&da, sizeof(h)); hipMalloc(&dout, n * 4);
  hipMemcpy(da, h, sizeof(h), hipMemcpyHostToDevice);
  k<<<1, 64>>>(da, dout, n);
  unsigned out[64];
  hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i)
    printf("in (%g, %g) -> (%g, %g)\n", h[2 * i], h[2 * i + 1], bf(out[i] & 0xffff), bf(out[i] >> 16));
  return 0;
}
