// Probe: the ring attention's rel_shift scratch, sheared-write (pitch 49 write / 48 read) against the
// read-side variant (aligned pitch-48 writes, 2-B aligned reads), one wave, f16 values = 100 * fr + e.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void probe(float* out_a, float* out_b) {
  __shared__ __attribute__((aligned(16))) _Float16 scr[2][16 * 49];
  const int lane = threadIdx.x, fr = lane & 15, g = lane >> 4;
  const unsigned sa = (unsigned)(size_t)(__attribute__((address_space(3))) char*)&scr[0][0];
  const unsigned sb = (unsigned)(size_t)(__attribute__((address_space(3))) char*)&scr[1][0];
  for (int pt = 0; pt < 3; ++pt) {
    float v[4];
    for (int r = 0; r < 4; ++r) v[r] = 100.f * fr + (16 * pt + 4 * g + r);
    const unsigned lo = __builtin_bit_cast(unsigned, (h2){(_Float16)v[0], (_Float16)v[1]});
    const unsigned hi = __builtin_bit_cast(unsigned, (h2){(_Float16)v[2], (_Float16)v[3]});
    const unsigned wa = sa + 2u * (unsigned)(fr * 49 + 1 + 16 * pt + 4 * g);
    asm volatile("ds_write_b16 %0, %1\n\tds_write_b16_d16_hi %0, %1 offset:2\n\t"
                 "ds_write_b16 %0, %2 offset:4\n\tds_write_b16_d16_hi %0, %2 offset:6" ::"v"(wa), "v"(lo), "v"(hi) : "memory");
    const unsigned wb = sb + 2u * (unsigned)(fr * 48 + 16 * pt + 4 * g);
    asm volatile("ds_write_b64 %0, %1" ::"v"(wb), "v"((u32x2){lo, hi}) : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  for (int st2 = 0; st2 < 2; ++st2) {
    h4 a, b;
    asm volatile("ds_read_b64 %0, %1" : "=v"(a) : "v"(sa + 2u * (unsigned)(fr * 48 + 16 + 16 * st2 + 4 * g)) : "memory");
    // read side: three dwords from the 4-B aligned address at or below the 2-B aligned start, then a
    // funnel shift by 0 or 16 bits (v_alignbit_b32) per output dword
    const unsigned ra = sb + 2u * (unsigned)(fr * 48 + 15 - fr + 16 * st2 + 4 * g);
    const unsigned al = ra & ~3u, sh = (ra & 2u) << 3;
    u32x2 d01;
    unsigned d2;
    asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:1" : "=v"(d01) : "v"(al) : "memory");
    asm volatile("ds_read_b32 %0, %1 offset:8" : "=v"(d2) : "v"(al) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(d01), "+v"(d2)::"memory");
    const u32x2 pr = {__builtin_amdgcn_alignbit(d01.y, d01.x, sh), __builtin_amdgcn_alignbit(d2, d01.y, sh)};
    b = __builtin_bit_cast(h4, pr);
    for (int r = 0; r < 4; ++r) {
      out_a[(lane * 2 + st2) * 4 + r] = (float)a[r];
      out_b[(lane * 2 + st2) * 4 + r] = (float)b[r];
    }
  }
}

int main() {
  float *a, *b;
  hipMalloc(&a, 512 * 4);
  hipMalloc(&b, 512 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b);
  float ha[512], hb[512];
  hipMemcpy(ha, a, 2048, hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 512; ++i) {
    const int lane = i / 8, st2 = (i / 4) & 1, r = i & 3, fr = lane & 15, g = lane >> 4;
    const float want = 100.f * fr + (15 - fr + 16 * st2 + 4 * g + r);
    if (ha[i] != want || hb[i] != want) {
      if (bad < 12) printf("lane %d st2 %d r %d: sheared %g read-side %g want %g\n", lane, st2, r, ha[i], hb[i], want);
      ++bad;
    }
  }
  printf("%d mismatches of 512\n", bad);
  return 0;
}
