// Diagnostic (not product): latency of dependent VALU chains and LDS round trips on one wave.
// Build: hipcc -O3 --offload-arch=gfx950 -o lat lat.hip ; run on the GPU box: ./lat
// latency microbenchmark (scratch, not product): one wave, chains of dependent ops
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k_lds(float* out, long long* cyc, int n, float a, float b) {
  __shared__ float s[64 * 32];
  int l = threadIdx.x;
  s[l * 32] = l;
  __syncthreads();
  unsigned addr = (unsigned)(size_t)&s[l * 32];
  float v = 0.f;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    v = __builtin_fmaf(v, a, b);
    asm volatile("ds_write_b32 %0, %1" :: "v"(addr), "v"(v) : "memory");
  }
  long long t1 = clock64();
  out[l] = v;
  if (l == 0) cyc[0] = t1 - t0;
}
__global__ void k_ldsr(float* out, long long* cyc, int n, float a, float b) {
  __shared__ unsigned s[64 * 32];
  int l = threadIdx.x;
  unsigned base = (unsigned)(size_t)&s[0];
  s[l * 32] = base + l * 128;  // points to itself
  __syncthreads();
  unsigned addr = base + l * 128;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    asm volatile("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)" : "+v"(addr) :: "memory");
  }
  long long t1 = clock64();
  out[l] = addr;
  if (l == 0) cyc[0] = t1 - t0;
}
__global__ void k_valu(float* out, long long* cyc, int n, float a, float b) {
  int l = threadIdx.x;
  float x = l;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 20; ++j) x = __builtin_fmaf(x, a, b);
  }
  long long t1 = clock64();
  out[l] = x;
  if (l == 0) cyc[0] = t1 - t0;
}
__global__ void k_valu_ilp(float* out, long long* cyc, int n, float a, float b) {
  int l = threadIdx.x;
  float x = l, y = l + 1, z = l + 2, w = l + 3;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 20; ++j) { x = __builtin_fmaf(x, a, b); y = __builtin_fmaf(y, a, b); z = __builtin_fmaf(z, a, b); w = __builtin_fmaf(w, a, b); }
  }
  long long t1 = clock64();
  out[l] = x + y + z + w;
  if (l == 0) cyc[0] = t1 - t0;
}
typedef __attribute__((ext_vector_type(2))) float f2;
__global__ void k_pk(float* out, long long* cyc, int n, float a, float b) {
  int l = threadIdx.x;
  f2 x = {(float)l, (float)l + 1};
  f2 A = {a, a}, B = {b, b};
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 20; ++j) x = __builtin_elementwise_fma(x, A, B);
  }
  long long t1 = clock64();
  out[l] = x.x + x.y;
  if (l == 0) cyc[0] = t1 - t0;
}
__global__ void k_wt(long long* cyc) {
  long long t0 = clock64();
  long long w0 = wall_clock64();
  long long t1 = t0, w1 = w0;
  while (t1 - t0 < 10000000) { t1 = clock64(); }
  w1 = wall_clock64();
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = w1 - w0; }
}
int main() {
  float* out; long long* cyc; hipMalloc(&out, 256 * 4); hipMalloc(&cyc, 64);
  long long h[2]; int n = 1000;
  k_wt<<<1, 64>>>(cyc); hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
  printf("clock64 %lld ticks vs wall_clock64 %lld ticks (100 MHz): %.2f GHz\n", h[0], h[1], h[0] / (h[1] / 100e6) / 1e9);
  for (int r = 0; r < 2; ++r) {
    k_lds<<<1, 64>>>(out, cyc, n, 0.999f, 0.001f); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("lds write->read->fma chain (b32): %.1f cycles/iter\n", (double)h[0] / n);
    k_ldsr<<<1, 64>>>(out, cyc, n, 0.999f, 0.001f); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("lds read pointer chase: %.1f cycles/iter\n", (double)h[0] / n);
    k_valu<<<1, 64>>>(out, cyc, n, 0.999f, 0.001f); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent v_fma: %.2f cycles/op\n", (double)h[0] / n / 20);
    k_valu_ilp<<<1, 64>>>(out, cyc, n, 0.999f, 0.001f); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("4 independent v_fma chains: %.2f cycles/op\n", (double)h[0] / n / 80);
    k_pk<<<1, 64>>>(out, cyc, n, 0.999f, 0.001f); hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("dependent v_pk_fma: %.2f cycles/op\n", (double)h[0] / n / 20);
  }
  return 0;
}
