// Diagnostic (not product): dependent-issue latency of the VALU instruction kinds in the contact
// solve's chain (one wave, s_memtime), 64 dependent instructions per kind, 100 repetitions.
// Build: hipcc -O3 --offload-arch=gfx950 -o deplat deplat.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

template <int K>
__global__ void lat(long long* out, float* sink, float seed) {
  float a = seed + threadIdx.x, b = 1.0001f, c = 0.5f;
  float a2 = a + 1.0f;
  long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < 101; ++rep) {
    if (rep == 1) t0 = clock64();
    if constexpr (K == 0) asm volatile(R64("v_add_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    if constexpr (K == 1) asm volatile(R64("v_fma_f32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == 2) asm volatile(R64("v_pk_add_f32 %0, %0, %1\n") : "+v"(*(double*)&a) : "v"(*(double*)&b));
    if constexpr (K == 3) asm volatile(R64("v_max_f32 %0, 0, %0\n") : "+v"(a));
    if constexpr (K == 4) asm volatile(R64("v_med3_f32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c));
    if constexpr (K == 5) asm volatile(R64("v_cmp_lt_f32 vcc, 0, %0\n v_cndmask_b32 %0, %1, %0, vcc\n") : "+v"(a) : "v"(b) : "vcc");
    if constexpr (K == 6) asm volatile(R64("v_add_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    if constexpr (K == 7) asm volatile(R64("v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2\n") : "+v"(a), "+v"(a2) : "v"(b));
  }
  t1 = clock64();
  sink[threadIdx.x] = a + a2;
  if (threadIdx.x == 0) out[K] = t1 - t0;
}

int main() {
  long long* d;
  float* s;
  hipMalloc(&d, 64 * 8);
  hipMalloc(&s, 64 * 4);
  const char* names[] = {"v_add_f32", "v_fma_f32", "v_pk_add_f32 (pairs)", "v_max_f32", "v_med3_f32",
                         "v_cmp vcc + v_cndmask (per pair of insts)", "v_add/v_mul alternating (per pair)",
                         "two independent v_add chains (per pair)"};
  for (int r = 0; r < 2; ++r) {
    lat<0><<<1, 64>>>(d, s, 1.f); lat<1><<<1, 64>>>(d, s, 1.f); lat<2><<<1, 64>>>(d, s, 1.f);
    lat<3><<<1, 64>>>(d, s, 1.f); lat<4><<<1, 64>>>(d, s, 1.f); lat<5><<<1, 64>>>(d, s, 1.f);
    lat<6><<<1, 64>>>(d, s, 1.f); lat<7><<<1, 64>>>(d, s, 1.f);
    hipDeviceSynchronize();
    long long h[8];
    hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
    for (int k = 0; k < 8; ++k) printf("%-44s %.2f cycles per dependent step\n", names[k], (double)h[k] / 100 / 64);
  }
  return 0;
}
