// Validation of the reduced-range division / sqrt sequences of ms_device.h (div_nr, sqrt_nr)
// against the compiler's IEEE fp32 division and sqrtf, bit for bit, on random operands of the
// domains the kernel guards for (frame_inputs_in_range): numerators 0 or 2^-100..2^30,
// divisors 2^-28..2^14 plus the obs constants, sqrt arguments 2^-90..2^126.
// Built and run by tests/test_fastdiv.py (GPU); prints the mismatch counts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <math.h>
#include "../../marl-soccer_amd/csrc/ms_device.h"
using ms::rcp_nr;
using ms::div_nr;
using ms::sqrt_nr;
using ms::div_nr2;
using ms::div_nr_nonneg;
__device__ __forceinline__ uint64_t mix(uint64_t z) { z += 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }
__device__ float logu(uint64_t h, float lo_e, float hi_e) {  // log-uniform magnitude 2^[lo,hi) with random mantissa
  float e = lo_e + (hi_e - lo_e) * (float)(h & 0xffffff) / 16777216.0f;
  int ie = (int)floorf(e);
  uint32_t mant = (uint32_t)(h >> 24) & 0x7fffff;
  return __uint_as_float(((uint32_t)(ie + 127) << 23) | mant);
}
__global__ void k(uint64_t base, unsigned long long* bad, unsigned long long* badsq, float* ex, unsigned long long* seen) {
  uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t h1 = mix(i), h2 = mix(i ^ 0xabcdef1234567ull), h3 = mix(i * 3 + 7);
  float n = logu(h1, -100.0f, 30.0f);
  if (h3 & 1) n = -n;
  if ((h3 & 0x3f0) == 0) n = 0.0f;
  float d;
  uint32_t sel = (h3 >> 10) & 15;
  if (sel == 0) d = 200.0f; else if (sel == 1) d = 10.0f; else if (sel == 2) d = 1000.0f; else if (sel == 3) d = 3.1415927410125732f;
  else d = logu(h2, -28.0f, 14.0f);
  float q0 = n / d, q1 = div_nr(n, d, rcp_nr(d));
  // the packed pair form (second component: an independent numerator) and the +0-safe form
  // must give the same bits as div_nr itself
  const float n2 = (h2 & 2) ? -logu(h3 ^ h2, -100.0f, 30.0f) : ((h2 & 0x7c) == 0 ? 0.0f : logu(h3 ^ h2, -100.0f, 30.0f));
  const ms::V2 qp = div_nr2(ms::V2{n, n2}, d, rcp_nr(d));
  const float q2 = n2 / d;
  bool wrong = __float_as_uint(qp.x) != __float_as_uint(q0) || __float_as_uint(qp.y) != __float_as_uint(q2);
  const float na = fabsf(n);
  wrong = wrong || __float_as_uint(div_nr_nonneg(na, d, rcp_nr(d))) != __float_as_uint(na / d);
  if (wrong || __float_as_uint(q0) != __float_as_uint(q1)) { unsigned long long c = atomicAdd(bad, 1ull); if (c < 4) { ex[4*c] = n; ex[4*c+1] = d; ex[4*c+2] = q0; ex[4*c+3] = q1; } }
  // also dx/mag with mag = sqrt(dx^2+dy^2) structure
  float x = logu(h2 ^ h1, -90.0f, 126.0f);
  float s0 = sqrtf(x), s1 = sqrt_nr(x);
  if (threadIdx.x == 0) atomicAdd(seen, (unsigned long long)blockDim.x);
  if (__float_as_uint(s0) != __float_as_uint(s1)) { unsigned long long c = atomicAdd(badsq, 1ull); if (c < 4) { ex[16+2*c] = x; ex[17+2*c] = s1; } }
}
int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 64;
  unsigned long long *bad, *badsq, *seen; float* ex;
  (void)hipMalloc(&seen, 8); (void)hipMemset(seen, 0, 8);
  hipMalloc(&bad, 8); hipMalloc(&badsq, 8); hipMalloc(&ex, 256);
  hipMemset(bad, 0, 8); hipMemset(badsq, 0, 8); hipMemset(ex, 0, 256);
  const uint64_t per = 1ull << 28;  // samples per launch
  for (int r = 0; r < rounds; ++r) hipLaunchKernelGGL(k, dim3(per / 256), dim3(256), 0, 0, (uint64_t)r * per, bad, badsq, ex, seen);
  hipDeviceSynchronize();
  unsigned long long hb, hs, hseen; float hex[64];
  printf("launch status: %s\n", hipGetErrorString(hipGetLastError()));
  (void)hipMemcpy(&hseen, seen, 8, hipMemcpyDeviceToHost);
  printf("samples executed %llu\n", hseen);
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(&hs, badsq, 8, hipMemcpyDeviceToHost); hipMemcpy(hex, ex, 256, hipMemcpyDeviceToHost);
  printf("samples %llu div mismatches %llu sqrt mismatches %llu\n", (unsigned long long)rounds * per, hb, hs);
  for (int c = 0; c < 4 && c < (int)hb; ++c) printf("  div n=%a d=%a ieee=%a nr=%a\n", hex[4*c], hex[4*c+1], hex[4*c+2], hex[4*c+3]);
  for (int c = 0; c < 4 && c < (int)hs; ++c) printf("  sqrt x=%a nr=%a\n", hex[16+2*c], hex[17+2*c]);
  return 0;
}
