// Exhaustive check of the one-correction division by a constant (diagnostic, not product code).
//
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -o div_check tools/div_check.hip && ./div_check
//
// For a divisor d and y = rcp_nr(d) (the kernels' refined reciprocal), the product's one-residual
// quotient div_k(n, d, y) (q0 = n y, r = fma(-d, q0, n), q1 = fma(r, y, q0)) is compared bit for bit
// with the IEEE quotient n / d for EVERY fp32 numerator n of a bit range (both signs), and for n >= +0
// also div_k_nonneg and the packed div_k2_nonneg of unit_mag2_pos (both components), for the divisors
// the frame arithmetic divides by: 1000 (magnitudes), 200 and 10 (the default obs_vmax, obs_wmax) and pi
// (angle_obs). The functions are ms_device.h's own (included), so a change to them is what this checks.
// Any mismatch is counted and the first few are printed; a clean run over a domain proves the shorter
// sequence equal there.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

// the product's own device functions (rcp_nr, div_k, div_k_nonneg, div_k2_nonneg), not copies
#include "../marl-soccer_amd/csrc/ms_device.h"

__global__ void check(float d, uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
  const float y = ms::rcp_nr(d);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= (uint64_t)(hi - lo); i += stride) {
    const uint32_t bits = lo + (uint32_t)i;
    float qn[2];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      const float n = __uint_as_float(bits | (sg ? 0x80000000u : 0u));
      const float ref = n / d;
      const float q1 = ms::div_k(n, d, y);
      bool same = __float_as_uint(q1) == __float_as_uint(ref) || (n == 0.0f && q1 == ref);
      if (sg == 0) {  // the non-negative forms (magnitudes): scalar and packed, this numerator paired with its neighbour
        const float q2 = ms::div_k_nonneg(n, d, y);
        const float nb = __uint_as_float(bits + 1u <= hi ? bits + 1u : bits);
        const ms::V2 q3 = ms::div_k2_nonneg(ms::V2{n, nb}, d, y);
        same = same && __float_as_uint(q2) == __float_as_uint(ref) && __float_as_uint(q3.x) == __float_as_uint(ref) &&
               __float_as_uint(q3.y) == __float_as_uint(nb / d);
      }
      qn[sg] = q1;
      if (!same) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 4) first[k] = __float_as_uint(n);
      }
    }
    (void)qn;
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 2;                                                                \
    }                                                                          \
  } while (0)

int main() {
  struct Case { const char* name; float d; uint32_t lo, hi; bool domain; };
  const Case cases[] = {
      // the fast path's numerator domain: 2^-100 .. 2^32 (frame_inputs_in_range / psnap_in_range)
      {"mag / 1000", 1000.0f, 0x0D800000u, 0x4F800000u, true},
      {"v / 200 (obs_vmax)", 200.0f, 0x0D800000u, 0x4F800000u, true},
      {"w / 10 (obs_wmax)", 10.0f, 0x0D800000u, 0x4F800000u, true},
      {"angle / pi", 3.1415927410125732f, 0x0D800000u, 0x40800000u, true},  // .. 4
      // every normal numerator (information: where the shorter sequence stops agreeing)
      {"mag / 1000 (normals)", 1000.0f, 0x00800000u, 0x7F000000u, false},
      {"v / 200 (normals)", 200.0f, 0x00800000u, 0x7F000000u, false},
      {"w / 10 (normals)", 10.0f, 0x00800000u, 0x7F000000u, false},
      {"angle / pi (normals)", 3.1415927410125732f, 0x00800000u, 0x7F000000u, false},
  };
  unsigned long long* bad;
  uint32_t* first;
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  CK(hipMalloc(&first, 4 * sizeof(uint32_t)));
  int fails = 0;
  for (const Case& c : cases) {
    CK(hipMemset(bad, 0, sizeof(unsigned long long)));
    CK(hipMemset(first, 0, 4 * sizeof(uint32_t)));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, c.d, c.lo, c.hi, bad, first);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long nb = 0;
    uint32_t f[4];
    CK(hipMemcpy(&nb, bad, sizeof(nb), hipMemcpyDeviceToHost));
    CK(hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost));
    printf("%-22s d=%a numerators [%08x, %08x] x 2 signs: %llu mismatches", c.name, c.d, c.lo, c.hi, nb);
    for (int k = 0; k < 4 && k < (int)nb; ++k) {
      float v;
      std::memcpy(&v, &f[k], 4);
      printf(" %08x(%a)", f[k], v);
    }
    printf("\n");
    fails += c.domain && nb != 0;  // (the rows over every normal numerator are information)
  }
  CK(hipFree(bad));
  CK(hipFree(first));
  return fails ? 1 : 0;
}
