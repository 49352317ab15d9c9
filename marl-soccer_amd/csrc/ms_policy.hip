// ms_policy.hip — fused actor-critic forward of the reference's PPO policy on gfx950.
//
// The reference's caller (marl-soccer.ipynb, train cell, rollout L299-313; eval.py:17-47, 69-81)
// normalises the blue agents' observations with its RunningMeanStd (clip((x - mean) /
// (sqrt(var) + 1e-8), -10, 10) in float64, then float32) and runs two tanh MLPs
// 66-512-256-128-64-{3, 1} (actor mean, critic value). Here one kernel does all of it per
// tile of 32 rows, with every hidden activation kept in registers:
//
//   * one wave per 32-row tile; every layer is C^T = W . H^T on the f32-input MFMA
//     v_mfma_f32_32x32x2_f32 (exact f32: a k-ordered fmaf chain, MI355X_MICROARCH.md):
//     the batch row is the lane's column of the 32x32 accumulator tile (lane & 31) and the
//     layer's output features are the tile's rows, 16 registers per lane;
//   * an accumulator tile is the next layer's B operand as it stands (no LDS, no lane moves):
//     k-step 16P + r of the next layer takes register r of input tile P, whose feature for lane
//     half h is 32P + (r & 3) + 8 (r >> 2) + 4h — the packed weights (A operand) follow that
//     order (marlsoccer/policy.py packs them);
//   * weights stream from L2 (both nets are 1.7 MB, resident) as one coalesced 16-B load per
//     lane per four MFMAs, issued a group ahead of their use;
//   * bias and tanh are applied to the accumulator registers in place.
//
// Layer geometry (T = 32-feature output tiles, G = groups of four k-steps of two features):
//   L1 66 -> 512 (T 16, G 9: 33 k-steps + 3 zero steps), L2 512 -> 256 (T 8, G 64),
//   L3 256 -> 128 (T 4, G 32), L4 128 -> 64 (T 2, G 16), L5 64 -> {3 | 1} (T 1, G 8).
// Packed net (floats): per layer W[T][G][64 lanes][4] then bias[T][2 halves][16 registers].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <type_traits>

#include "../../include/marl_soccer.h"

namespace pol {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TM = 32;  // rows per wave
#ifndef MS_POL_DEPTH
#define MS_POL_DEPTH 2
#endif
#ifndef MS_POL_CH
#define MS_POL_CH 4
#endif
constexpr int DEPTH = MS_POL_DEPTH;  // A-operand groups in flight
constexpr int CH = MS_POL_CH;        // output tiles accumulated at once (layers 1-3)
constexpr int T1 = 16, T2 = 8, T3 = 4, T4 = 2, T5 = 1;
constexpr int G1 = 9, G2 = 64, G3 = 32, G4 = 16, G5 = 8;
constexpr int OW1 = 0, OB1 = OW1 + T1 * G1 * 256;
constexpr int OW2 = OB1 + T1 * 32, OB2 = OW2 + T2 * G2 * 256;
constexpr int OW3 = OB2 + T2 * 32, OB3 = OW3 + T3 * G3 * 256;
constexpr int OW4 = OB3 + T3 * 32, OB4 = OW4 + T4 * G4 * 256;
constexpr int OW5 = OB4 + T4 * 32, OB5 = OW5 + T5 * G5 * 256;
constexpr int NET = OB5 + T5 * 32;
static_assert(NET == MS_POLICY_NET_FLOATS, "packed layout of include/marl_soccer.h");

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// tanh(x) = sign(x) (1 - 2 / (exp(2|x|) + 1)) on the hardware exp2 and reciprocal (absolute
// error ~2e-7: the hidden activations' rounding, far below the 1e-5 output bound)
__device__ __forceinline__ float tanh_fast(float x) {
  const float ax = __builtin_fabsf(x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);  // 2 log2(e)
  const float t = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
  return __builtin_copysignf(t, x);
}

// One dense layer C^T = W . H^T (+ bias, tanh unless LAST) for T_OUT output tiles, CH tiles at
// a time. bop(s) gives this lane's B operand of k-step s (compile-time s); W/b the layer's
// packed weights and biases.
template <int T_OUT, int G, int CH, bool LAST, typename BOP>
__device__ __forceinline__ void dense(BOP&& bop, f32x16 (&Y)[T_OUT], const float* __restrict__ W,
                                      const float* __restrict__ b, int lane) {
  const int h = lane >> 5;
  static_for<0, T_OUT / CH>([&](auto cc) __attribute__((always_inline)) {
    constexpr int c = decltype(cc)::value;
    f32x16 acc[CH];
    static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
      acc[decltype(tc)::value] = f32x16{0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f,
                                        0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    });
    // A operands of the current group and the next DEPTH - 1 groups (a ring: each group's
    // 16-B loads are issued DEPTH - 1 groups, 4 (DEPTH - 1) CH MFMAs, ahead of their use)
    f32x4 a[DEPTH][CH];
    static_for<0, DEPTH - 1>([&](auto pc) __attribute__((always_inline)) {
      constexpr int g = decltype(pc)::value;
      if constexpr (g < G) {
        static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          a[g][t] = *(const f32x4*)(W + (((c * CH + t) * G + g) * 64 + lane) * 4);
        });
      }
    });
    static_for<0, G>([&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g + DEPTH - 1 < G) {
        static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          a[(g + DEPTH - 1) % DEPTH][t] = *(const f32x4*)(W + (((c * CH + t) * G + g + DEPTH - 1) * 64 + lane) * 4);
        });
      }
      static_for<0, 4>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const float bv = bop(std::integral_constant<int, 4 * g + j>{});
        static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g % DEPTH][t][j], bv, acc[t], 0, 0, 0);
        });
      });
    });
    static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      const f32x4* bb = (const f32x4*)(b + ((c * CH + t) * 2 + h) * 16);
      f32x16 y = acc[t];
      static_for<0, 4>([&](auto qc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        const f32x4 bq = bb[q];
        static_for<0, 4>([&](auto ec) __attribute__((always_inline)) {
          constexpr int e = decltype(ec)::value;
          const float v = y[4 * q + e] + bq[e];
          y[4 * q + e] = LAST ? v : tanh_fast(v);
        });
      });
      Y[c * CH + t] = y;
    });
  });
}

// One net (actor or critic) on the normalised inputs xk (k-step s of layer 1: feature 2s + h,
// s < 36; steps 33-35 are zero). Returns the last layer's tile (rows 0..NOUT-1 of lane half 0).
__device__ __forceinline__ f32x16 net_forward(const float (&xk)[36], const float* __restrict__ P, int lane) {
  f32x16 H1[T1];
  dense<T1, G1, CH, false>([&](auto s) __attribute__((always_inline)) { return xk[decltype(s)::value]; }, H1, P + OW1,
                          P + OB1, lane);
  f32x16 H2[T2];
  dense<T2, G2, CH, false>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H1[k >> 4][k & 15];
  }, H2, P + OW2, P + OB2, lane);
  f32x16 H3[T3];
  dense<T3, G3, CH, false>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H2[k >> 4][k & 15];
  }, H3, P + OW3, P + OB3, lane);
  f32x16 H4[T4];
  dense<T4, G4, 2, false>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H3[k >> 4][k & 15];
  }, H4, P + OW4, P + OB4, lane);
  f32x16 H5[T5];
  dense<T5, G5, 1, true>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H4[k >> 4][k & 15];
  }, H5, P + OW5, P + OB5, lane);
  return H5[0];
}

// Row r of the input: x + (r / group_rows) * group_stride + (r % group_rows) * row_stride.
__global__ __launch_bounds__(64) void policy_forward_kernel(const float* __restrict__ x, int64_t rows, int group_rows,
                                                            int64_t group_stride, int64_t row_stride,
                                                            const double* __restrict__ mean,
                                                            const double* __restrict__ den,
                                                            const float* __restrict__ actor,
                                                            const float* __restrict__ critic,
                                                            float* __restrict__ act_mean, float* __restrict__ value) {
  const int lane = threadIdx.x;
  const int h = lane >> 5;
  const int64_t row = (int64_t)blockIdx.x * TM + (lane & 31);
  const bool valid = row < rows;
  const int64_t rr = valid ? row : rows - 1;
  const float* xr = x + (rr / group_rows) * group_stride + (rr % group_rows) * row_stride;
  // layer-1 B operand: feature 2s + h of this lane's row, normalised as RunningMeanStd.normalize
  // (float64 (x - mean) / (sqrt(var) + 1e-8), clip to [-10, 10], float32)
  float xk[36];
#pragma unroll
  for (int s = 0; s < 33; ++s) {
    const int f = 2 * s + h;
    const float v = xr[f];
    if (mean) {
      double y = ((double)v - mean[f]) / den[f];
      y = y < -10.0 ? -10.0 : (y > 10.0 ? 10.0 : y);
      xk[s] = (float)y;
    } else {
      xk[s] = v;
    }
  }
  xk[33] = 0.0f; xk[34] = 0.0f; xk[35] = 0.0f;
  if (actor) {
    const f32x16 m = net_forward(xk, actor, lane);
    if (valid && h == 0) {  // rows 0..2 of the tile = the three action components, lane half 0
      act_mean[row * 3 + 0] = m[0];
      act_mean[row * 3 + 1] = m[1];
      act_mean[row * 3 + 2] = m[2];
    }
  }
  if (critic) {
    const f32x16 v = net_forward(xk, critic, lane);
    if (valid && h == 0) value[row] = v[0];
  }
}

}  // namespace pol

static thread_local std::string g_pol_err;

extern "C" {

const char* ms_policy_last_error(void) { return g_pol_err.c_str(); }

int ms_policy_forward(const float* x, int64_t rows, int group_rows, int64_t group_stride, int64_t row_stride,
                      const double* mean, const double* den, const float* actor, const float* critic, float* act_mean,
                      float* value, void* stream) {
  if (!x || rows <= 0 || group_rows <= 0 || (!actor && !critic) || (actor && !act_mean) || (critic && !value) ||
      (!mean) != (!den)) {
    g_pol_err = "ms_policy_forward: bad arguments";
    return MS_ERR_INVALID_ARGUMENT;
  }
  if (((uintptr_t)actor & 15u) || ((uintptr_t)critic & 15u)) {
    g_pol_err = "ms_policy_forward: packed weights must be 16-B aligned";
    return MS_ERR_INVALID_ARGUMENT;
  }
  const unsigned grid = (unsigned)((rows + pol::TM - 1) / pol::TM);
  hipLaunchKernelGGL(pol::policy_forward_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, x, rows, group_rows,
                     group_stride, row_stride, mean, den, actor, critic, act_mean, value);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_pol_err = std::string("ms_policy_forward: ") + hipGetErrorString(e);
    return MS_ERR_HIP;
  }
  return MS_OK;
}

}  // extern "C"
