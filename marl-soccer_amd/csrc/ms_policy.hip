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
//   * the accumulators start at the bias; each chunk's tanh is applied to its accumulator
//     registers in place, interleaved with the MFMAs of the next chunk (or of the next layer's
//     first k-steps, which read earlier tiles): VALU work under the matrix pipe's 64 cycles.
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

// One dense layer C^T = W . H^T + bias for T_OUT output tiles, CH tiles at a time. The
// accumulators start at the bias (so the epilogue is the tanh alone), and the tanh of a chunk
// is software-pipelined into the MFMA stream: chunk c's tanh runs one element at a time between
// the MFMAs of chunk c + 1 (they are independent), and the last chunk's tanh is handed back as
// `pending` work that the next layer interleaves with its first k-steps (which read earlier
// tiles only). prev(s) is the previous layer's pending work for this layer's k-step s
// (chunk 0); bop(s) this lane's B operand of k-step s; W/b the packed weights and biases.
template <int T_OUT, int BASE, int CH>
struct Pending {  // the tanh of tiles [BASE, BASE + CH) of Y, to be spread over k-steps
  f32x16 (&Y)[T_OUT];
  template <int S, int SPAN>
  __device__ __forceinline__ void step() {  // element share of step S of SPAN steps
    constexpr int E = CH * 16;
    constexpr int lo = S * E / SPAN, hi = (S + 1) * E / SPAN;
    static_for<lo, hi>([&](auto ec) __attribute__((always_inline)) {
      constexpr int e = decltype(ec)::value;
      Y[BASE + e / 16][e % 16] = tanh_fast(Y[BASE + e / 16][e % 16]);
    });
  }
};
struct NoPending {
  template <int S, int SPAN>
  __device__ __forceinline__ void step() {}
};

template <int T_OUT, int G, int CH, bool LAST, int SLACK, typename BOP, typename PREV>
__device__ __forceinline__ void dense(BOP&& bop, PREV& prev, f32x16 (&Y)[T_OUT], const float* __restrict__ W,
                                      const float* __restrict__ b, int lane) {
  const int h = lane >> 5;
  constexpr int S = 4 * G;  // k-steps
  static_for<0, T_OUT / CH>([&](auto cc) __attribute__((always_inline)) {
    constexpr int c = decltype(cc)::value;
    f32x16 acc[CH];
    static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      const f32x4* bb = (const f32x4*)(b + ((c * CH + t) * 2 + h) * 16);
      const f32x4 b0 = bb[0], b1 = bb[1], b2 = bb[2], b3 = bb[3];
      acc[t] = f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                      b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
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
        constexpr int s = 4 * g + j;
        const float bv = bop(std::integral_constant<int, s>{});
        static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g % DEPTH][t][j], bv, acc[t], 0, 0, 0);
        });
        // interleaved VALU work: the previous layer's pending tanh (chunk 0, within the k-steps
        // that do not read it yet) or this layer's previous chunk's tanh
        if constexpr (c == 0) {
          if constexpr (s < SLACK) prev.template step<s, SLACK>();
        } else if constexpr (!LAST) {
          Pending<T_OUT, (c - 1) * CH, CH>{Y}.template step<s, S>();
        }
      });
    });
    if constexpr (c == 0 && SLACK > S) {  // a chunk shorter than the slack: finish the rest
      static_for<S, SLACK>([&](auto sc) __attribute__((always_inline)) {
        prev.template step<decltype(sc)::value, SLACK>();
      });
    }
    static_for<0, CH>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      Y[c * CH + t] = acc[t];
    });
  });
}

// One net (actor or critic) on the normalised inputs xk (k-step s of layer 1: feature 2s + h,
// s < 36; steps 33-35 are zero). Returns the last layer's tile (rows 0..NOUT-1 of lane half 0).
// The SLACK of a layer: the k-steps before it first reads the previous layer's last chunk
// (16 (T_prev - CH_prev)); a previous layer with a single chunk gets its tanh done up front.
__device__ __forceinline__ f32x16 net_forward(const float (&xk)[36], const float* __restrict__ P, int lane) {
  NoPending none;
  f32x16 H1[T1];
  dense<T1, G1, CH, false, 0>([&](auto s) __attribute__((always_inline)) { return xk[decltype(s)::value]; }, none, H1,
                              P + OW1, P + OB1, lane);
  Pending<T1, T1 - CH, CH> p1{H1};
  f32x16 H2[T2];
  dense<T2, G2, CH, false, 16 * (T1 - CH)>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H1[k >> 4][k & 15];
  }, p1, H2, P + OW2, P + OB2, lane);
  Pending<T2, T2 - CH, CH> p2{H2};
  f32x16 H3[T3];
  dense<T3, G3, CH, false, 16 * (T2 - CH)>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H2[k >> 4][k & 15];
  }, p2, H3, P + OW3, P + OB3, lane);
  // layer 3 is one chunk (T3 = CH): its tanh before layer 4, which reads it from k-step 0
  static_for<0, T3 * 16>([&](auto ec) __attribute__((always_inline)) {
    constexpr int e = decltype(ec)::value;
    H3[e / 16][e % 16] = tanh_fast(H3[e / 16][e % 16]);
  });
  f32x16 H4[T4];
  dense<T4, G4, 2, false, 0>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H3[k >> 4][k & 15];
  }, none, H4, P + OW4, P + OB4, lane);
  static_for<0, T4 * 16>([&](auto ec) __attribute__((always_inline)) {
    constexpr int e = decltype(ec)::value;
    H4[e / 16][e % 16] = tanh_fast(H4[e / 16][e % 16]);
  });
  f32x16 H5[T5];
  dense<T5, G5, 1, true, 0>([&](auto s) __attribute__((always_inline)) {
    constexpr int k = decltype(s)::value;
    return H4[k >> 4][k & 15];
  }, none, H5, P + OW5, P + OB5, lane);
  return H5[0];
}

// Row r of the input: obs + (r / group_rows) * group_stride + (r % group_rows) * row_stride.
// One launch per rollout step (ms_policy_run, include/marl_soccer.h): NULL outputs are skipped
// (wave-uniform branches).
__global__ __launch_bounds__(64) void policy_kernel(const ms_policy_io io) {
  const int lane = threadIdx.x;
  const int h = lane >> 5;
  const int64_t row = (int64_t)blockIdx.x * TM + (lane & 31);
  const bool valid = row < io.rows;
  const int64_t rr = valid ? row : io.rows - 1;
  const float* xr = io.obs + (rr / io.group_rows) * io.group_stride + (rr % io.group_rows) * io.row_stride;
  // the rollout's obs storage: the tile's rows as 8-B pieces, lanes over consecutive pieces of
  // the contiguous destination (a row's 66 features are contiguous in the source as well)
  const bool copy_pairs = io.obs_copy && !(((uintptr_t)io.obs | (uintptr_t)io.obs_copy) & 7u) &&
                          !((io.row_stride | io.group_stride) & 1);
  if (copy_pairs) {
    const int64_t row0 = (int64_t)blockIdx.x * TM;
    const int nr = (int)(io.rows - row0 < TM ? io.rows - row0 : TM);
    for (int i = lane; i < nr * 33; i += 64) {
      const int r = i / 33, c = i - 33 * r;
      const int64_t q = row0 + r;
      const float2 v = *(const float2*)(io.obs + (q / io.group_rows) * io.group_stride +
                                        (q % io.group_rows) * io.row_stride + 2 * c);
      *(float2*)(io.obs_copy + q * 66 + 2 * c) = v;
    }
  }
  // layer-1 B operand: feature 2s + h of this lane's row, normalised as RunningMeanStd.normalize
  // (float64 (x - mean) / (sqrt(var) + 1e-8), clip to [-10, 10], float32)
  float xk[36];
#pragma unroll
  for (int s = 0; s < 33; ++s) {
    const int f = 2 * s + h;
    const float v = xr[f];
    if (io.obs_copy && !copy_pairs && valid) io.obs_copy[row * 66 + f] = v;  // unaligned fallback
    if (io.mean) {
      double y = ((double)v - io.mean[f]) / io.den[f];
      y = y < -10.0 ? -10.0 : (y > 10.0 ? 10.0 : y);
      xk[s] = (float)y;
    } else {
      xk[s] = v;
    }
  }
  xk[33] = 0.0f; xk[34] = 0.0f; xk[35] = 0.0f;
  if (io.actor) {
    const f32x16 m = net_forward(xk, io.actor, lane);
    if (valid && h == 0) {  // rows 0..2 of the tile = the three action components, lane half 0
      float act[3];
      float lp = 0.0f;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (io.act_mean) io.act_mean[row * 3 + c] = m[c];
        act[c] = m[c];
        if (io.eps) {  // Agent.sample: eps * exp(logstd) + mean; Normal(mean, std).log_prob summed
          const float ls = io.logstd[c];
          const float sd = expf(ls);
          act[c] = io.eps[row * 3 + c] * sd + m[c];
          const float d = act[c] - m[c];
          lp += -(d * d) / (2.0f * (sd * sd)) - ls - 0.91893853320467274f;  // log sqrt(2 pi)
        }
        if (io.action) io.action[row * 3 + c] = act[c];
        if (io.env_actions) io.env_actions[((row >> 1) * 4 + (row & 1)) * 3 + c] = act[c];
        if (io.env_actions && io.red_uniform)
          io.env_actions[((row >> 1) * 4 + 2 + (row & 1)) * 3 + c] = io.red_uniform[row * 3 + c] * 2.0f - 1.0f;
      }
      if (io.logprob) io.logprob[row] = lp;
    }
  }
  if (io.critic) {
    const f32x16 v = net_forward(xk, io.critic, lane);
    if (valid && h == 0 && io.value) io.value[row] = v[0];
  }
}

// ms_rollout_record: one env per lane; the finished-episode count and scores reduced per wave
// (cross-lane adds), one device atomic per wave and counter.
__global__ __launch_bounds__(256) void rollout_record_kernel(int64_t n, const float* __restrict__ rew,
                                                             const uint8_t* __restrict__ term,
                                                             const uint8_t* __restrict__ trunc,
                                                             const int32_t* __restrict__ score,
                                                             float* __restrict__ rewards, float* __restrict__ next_done,
                                                             float* __restrict__ dones_next, int64_t* episodes,
                                                             int64_t* score_sum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int fin = 0, sb = 0, sr = 0;
  if (i < n) {
    const float2 r = *(const float2*)(rew + i * 4);
    *(float2*)(rewards + i * 2) = r;
    const uint32_t te = *(const uint32_t*)(term + i * 4), tr = *(const uint32_t*)(trunc + i * 4);
    const uint32_t d = te | tr;
    const float2 dn = make_float2((d & 0xffu) ? 1.0f : 0.0f, (d & 0xff00u) ? 1.0f : 0.0f);
    *(float2*)(next_done + i * 2) = dn;
    if (dones_next) *(float2*)(dones_next + i * 2) = dn;
    if (tr & 0xffu) {
      fin = 1;
      sb = score[i * 2];
      sr = score[i * 2 + 1];
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    fin += __shfl_xor(fin, m);
    sb += __shfl_xor(sb, m);
    sr += __shfl_xor(sr, m);
  }
  if ((threadIdx.x & 63) == 0 && fin) {
    atomicAdd((unsigned long long*)episodes, (unsigned long long)fin);
    atomicAdd((unsigned long long*)score_sum, (unsigned long long)(int64_t)sb);
    atomicAdd((unsigned long long*)(score_sum + 1), (unsigned long long)(int64_t)sr);
  }
}

}  // namespace pol

static thread_local std::string g_pol_err;

extern "C" {

const char* ms_policy_last_error(void) { return g_pol_err.c_str(); }

static int launch(const ms_policy_io& io, void* stream, const char* who) {
  const unsigned grid = (unsigned)((io.rows + pol::TM - 1) / pol::TM);
  hipLaunchKernelGGL(pol::policy_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, io);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_pol_err = std::string(who) + ": " + hipGetErrorString(e);
    return MS_ERR_HIP;
  }
  return MS_OK;
}

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
  ms_policy_io io = {};
  io.obs = x; io.rows = rows; io.group_rows = group_rows; io.group_stride = group_stride; io.row_stride = row_stride;
  io.mean = mean; io.den = den; io.actor = actor; io.critic = critic; io.act_mean = act_mean; io.value = value;
  return launch(io, stream, "ms_policy_forward");
}

int ms_policy_run(const ms_policy_io* io, void* stream) {
  if (!io || !io->obs || io->rows <= 0 || io->group_rows <= 0 || (!io->actor && !io->critic) ||
      (!io->mean) != (!io->den) || (io->eps && !io->logstd) || (io->eps && !io->actor) ||
      (io->env_actions && (!io->actor || (io->rows & 1))) || (io->red_uniform && !io->env_actions) ||
      ((io->act_mean || io->action || io->logprob || io->env_actions) && !io->actor) || (io->value && !io->critic)) {
    g_pol_err = "ms_policy_run: bad arguments";
    return MS_ERR_INVALID_ARGUMENT;
  }
  if (((uintptr_t)io->actor & 15u) || ((uintptr_t)io->critic & 15u)) {
    g_pol_err = "ms_policy_run: packed weights must be 16-B aligned";
    return MS_ERR_INVALID_ARGUMENT;
  }
  return launch(*io, stream, "ms_policy_run");
}

int ms_rollout_record(int64_t n_envs, const float* rew, const uint8_t* term, const uint8_t* trunc,
                      const int32_t* score, float* rewards, float* next_done, float* dones_next, int64_t* episodes,
                      int64_t* score_sum, void* stream) {
  if (n_envs <= 0 || !rew || !term || !trunc || !score || !rewards || !next_done || !episodes || !score_sum ||
      (((uintptr_t)rew | (uintptr_t)rewards | (uintptr_t)next_done | (uintptr_t)dones_next | (uintptr_t)episodes |
        (uintptr_t)score_sum) & 7u) ||
      (((uintptr_t)term | (uintptr_t)trunc | (uintptr_t)score) & 3u)) {
    g_pol_err = "ms_rollout_record: bad arguments (NULL or misaligned pointers)";
    return MS_ERR_INVALID_ARGUMENT;
  }
  const unsigned grid = (unsigned)((n_envs + 255) / 256);
  hipLaunchKernelGGL(pol::rollout_record_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_envs, rew, term,
                     trunc, score, rewards, next_done, dones_next, episodes, score_sum);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_pol_err = std::string("ms_rollout_record: ") + hipGetErrorString(e);
    return MS_ERR_HIP;
  }
  return MS_OK;
}

}  // extern "C"
