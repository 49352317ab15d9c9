// ms_env.hip — MI355X-native batched 2v2 soccer env: HIP kernels + the C-ABI of
// include/marl_soccer.h.
//
// One fused kernel advances every environment by one env.step (SoccerEnv.step ->
// Game.step -> pymunk Space.step(1/60); soccer_env.py:100-154, game/game.py:378-437).
// One lane owns one env for the whole step: the physics of one env is a short sequential
// Gauss-Seidel solve over at most a few contacts, so parallelism comes from the batch.
//
// HBM layout: state blocks. Block b holds the state of envs [64b, 64b + 64) — one wave's envs —
// as planes of 64 lane elements (16-B elements, 4-B for the cache headers), so one wave
// instruction moves 1 KiB of contiguous memory and fetches four fields per lane, and every plane
// sits at a compile-time offset from the block base (no per-plane base address is held in a
// register):
//   B4 float4 [11][64]     bodies, flat field i in plane i/4 (agent b: 9b + px py vx vy angle w
//                          vbx vby wb; ball: 36 + px py vx vy w vbx vby wb)
//   H4 float4 [7][64]      obs-history snapshot of step t-2 (26 floats, 2 pad). The snapshot of
//                          t-1 is the body state itself at the start of the step.
//   I4 int4   [64]         steps, score (blue | red << 16), meta bits, PCG64 buffered u32
//   R2 u64x2  [2][64]      PCG64 (state hi, lo), (inc hi, lo): touched by resets and goal respawns
//   CH u32    [2][MAXA][64] arbiter-cache headers, ping-pong by a per-env parity bit
//   CJ float4 [2][MAXA][64] arbiter-cache accumulated impulses (jn0, jt0, jn1, jt1)
// The last block is padded to 64 envs; the padding lanes run with zeroed state and store nothing.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <random>
#include <string>
#include <type_traits>

#include "ms_device.h"

using namespace ms;

#ifndef MS_BLOCK
#define MS_BLOCK 64
#endif
#define MAXA MS_MAX_ARBITERS

// ---- group indices -----------------------------------------------------------------------
enum {
  F_BALL = 36,      // flat body field of the ball's px (agent b: 9b)
  G_BODY = 11,      // float4 groups of body state (44 floats)
  G_SNAP = 7        // float4 groups of one snapshot (MS_SNAP_SIZE = 26 floats + 2 pad)
};
// META bits: 0-1 spawn mode, 2 hist_empty, 4 cache parity, 8-13 n_cache, 16 PCG64 has_uint32
#define META_MODE(m) ((m) & 3)
#define META_HE 4u
#define META_PAR 16u
#define META_NC(m) (((m) >> 8) & 63)
#define META_H32 (1u << 16)

// state block layout (bytes from the block base)
constexpr int BLK = 64;  // envs per state block = lanes per wave
static_assert(MS_BLOCK == BLK, "the step kernel maps one wave to one state block");
constexpr int OFF_B4 = 0;
constexpr int OFF_H4 = OFF_B4 + G_BODY * BLK * 16;
constexpr int OFF_I4 = OFF_H4 + G_SNAP * BLK * 16;
constexpr int OFF_R2 = OFF_I4 + BLK * 16;
constexpr int OFF_CH = OFF_R2 + 2 * BLK * 16;
constexpr int OFF_CJ = OFF_CH + 2 * MAXA * BLK * 4;
constexpr int BLOCK_BYTES = OFF_CJ + 2 * MAXA * BLK * 16;

// Per-block counts since ms_reset_stats, summed by ms_get_stats: arbiter-cache entries read (the
// previous step's cache) and written, env-steps taken. 64-bit, so a block's counts never wrap.
struct Tally {
  unsigned long long read, written, steps, pad;
};

struct DevState {
  unsigned long long* stamps;  // MS_STAMPS diagnostic builds only: [wave][MS_NSTAMP] s_memtime
  char* blocks;                // [ceil(n / 64)] state blocks
  void* SP;  // contacts past an env's register / LDS slots (pile-ups only): [env][SPW] CSlot
  struct Tally* tally;  // [ceil(n / 64)] per-block counts since ms_reset_stats (64-bit: no wrap in a run)
  int64_t n;
};

// An env's place in the state: its block's base and its lane in the block. The step kernel
// builds it from blockIdx.x (a wave-uniform block base); the other kernels from the env index.
struct At {
  char* blk;
  int lane;
};
__device__ __forceinline__ At env_at(const DevState& S, int64_t e) {
  return At{S.blocks + (int64_t)((uint64_t)e / BLK) * BLOCK_BYTES, (int)((uint64_t)e % BLK)};
}
// element `lane` of plane p of the region at byte offset `off` (planes of BLK elements of T)
template <typename T>
__device__ __forceinline__ T* plane(At a, int off, int p) {
  return (T*)(a.blk + off + p * (BLK * (int)sizeof(T))) + a.lane;
}
// global-memory pointer type for the rare HBM reads that sit next to an LDS read of the same
// value: distinct address spaces keep the compiler from merging the two into one flat load
typedef __attribute__((address_space(1))) const uint32_t gu32_t;

struct Counters {
  unsigned long long overflow;
  unsigned long long nonfinite;
  long long first_bad;
};


#include "ms_diag.h"  // STAMP / ACC_* phase stamps (empty unless -DMS_STAMPS)

// ---- per-lane env register file ------------------------------------------------------------
struct Env {
  float px[5], py[5], vx[5], vy[5], ang[4], w[5], vbx[5], vby[5], wb[5];
  int steps, score_blue, score_red;
  uint32_t meta;
  Rng rng;
};

__device__ __forceinline__ void unpack_bodies(const float f[44], Env& E) {
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    E.px[b] = f[9 * b + 0]; E.py[b] = f[9 * b + 1]; E.vx[b] = f[9 * b + 2]; E.vy[b] = f[9 * b + 3];
    E.ang[b] = f[9 * b + 4]; E.w[b] = f[9 * b + 5];
    E.vbx[b] = f[9 * b + 6]; E.vby[b] = f[9 * b + 7]; E.wb[b] = f[9 * b + 8];
  }
  E.px[4] = f[F_BALL + 0]; E.py[4] = f[F_BALL + 1]; E.vx[4] = f[F_BALL + 2]; E.vy[4] = f[F_BALL + 3];
  E.w[4] = f[F_BALL + 4]; E.vbx[4] = f[F_BALL + 5]; E.vby[4] = f[F_BALL + 6]; E.wb[4] = f[F_BALL + 7];
}

__device__ __forceinline__ void load_bodies(At a, Env& E) {
  float f[44];
#pragma unroll
  for (int g = 0; g < G_BODY; ++g) {
    const float4 v = *plane<float4>(a, OFF_B4, g);
    f[4 * g] = v.x; f[4 * g + 1] = v.y; f[4 * g + 2] = v.z; f[4 * g + 3] = v.w;
  }
  unpack_bodies(f, E);
}

__device__ __forceinline__ void store_bodies(At a, const Env& E) {
  float f[44];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    f[9 * b + 0] = E.px[b]; f[9 * b + 1] = E.py[b]; f[9 * b + 2] = E.vx[b]; f[9 * b + 3] = E.vy[b];
    f[9 * b + 4] = E.ang[b]; f[9 * b + 5] = E.w[b];
    f[9 * b + 6] = E.vbx[b]; f[9 * b + 7] = E.vby[b]; f[9 * b + 8] = E.wb[b];
  }
  f[F_BALL + 0] = E.px[4]; f[F_BALL + 1] = E.py[4]; f[F_BALL + 2] = E.vx[4]; f[F_BALL + 3] = E.vy[4];
  f[F_BALL + 4] = E.w[4]; f[F_BALL + 5] = E.vbx[4]; f[F_BALL + 6] = E.vby[4]; f[F_BALL + 7] = E.wb[4];
#pragma unroll
  for (int g = 0; g < G_BODY; ++g) *plane<float4>(a, OFF_B4, g) = make_float4(f[4 * g], f[4 * g + 1], f[4 * g + 2], f[4 * g + 3]);
}

__device__ __forceinline__ void load_rng(At a, Env& E) {
  const ulonglong2 st = *plane<ulonglong2>(a, OFF_R2, 0), inc = *plane<ulonglong2>(a, OFF_R2, 1);
  E.rng.shi = st.x; E.rng.slo = st.y;
  E.rng.ihi = inc.x; E.rng.ilo = inc.y;
  E.rng.has32 = (E.meta & META_H32) ? 1u : 0u;
}
__device__ __forceinline__ void store_rng(At a, Env& E) {
  ulonglong2 st, inc;
  st.x = E.rng.shi; st.y = E.rng.slo;
  inc.x = E.rng.ihi; inc.y = E.rng.ilo;
  *plane<ulonglong2>(a, OFF_R2, 0) = st;
  *plane<ulonglong2>(a, OFF_R2, 1) = inc;
  E.meta = (E.meta & ~META_H32) | (E.rng.has32 ? META_H32 : 0u);
}

// ---- LDS scratchpad ------------------------------------------------------------------------
// Layouts are [field][index][lane]: the 64 lanes of a wave hit 64 distinct dwords (or 8-byte
// pairs) whatever body/box each lane selects, so dynamic per-lane indexing is conflict free.
// x/y pairs are stored together so that they load into register pairs for packed math.

constexpr int KC = 4;  // old arbiter-cache entries staged in LDS; entries KC.. are read from HBM (pile-ups)
constexpr int NLDS = 3;  // overflow contacts staged in LDS during the solver (union with the narrowphase scratch)

struct Lds {
  Seg seg[8];  // static segments (walls, goal lines), read with per-lane indices
  struct {
    V2 p[6][MS_BLOCK];             // body position (body 5 = static, all 0)
    float4 vw[6][MS_BLOCK];        // velocity x, y, angular velocity (one 12-B access per body)
    float4 bw[6][MS_BLOCK];        // bias velocity x, y, bias angular velocity
    float4 box[4][MS_BLOCK];  // agent box transform (px, py, cos, sin): one 16-B read per box
  } ph;
  float4 h1[7][MS_BLOCK];  // the t-1 snapshot (step-start state) across the physics
  union {
    struct {
      // previous step's arbiter cache, entries 0..KC-1 (loaded with the state at kernel start)
      uint32_t ch[KC][MS_BLOCK];
      float4 cj[KC][MS_BLOCK];
      // static-agent pair tests shared out over the wave: task (owner lane << 5 | pair bit)
      // and its Col result (n, p1[0]; p2[0], p1[1]; p2[1], hash[0] | count << 16, hash[1]);
      // feature hashes are 8-bit (MS_FEATURE_HASH)
      struct {
        uint32_t task[MS_BLOCK];
        float4 res[3][MS_BLOCK];
      } nt;
    } np;  // narrowphase
    // prestep, warm start, solver: contacts KREG .. KREG+NLDS-1 (pile-ups), four 16-B records
    // (r1, r2 | n, u, nMass | tMass, bias, bounce, jn | jt, jb, m, -) per lane
    float4 ov[NLDS][4][MS_BLOCK];
  } u;
};

// body velocity (v, w) and bias velocity (vb, wb) of body b in LDS
// full 16-B reads (ds_read_b128: 4 LDS cycles per wave-instruction; the 12-B ds_read_b96 the
// compiler narrows a 3-float use to takes 8)
typedef float F4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ F4 lds_f4(const float4* p) { return __builtin_nontemporal_load((const F4*)p); }
__device__ __forceinline__ void ld_v(const Lds& L, int b, int lane, V2& v, float& w) {
  const F4 q = lds_f4(&L.ph.vw[b][lane]);
  v = v2(q.x, q.y); w = q.z;
}
__device__ __forceinline__ void st_v(Lds& L, int b, int lane, V2 v, float w) {
  float* d = (float*)&L.ph.vw[b][lane];
  d[0] = v.x; d[1] = v.y; d[2] = w;
}
__device__ __forceinline__ void ld_vb(const Lds& L, int b, int lane, V2& v, float& w) {
  const F4 q = lds_f4(&L.ph.bw[b][lane]);
  v = v2(q.x, q.y); w = q.z;
}
__device__ __forceinline__ void st_vb(Lds& L, int b, int lane, V2 v, float w) {
  float* d = (float*)&L.ph.bw[b][lane];
  d[0] = v.x; d[1] = v.y; d[2] = w;
}

// Compile-time loop: every reg[] access below uses a constant index from the first IR on,
// so the slots are promoted to registers (an unrolled runtime loop is not: SROA runs first).
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ---- frames -----------------------------------------------------------------------------
__device__ __forceinline__ void frame_of(const Params& P, const Env& E, int agent, float* o) {
  switch (agent) {
    case 0: agent_frame<0>(P, E.px, E.py, E.vx, E.vy, E.ang, E.w, o); break;
    case 1: agent_frame<1>(P, E.px, E.py, E.vx, E.vy, E.ang, E.w, o); break;
    case 2: agent_frame<2>(P, E.px, E.py, E.vx, E.vy, E.ang, E.w, o); break;
    default: agent_frame<3>(P, E.px, E.py, E.vx, E.vy, E.ang, E.w, o); break;
  }
}

// Snapshot of the obs inputs (include/marl_soccer.h MS_SNAP_SIZE)
struct Snap {
  float px[5], py[5], vx[4], vy[4], ang[4], w[4];
};
__device__ __forceinline__ void snap_of(const Env& E, Snap& s) {
#pragma unroll
  for (int b = 0; b < 5; ++b) { s.px[b] = E.px[b]; s.py[b] = E.py[b]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { s.vx[i] = E.vx[i]; s.vy[i] = E.vy[i]; s.ang[i] = E.ang[i]; s.w[i] = E.w[i]; }
}
// the t-2 snapshot (H4): px[5] py[5] vx[4] vy[4] angle[4] w[4] in 7 float4 groups
__device__ __forceinline__ void snap_load(At a, Snap& s) {
  float f[28];
#pragma unroll
  for (int g = 0; g < G_SNAP; ++g) {
    const float4 v = *plane<float4>(a, OFF_H4, g);
    f[4 * g] = v.x; f[4 * g + 1] = v.y; f[4 * g + 2] = v.z; f[4 * g + 3] = v.w;
  }
#pragma unroll
  for (int b = 0; b < 5; ++b) { s.px[b] = f[b]; s.py[b] = f[5 + b]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { s.vx[i] = f[10 + i]; s.vy[i] = f[14 + i]; s.ang[i] = f[18 + i]; s.w[i] = f[22 + i]; }
}
__device__ __forceinline__ void snap_store(At a, const Snap& s) {
  float f[28];
#pragma unroll
  for (int b = 0; b < 5; ++b) { f[b] = s.px[b]; f[5 + b] = s.py[b]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[10 + i] = s.vx[i]; f[14 + i] = s.vy[i]; f[18 + i] = s.ang[i]; f[22 + i] = s.w[i]; }
  f[26] = 0.0f; f[27] = 0.0f;
#pragma unroll
  for (int g = 0; g < G_SNAP; ++g) *plane<float4>(a, OFF_H4, g) = make_float4(f[4 * g], f[4 * g + 1], f[4 * g + 2], f[4 * g + 3]);
}
__device__ __forceinline__ void obs_put(float4* d, float4 v) { *d = v; }
__device__ __forceinline__ void obs_put(float2* d, float2 v) { *d = v; }

// The six agent-agent vectors of a snapshot, computed once per pair: agent j's vector to agent
// i is the exact negation of i's to j (IEEE a-b = -(b-a), same magnitude).
template <bool FAST>
__device__ __forceinline__ void pair_vectors(const Snap& s, float aa[6][3]) {
  constexpr int PI_[6] = {0, 0, 0, 1, 1, 2}, PJ_[6] = {1, 2, 3, 2, 3, 3};
#pragma unroll
  for (int p = 0; p < 6; ++p) unit_mag<FAST>(s.px[PJ_[p]] - s.px[PI_[p]], s.py[PJ_[p]] - s.py[PI_[p]], aa[p]);
}

// Agent A's 22-float frame of a snapshot (Game._get_observations, game.py:258-322), stored as
// stacked-frame slot K (0 = t-2, 1 = t-1, 2 = t; soccer_env.py:130-140) of its 66-float row.
// A mirrored pair vector is written as 0 - u so that a zero component stays +0 as the direct
// evaluation gives.
template <bool FAST, int A, int K>
__device__ __forceinline__ void agent_frame_store(const Params& P, const Snap& s, const float aa[6][3],
                                                  float* __restrict__ row0) {
  // obs slots 4 (teammate), 7, 10 (opponents in index order) -> (pair, mirrored)
  constexpr int TEAM = A ^ 1, O1 = A < 2 ? 2 : 0, O2 = A < 2 ? 3 : 1;
  constexpr int OTH[3] = {TEAM, O1, O2};
  float f[22];
  if constexpr (FAST) {
    f[0] = obs_div(s.vx[A], P.obs_vmax);
    f[1] = obs_div(s.vy[A], P.obs_vmax);
    f[3] = obs_div(s.w[A], P.obs_wmax);
  } else {
    f[0] = s.vx[A] / P.obs_vmax;
    f[1] = s.vy[A] / P.obs_vmax;
    f[3] = s.w[A] / P.obs_wmax;
  }
  f[2] = angle_obs<FAST>(s.ang[A]);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int B = OTH[k];
    const int lo = A < B ? A : B, hi = A < B ? B : A;
    const int p = lo == 0 ? hi - 1 : (lo == 1 ? hi + 1 : 5);
    if (A < B) {
      f[4 + 3 * k] = aa[p][0]; f[5 + 3 * k] = aa[p][1];
    } else {
      f[4 + 3 * k] = 0.0f - aa[p][0]; f[5 + 3 * k] = 0.0f - aa[p][1];
    }
    f[6 + 3 * k] = aa[p][2];
  }
  unit_mag<FAST>(s.px[4] - s.px[A], s.py[4] - s.py[A], f + 13);
  const float own_x = A < 2 ? 10.0f : 790.0f, opp_x = A < 2 ? 790.0f : 10.0f;
  unit_mag<FAST>(own_x - s.px[A], 300.0f - s.py[A], f + 16);
  unit_mag<FAST>(opp_x - s.px[A], 300.0f - s.py[A], f + 19);
  float* d = row0 + A * 66 + K * 22;
  if constexpr (((A + K) & 1) == 0) {  // 16-B aligned: five 16-B stores and one 8-B store
#pragma unroll
    for (int q = 0; q < 5; ++q) obs_put((float4*)(d + 4 * q), make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]));
    obs_put((float2*)(d + 20), make_float2(f[20], f[21]));
  } else {  // starts half-way into a 16-B word: the 8-B store first
    obs_put((float2*)d, make_float2(f[0], f[1]));
#pragma unroll
    for (int q = 0; q < 5; ++q)
      obs_put((float4*)(d + 2 + 4 * q), make_float4(f[2 + 4 * q], f[3 + 4 * q], f[4 + 4 * q], f[5 + 4 * q]));
  }
}

// The four agents' frames of one snapshot, stored as slot K of every agent's row.
template <bool FAST, int K>
__device__ __forceinline__ void emit_snapshot_impl(const Params& P, const Snap& s, float* __restrict__ row0) {
  float aa[6][3];
  pair_vectors<FAST>(s, aa);
  static_for<0, 4>([&](auto ac) __attribute__((always_inline)) {
    agent_frame_store<FAST, decltype(ac)::value, K>(P, s, aa, row0);
  });
}

// Operands of a snapshot's frames inside the domains of div_nr / sqrt_nr (ms_device.h):
// positions 0 or 2^-70..2^28 (so every difference is 0 or 2^-93..2^29), velocities, spins and
// angles 0 or 2^-100..2^30. Two max/min reductions over the raw magnitudes (0 maps to ~0u).
__device__ __forceinline__ bool frame_inputs_in_range(const Params& P, const Snap& s) {
  uint32_t pmax = 0u, pmin = ~0u, vmax = 0u, vmin = ~0u;
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    const uint32_t x = __float_as_uint(s.px[b]) & 0x7fffffffu, y = __float_as_uint(s.py[b]) & 0x7fffffffu;
    pmax = max(pmax, max(x, y));
    pmin = min(pmin, min(x - 1u, y - 1u));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t a = __float_as_uint(s.vx[i]) & 0x7fffffffu, b = __float_as_uint(s.vy[i]) & 0x7fffffffu;
    const uint32_t c = __float_as_uint(s.w[i]) & 0x7fffffffu, d = __float_as_uint(s.ang[i]) & 0x7fffffffu;
    vmax = max(vmax, max(max(a, b), max(c, d)));
    vmin = min(vmin, min(min(a - 1u, b - 1u), min(c - 1u, d - 1u)));
  }
  return P.fast_div && pmax <= 0x4D800000u && pmin >= 0x1C800000u - 1u && vmax <= 0x4E800000u &&
         vmin >= 0x0D800000u - 1u;
}

template <int K>
__device__ __forceinline__ void emit_snapshot(const Params& P, const Snap& s, float* __restrict__ row0) {
  if (frame_inputs_in_range(P, s)) emit_snapshot_impl<true, K>(P, s, row0);
  else emit_snapshot_impl<false, K>(P, s, row0);
}

// Frames t-2, t-1, t of every agent. Agent-major order finishes each 264-B row segment of an
// agent in one burst of stores. Every lane runs the reduced-range arithmetic as one straight
// path; a lane whose operands fall outside its domain (never in play: velocities or spins below
// 2^-100, a non-default vmax outside div_nr's divisor domain) then rewrites its whole row by
// the IEEE path — same bytes as an if/else per lane, 1.6 us less per launch at 65,536 envs
// than the if/else (the divergent branch around the hot path cost more than the
// range test).
__device__ __forceinline__ void emit_three(const Params& P, const Snap& s2, const Snap& s1, const Snap& s0,
                                           float* __restrict__ row0) {
  const bool fast = frame_inputs_in_range(P, s2) && frame_inputs_in_range(P, s1) && frame_inputs_in_range(P, s0);
  {
    float a2[6][3], a1[6][3], a0[6][3];
    pair_vectors<true>(s2, a2);
    pair_vectors<true>(s1, a1);
    pair_vectors<true>(s0, a0);
    static_for<0, 4>([&](auto ac) __attribute__((always_inline)) {
      constexpr int A = decltype(ac)::value;
      agent_frame_store<true, A, 0>(P, s2, a2, row0);
      agent_frame_store<true, A, 1>(P, s1, a1, row0);
      agent_frame_store<true, A, 2>(P, s0, a0, row0);
    });
  }
  if (!fast) {  // same lane, same addresses: these stores land after the ones above
    emit_snapshot_impl<false, 0>(P, s2, row0);
    emit_snapshot_impl<false, 1>(P, s1, row0);
    emit_snapshot_impl<false, 2>(P, s0, row0);
  }
}

// Frames of a reset (soccer_env.py:90-96): all three stacked frames are the current one, and
// the history slot (t-2 for the next step) is the current snapshot too.
__device__ __forceinline__ void snap_to_lds(float4 (*dst)[MS_BLOCK], int lane, const Snap& s) {
  float f[28];
#pragma unroll
  for (int b = 0; b < 5; ++b) { f[b] = s.px[b]; f[5 + b] = s.py[b]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[10 + i] = s.vx[i]; f[14 + i] = s.vy[i]; f[18 + i] = s.ang[i]; f[22 + i] = s.w[i]; }
  f[26] = 0.0f; f[27] = 0.0f;
#pragma unroll
  for (int g = 0; g < 7; ++g) dst[g][lane] = make_float4(f[4 * g], f[4 * g + 1], f[4 * g + 2], f[4 * g + 3]);
}
__device__ __forceinline__ void snap_from_lds(const float4 (*src)[MS_BLOCK], int lane, Snap& s) {
  float f[28];
#pragma unroll
  for (int g = 0; g < 7; ++g) {
    const float4 v = src[g][lane];
    f[4 * g] = v.x; f[4 * g + 1] = v.y; f[4 * g + 2] = v.z; f[4 * g + 3] = v.w;
  }
#pragma unroll
  for (int b = 0; b < 5; ++b) { s.px[b] = f[b]; s.py[b] = f[5 + b]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { s.vx[i] = f[10 + i]; s.vy[i] = f[14 + i]; s.ang[i] = f[18 + i]; s.w[i] = f[22 + i]; }
}

__device__ __forceinline__ void emit_fill3(At a, const Params& P, int64_t e, const Snap& s0,
                                           float* __restrict__ obs) {
  if (obs) {
    float* dst = obs + e * 264;
    emit_snapshot<0>(P, s0, dst);
    emit_snapshot<1>(P, s0, dst);
    emit_snapshot<2>(P, s0, dst);
  }
  snap_store(a, s0);
}

// ---- frame-ring observations (ms_step_ring) -------------------------------------------------
// The stacked observation as a window of three consecutive frames of a per-env, per-agent ring
// of R 22-float frames: row [env][agent] holds R frames, the step's obs is frames pos..pos+2
// (t-2, t-1, t), which the caller views as an (N, 4, 66) tensor with a row stride of R*22
// floats. A step writes frame t only (at pos+2); frames t-2 and t-1 are the previous steps'
// frames t, already in place. When the window wraps to the start of the ring (pos = 0) the step
// writes all three (t-2 and t-1 from their snapshots), and a refilled stack (reset, auto-reset)
// writes frame t three times, as the contiguous layout does.
struct Ring {
  float* frames;
  int R;     // frames per ring row (even: every frame slot of an even index is 16-B aligned)
  int pos;   // ring slot of frame t-2 in this step's window
  int wrap;  // 1: frames t-2, t-1 are written too
};

// agent_frame_store with the destination and its 16-B alignment (`al`) as runtime values. The
// arithmetic is agent_frame_store's, restated rather than shared on purpose: factoring the two
// through one helper changes the register allocation of ms_step_kernel (its ISA is otherwise
// instruction-for-instruction what it was before the ring existed; checked with --cuda-device-only -S).
template <bool FAST, int A>
__device__ __forceinline__ void frame_store_at(const Params& P, const Snap& s, const float aa[6][3],
                                               float* __restrict__ d, bool al) {
  // obs slots 4 (teammate), 7, 10 (opponents in index order) -> (pair, mirrored)
  constexpr int TEAM = A ^ 1, O1 = A < 2 ? 2 : 0, O2 = A < 2 ? 3 : 1;
  constexpr int OTH[3] = {TEAM, O1, O2};
  float f[22];
  if constexpr (FAST) {
    f[0] = obs_div(s.vx[A], P.obs_vmax);
    f[1] = obs_div(s.vy[A], P.obs_vmax);
    f[3] = obs_div(s.w[A], P.obs_wmax);
  } else {
    f[0] = s.vx[A] / P.obs_vmax;
    f[1] = s.vy[A] / P.obs_vmax;
    f[3] = s.w[A] / P.obs_wmax;
  }
  f[2] = angle_obs<FAST>(s.ang[A]);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int B = OTH[k];
    const int lo = A < B ? A : B, hi = A < B ? B : A;
    const int p = lo == 0 ? hi - 1 : (lo == 1 ? hi + 1 : 5);
    if (A < B) {
      f[4 + 3 * k] = aa[p][0]; f[5 + 3 * k] = aa[p][1];
    } else {
      f[4 + 3 * k] = 0.0f - aa[p][0]; f[5 + 3 * k] = 0.0f - aa[p][1];
    }
    f[6 + 3 * k] = aa[p][2];
  }
  unit_mag<FAST>(s.px[4] - s.px[A], s.py[4] - s.py[A], f + 13);
  const float own_x = A < 2 ? 10.0f : 790.0f, opp_x = A < 2 ? 790.0f : 10.0f;
  unit_mag<FAST>(own_x - s.px[A], 300.0f - s.py[A], f + 16);
  unit_mag<FAST>(opp_x - s.px[A], 300.0f - s.py[A], f + 19);
  if (al) {  // 16-B aligned: five 16-B stores and one 8-B store
#pragma unroll
    for (int q = 0; q < 5; ++q) obs_put((float4*)(d + 4 * q), make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]));
    obs_put((float2*)(d + 20), make_float2(f[20], f[21]));
  } else {  // starts half-way into a 16-B word: the 8-B store first
    obs_put((float2*)d, make_float2(f[0], f[1]));
#pragma unroll
    for (int q = 0; q < 5; ++q)
      obs_put((float4*)(d + 2 + 4 * q), make_float4(f[2 + 4 * q], f[3 + 4 * q], f[4 + 4 * q], f[5 + 4 * q]));
  }
}

// The four agents' frames of snapshot s at ring slot `slot` of the env's rows; AL: slot is even
// (16-B aligned). The alignment is a template argument so every frame is stored as 16-B and 8-B
// vector stores: with a runtime alignment the two store sequences are merged at 4-B alignment
// and split into single dwords.
template <bool AL>
__device__ __forceinline__ void ring_emit(const Params& P, const Snap& s, float* __restrict__ row, int R, int slot) {
  float* d0 = row + slot * 22;
  const bool fast = frame_inputs_in_range(P, s);
  {  // every lane: the reduced-range path; out-of-domain lanes rewrite by the IEEE path (emit_three)
    float aa[6][3];
    pair_vectors<true>(s, aa);
    static_for<0, 4>([&](auto ac) __attribute__((always_inline)) {
      constexpr int A = decltype(ac)::value;
      frame_store_at<true, A>(P, s, aa, d0 + A * R * 22, AL);
    });
  }
  if (!fast) {
    float aa[6][3];
    pair_vectors<false>(s, aa);
    static_for<0, 4>([&](auto ac) __attribute__((always_inline)) {
      constexpr int A = decltype(ac)::value;
      frame_store_at<false, A>(P, s, aa, d0 + A * R * 22, AL);
    });
  }
}

__device__ __forceinline__ void snap_select(bool c, const Snap& a, const Snap& b, Snap& o) {
#pragma unroll
  for (int q = 0; q < 5; ++q) { o.px[q] = c ? a.px[q] : b.px[q]; o.py[q] = c ? a.py[q] : b.py[q]; }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o.vx[q] = c ? a.vx[q] : b.vx[q]; o.vy[q] = c ? a.vy[q] : b.vy[q];
    o.ang[q] = c ? a.ang[q] : b.ang[q]; o.w[q] = c ? a.w[q] : b.w[q];
  }
}

// The frames a step writes into its window pos..pos+2: frame t (s0) at pos+2 always; with
// `refill` (reset, auto-reset) s0 at pos and pos+1 too, else on a wrap t-2 (h2) and t-1 (h1).
// One loop over the slots keeps a single copy of the frame code per alignment.
__device__ __forceinline__ void ring_emit_window(const Params& P, const Snap& h2, const Snap& h1, const Snap& s0,
                                                 bool refill, float* __restrict__ row, const Ring& rg) {
  const int k0 = (refill || rg.wrap) ? 0 : 2;
#pragma unroll 1
  for (int k = k0; k < 3; ++k) {
    Snap s;
    snap_select(k == 2 || refill, s0, k == 0 ? h2 : h1, s);
    const int slot = rg.pos + k;
    if (slot & 1) ring_emit<false>(P, s, row, rg.R, slot);
    else ring_emit<true>(P, s, row, rg.R, slot);
  }
}

// Game.reset (game.py:76-118): fresh bodies, score/steps 0, arbiters dropped, spawn.
__device__ __forceinline__ void reset_env_regs(Env& E, int mode) {
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    E.vx[b] = 0.0f; E.vy[b] = 0.0f; E.w[b] = 0.0f;
    E.vbx[b] = 0.0f; E.vby[b] = 0.0f; E.wb[b] = 0.0f;
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) E.ang[b] = b < 2 ? 0.0f : 3.14159265358979323846f;
  E.steps = 0; E.score_blue = 0; E.score_red = 0;
  E.meta = (E.meta & (META_H32 | META_PAR)) | (uint32_t)(mode & 3);  // n_cache = 0
  spawn_positions(E.rng, mode, E.px, E.py);
}

// Goal soft reset (Game._reset_positions, game.py:120-127): bias velocities, ball spin and
// the arbiter cache survive.
__device__ __forceinline__ void soft_reset_regs(Env& E) {
  spawn_positions(E.rng, META_MODE(E.meta), E.px, E.py);
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    E.vx[b] = 0.0f; E.vy[b] = 0.0f; E.w[b] = 0.0f;
    E.ang[b] = b < 2 ? 0.0f : 3.14159265358979323846f;
  }
  E.vx[4] = 0.0f; E.vy[4] = 0.0f;
}

// copy the segment table from the kernel arguments with constant indices (a per-lane index
// into the by-value Params would make the compiler copy all of Params to scratch)
__device__ __forceinline__ void stage_segments(const Params& P, Lds& L, int lane) {
  // field by field: a whole-struct copy becomes a memcpy out of a private copy of Params
  // (scratch stores in every lane)
  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      L.seg[s].ax = P.seg[s].ax; L.seg[s].ay = P.seg[s].ay; L.seg[s].bx = P.seg[s].bx; L.seg[s].by = P.seg[s].by;
      L.seg[s].nx = P.seg[s].nx; L.seg[s].ny = P.seg[s].ny; L.seg[s].r = P.seg[s].r;
#pragma unroll
      for (int k = 0; k < 4; ++k) L.seg[s].bb[k] = P.seg[s].bb[k];
    }
  }
  __syncthreads();
}

// ---- physics: cpSpaceStep restated ---------------------------------------------------------
// One contact of the per-step arbiter list (cpArbiter + cpContact fields the solver uses).
struct CSlot {
  V2 r1, r2, n;
  float u, nMass, tMass, bias, bounce, jn, jt, jb;
  uint32_t m;  // ba 0-2 | bb 3-5 | warm 6 | cidx 7 | count 8-9 | hash 10-17 | cache pos 18-23 | pair 24-29
};
#define CS_BA(m) ((int)((m) & 7u))
#define CS_BB(m) ((int)(((m) >> 3) & 7u))
#define CS_WARM(m) (((m) >> 6) & 1u)
#define CS_CIDX(m) (((m) >> 7) & 1u)
#define CS_COUNT(m) (((m) >> 8) & 3u)
#define CS_HASH(m) (((m) >> 10) & 0xffu)
#define CS_POS(m) ((int)(((m) >> 18) & 63u))
#define CS_PAIR(m) ((int)(((m) >> 24) & 63u))

constexpr int KREG = 8;  // contacts held in registers; further ones go to the global spill (pile-ups)
constexpr int PRE_GROUP = 2;  // register slots per wave-uniform prestep group (2: 53.3 us, 4: 53.7, 8: 54.3, per-lane: 53.9)
static_assert(KREG % PRE_GROUP == 0, "prestep groups must cover every register slot");
#define MAXC (2 * MAXA)                 // contact capacity (2 per arbiter)
// contact-spill slots per env (S.SP): the per-lane kernel spills contacts KREG.., the lane-pair
// kernel contacts pr::KP.. (4-6), the lane-group kernel contacts grp::GCAP..
constexpr int SPW = MAXC - 4;

__device__ __forceinline__ void cache_write(At a, int par, int k, uint32_t hdr, float4 j) {
  *plane<uint32_t>(a, OFF_CH, par * MAXA + k) = hdr;
  *plane<float4>(a, OFF_CJ, par * MAXA + k) = j;
}

// Per-lane working set of the contact pipeline.
struct Contacts {
  CSlot reg[KREG];
  int nc, na;
};

// d = c ? s : d, field by field with unconditional stores: a conditional whole-struct store
// lets the optimizer merge the KREG stores into one store through a phi of slot pointers,
// which pins the slots in scratch memory. Only the fields the narrowphase defines (bias holds
// the separation (p2 - p1) . n until prestep_one turns it into the bias velocity): u, nMass,
// tMass, bounce and jb are written by prestep_one before anything reads them.
__device__ __forceinline__ void slot_select(CSlot& d, const CSlot& s, bool c) {
  d.r1 = c ? s.r1 : d.r1; d.r2 = c ? s.r2 : d.r2; d.n = c ? s.n : d.n; d.bias = c ? s.bias : d.bias;
  d.jn = c ? s.jn : d.jn; d.jt = c ? s.jt : d.jt; d.m = c ? s.m : d.m;
}

// overflow slots KREG..MAXC-1 live in the global spill buffer; only pile-ups reach them
__device__ __forceinline__ void slot_put(Contacts& C, CSlot* ovf, int k, const CSlot& s) {
  static_for<0, KREG>([&](auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    slot_select(C.reg[q], s, q == k);
  });
  if (k >= KREG) ovf[k - KREG] = s;
}

// overflow contact KREG + j staged in LDS (Lds::u.ov) for prestep, warm start and solver
__device__ __forceinline__ void ov_get(const Lds& L, int j, int lane, CSlot& c) {
  const F4 q0 = lds_f4(&L.u.ov[j][0][lane]), q1 = lds_f4(&L.u.ov[j][1][lane]);
  const F4 q2 = lds_f4(&L.u.ov[j][2][lane]), q3 = lds_f4(&L.u.ov[j][3][lane]);
  c.r1 = v2(q0.x, q0.y); c.r2 = v2(q0.z, q0.w); c.n = v2(q1.x, q1.y); c.u = q1.z; c.nMass = q1.w;
  c.tMass = q2.x; c.bias = q2.y; c.bounce = q2.z; c.jn = q2.w;
  c.jt = q3.x; c.jb = q3.y; c.m = __float_as_uint(q3.z);
}
__device__ __forceinline__ void ov_put(Lds& L, int j, int lane, const CSlot& c) {
  L.u.ov[j][0][lane] = make_float4(c.r1.x, c.r1.y, c.r2.x, c.r2.y);
  L.u.ov[j][1][lane] = make_float4(c.n.x, c.n.y, c.u, c.nMass);
  L.u.ov[j][2][lane] = make_float4(c.tMass, c.bias, c.bounce, c.jn);
  L.u.ov[j][3][lane] = make_float4(c.jt, c.jb, __uint_as_float(c.m), 0.0f);
}
// contact k >= KREG after the solver: from LDS or from the global spill
__device__ __forceinline__ CSlot over_slot(const Lds& L, int lane, const CSlot* ovf, int k) {
  CSlot c;
  if (k < KREG + NLDS) ov_get(L, k - KREG, lane, c);
  else c = ovf[k - KREG];
  return c;
}

// per-body inverse mass / moment without a per-lane indexed parameter load
__device__ __forceinline__ float body_minv(const Params& P, int b) {
  return b < 4 ? P.m_inv[0] : (b == 4 ? P.m_inv[4] : 0.0f);
}
__device__ __forceinline__ float body_iinv(const Params& P, int b) {
  return b < 4 ? P.i_inv[0] : (b == 4 ? P.i_inv[4] : 0.0f);
}
// shape b of an arbiter is never the ball (the ball is shape a of its agent pairs and of its
// wall pairs, DESIGN.md pair table): an agent or the static body
__device__ __forceinline__ float body_b_minv(const Params& P, int b) { return b < 4 ? P.m_inv[0] : 0.0f; }
__device__ __forceinline__ float body_b_iinv(const Params& P, int b) { return b < 4 ? P.i_inv[0] : 0.0f; }

// Body velocity records of the contact solve: the step kernel's per-lane LDS layout (LaneBodies)
// or one env's records of the lane-group kernel (ms_group.inc). The contact arithmetic below is
// shared, so both kernels compute every impulse with the same operations in the same order.
struct LaneBodies {
  Lds& L;
  int lane;
  __device__ __forceinline__ void ld_v(int b, V2& v, float& w) const { ::ld_v(L, b, lane, v, w); }
  __device__ __forceinline__ void st_v(int b, V2 v, float w) const { ::st_v(L, b, lane, v, w); }
  __device__ __forceinline__ void ld_vb(int b, V2& v, float& w) const { ::ld_vb(L, b, lane, v, w); }
  __device__ __forceinline__ void st_vb(int b, V2 v, float w) const { ::st_vb(L, b, lane, v, w); }
};

// cpArbiterPreStep for one contact (velocities: previous step's post-solve values)
template <class BR>
__device__ __forceinline__ void prestep_t(const Params& P, CSlot& c, const BR& B) {
  const int ba = CS_BA(c.m), bb = CS_BB(c.m);
  const float ma = body_minv(P, ba), ia = body_iinv(P, ba), mb = body_b_minv(P, bb), ib = body_b_iinv(P, bb);
  const int p = CS_PAIR(c.m);
  const float e_s = ((p - 10) & 7) < 6 ? P.e_aw : P.e_ag;
  const float e = p < 6 ? P.e_aa : (p < 10 ? P.e_ab : (p < 42 ? e_s : P.e_bw));
  const float u_s = ((p - 10) & 7) < 6 ? P.u_aw : P.u_ag;
  c.u = p < 6 ? P.u_aa : (p < 10 ? P.u_ab : (p < 42 ? u_s : P.u_bw));
  const V2 n = c.n;
  V2 va, vb;
  float wa, wbv;
  B.ld_v(ba, va, wa);
  B.ld_v(bb, vb, wbv);
  const V2 r1 = c.r1, r2 = c.r2;
  const float rcn1 = vcross(r1, n), rcn2 = vcross(r2, n);
  c.nMass = 1.0f / ((ma + ia * rcn1 * rcn1) + (mb + ib * rcn2 * rcn2));
  const V2 t = vperp(n);
  const float rct1 = vcross(r1, t), rct2 = vcross(r2, t);
  c.tMass = 1.0f / ((ma + ia * rct1 * rct1) + (mb + ib * rct2 * rct2));
  const float dist = c.bias;  // (p2 - p1) . n from the narrowphase frame (add_arbiter)
  c.bias = -P.bias_coef * fminr(0.0f, dist + P.slop) / P.dt;
  c.jb = 0.0f;
  const V2 v1 = vadd(va, vmult(vperp(r1), wa));
  const V2 v2s = vadd(vb, vmult(vperp(r2), wbv));
  c.bounce = vdot(vsub(v2s, v1), n) * e;
}
__device__ __forceinline__ void prestep_one(const Params& P, CSlot& c, const Lds& L, int lane) {
  prestep_t(P, c, LaneBodies{const_cast<Lds&>(L), lane});
}

// cpArbiterApplyCachedImpulse for one contact (dt_coef = 1)
template <class BR>
__device__ __forceinline__ void warm_t(const Params& P, const CSlot& c, const BR& B) {
  if (!CS_WARM(c.m)) return;
  const int ba = CS_BA(c.m), bb = CS_BB(c.m);
  const float ma = body_minv(P, ba), ia = body_iinv(P, ba), mb = body_b_minv(P, bb), ib = body_b_iinv(P, bb);
  const V2 j = vrotate(c.n, v2(c.jn, c.jt));
  const V2 nj = vneg(j);
  V2 va, vb;
  float wa, wbv;
  B.ld_v(ba, va, wa);
  B.st_v(ba, vmadd(nj, ma, va), __builtin_fmaf(ia, vcross(c.r1, nj), wa));
  B.ld_v(bb, vb, wbv);
  B.st_v(bb, vmadd(j, mb, vb), __builtin_fmaf(ib, vcross(c.r2, j), wbv));
}
__device__ __forceinline__ void warm_one(const Params& P, const CSlot& c, Lds& L, int lane) {
  warm_t(P, c, LaneBodies{L, lane});
}

// cpArbiterApplyImpulse for one contact, with its bodies' inverse masses and moments given
template <class BR>
__device__ __forceinline__ void solve_m(CSlot& c, const BR& B, float ma, float ia, float mb, float ib) {
  const int ba = CS_BA(c.m), bb = CS_BB(c.m);
  const V2 n = c.n;
  const V2 r1 = c.r1, r2 = c.r2;
  V2 vba, vbb, va, vb;
  float wba, wbb, wa, wb_;
  B.ld_vb(ba, vba, wba);
  B.ld_vb(bb, vbb, wbb);
  B.ld_v(ba, va, wa);
  B.ld_v(bb, vb, wb_);
  const V2 vb1 = vmadd(vperp(r1), wba, vba);
  const V2 vb2 = vmadd(vperp(r2), wbb, vbb);
  const V2 vs1 = vmadd(vperp(r1), wa, va);
  const V2 vs2 = vmadd(vperp(r2), wb_, vb);
  const V2 vr = vsub(vs2, vs1);
  const float vbn = vdot(vsub(vb2, vb1), n);
  const float vrn = vdot(vr, n);
  const float vrt = vdot(vr, vperp(n));

  const float jbn = (c.bias - vbn) * c.nMass;
  const float jbnOld = c.jb;
  c.jb = fmaxr(jbnOld + jbn, 0.0f);

  const float jn = -(c.bounce + vrn) * c.nMass;
  const float jnOld = c.jn;
  c.jn = fmaxr(jnOld + jn, 0.0f);

  const float jtMax = c.u * c.jn;
  const float jt = -vrt * c.tMass;
  const float jtOld = c.jt;
  c.jt = fclamp_sym(jtOld + jt, jtMax);

  const V2 jbv = vmult(n, c.jb - jbnOld);
  const V2 njb = vneg(jbv);
  const V2 j = vrotate(n, v2(c.jn - jnOld, c.jt - jtOld));
  const V2 nj = vneg(j);
  // body a first, then body b (apply_bias_impulses then apply_impulses, cpArbiter.c);
  // a and b are distinct bodies, so the four updates commute per body.
  B.st_vb(ba, vmadd(njb, ma, vba), __builtin_fmaf(ia, vcross(r1, njb), wba));
  B.st_vb(bb, vmadd(jbv, mb, vbb), __builtin_fmaf(ib, vcross(r2, jbv), wbb));
  B.st_v(ba, vmadd(nj, ma, va), __builtin_fmaf(ia, vcross(r1, nj), wa));
  B.st_v(bb, vmadd(j, mb, vb), __builtin_fmaf(ib, vcross(r2, j), wb_));
}
template <class BR>
__device__ __forceinline__ void solve_t(const Params& P, CSlot& c, const BR& B) {
  const int ba = CS_BA(c.m), bb = CS_BB(c.m);
  solve_m(c, B, body_minv(P, ba), body_iinv(P, ba), body_b_minv(P, bb), body_b_iinv(P, bb));
}
__device__ __forceinline__ void solve_one(const Params& P, CSlot& c, Lds& L, int lane) {
  solve_t(P, c, LaneBodies{L, lane});
}

// Cross-lane hand-off through LDS inside one wave: every lane's LDS writes before it are
// visible to every lane's LDS reads after it. A wave's LDS instructions execute in order, so no
// wait is needed; the fences (wavefront scope) and the wave barrier keep the compiler and the
// machine scheduler from moving LDS accesses across the hand-off, whatever the scheduling
// strategy ("Faults").
__device__ __forceinline__ void wave_lds_handoff() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// number of set bits of m below this lane
__device__ __forceinline__ int lane_rank(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}


// Old-cache cursor: the previous step's arbiter cache (sorted by pair id) is streamed once,
// merged with this step's touched arbiters into the other (ping-pong) buffer. Entries below KC
// come from LDS (staged at kernel start), the rest from HBM. The cursor decisions (pair id and
// idle count of the entry under it) come from one key byte per entry packed into two registers
// at the load, so advancing the cursor never waits for an LDS read; the full header and the
// impulses are read only for an entry that is aged or matched.
struct CacheWalk {
  int par, nc_old, cur, out;
  uint32_t pk;  // key bytes (pair | idle << 6) of entries 0..KC-1
};
__device__ __forceinline__ uint32_t cache_key(uint32_t hdr) { return (hdr & 63u) | (((hdr >> 8) & 3u) << 6); }

// (the HBM fallback reads through address-space-1 pointers: with generic pointers the optimizer
// merges the LDS and the global read into one flat-address load through a selected address)
__device__ __forceinline__ uint32_t old_hdr(At a, const Lds& L, int par, int k) {
  if (k < KC) return L.u.np.ch[k][a.lane];
  return __builtin_nontemporal_load((gu32_t*)plane<uint32_t>(a, OFF_CH, par * MAXA + k));
}
__device__ __forceinline__ float4 old_imp(At a, const Lds& L, int par, int k) {
  if (k < KC) return L.u.np.cj[k][a.lane];
  gu32_t* g = (gu32_t*)plane<float4>(a, OFF_CJ, par * MAXA + k);
  return make_float4(__uint_as_float(__builtin_nontemporal_load(g)), __uint_as_float(__builtin_nontemporal_load(g + 1)),
                     __uint_as_float(__builtin_nontemporal_load(g + 2)), __uint_as_float(__builtin_nontemporal_load(g + 3)));
}

// key byte of the entry under the cursor (cur < nc_old)
__device__ __forceinline__ uint32_t cur_key(At a, const CacheWalk& W) {
  if (W.cur < KC) return (W.pk >> (8 * W.cur)) & 0xffu;
  return cache_key(__builtin_nontemporal_load((gu32_t*)plane<uint32_t>(a, OFF_CH, W.par * MAXA + W.cur)));
}
// pair id under the cursor, 64 past the end of the old cache
__device__ __forceinline__ int cur_pair(At a, const CacheWalk& W) {
  return W.cur < W.nc_old ? (int)(cur_key(a, W) & 63u) : 64;
}

// emit the old entry under the cursor aged by one step (dropped at idle 3, cpSpaceArbiterSetFilter)
__device__ __forceinline__ void cache_age_current(At a, const Lds& L, CacheWalk& W, unsigned long long* overflow_acc) {
  const uint32_t idle = (cur_key(a, W) >> 6) + 1u;
  if (idle < 3u) {
    if (W.out < MAXA) {
      const uint32_t h = old_hdr(a, L, W.par, W.cur);
      cache_write(a, W.par ^ 1, W.out, (h & ~(3u << 8)) | (idle << 8), old_imp(a, L, W.par, W.cur));
      ++W.out;
    } else {
      (*overflow_acc)++;
    }
  }
  ++W.cur;
}

// cpSpaceCollideShapes + cpArbiterUpdate for one touching pair. The collision `col` is in the
// pair's narrowphase frame, in which bodies a and b sit at oa and ob (one of them the origin,
// exactly 0): lever arms r1 = p1 - oa, r2 = p2 - ob and the separation
// (p2 - p1) . n never pass through world coordinates.
__device__ __forceinline__ void add_arbiter(At a, const Lds& L, Contacts& C, CSlot* ovf, CacheWalk& W, int p, int ba,
                                            int bb, const Col& col, V2 oa, V2 ob, unsigned long long* overflow_acc) {
  if (C.na >= MAXA) { (*overflow_acc)++; return; }
  while (cur_pair(a, W) < p) cache_age_current(a, L, W, overflow_acc);
  const bool found = cur_pair(a, W) == p;
  uint32_t oh = 0u;
  float oj[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (found) {
    oh = old_hdr(a, L, W.par, W.cur);
    const float4 j = old_imp(a, L, W.par, W.cur);
    oj[0] = j.x; oj[1] = j.y; oj[2] = j.z; oj[3] = j.w;
    ++W.cur;
  }
  int pos = W.out;
  if (W.out < MAXA) ++W.out; else { (*overflow_acc)++; pos = 63; }
  C.na++;
  const uint32_t warm = (found && ((oh >> 8) & 3u) == 0u) ? 1u : 0u;
  // the old arbiter's contact hashes (cpArbiterUpdate matches contacts by feature hash; a later
  // old contact wins, as in the loop over the old contact list)
  const int ocount = found ? (int)((oh >> 6) & 3u) : 0;
  const int oh0 = (int)((oh >> 16) & 0xffu), oh1 = (int)((oh >> 24) & 0xffu);
  // the one or two contacts of the collision, unrolled (no loop control in the hot path)
  static_for<0, 2>([&](auto kc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value;
    if (k == 0 || col.count > 1) {
      CSlot s;
      const int h = col.hash[k];
      s.r1 = vsub(col.p1[k], oa);
      s.r2 = vsub(col.p2[k], ob);
      s.n = col.n;
      s.bias = vdot(vsub(col.p2[k], col.p1[k]), col.n);
      float jn = 0.0f, jt = 0.0f;
      if (ocount > 0 && oh0 == h) { jn = oj[0]; jt = oj[1]; }
      if (ocount > 1 && oh1 == h) { jn = oj[2]; jt = oj[3]; }
      s.jn = jn; s.jt = jt;
      s.m = (uint32_t)ba | ((uint32_t)bb << 3) | (warm << 6) | ((uint32_t)k << 7) | ((uint32_t)col.count << 8) |
            ((uint32_t)(h & 0xff) << 10) | ((uint32_t)pos << 18) | ((uint32_t)p << 24);
      slot_put(C, ovf, C.nc + k, s);
    }
  });
  C.nc += col.count;
}

// cache entry of a touched arbiter from its first contact c0 (and c1 when it has two)
__device__ __forceinline__ void write_arbiter_cache(At a, int npar, const CSlot& c0, const CSlot& c1) {
  if (CS_CIDX(c0.m) != 0 || CS_POS(c0.m) >= MAXA) return;
  const bool two = CS_COUNT(c0.m) > 1;
  const uint32_t hdr = (uint32_t)CS_PAIR(c0.m) | (CS_COUNT(c0.m) << 6) | (CS_HASH(c0.m) << 16) |
                       ((two ? CS_HASH(c1.m) : 0u) << 24);
  cache_write(a, npar, CS_POS(c0.m), hdr, make_float4(c0.jn, c0.jt, two ? c1.jn : 0.0f, two ? c1.jt : 0.0f));
}

#define FOR_CONTACTS(C, OVF, BODY)                                    \
  {                                                                   \
    static_for<0, KREG>([&](auto kc_) __attribute__((always_inline)) {                             \
      constexpr int k_ = decltype(kc_)::value;                        \
      if (k_ < (C).nc) {                                              \
        CSlot& c_ = (C).reg[k_];                                      \
        BODY;                                                         \
      }                                                               \
    });                                                               \
    for (int k_ = KREG; k_ < (C).nc; ++k_) {                          \
      if (k_ < KREG + NLDS) {                                         \
        CSlot c_;                                                     \
        ov_get(L, k_ - KREG, lane, c_);                               \
        BODY;                                                         \
        ov_put(L, k_ - KREG, lane, c_);                               \
      } else {                                                        \
        CSlot& c_ = (OVF)[k_ - KREG];                                 \
        BODY;                                                         \
      }                                                               \
    }                                                                 \
  }

__device__ __forceinline__ void physics_step(const DevState& S, At a, int64_t e, const Params& P, Env& E, float fx[4],
                                             float fy[4], float tq[4], Lds& L, unsigned long long* overflow_acc,
                                             Snap& h2, uint32_t pk0, bool need_h2) {
  const int lane = a.lane;
  const float dt = P.dt;
#ifdef MS_STAMPS
  const int64_t stamp_row = (a.blk - S.blocks) / BLOCK_BYTES;  // the state block (STAMP's row)
#endif
  // cpBodyUpdatePosition
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    E.px[b] = E.px[b] + (E.vx[b] + E.vbx[b]) * dt;
    E.py[b] = E.py[b] + (E.vy[b] + E.vby[b]) * dt;
    if (b < 4) E.ang[b] = E.ang[b] + (E.w[b] + E.wb[b]) * dt;
    E.vbx[b] = 0.0f; E.vby[b] = 0.0f; E.wb[b] = 0.0f;
  }
  // shape caches; agents' transforms go to LDS for per-lane dynamic access
  float bb_[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    float s, c;
    sincos_contract(E.ang[b], &s, &c);
    Box bx;
    box_world(E.px[b], E.py[b], c, s, bx);
#pragma unroll
    for (int q = 0; q < 4; ++q) bb_[b][q] = bx.bb[q];
    L.ph.box[b][lane] = make_float4(E.px[b], E.py[b], c, s);
  }
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    L.ph.p[b][lane] = v2(E.px[b], E.py[b]);
    st_v(L, b, lane, v2(E.vx[b], E.vy[b]), E.w[b]);
    st_vb(L, b, lane, v2(0.0f, 0.0f), 0.0f);
  }
  L.ph.p[5][lane] = v2(0.0f, 0.0f);
  st_v(L, 5, lane, v2(0.0f, 0.0f), 0.0f);
  st_vb(L, 5, lane, v2(0.0f, 0.0f), 0.0f);
  const V2 ballc = v2(E.px[4], E.py[4]);
  const float BR = 10.0f;
  const float ballbb[4] = {ballc.x - BR, ballc.y - BR, ballc.x + BR, ballc.y + BR};

  // broadphase: AABB masks per pair class (cpBBIntersects), no divergence
  STAMP(2);
  uint32_t mAA = 0, mBA = 0, mSA = 0, mBS = 0;
  {
    const int AI[6] = {0, 0, 0, 1, 1, 2}, AJ[6] = {1, 2, 3, 2, 3, 3};
#pragma unroll
    for (int p = 0; p < 6; ++p)
      if (bb_intersects(bb_[AI[p]], bb_[AJ[p]])) mAA |= 1u << p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (bb_intersects(ballbb, bb_[i])) mBA |= 1u << i;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        if (bb_intersects(P.seg[s].bb, bb_[i])) mSA |= 1u << (i * 8 + s);
    }
#pragma unroll
    for (int s = 0; s < 6; ++s)
      if (bb_intersects(ballbb, P.seg[s].bb)) mBS |= 1u << s;
  }

  CSlot* ovf = (CSlot*)S.SP + e * SPW;
  Contacts C;
  C.nc = 0;
  C.na = 0;
  // a slot no contact reaches still gets prestep_one (below): body indices 0, not undefined
  static_for<0, KREG>([&](auto qc) __attribute__((always_inline)) { C.reg[decltype(qc)::value].m = 0u; });
  CacheWalk W;
  W.par = (E.meta & META_PAR) ? 1 : 0;
  W.nc_old = META_NC(E.meta);
  W.cur = 0;
  W.out = 0;
  W.pk = pk0;

  ACC_DECL(aa_col); ACC_DECL(aa_add); ACC_DECL(sa_col); ACC_DECL(sa_add);
#ifdef MS_STAMPS
  unsigned long long aa_n = 0, sa_n = 0;
#endif
  // narrowphase, one compacted loop per pair class so each lane visits only its own touching
  // pairs; class order + ctz order = canonical pair order (DESIGN.md pair table)
  while (mAA) {
    const int p = __builtin_ctz(mAA);
    mAA &= mAA - 1;
    const int i = p < 3 ? 0 : (p < 5 ? 1 : 2);
    const int j = p < 3 ? p + 1 : (p < 5 ? p - 1 : 3);
    // frame of agent i: box i at the origin, box j at p_j - p_i
    const F4 ta = lds_f4(&L.ph.box[i][lane]), tb = lds_f4(&L.ph.box[j][lane]);
    const V2 ob = v2(tb.x - ta.x, tb.y - ta.y);
    Box A, B;
    box_world(0.0f, 0.0f, ta.z, ta.w, A);
    box_world(ob.x, ob.y, tb.z, tb.w, B);
    Col col; col.count = 0; col.n = v2(0.0f, 0.0f);
    ACC_BEGIN(aa_col);
    col_box_box(A, B, col);
    ACC_END(aa_col);
    ACC_BEGIN(aa_add);
    if (col.count) add_arbiter(a, L, C, ovf, W, p, i, j, col, v2(0.0f, 0.0f), ob, overflow_acc);
    ACC_END(aa_add);
    ACC_INC(aa_n);
  }
  while (mBA) {
    const int i = __builtin_ctz(mBA);
    mBA &= mBA - 1;
    // frame of the ball: the ball at the origin, box i at p_i - p_ball
    const F4 tb = lds_f4(&L.ph.box[i][lane]);
    const V2 ob = v2(tb.x - ballc.x, tb.y - ballc.y);
    Box B;
    box_world(ob.x, ob.y, tb.z, tb.w, B);
    Col col; col.count = 0; col.n = v2(0.0f, 0.0f);
    col_circle_box(v2(0.0f, 0.0f), BR, B, col);
    if (col.count) add_arbiter(a, L, C, ovf, W, 6 + i, 4, i, col, v2(0.0f, 0.0f), ob, overflow_acc);
  }
  STAMP(11);
  // Static-agent pairs: the tests (col_seg_box, the costly part) are spread over the wave's
  // active lanes instead of run by each env's lane in turn — a lane whose env has k touching
  // pairs would otherwise hold the wave for k tests while the others idle. Tasks are numbered in
  // (lane, ctz) order; each window of `nact` tasks is tested by the active lanes (rank r takes
  // task base + r), then every lane inserts its own results in ctz order, so the arbiter order
  // and every value are those of the per-lane loop. Prefix sums by bit-sliced ballots (exact
  // with inactive lanes, which hold no tasks).
  {
    const uint64_t act = __builtin_amdgcn_read_exec();
    const int nact = __builtin_popcountll(act);
    const int rank = lane_rank(act);
    const int cnt = __builtin_popcount(mSA);
    int pre = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const uint64_t m = __ballot((cnt >> b) & 1);
      pre += lane_rank(m) << b;
      total += __builtin_popcountll(m) << b;
    }
    int tf = pre, tc = pre;  // global index of this lane's next task to post / to insert
    uint32_t mf = mSA, mc = mSA;
    for (int base = 0; base < total; base += nact) {
      while (mf && tf < base + nact) {
        const int q = __builtin_ctz(mf);
        mf &= mf - 1;
        L.u.np.nt.task[tf - base] = (uint32_t)(lane << 5) | (uint32_t)q;
        ++tf;
      }
      wave_lds_handoff();  // tasks posted -> read by the testing lanes
      ACC_BEGIN(sa_col);
      if (rank < total - base) {
        const uint32_t v = L.u.np.nt.task[rank];
        const int q = (int)(v & 31u);
        // frame of the owner's agent: its box at the origin, the segment moved by -p_agent
        const F4 t = lds_f4(&L.ph.box[q >> 3][(int)(v >> 5)]);
        Box B;
        box_world(0.0f, 0.0f, t.z, t.w, B);
        Col col; col.count = 0; col.n = v2(0.0f, 0.0f);
        Seg sg = L.seg[q & 7];
        sg.ax = sg.ax - t.x; sg.ay = sg.ay - t.y;
        sg.bx = sg.bx - t.x; sg.by = sg.by - t.y;
        col_seg_box(sg, B, col);
        L.u.np.nt.res[0][rank] = make_float4(col.n.x, col.n.y, col.p1[0].x, col.p1[0].y);
        L.u.np.nt.res[1][rank] = make_float4(col.p2[0].x, col.p2[0].y, col.p1[1].x, col.p1[1].y);
        L.u.np.nt.res[2][rank] = make_float4(col.p2[1].x, col.p2[1].y, __int_as_float((col.count ? col.hash[0] & 0xffff : 0) | (col.count << 16)),
                                             __int_as_float(col.hash[1]));
      }
      ACC_END(sa_col);
      wave_lds_handoff();  // results written -> read by the owner lanes
      ACC_BEGIN(sa_add);
      while (mc && tc < base + nact) {
        const int q = __builtin_ctz(mc);
        mc &= mc - 1;
        const int t = tc - base, i = q >> 3;
        ++tc;
        // one round trip: the count travels with the hashes
        const F4 r0 = lds_f4(&L.u.np.nt.res[0][t]), r1 = lds_f4(&L.u.np.nt.res[1][t]), r2 = lds_f4(&L.u.np.nt.res[2][t]);
        Col col;
        col.count = __float_as_int(r2.z) >> 16;
        if (col.count) {
          col.n = v2(r0.x, r0.y);
          col.p1[0] = v2(r0.z, r0.w); col.p2[0] = v2(r1.x, r1.y);
          col.p1[1] = v2(r1.z, r1.w); col.p2[1] = v2(r2.x, r2.y);
          col.hash[0] = __float_as_int(r2.z) & 0xffff; col.hash[1] = __float_as_int(r2.w);
          add_arbiter(a, L, C, ovf, W, 10 + q, 5, i, col, v2(0.0f, 0.0f), v2(0.0f, 0.0f), overflow_acc);
        }
        ACC_INC(sa_n);
      }
      ACC_END(sa_add);
      wave_lds_handoff();  // results read -> the next window's tasks and results overwrite them
    }
  }
  STAMP(13);
  while (mBS) {
    const int s = __builtin_ctz(mBS);
    mBS &= mBS - 1;
    // frame of the ball: the ball at the origin, the segment moved by -p_ball
    Col col; col.count = 0; col.n = v2(0.0f, 0.0f);
    Seg sg = L.seg[s];
    sg.ax = sg.ax - ballc.x; sg.ay = sg.ay - ballc.y;
    sg.bx = sg.bx - ballc.x; sg.by = sg.by - ballc.y;
    col_circle_seg(v2(0.0f, 0.0f), BR, sg, col);
    if (col.count) add_arbiter(a, L, C, ovf, W, 42 + s, 4, 5, col, v2(0.0f, 0.0f), v2(0.0f, 0.0f), overflow_acc);
  }
  while (W.cur < W.nc_old) cache_age_current(a, L, W, overflow_acc);
  // contacts KREG.. of a pile-up from the global spill into LDS for the 12 passes over them
  // (the narrowphase scratch they share LDS with is dead from here on)
  asm volatile("" ::: "memory");
  for (int k = KREG; k < C.nc && k < KREG + NLDS; ++k) ov_put(L, k - KREG, lane, ovf[k - KREG]);
  STAMP(3);
#ifdef MS_STAMPS
  ACC_STORE(aa_col, 16); ACC_STORE(aa_add, 17); ACC_STORE(aa_n, 18);
  ACC_STORE(sa_col, 19); ACC_STORE(sa_add, 20); ACC_STORE(sa_n, 21);
  {
    int mx = C.nc;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0 && S.stamps) S.stamps[stamp_row * MS_NSTAMP + 12] = (unsigned long long)mx;
  }
#endif

  // cpArbiterPreStep. prestep_one of one contact reads only body state and writes only its own
  // slot, so the register slots go in groups of PRE_GROUP under one wave-uniform test (does any
  // lane have a contact in the group) and without a per-lane test inside: the compiler can then
  // overlap the group's LDS reads and divisions. A lane's slots past its last contact get values
  // nothing reads (warm start, solver and cache writes test k < nc).
  static_for<0, KREG / PRE_GROUP>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    if (__ballot(PRE_GROUP * g < C.nc) != 0) {
      static_for<0, PRE_GROUP>([&](auto kc) __attribute__((always_inline)) {
        prestep_one(P, C.reg[PRE_GROUP * g + decltype(kc)::value], L, lane);
      });
    }
  });
  for (int k_ = KREG; k_ < C.nc; ++k_) {
    if (k_ < KREG + NLDS) {
      CSlot c_;
      ov_get(L, k_ - KREG, lane, c_);
      prestep_one(P, c_, L, lane);
      ov_put(L, k_ - KREG, lane, c_);
    } else {
      prestep_one(P, ovf[k_ - KREG], L, lane);
    }
  }
  STAMP(14);

  // cpBodyUpdateVelocity + entities.py velocity_func (damping, max-velocity clamp)
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    const float mi = P.m_inv[b], ii = P.i_inv[b];
    const float ffx = b < 4 ? fx[b] : 0.0f, ffy = b < 4 ? fy[b] : 0.0f, tt = b < 4 ? tq[b] : 0.0f;
    float nvx = E.vx[b] * 1.0f + (0.0f + ffx * mi) * dt;
    float nvy = E.vy[b] * 1.0f + (0.0f + ffy * mi) * dt;
    float nw = E.w[b] * 1.0f + tt * ii * dt;
    const float damp = b < 4 ? P.agent_damp : P.ball_damp;
    nvx = nvx * damp;
    nvy = nvy * damp;
    if (b < 4) nw = nw * damp;
    const float len = sqrtf(nvx * nvx + nvy * nvy);
    if (len > P.vmax) {
      nvx = (nvx / len) * P.vmax;
      nvy = (nvy / len) * P.vmax;
    }
    E.vx[b] = nvx; E.vy[b] = nvy; E.w[b] = nw;
    st_v(L, b, lane, v2(nvx, nvy), nw);
  }

  STAMP(4);
  if (need_h2) snap_load(a, h2);  // arrives during the solver
  if (C.nc > 0) {
    // cpArbiterApplyCachedImpulse, then cpArbiterApplyImpulse x 10 (pymunk Space default)
    FOR_CONTACTS(C, ovf, { warm_one(P, c_, L, lane); });
    STAMP(15);
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
      asm volatile("; MS_SOLVER_ITER_BEGIN" ::: "memory");
      FOR_CONTACTS(C, ovf, { solve_one(P, c_, L, lane); });
      asm volatile("; MS_SOLVER_ITER_END" ::: "memory");
    }
    STAMP(5);
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      V2 v, vbv;
      ld_v(L, b, lane, v, E.w[b]);
      ld_vb(L, b, lane, vbv, E.wb[b]);
      E.vx[b] = v.x; E.vy[b] = v.y;
      E.vbx[b] = vbv.x; E.vby[b] = vbv.y;
    }
    // touched arbiters' cache entries at the positions reserved in merge order
    static_for<0, KREG - 1>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      if (k < C.nc) write_arbiter_cache(a, W.par ^ 1, C.reg[k], C.reg[k + 1]);
    });
    if (KREG - 1 < C.nc) {
      CSlot next = C.reg[KREG - 1];
      if (KREG < C.nc) next = over_slot(L, lane, ovf, KREG);
      write_arbiter_cache(a, W.par ^ 1, C.reg[KREG - 1], next);
    }
    // the contact after the last one is never read (count > 1 only for an arbiter's first contact,
    // whose second contact exists); k + 1 stays inside the env's spill slice
    for (int k = KREG; k < C.nc; ++k)
      write_arbiter_cache(a, W.par ^ 1, over_slot(L, lane, ovf, k), over_slot(L, lane, ovf, k + 1 < MAXC ? k + 1 : k));
  }
  STAMP(6);
  const int nn = W.out < MAXA ? W.out : MAXA;
  E.meta = (E.meta & ~((63u << 8) | META_PAR)) | ((uint32_t)nn << 8) | (W.par ? 0u : META_PAR);
}

// ---- kernels ---------------------------------------------------------------------------------
__device__ __forceinline__ void unpack_scalars(int4 v, Env& E) {
  E.steps = v.x;
  E.score_blue = (int)((uint32_t)v.y & 0xffffu);
  E.score_red = (int)((uint32_t)v.y >> 16);
  E.meta = (uint32_t)v.z;
  E.rng.u32 = (uint32_t)v.w;
}
__device__ __forceinline__ void load_scalars(At a, Env& E) { unpack_scalars(*plane<int4>(a, OFF_I4, 0), E); }

// The outputs of an env-step skipped for a non-finite action (SoccerEnv.step raises ValueError there,
// soccer_env.py:116-117, and the env is not stepped): defined values, so that a caller who does not
// look at the NaN reward reads no stale or uninitialised episode end (a ms_step_n output slot would
// otherwise keep whatever it held). Reward (NaN, NaN, 0, 0), term / trunc / goal 0, the env's current
// score (sc: its scalars group), the stacked observation all NaN. `part` of `parts` cooperating lanes
// writes every parts-th 16-B piece of the 1,056-B obs row; lane part 0 writes the rest.
__device__ __forceinline__ void skipped_outputs(int64_t e, int4 sc, int part, int parts, float* __restrict__ obs,
                                                float* __restrict__ rew, uint8_t* __restrict__ term,
                                                uint8_t* __restrict__ trunc, int8_t* __restrict__ goal_out,
                                                int32_t* __restrict__ score_out) {
  const float qn = __builtin_nanf("");
  if (obs) {
    float4* row = (float4*)(obs + e * 264);
    for (int q = part; q < 66; q += parts) row[q] = make_float4(qn, qn, qn, qn);
  }
  if (part != 0) return;
  if (rew) *(float4*)(rew + e * 4) = make_float4(qn, qn, 0.0f, 0.0f);
  if (term) *(uint32_t*)(term + e * 4) = 0u;
  if (trunc) *(uint32_t*)(trunc + e * 4) = 0u;
  if (goal_out) goal_out[e] = 0;
  if (score_out) *(int2*)(score_out + e * 2) = make_int2((int)((uint32_t)sc.y & 0xffffu), (int)((uint32_t)sc.y >> 16));
}
__device__ __forceinline__ void store_scalars(At a, const Env& E) {
  *plane<int4>(a, OFF_I4, 0) = make_int4(E.steps, (int32_t)(((uint32_t)E.score_blue & 0xffffu) | ((uint32_t)E.score_red << 16)),
                      (int32_t)E.meta, (int32_t)E.rng.u32);
}

// The reference's default config.json physics and rewards (make_params of ms_config_default,
// bit for bit; ms_create compares the two and launches the specialised step kernel only when
// they are identical). As compile-time constants the masses, restitution/friction products,
// reward multipliers and the segment table fold into the instructions that use them.
__host__ __device__ constexpr Params default_params() {
  return Params{
    0x1.111112p-6f, 0x1.99999ap-4f, 0x1.99999ap-4f,
    {0x1.99999ap-4f, 0x1.99999ap-4f, 0x1.99999ap-4f, 0x1.99999ap-4f, 0x1p+0f, 0.0f},
    {0x1.47ae14p-7f, 0x1.47ae14p-7f, 0x1.47ae14p-7f, 0x1.47ae14p-7f, 0x1.99999ap-4f, 0.0f},
    0x1.fae148p-1f, 0x1.f0a3d8p-1f, 200.0f, 150000.0f, 1000.0f, 200.0f, 10.0f,
    0x1.47ae16p-5f, 0x1.47ae16p-1f, 0x1.851eb8p-3f, 0x1.47ae16p-3f, 0x1.851eb8p-3f, 0x1.47ae16p-3f,
    0x1.851eb8p-3f, 0.0f, 0x1.ce147ap-1f, 0x1.47ae16p-5f,
    0x1.0624dep-9f, 0x1.99999ap-4f, 0x1.4f8b58p-17f, 4.0f, 0.0f, 0.0f,
    1000, 1, 1,
    {{10.0f, 10.0f, 790.0f, 10.0f, -0.0f, 1.0f, 2.0f, {8.0f, 8.0f, 792.0f, 12.0f}},
     {10.0f, 590.0f, 790.0f, 590.0f, -0.0f, 1.0f, 2.0f, {8.0f, 588.0f, 792.0f, 592.0f}},
     {10.0f, 10.0f, 10.0f, 225.0f, -1.0f, 0.0f, 2.0f, {8.0f, 8.0f, 12.0f, 227.0f}},
     {10.0f, 375.0f, 10.0f, 590.0f, -1.0f, 0.0f, 2.0f, {8.0f, 373.0f, 12.0f, 592.0f}},
     {790.0f, 10.0f, 790.0f, 225.0f, -1.0f, 0.0f, 2.0f, {788.0f, 8.0f, 792.0f, 227.0f}},
     {790.0f, 375.0f, 790.0f, 590.0f, -1.0f, 0.0f, 2.0f, {788.0f, 373.0f, 792.0f, 592.0f}},
     {10.0f, 225.0f, 10.0f, 375.0f, -1.0f, 0.0f, 1.0f, {9.0f, 224.0f, 11.0f, 376.0f}},
     {790.0f, 225.0f, 790.0f, 375.0f, -1.0f, 0.0f, 1.0f, {789.0f, 224.0f, 791.0f, 376.0f}}}};
}

// The parameters a step kernel computes with, by its specialisation mode PM (ms_config_specialised):
// 1 = the reference's defaults as compile-time constants, 2 = the default physics as constants with
// the reward multipliers from the kernel arguments (a reward-shaping config keeps the physics folded
// into the instructions), 0 = everything from the kernel arguments. max_steps and autoreset are
// always runtime values.
template <int PM>
__device__ __forceinline__ Params kernel_params(const Params& Pin) {
  if constexpr (PM == 0) {
    return Pin;
  } else {
    Params P = default_params();
    P.max_steps = Pin.max_steps;
    P.autoreset = Pin.autoreset;
    if constexpr (PM == 2) {
      P.prox_mult = Pin.prox_mult;
      P.goal_mult = Pin.goal_mult;
      P.alive = Pin.alive;
      P.goal_reward = Pin.goal_reward;
      P.concede_penalty = Pin.concede_penalty;
      P.score_diff_mult = Pin.score_diff_mult;
    }
    return P;
  }
}
// The parameters a lane-pair or lane-group kernel steps with: PM 0 the kernel argument in the
// kernel-argument segment itself (every such kernel takes (DevState, Params, ...), laid out as KArgHead; read
// per phase: param_phase — a reference to the by-value parameter would be a copy in scratch), the
// others kernel_params' folded constants
struct KArgHead {
  DevState S;
  Params P;
};
template <int PM>
__device__ __forceinline__ const Params& step_params(const Params& Pin, Params& tmp) {
  if constexpr (PM == 0) {
    const __attribute__((address_space(4))) char* ka =
        (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
    return *(const Params*)(const __attribute__((address_space(4))) Params*)(ka + offsetof(KArgHead, P));
  } else {
    tmp = kernel_params<PM>(Pin);
    return tmp;
  }
}

// PM 0: the step's parameters are a phase-local copy (Pv), re-read from the kernel-argument
// segment at every phase boundary through a pointer the compiler cannot see through: each phase
// loads (s_load) only the fields it uses, at its start, instead of one load per field held in SGPRs
// from its first to its last use across the step (the spills of the generic kernels). A copy, not
// per-use loads: a per-lane select between two parameters loaded at the select would be folded into
// one per-lane vector load from a selected address. (Pa must be the kernel argument in the argument
// segment itself, pair_params; the default-physics kernels copy their folded constants.)
__device__ __forceinline__ const Params* param_phase(const Params* p) {
  auto q = (const __attribute__((address_space(4))) Params*)p;
  asm volatile("" : "+s"(q));
  return (const Params*)q;
}

// The K-step kernels' arguments as laid out in the kernel-argument segment (ms_step_pair_n_kernel;
// ms_step_group_n_kernel adds `int solve` after them)
struct KStepArgs {
  DevState S;
  Params P;
  int K;
  const float* actions;
  float* obs;
  float* rew;
  uint8_t* term;
  uint8_t* trunc;
  int8_t* goal_out;
  int32_t* score_out;
  Counters* ctr;
};
// The first HBM batch of one state block (one wave's 64 envs): scalars, bodies, actions, the
// previous step's arbiter-cache entries 0..KC-1 and PCG64. The scalars come first and alone
// (fetch_scalars): the cache entries' addresses depend on them (parity bit, entry count).
struct Fetch {
  int4 sc;
  float4 b[G_BODY];
  float4 a[3];
  uint32_t ch[KC];
  float4 cj[KC];
  ulonglong2 r0, r1;
};
__device__ __forceinline__ void fetch_scalars(const DevState& S, int64_t blk, int lane, Fetch& F) {
  const At at{S.blocks + blk * BLOCK_BYTES, lane};
  F.sc = *plane<int4>(at, OFF_I4, 0);
}
// Loads are unconditional (a padding lane of the last block reads its zeroed slot and the last
// env's actions): loads under a lane branch make the compiler copy the loaded registers at the
// join, and every copy waits for its load. A lane without cache entry k re-reads its own
// scalars/bodies, which are in L1, instead.
__device__ __forceinline__ void fetch_rest(const DevState& S, int64_t blk, int lane, const float* __restrict__ actions,
                                           Fetch& F) {
  const At at{S.blocks + blk * BLOCK_BYTES, lane};
  const int64_t e = blk * MS_BLOCK + lane;
#pragma unroll
  for (int g = 0; g < G_BODY; ++g) F.b[g] = *plane<float4>(at, OFF_B4, g);
  const float4* ap = (const float4*)(actions + (e < S.n ? e : S.n - 1) * 12);
#pragma unroll
  for (int q = 0; q < 3; ++q) F.a[q] = ap[q];
  const uint32_t meta = (uint32_t)F.sc.z;
  const int nco = META_NC(meta);
  const int par0 = (meta & META_PAR) ? 1 : 0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const bool need = k < nco;
    const uint32_t* hp = need ? plane<uint32_t>(at, OFF_CH, par0 * MAXA + k) : (const uint32_t*)plane<int4>(at, OFF_I4, 0);
    const float4* jp = need ? plane<float4>(at, OFF_CJ, par0 * MAXA + k) : plane<float4>(at, OFF_B4, 0);
    F.ch[k] = *hp;
    F.cj[k] = *jp;
  }
  F.r0 = *plane<ulonglong2>(at, OFF_R2, 0);
  F.r1 = *plane<ulonglong2>(at, OFF_R2, 1);
}

// One env.step of every env of state block `blk` (SoccerEnv.step -> Game.step,
// soccer_env.py:100-154, game/game.py:378-437), one lane per env. Order inside a lane:
//   1. the first HBM batch (Fetch, loaded by the caller): scalars, bodies, actions, the old
//      arbiter cache (entries < KC, staged in LDS) and PCG64; the t-1 snapshot (= the body state
//      before this step) is staged in LDS;
//   2. physics; the t-2 snapshot is loaded just before the solver and arrives while it runs;
//      no other HBM read follows (gfx9 has one vmcnt for loads and stores, so a read after
//      the stores would wait for them);
//   3. goal, rewards, outputs, goal respawn, vec auto-reset;
//   4. frames t-2, t-1, t of agent 0, then agent 1, ... (each 264-B row segment in one burst
//      of stores), the history slot (t-1 becomes the next step's t-2) and the
//      state. A lane whose stack is refilled (first step after a reset, or an auto-reset this
//      step) writes three copies of frame t and the slot instead.
template <bool RING>
__device__ __forceinline__ void step_block(const DevState& S, const Params& P, Lds& L, const int64_t blk, const Fetch& F,
                                           const float* __restrict__ actions,
                                           float* __restrict__ obs, float* __restrict__ rew,
                                           uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                           int8_t* __restrict__ goal_out, int32_t* __restrict__ score_out,
                                           Counters* ctr, const Ring rg) {
  const int lane = threadIdx.x;
  const int64_t e = blk * MS_BLOCK + lane;
  bool active = e < S.n;
  // the wave's state block: a wave-uniform base and this lane's slot in it
  const At at{S.blocks + blk * BLOCK_BYTES, lane};
#ifdef MS_STAMPS
  const int64_t stamp_row = blk;
#endif
  STAMP(0);

  Env E;
  unpack_scalars(F.sc, E);
  {
    float f[44];
#pragma unroll
    for (int g = 0; g < G_BODY; ++g) {
      f[4 * g] = F.b[g].x; f[4 * g + 1] = F.b[g].y; f[4 * g + 2] = F.b[g].z; f[4 * g + 3] = F.b[g].w;
    }
    unpack_bodies(f, E);
  }
  Snap h2;  // obs-history snapshot t-2
  float a[12];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    a[4 * q] = F.a[q].x; a[4 * q + 1] = F.a[q].y; a[4 * q + 2] = F.a[q].z; a[4 * q + 3] = F.a[q].w;
  }
  const int nco = META_NC(E.meta);
  uint32_t pk0 = 0u;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    L.u.np.ch[k][lane] = F.ch[k];
    L.u.np.cj[k][lane] = F.cj[k];
    pk0 |= cache_key(F.ch[k]) << (8 * k);
  }
  bool fill3 = false, rng_dirty = false;
  E.rng.shi = F.r0.x; E.rng.slo = F.r0.y;
  E.rng.ihi = F.r1.x; E.rng.ilo = F.r1.y;
  E.rng.has32 = (E.meta & META_H32) ? 1u : 0u;
  Snap h1;  // obs-history snapshot t-1: the body state before this step
  if (active) {
    // SoccerEnv.step validation (soccer_env.py:101-117): a non-finite action skips the env
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 12; ++k) finite = finite && isfinite(a[k]);
    if (!finite) {
      atomicAdd(&ctr->nonfinite, 1ULL);
      atomicMin(&ctr->first_bad, (long long)e);
      // the env is not stepped; its reward is poisoned so that no caller reads the previous
      // step's value as this one's (the reference raises ValueError here), and its other outputs
      // get defined values (skipped_outputs; the frame ring writes no frame: FrameRingBatch)
      skipped_outputs(e, F.sc, 0, 1, RING ? nullptr : obs, rew, term, trunc, goal_out, score_out);
      active = false;
    }
  }
  if (active) {
    E.steps += 1;
    const bool done_now = P.max_steps > 0 && E.steps >= P.max_steps;
    // the stack is refilled instead of shifted after a reset (hist_empty) or an auto-reset at
    // the end of this step
    fill3 = (E.meta & META_HE) != 0 || (P.autoreset && done_now);
    snap_of(E, h1);
    snap_to_lds(L.h1, lane, h1);  // back at the end: not held in registers across the physics
  }

  float pvx[5], pvy[5];
  int ncw = 0;  // arbiter-cache entries this step wrote
  if (active) {
    float fx[4], fy[4], tq[4];
#pragma unroll
    for (int b = 0; b < 5; ++b) { pvx[b] = E.px[b]; pvy[b] = E.py[b]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float Fo[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float v = a[i * 3 + k];
        v = v < -1.0f ? -1.0f : (v > 1.0f ? 1.0f : v);
        Fo[k] = v * (k < 2 ? P.force_max : P.torque_max);
      }
      float sn, cs;
      sincos_contract(E.ang[i], &sn, &cs);
      fx[i] = 0.0f + (cs * Fo[0] + (-sn) * Fo[1]);
      fy[i] = 0.0f + (sn * Fo[0] + cs * Fo[1]);
      tq[i] = Fo[2];
    }

    unsigned long long ovf = 0;
    STAMP(1);
    physics_step(S, at, e, P, E, fx, fy, tq, L, &ovf, h2, pk0, !RING || rg.wrap != 0);
    ncw = META_NC(E.meta);
    // positions back from LDS (written by the position phase, unchanged since)
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const V2 p = L.ph.p[b][lane];
      E.px[b] = p.x; E.py[b] = p.y;
    }
    snap_from_lds(L.h1, lane, h1);
#pragma unroll
    for (int b = 0; b < 5; ++b) { pvx[b] = h1.px[b]; pvy[b] = h1.py[b]; }
    STAMP(7);
    if (ovf) atomicAdd(&ctr->overflow, ovf);
  }
  if (active) {
    // goal detection (game.py:401-412)
    int goal = 0;
    const float bx = E.px[4], by = E.py[4];
    if (bx < 10.0f && 225.0f < by && by < 375.0f) { goal = 2; E.score_red += 1; }
    else if (bx > 790.0f && 225.0f < by && by < 375.0f) { goal = 1; E.score_blue += 1; }
    const bool done = P.max_steps > 0 && E.steps >= P.max_steps;
    float r = blue_reward(P, pvx, pvy, E.px, E.py, goal, false, 0, 0);
    if (goal) {
      rng_dirty = true;
      soft_reset_regs(E);
    }
    if (done) r = blue_reward(P, pvx, pvy, E.px, E.py, goal, true, E.score_blue, E.score_red);

    // outputs of this step (before a vec auto-reset)
    if (rew) *(float4*)(rew + e * 4) = make_float4(r, r, 0.0f, 0.0f);
    if (term) *(uint32_t*)(term + e * 4) = 0u;
    if (trunc) *(uint32_t*)(trunc + e * 4) = done ? 0x01010101u : 0u;
    if (goal_out) goal_out[e] = (int8_t)goal;
    if (score_out) *(int2*)(score_out + e * 2) = make_int2(E.score_blue, E.score_red);

    if (done && P.autoreset) {
      // marl_vecenv.py:48-51: env.reset(options={"use_full_random_positions": True})
      rng_dirty = true;
      reset_env_regs(E, MS_SPAWN_FULL_RANDOM);
    }
  }
  STAMP(8);
  if (active) {
    // (4) frame t; refilled stacks get all three frames and the history slot
    Snap s0;
    snap_of(E, s0);
    if constexpr (RING) {
      ring_emit_window(P, h2, h1, s0, fill3, rg.frames + e * (int64_t)(4 * rg.R * 22), rg);
      if (fill3) {
        snap_store(at, s0);
        E.meta &= ~META_HE;
      } else {
        snap_store(at, h1);  // t-1 becomes the next step's t-2
      }
    } else if (fill3) {
      emit_fill3(at, P, e, s0, obs);
      E.meta &= ~META_HE;
    } else {
      if (obs) emit_three(P, h2, h1, s0, obs + e * 264);
      snap_store(at, h1);  // t-1 becomes the next step's t-2
    }
    STAMP(9);
    if (rng_dirty) store_rng(at, E);
    store_bodies(at, E);
    store_scalars(at, E);
  }
  STAMP(10);
  // The wave's tally of arbiter-cache entries read (the previous step's cache) and written, and
  // of env-steps taken: the cache term of the algorithmic byte count, measured inside the timed
  // launches (ms_get_stats). Packed as read | written << 12 | steps << 24 (64 lanes x <= 32
  // entries < 2^12), summed over the wave, then three no-return vector atomics by lane 0 to the
  // block's own counters (no address is shared between waves).
  {
    uint32_t v = active ? ((uint32_t)nco | ((uint32_t)ncw << 12) | (1u << 24)) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) {
      Tally* t = S.tally + blk;
      atomicAdd(&t->read, (unsigned long long)(v & 0xfffu));
      atomicAdd(&t->written, (unsigned long long)((v >> 12) & 0xfffu));
      atomicAdd(&t->steps, (unsigned long long)(v >> 24));
    }
  }
}

// One wave per state block (grid = blocks).
template <bool RING>
__device__ __forceinline__ void step_envs(const DevState& S, const Params& P, const float* __restrict__ actions,
                                          float* __restrict__ obs, float* __restrict__ rew,
                                          uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                          int8_t* __restrict__ goal_out, int32_t* __restrict__ score_out,
                                          Counters* ctr, const Ring rg) {
  __shared__ Lds L;
  const int lane = threadIdx.x;
  const int64_t blk = blockIdx.x;
  Fetch F;
  fetch_scalars(S, blk, lane, F);
  fetch_rest(S, blk, lane, actions, F);
  stage_segments(P, L, lane);
  step_block<RING>(S, P, L, blk, F, actions, obs, rew, term, trunc, goal_out, score_out, ctr, rg);
}

template <bool DEFAULT_PARAMS>
__global__ __launch_bounds__(MS_BLOCK) void ms_step_kernel(DevState S, Params Pin, const float* __restrict__ actions,
                                                           float* __restrict__ obs, float* __restrict__ rew,
                                                           uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                                           int8_t* __restrict__ goal_out, int32_t* __restrict__ score_out,
                                                           Counters* ctr) {
  const Ring none{nullptr, 0, 0, 0};
  if constexpr (DEFAULT_PARAMS) {
    Params Pd = default_params();
    Pd.max_steps = Pin.max_steps;  // episode length and auto-reset stay runtime values
    Pd.autoreset = Pin.autoreset;
    step_envs<false>(S, Pd, actions, obs, rew, term, trunc, goal_out, score_out, ctr, none);
  } else {
    step_envs<false>(S, Pin, actions, obs, rew, term, trunc, goal_out, score_out, ctr, none);
  }
}

// ms_step with the observation as a frame-ring window (ms_step_ring)
template <bool DEFAULT_PARAMS>
__global__ __launch_bounds__(MS_BLOCK) void ms_step_ring_kernel(DevState S, Params Pin, const float* __restrict__ actions,
                                                                Ring rg, float* __restrict__ rew,
                                                                uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                                                int8_t* __restrict__ goal_out,
                                                                int32_t* __restrict__ score_out, Counters* ctr) {
  if constexpr (DEFAULT_PARAMS) {
    Params Pd = default_params();
    Pd.max_steps = Pin.max_steps;
    Pd.autoreset = Pin.autoreset;
    step_envs<true>(S, Pd, actions, nullptr, rew, term, trunc, goal_out, score_out, ctr, rg);
  } else {
    step_envs<true>(S, Pin, actions, nullptr, rew, term, trunc, goal_out, score_out, ctr, rg);
  }
}

#ifndef MS_KSTEP_TU  // (ms_kstep.hip includes this file for the device code of the K-step kernels only)
__global__ __launch_bounds__(MS_BLOCK) void ms_reset_kernel(DevState S, Params P, const uint64_t* __restrict__ pcg,
                                                            const uint8_t* __restrict__ mask, int mode, int set_hist_empty,
                                                            float* __restrict__ obs, const Ring rg) {
  const int64_t e = (int64_t)blockIdx.x * MS_BLOCK + threadIdx.x;
  const bool active = e < S.n && (!mask || mask[e]);
  if (!active) return;
  const At a = env_at(S, e);
  Env E;
  load_scalars(a, E);
  if (pcg) {
    E.rng.shi = pcg[e * 4 + 0]; E.rng.slo = pcg[e * 4 + 1];
    E.rng.ihi = pcg[e * 4 + 2]; E.rng.ilo = pcg[e * 4 + 3];
    E.rng.has32 = 0; E.rng.u32 = 0;
  } else {
    load_rng(a, E);
  }
  reset_env_regs(E, mode);
  Snap s0;
  snap_of(E, s0);
  emit_fill3(a, P, e, s0, obs);
  if (rg.frames) {
    ring_emit_window(P, s0, s0, s0, true, rg.frames + e * (int64_t)(4 * rg.R * 22), rg);
  }
  E.meta &= ~META_HE;
  if (set_hist_empty) E.meta |= META_HE;
  store_rng(a, E);
  store_bodies(a, E);
  store_scalars(a, E);
}

__global__ __launch_bounds__(MS_BLOCK) void ms_observe_kernel(DevState S, Params P, float* __restrict__ frames) {
  const int64_t e = (int64_t)blockIdx.x * MS_BLOCK + threadIdx.x;
  if (e >= S.n) return;
  const At a = env_at(S, e);
  Env E;
  load_scalars(a, E);
  load_bodies(a, E);
#pragma unroll 1
  for (int a = 0; a < 4; ++a) {
    float f[22];
    frame_of(P, E, a, f);
#pragma unroll
    for (int k = 0; k < 22; ++k) frames[e * 88 + a * 22 + k] = f[k];
  }
}

__global__ void ms_export_kernel(DevState S, ms_env_state* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const At a = env_at(S, e);
  Env E;
  load_scalars(a, E);
  load_bodies(a, E);
  load_rng(a, E);
  ms_env_state& o = out[e];
  for (int b = 0; b < 5; ++b) {
    ms_body_state& d = o.body[b];
    d.px = E.px[b]; d.py = E.py[b]; d.vx = E.vx[b]; d.vy = E.vy[b];
    d.angle = b < 4 ? E.ang[b < 4 ? b : 0] : 0.0f;
    d.w = E.w[b]; d.vbx = E.vbx[b]; d.vby = E.vby[b]; d.wb = E.wb[b];
  }
  Snap h2, h1;
  snap_load(a, h2);
  snap_of(E, h1);  // the t-1 snapshot is the current body state
  for (int b = 0; b < 5; ++b) {
    o.snap[0][b] = h2.px[b]; o.snap[0][5 + b] = h2.py[b];
    o.snap[1][b] = h1.px[b]; o.snap[1][5 + b] = h1.py[b];
  }
  for (int i = 0; i < 4; ++i) {
    o.snap[0][10 + i] = h2.vx[i]; o.snap[0][14 + i] = h2.vy[i]; o.snap[0][18 + i] = h2.ang[i]; o.snap[0][22 + i] = h2.w[i];
    o.snap[1][10 + i] = h1.vx[i]; o.snap[1][14 + i] = h1.vy[i]; o.snap[1][18 + i] = h1.ang[i]; o.snap[1][22 + i] = h1.w[i];
  }
  o.steps = E.steps; o.score_blue = E.score_blue; o.score_red = E.score_red;
  o.mode = (uint8_t)META_MODE(E.meta);
  o.hist_empty = (E.meta & META_HE) ? 1 : 0;
  o.has_uint32 = E.rng.has32 ? 1 : 0;
  o.uinteger = E.rng.u32;
  o.pad = 0;
  o.pcg_state_hi = E.rng.shi; o.pcg_state_lo = E.rng.slo;
  o.pcg_inc_hi = E.rng.ihi; o.pcg_inc_lo = E.rng.ilo;
  const int par = (E.meta & META_PAR) ? 1 : 0;
  const int nc = META_NC(E.meta);
  o.n_arb = (uint8_t)nc;
  for (int k = 0; k < MAXA; ++k) {
    ms_arbiter_state& A = o.arb[k];
    memset(&A, 0, sizeof(A));
    if (k >= nc) continue;
    const uint32_t h = *plane<uint32_t>(a, OFF_CH, par * MAXA + k);
    A.pair = h & 63u; A.count = (h >> 6) & 3u; A.idle = (h >> 8) & 3u;
    A.hash[0] = (h >> 16) & 0xffu; A.hash[1] = (h >> 24) & 0xffu;
    const float4 j = *plane<float4>(a, OFF_CJ, par * MAXA + k);
    A.jn[0] = j.x; A.jt[0] = j.y; A.jn[1] = j.z; A.jt[1] = j.w;
  }
}

// snap[1] (t-1) is not stored: it is the body state itself, which every state the library or
// the oracle exports satisfies.
__global__ void ms_import_kernel(DevState S, const ms_env_state* __restrict__ in) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const At a = env_at(S, e);
  const ms_env_state& o = in[e];
  Env E;
  for (int b = 0; b < 5; ++b) {
    const ms_body_state& d = o.body[b];
    E.px[b] = d.px; E.py[b] = d.py; E.vx[b] = d.vx; E.vy[b] = d.vy;
    if (b < 4) E.ang[b] = d.angle;
    E.w[b] = d.w; E.vbx[b] = d.vbx; E.vby[b] = d.vby; E.wb[b] = d.wb;
  }
  E.steps = o.steps; E.score_blue = o.score_blue; E.score_red = o.score_red;
  const int nc = o.n_arb > MAXA ? MAXA : o.n_arb;
  E.meta = (uint32_t)(o.mode & 3) | (o.hist_empty ? META_HE : 0u) | ((uint32_t)nc << 8) | (o.has_uint32 ? META_H32 : 0u);
  E.rng.shi = o.pcg_state_hi; E.rng.slo = o.pcg_state_lo; E.rng.ihi = o.pcg_inc_hi; E.rng.ilo = o.pcg_inc_lo;
  E.rng.has32 = o.has_uint32; E.rng.u32 = o.uinteger;
  Snap h2;
  for (int b = 0; b < 5; ++b) { h2.px[b] = o.snap[0][b]; h2.py[b] = o.snap[0][5 + b]; }
  for (int i = 0; i < 4; ++i) {
    h2.vx[i] = o.snap[0][10 + i]; h2.vy[i] = o.snap[0][14 + i]; h2.ang[i] = o.snap[0][18 + i]; h2.w[i] = o.snap[0][22 + i];
  }
  snap_store(a, h2);
  for (int k = 0; k < nc; ++k) {
    const ms_arbiter_state& A = o.arb[k];
    *plane<uint32_t>(a, OFF_CH, k) = (uint32_t)(A.pair & 63u) | ((uint32_t)(A.count & 3u) << 6) |
                                 ((uint32_t)(A.idle & 3u) << 8) | ((uint32_t)A.hash[0] << 16) | ((uint32_t)A.hash[1] << 24);
    *plane<float4>(a, OFF_CJ, k) = make_float4(A.jn[0], A.jt[0], A.jn[1], A.jt[1]);
  }
  store_rng(a, E);
  store_bodies(a, E);
  store_scalars(a, E);
}

__global__ void ms_debug_rewards_kernel(Params P, int64_t n, const float* __restrict__ prev, const float* __restrict__ cur,
                                        const int8_t* __restrict__ goal, const uint8_t* __restrict__ terminal,
                                        const int32_t* __restrict__ score, float* __restrict__ rew) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float pvx[5], pvy[5], cux[5], cuy[5];
  for (int b = 0; b < 5; ++b) {
    pvx[b] = prev[e * 10 + 2 * b]; pvy[b] = prev[e * 10 + 2 * b + 1];
    cux[b] = cur[e * 10 + 2 * b]; cuy[b] = cur[e * 10 + 2 * b + 1];
  }
  const float r = blue_reward(P, pvx, pvy, cux, cuy, goal[e], terminal[e] != 0, score[2 * e], score[2 * e + 1]);
  rew[2 * e] = r;
  rew[2 * e + 1] = r;
}

#endif  // MS_KSTEP_TU

// small batches: one env per lane group (ms_step when envs x 8 <= the device's lanes)
#include "ms_group.inc"
// two lanes per env, two waves per SIMD
#include "ms_pair.inc"

// ms_kstep.hip: launch the K-step kernel of lane group G (2: lane pairs; 8, 16: lane groups) on stream st
hipError_t ms_kstep_launch(int G, int param_mode, dim3 grid, hipStream_t st, const DevState& S, const Params& P, int K,
                           const float* actions, float* obs, float* rew, uint8_t* term, uint8_t* trunc, int8_t* goal,
                           int32_t* score, Counters* ctr, int group_solve);

#ifndef MS_KSTEP_TU
// =============================================================================================
// Host side: the C-ABI
// =============================================================================================
struct ms_env {
  int device;
  hipStream_t stream;
  int64_t n;
  int group;       // ms_step: lanes per env of the lane-group kernel (8 or 16), 0: one lane per env
  int group_solve; // the lane-group kernel's contact-solve schedule (ms_set_group_solve)
  int64_t lanes;   // the device's wave slots at one wave per SIMD x 64 (4 x CUs x 64)
  Params P;
  bool default_params;  // P == default_params() up to max_steps/autoreset: specialised kernel
  int param_mode;       // kernel_params' mode of the lane-pair and lane-group kernels (2: default physics)
  DevState S;
  void* mem;
  Counters* ctr;
  ms_config cfg;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                                      \
  do {                                                                                                 \
    hipError_t _e = (x);                                                                               \
    if (_e != hipSuccess) return fail(MS_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e));     \
  } while (0)

extern "C" {

const char* ms_last_error(void) { return g_err.c_str(); }
int ms_abi_version(void) { return MS_ABI_VERSION; }

void ms_config_default(ms_config* c) {
  memset(c, 0, sizeof(*c));
  c->max_velocity = 200; c->agent_mass = 10; c->ball_mass = 1; c->agent_moment = 100;
  c->ball_moment = 10; c->agent_friction = 0.99; c->ball_friction = 0.97;
  c->agent_elasticity = 0.2; c->agent_surface_friction = 0.8; c->ball_elasticity = 0.95;
  c->ball_surface_friction = 0.2; c->action_force_max = 150000.0; c->action_torque_max = 1000.0;
  c->max_angular_velocity = 1000.0 / 100.0;
  c->ball_proximity_multiplier = 0.002; c->move_ball_to_goal_multiplier = 0.1;
  c->alive_penalty = 0.00001; c->goal_scored_reward = 4.0; c->goal_conceded_penalty = 0.0;
  c->score_difference_multiplier = 0.0; c->max_steps = 1000; c->autoreset = 1;
}

// --- numpy SeedSequence (bit_generator.pyx) -> PCG64 seeding (pcg64.c pcg64_set_seed) ------
static void seed_sequence_pcg64(const uint32_t* entropy, int n_words, uint64_t out[4]) {
  const uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
  const uint32_t MIX_MULT_L = 0xca01f9ddu, MIX_MULT_R = 0x4973f715u;
  uint32_t pool[4];
  uint32_t hash_const = INIT_A;
  auto hashmix = [&](uint32_t value) {
    value ^= hash_const;
    hash_const *= MULT_A;
    value *= hash_const;
    value ^= value >> 16;
    return value;
  };
  auto mix = [](uint32_t x, uint32_t y) {
    uint32_t result = MIX_MULT_L * x - MIX_MULT_R * y;
    result ^= result >> 16;
    return result;
  };
  for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < n_words ? entropy[i] : 0u);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
  for (int s = 4; s < n_words; ++s)
    for (int d = 0; d < 4; ++d) pool[d] = mix(pool[d], hashmix(entropy[s]));
  uint32_t words[8];
  uint32_t hc = INIT_B;
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i % 4];
    v ^= hc;
    hc *= MULT_B;
    v *= hc;
    v ^= v >> 16;
    words[i] = v;
  }
  uint64_t v[4];
  for (int i = 0; i < 4; ++i) v[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
  // pcg64_set_seed(seed = v[0:2], inc = v[2:4]); PCG_128BIT_CONSTANT(high, low)
  typedef unsigned __int128 u128;
  const u128 MULT = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
  u128 initstate = ((u128)v[0] << 64) | v[1];
  u128 initseq = ((u128)v[2] << 64) | v[3];
  u128 inc = (initseq << 1) | 1u;
  u128 st = 0;
  st = st * MULT + inc;
  st += initstate;
  st = st * MULT + inc;
  out[0] = (uint64_t)(st >> 64); out[1] = (uint64_t)st;
  out[2] = (uint64_t)(inc >> 64); out[3] = (uint64_t)inc;
}

int ms_seed_pcg64(const uint32_t* entropy, int n_words, uint64_t out[4]) {
  if (!entropy || n_words < 1 || !out) return fail(MS_ERR_INVALID_ARGUMENT, "ms_seed_pcg64: bad arguments");
  seed_sequence_pcg64(entropy, n_words, out);
  return MS_OK;
}

int ms_seed_pcg64_range(uint64_t seed0, int64_t n, uint64_t* out) {
  if (!out || n < 0) return fail(MS_ERR_INVALID_ARGUMENT, "ms_seed_pcg64_range: bad arguments");
  for (int64_t i = 0; i < n; ++i) {
    uint64_t s = seed0 + (uint64_t)i;
    uint32_t w[2] = {(uint32_t)s, (uint32_t)(s >> 32)};
    seed_sequence_pcg64(w, w[1] ? 2 : 1, out + 4 * i);
  }
  return MS_OK;
}

// --- parameter setup: identical float arithmetic to oracle orc_params_init (ORC_F32) -------
static void make_params(const ms_config* cfg, Params* P) {
  memset(P, 0, sizeof(*P));
  P->dt = (float)(1.0 / 60.0);
  P->bias_coef = (float)(1.0 - pow(pow(1.0 - 0.1, 60.0), 1.0 / 60.0));
  P->slop = 0.1f;
  const float am = (float)cfg->agent_mass, bm = (float)cfg->ball_mass;
  const float ai = (float)cfg->agent_moment, bi = (float)cfg->ball_moment;
  for (int i = 0; i < 4; ++i) { P->m_inv[i] = 1.0f / am; P->i_inv[i] = 1.0f / ai; }
  P->m_inv[4] = 1.0f / bm; P->i_inv[4] = 1.0f / bi;
  P->m_inv[5] = 0.0f; P->i_inv[5] = 0.0f;
  P->agent_damp = (float)cfg->agent_friction;
  P->ball_damp = (float)cfg->ball_friction;
  P->vmax = (float)cfg->max_velocity;
  P->force_max = (float)cfg->action_force_max;
  P->torque_max = (float)cfg->action_torque_max;
  P->obs_vmax = (float)(cfg->max_velocity > 1e-6 ? cfg->max_velocity : 1e-6);
  P->obs_wmax = (float)(cfg->max_angular_velocity > 1e-6 ? cfg->max_angular_velocity : 1e-6);
  P->fast_div = (P->obs_vmax >= 0x1p-20f && P->obs_vmax <= 0x1p12f && P->obs_wmax >= 0x1p-20f &&
                 P->obs_wmax <= 0x1p12f) ? 1 : 0;
  const float ea = (float)cfg->agent_elasticity, ua = (float)cfg->agent_surface_friction;
  const float eb = (float)cfg->ball_elasticity, ub = (float)cfg->ball_surface_friction;
  const float ew = 0.95f, uw = 0.2f, eg = 0.95f, ug = 0.0f;
  P->e_aa = ea * ea; P->u_aa = ua * ua;
  P->e_ab = eb * ea; P->u_ab = ub * ua;
  P->e_aw = ew * ea; P->u_aw = uw * ua;
  P->e_ag = eg * ea; P->u_ag = ug * ua;
  P->e_bw = eb * ew; P->u_bw = ub * uw;
  P->prox_mult = (float)cfg->ball_proximity_multiplier;
  P->goal_mult = (float)cfg->move_ball_to_goal_multiplier;
  P->alive = (float)cfg->alive_penalty;
  P->goal_reward = (float)cfg->goal_scored_reward;
  P->concede_penalty = (float)cfg->goal_conceded_penalty;
  P->score_diff_mult = (float)cfg->score_difference_multiplier;
  P->max_steps = cfg->max_steps;
  P->autoreset = cfg->autoreset;
  static const double DEF[8][5] = {{10, 10, 790, 10, 2},   {10, 590, 790, 590, 2}, {10, 10, 10, 225, 2},
                                   {10, 375, 10, 590, 2},  {790, 10, 790, 225, 2}, {790, 375, 790, 590, 2},
                                   {10, 225, 10, 375, 1},  {790, 225, 790, 375, 1}};
  for (int s = 0; s < 8; ++s) {
    Seg& g = P->seg[s];
    g.ax = (float)DEF[s][0]; g.ay = (float)DEF[s][1]; g.bx = (float)DEF[s][2]; g.by = (float)DEF[s][3];
    g.r = (float)DEF[s][4];
    const float dx = g.bx - g.ax, dy = g.by - g.ay;
    const float len = sqrtf(dx * dx + dy * dy);
    const float inv = 1.0f / (len + 1.17549435082228750797e-38f);
    const float ux = dx * inv, uy = dy * inv;
    g.nx = -uy; g.ny = ux;
    float l, r, bt, t;
    if (g.ax < g.bx) { l = g.ax; r = g.bx; } else { l = g.bx; r = g.ax; }
    if (g.ay < g.by) { bt = g.ay; t = g.by; } else { bt = g.by; t = g.ay; }
    g.bb[0] = l - g.r; g.bb[1] = bt - g.r; g.bb[2] = r + g.r; g.bb[3] = t + g.r;
  }
}

// P equals the compile-time default_params() bit for bit, apart from the runtime fields
static bool params_are_default(const Params& P) {
  Params d = default_params();
  d.max_steps = P.max_steps;
  d.autoreset = P.autoreset;
  return memcmp(&d, &P, sizeof(Params)) == 0;
}
// kernel_params' mode for P: 1 all default, 2 default physics (any reward multipliers), 0 otherwise
static int param_mode(const Params& P) {
  if (params_are_default(P)) return 1;
  Params d = default_params();
  d.max_steps = P.max_steps;
  d.autoreset = P.autoreset;
  d.prox_mult = P.prox_mult;
  d.goal_mult = P.goal_mult;
  d.alive = P.alive;
  d.goal_reward = P.goal_reward;
  d.concede_penalty = P.concede_penalty;
  d.score_diff_mult = P.score_diff_mult;
  return memcmp(&d, &P, sizeof(Params)) == 0 ? 2 : 0;
}

int ms_config_specialised(const ms_config* cfg) {
  if (!cfg) return fail(MS_ERR_INVALID_ARGUMENT, "ms_config_specialised: null config") * -1;
  Params P;
  make_params(cfg, &P);
  return param_mode(P);
}

static inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

// ms_step's default kernel: the lane-group kernel (8 lanes per env) while the batch fits the
// device's SIMDs at one wave each with 8 lanes per env, the lane-pair kernel (two lanes per env,
// two waves per SIMD) above that — faster than one lane per env at every size measured
// (16,384-262,144 envs)
static int auto_group(int64_t n, int64_t lanes) { return n * 8 <= lanes ? 8 : 2; }

int ms_create(const ms_config* cfg, int64_t n_envs, int device, void* stream, ms_env** out) {
  if (!out || n_envs <= 0) return fail(MS_ERR_INVALID_ARGUMENT, "ms_create: n_envs must be > 0");
  if (n_envs > ((int64_t)1 << 31)) return fail(MS_ERR_INVALID_ARGUMENT, "ms_create: n_envs too large");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MS_ERR_NO_DEVICE, "ms_create: no HIP device");
  if (device < 0 || device >= ndev) return fail(MS_ERR_INVALID_ARGUMENT, "ms_create: bad device index");
  HIPCHK(hipSetDevice(device));
  ms_env* h = new ms_env();
  h->device = device;
  h->stream = (hipStream_t)stream;
  h->n = n_envs;
  if (cfg) h->cfg = *cfg; else ms_config_default(&h->cfg);
  make_params(&h->cfg, &h->P);
  h->default_params = params_are_default(h->P);
  h->param_mode = param_mode(h->P);
  {  // ms_step's default kernel by batch size (auto_group)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    h->lanes = (int64_t)4 * cus * 64;
    h->group = auto_group(n_envs, h->lanes);
  }
  const size_t n = (size_t)n_envs;
  const size_t total = (size_t)((n + BLK - 1) / BLK) * BLOCK_BYTES;  // state blocks, the last one padded
  char* base = nullptr;
  if (hipMalloc((void**)&base, total) != hipSuccess) {
    delete h;
    return fail(MS_ERR_OUT_OF_MEMORY, "ms_create: hipMalloc of device state failed");
  }
  h->mem = base;
  h->S.blocks = base;
  h->S.n = n_envs;
  h->S.stamps = nullptr;
  // contact-slot spill for pile-ups beyond KREG contacts: reserved address space, touched
  // only by envs with more than KREG contacts (no traffic in ordinary play)
  if (hipMalloc(&h->S.SP, sizeof(CSlot) * SPW * n) != hipSuccess) {
    (void)hipFree(h->mem);
    delete h;
    return fail(MS_ERR_OUT_OF_MEMORY, "ms_create: hipMalloc of the contact spill buffer failed");
  }
#ifdef MS_STAMPS
  // one row per wave: 64-env blocks, or the lane-group kernel's waves of 64 / G envs (G <= 16)
  if (hipMalloc((void**)&h->S.stamps, sizeof(unsigned long long) * MS_NSTAMP * ((n + 3) / 4)) != hipSuccess)
    return fail(MS_ERR_OUT_OF_MEMORY, "stamps");
  (void)hipMemsetAsync(h->S.stamps, 0, sizeof(unsigned long long) * MS_NSTAMP * ((n + 3) / 4), h->stream);
#endif
  const size_t nblk = (n + BLK - 1) / BLK;
  if (hipMalloc((void**)&h->ctr, sizeof(Counters)) != hipSuccess ||
      hipMalloc((void**)&h->S.tally, sizeof(Tally) * nblk) != hipSuccess) {
    (void)hipFree(h->mem);
    (void)hipFree(h->S.SP);
    (void)hipFree(h->ctr);
    delete h;
    return fail(MS_ERR_OUT_OF_MEMORY, "ms_create: hipMalloc of counters failed");
  }
  HIPCHK(hipMemsetAsync(h->S.tally, 0, sizeof(Tally) * nblk, h->stream));
  HIPCHK(hipMemsetAsync(h->mem, 0, total, h->stream));
  Counters c0 = {0, 0, (long long)INT64_MAX};
  HIPCHK(hipMemcpyAsync(h->ctr, &c0, sizeof(c0), hipMemcpyHostToDevice, h->stream));
  // Game.__init__: entropy-seeded default_rng() + reset() (game.py:17, 74)
  uint64_t* hp = (uint64_t*)malloc(sizeof(uint64_t) * 4 * n);
  std::random_device rd;
  for (size_t i = 0; i < n; ++i) {
    uint32_t w[4] = {rd(), rd(), rd(), rd()};
    seed_sequence_pcg64(w, 4, hp + 4 * i);
  }
  uint64_t* dp = nullptr;
  if (hipMalloc((void**)&dp, sizeof(uint64_t) * 4 * n) != hipSuccess) {
    free(hp);
    return fail(MS_ERR_OUT_OF_MEMORY, "ms_create: hipMalloc of seed buffer failed");
  }
  HIPCHK(hipMemcpyAsync(dp, hp, sizeof(uint64_t) * 4 * n, hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(ms_reset_kernel, dim3(grid_for(n_envs, MS_BLOCK)), dim3(MS_BLOCK), 0, h->stream, h->S, h->P,
                     (const uint64_t*)dp, (const uint8_t*)nullptr, (int)MS_SPAWN_RANDOM, 1, (float*)nullptr,
                     Ring{nullptr, 0, 0, 0});
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  (void)hipFree(dp);
  free(hp);
  *out = h;
  return MS_OK;
}

int ms_destroy(ms_env* h) {
  if (!h) return MS_OK;
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->stream);
  (void)hipFree(h->mem);
  (void)hipFree(h->S.SP);
  (void)hipFree(h->ctr);
  (void)hipFree(h->S.tally);
  delete h;
  return MS_OK;
}

int ms_set_stream(ms_env* h, void* stream) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_set_stream: null handle");
  h->stream = (hipStream_t)stream;
  return MS_OK;
}

int64_t ms_num_envs(const ms_env* h) { return h ? h->n : -1; }

int ms_reset(ms_env* h, const uint64_t* pcg, const uint8_t* mask, int mode, float* obs) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_reset: null handle");
  if (mode < 0 || mode > 2) return fail(MS_ERR_INVALID_ARGUMENT, "ms_reset: mode must be 0, 1 or 2");
  hipLaunchKernelGGL(ms_reset_kernel, dim3(grid_for(h->n, MS_BLOCK)), dim3(MS_BLOCK), 0, h->stream, h->S, h->P, pcg,
                     mask, mode, 0, obs, Ring{nullptr, 0, 0, 0});
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_step(ms_env* h, const float* actions, float* obs, float* rew, uint8_t* term, uint8_t* trunc, int8_t* goal,
            int32_t* score) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step: null handle");
  if (!actions || !obs) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step: actions and obs are required");
  if (((uintptr_t)actions & 15u) || ((uintptr_t)obs & 7u) || ((uintptr_t)rew & 15u) || ((uintptr_t)term & 3u) ||
      ((uintptr_t)trunc & 3u) || ((uintptr_t)score & 7u))
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_step: misaligned buffer (actions/rew 16 B, obs/score 8 B, flags 4 B)");
  [[maybe_unused]] const unsigned nblk = grid_for(h->n, MS_BLOCK);
  if (h->group == 2) {
    const dim3 grid(grid_for(h->n, pr::EPW)), blk(64);
    if (h->param_mode == 1)
      hipLaunchKernelGGL(ms_step_pair_kernel<1>, grid, blk, 0, h->stream, h->S, h->P, actions, obs, rew, term,
                         trunc, goal, score, h->ctr);
    else if (h->param_mode == 2)
      hipLaunchKernelGGL(ms_step_pair_kernel<2>, grid, blk, 0, h->stream, h->S, h->P, actions, obs, rew, term,
                         trunc, goal, score, h->ctr);
    else
      hipLaunchKernelGGL(ms_step_pair_kernel<0>, grid, blk, 0, h->stream, h->S, h->P, actions, obs, rew,
                         term, trunc, goal, score, h->ctr);
  } else {
#ifdef MS_PAIR_ONLY  // experiment builds (tools/variants.py): the lane-pair kernels only
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_step: this experiment build has the lane-pair kernel only");
#else
  if (h->group > 0) {
    const int G = h->group;
    const dim3 grid(grid_for(h->n, 64 / G));
#define MS_GROUP_LAUNCH(PM, GG)                                                                                  \
  hipLaunchKernelGGL((ms_step_group_kernel<PM, GG>), grid, dim3(64), 0, h->stream, h->S, h->P, actions, obs, rew, term, \
                     trunc, goal, score, h->ctr, h->group_solve)
    if (G == 8) {
      if (h->param_mode == 1) MS_GROUP_LAUNCH(1, 8);
      else if (h->param_mode == 2) MS_GROUP_LAUNCH(2, 8);
      else MS_GROUP_LAUNCH(0, 8);
    } else {
      if (h->param_mode == 1) MS_GROUP_LAUNCH(1, 16);
      else if (h->param_mode == 2) MS_GROUP_LAUNCH(2, 16);
      else MS_GROUP_LAUNCH(0, 16);
    }
#undef MS_GROUP_LAUNCH
  } else if (h->default_params) {
    hipLaunchKernelGGL(ms_step_kernel<true>, dim3(nblk), dim3(MS_BLOCK), 0, h->stream, h->S, h->P, actions, obs, rew,
                       term, trunc, goal, score, h->ctr);
  } else {
    hipLaunchKernelGGL(ms_step_kernel<false>, dim3(nblk), dim3(MS_BLOCK), 0, h->stream, h->S, h->P, actions, obs,
                       rew, term, trunc, goal, score, h->ctr);
  }
#endif
  }
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_step_n(ms_env* h, int K, const float* actions, float* obs, float* rew, uint8_t* term, uint8_t* trunc,
              int8_t* goal, int32_t* score) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_n: null handle");
  if (K < 1) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_n: K < 1");
  if (!actions || !obs) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_n: actions and obs are required");
  if (((uintptr_t)actions & 15u) || ((uintptr_t)obs & 7u) || ((uintptr_t)rew & 15u) || ((uintptr_t)term & 3u) ||
      ((uintptr_t)trunc & 3u) || ((uintptr_t)score & 7u))
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_n: misaligned buffer (actions/rew 16 B, obs/score 8 B, flags 4 B)");
  // the K-step kernels live in their own translation unit (ms_kstep.hip, built without machine LICM)
  const int G = h->group;
#ifdef MS_PAIR_ONLY
  if (G == 2) {
#else
  if (G == 2 || G == 8 || G == 16) {
#endif
    const dim3 grid(grid_for(h->n, G == 2 ? pr::EPW : 64 / G));
    HIPCHK(ms_kstep_launch(G, h->param_mode, grid, h->stream, h->S, h->P, K, actions, obs, rew, term, trunc, goal,
                           score, h->ctr, h->group_solve));
    return MS_OK;
  }
  const int64_t n = h->n;
  for (int k = 0; k < K; ++k) {
    const int64_t o = (int64_t)k * n;
    const int rc = ms_step(h, actions + o * 12, obs + o * 264, rew ? rew + o * 4 : nullptr, term ? term + o * 4 : nullptr,
                           trunc ? trunc + o * 4 : nullptr, goal ? goal + o : nullptr, score ? score + o * 2 : nullptr);
    if (rc != MS_OK) return rc;
  }
  return MS_OK;
}

int ms_set_lane_group(ms_env* h, int lanes) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_set_lane_group: null handle");
  if (lanes < 0) lanes = auto_group(h->n, h->lanes);
  if (lanes != 0 && lanes != 2 && lanes != 8 && lanes != 16)
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_set_lane_group: lanes per env must be 0, 2, 8, 16 or negative (automatic)");
  h->group = lanes;
  return MS_OK;
}

int ms_get_lane_group(const ms_env* h) { return h ? h->group : -1; }

int ms_set_group_solve(ms_env* h, int mode) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_set_group_solve: null handle");
  if (mode < 0 || mode > 2)
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_set_group_solve: mode must be 0 (automatic), 1 (serial) or 2 (rounds)");
  h->group_solve = mode;
  return MS_OK;
}

int ms_get_group_solve(const ms_env* h) { return h ? h->group_solve : -1; }

const char* ms_step_kernel_name(const ms_env* h) {
  if (!h) return "";
  if (h->group == 2) return "ms_step_pair_kernel";
  if (h->group > 0) return "ms_step_group_kernel";
  return "ms_step_kernel";
}

// Frame-ring arguments: frames 16-B aligned, R even and >= 4, window pos..pos+2 inside the row.
static int ring_check(const char* fn, const float* frames, int R, int pos, int wrap) {
  if (!frames || ((uintptr_t)frames & 15u) || R < 4 || (R & 1) || pos < 0 || pos + 3 > R || (wrap != 0 && wrap != 1)) {
    const std::string msg = std::string(fn) +
                            ": bad frame ring (frames 16-B aligned, R even >= 4, 0 <= pos <= R-3, wrap 0 or 1; got R=" +
                            std::to_string(R) + " pos=" + std::to_string(pos) + " wrap=" + std::to_string(wrap) + ")";
    return fail(MS_ERR_INVALID_ARGUMENT, msg);
  }
  return MS_OK;
}

int ms_reset_ring(ms_env* h, const uint64_t* pcg, const uint8_t* mask, int mode, float* frames, int R, int pos) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_reset_ring: null handle");
  if (mode < 0 || mode > 2) return fail(MS_ERR_INVALID_ARGUMENT, "ms_reset_ring: mode must be 0, 1 or 2");
  if (int rc = ring_check("ms_reset_ring", frames, R, pos, 0)) return rc;
  hipLaunchKernelGGL(ms_reset_kernel, dim3(grid_for(h->n, MS_BLOCK)), dim3(MS_BLOCK), 0, h->stream, h->S, h->P, pcg,
                     mask, mode, 0, (float*)nullptr, Ring{frames, R, pos, 0});
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_step_ring(ms_env* h, const float* actions, float* frames, int R, int pos, int wrap, float* rew, uint8_t* term,
                 uint8_t* trunc, int8_t* goal, int32_t* score) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_ring: null handle");
  if (!actions) return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_ring: actions are required");
  if (int rc = ring_check("ms_step_ring", frames, R, pos, wrap)) return rc;
  if (((uintptr_t)actions & 15u) || ((uintptr_t)rew & 15u) || ((uintptr_t)term & 3u) || ((uintptr_t)trunc & 3u) ||
      ((uintptr_t)score & 7u))
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_ring: misaligned buffer (actions/rew 16 B, score 8 B, flags 4 B)");
  const Ring rg{frames, R, pos, wrap};
#ifdef MS_PAIR_ONLY
  (void)rg;
  return fail(MS_ERR_INVALID_ARGUMENT, "ms_step_ring: this experiment build has the lane-pair kernel only");
#else
  if (h->group == 2) {  // the lane-pair launch (ms_pair.inc), as ms_step takes it
    const dim3 grid(grid_for(h->n, pr::EPW));
    if (h->param_mode == 1)
      hipLaunchKernelGGL(ms_step_pair_ring_kernel<1>, grid, dim3(64), 0, h->stream, h->S, h->P, actions, rg, rew, term,
                         trunc, goal, score, h->ctr);
    else if (h->param_mode == 2)
      hipLaunchKernelGGL(ms_step_pair_ring_kernel<2>, grid, dim3(64), 0, h->stream, h->S, h->P, actions, rg, rew, term,
                         trunc, goal, score, h->ctr);
    else
      hipLaunchKernelGGL(ms_step_pair_ring_kernel<0>, grid, dim3(64), 0, h->stream, h->S, h->P, actions, rg, rew, term,
                         trunc, goal, score, h->ctr);
  } else if (h->default_params)
    hipLaunchKernelGGL(ms_step_ring_kernel<true>, dim3(grid_for(h->n, MS_BLOCK)), dim3(MS_BLOCK), 0, h->stream, h->S,
                       h->P, actions, rg, rew, term, trunc, goal, score, h->ctr);
  else
    hipLaunchKernelGGL(ms_step_ring_kernel<false>, dim3(grid_for(h->n, MS_BLOCK)), dim3(MS_BLOCK), 0, h->stream, h->S,
                       h->P, actions, rg, rew, term, trunc, goal, score, h->ctr);
#endif
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_observe(ms_env* h, float* frames) {
  if (!h || !frames) return fail(MS_ERR_INVALID_ARGUMENT, "ms_observe: bad arguments");
  hipLaunchKernelGGL(ms_observe_kernel, dim3(grid_for(h->n, MS_BLOCK)), dim3(MS_BLOCK), 0, h->stream, h->S, h->P,
                     frames);
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_export_state(ms_env* h, ms_env_state* dst) {
  if (!h || !dst) return fail(MS_ERR_INVALID_ARGUMENT, "ms_export_state: bad arguments");
  hipLaunchKernelGGL(ms_export_kernel, dim3(grid_for(h->n, 128)), dim3(128), 0, h->stream, h->S, dst);
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_import_state(ms_env* h, const ms_env_state* src) {
  if (!h || !src) return fail(MS_ERR_INVALID_ARGUMENT, "ms_import_state: bad arguments");
  hipLaunchKernelGGL(ms_import_kernel, dim3(grid_for(h->n, 128)), dim3(128), 0, h->stream, h->S, src);
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_debug_rewards(ms_env* h, const float* prev_pos, const float* cur_pos, const int8_t* goal,
                     const uint8_t* terminal, const int32_t* score, float* rew) {
  if (!h || !prev_pos || !cur_pos || !goal || !terminal || !score || !rew)
    return fail(MS_ERR_INVALID_ARGUMENT, "ms_debug_rewards: bad arguments");
  hipLaunchKernelGGL(ms_debug_rewards_kernel, dim3(grid_for(h->n, 128)), dim3(128), 0, h->stream, h->P, h->n,
                     prev_pos, cur_pos, goal, terminal, score, rew);
  HIPCHK(hipGetLastError());
  return MS_OK;
}

int ms_get_stats(ms_env* h, ms_stats* out) {
  if (!h || !out) return fail(MS_ERR_INVALID_ARGUMENT, "ms_get_stats: bad arguments");
  Counters c;
  HIPCHK(hipMemcpyAsync(&c, h->ctr, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  out->arbiter_overflow = c.overflow;
  out->nonfinite_envs = c.nonfinite;
  out->first_nonfinite_env = c.first_bad == (long long)INT64_MAX ? -1 : c.first_bad;
  const size_t nblk = (size_t)((h->n + BLK - 1) / BLK);
  Tally* t = (Tally*)malloc(sizeof(Tally) * nblk);
  if (!t) return fail(MS_ERR_OUT_OF_MEMORY, "ms_get_stats: host buffer");
  if (hipMemcpy(t, h->S.tally, sizeof(Tally) * nblk, hipMemcpyDeviceToHost) != hipSuccess) {
    free(t);
    return fail(MS_ERR_HIP, "ms_get_stats: reading the per-block tally failed");
  }
  out->env_steps = out->cache_entries_read = out->cache_entries_written = 0;
  for (size_t b = 0; b < nblk; ++b) {
    out->cache_entries_read += t[b].read;
    out->cache_entries_written += t[b].written;
    out->env_steps += t[b].steps;
  }
  free(t);
  return MS_OK;
}

#ifdef MS_STAMPS
int ms_debug_stamps(ms_env* h, void** ptr, int64_t* n_waves) {
  *ptr = h->S.stamps;
  *n_waves = h->group > 0 ? (h->n + 64 / h->group - 1) / (64 / h->group) : (h->n + MS_BLOCK - 1) / MS_BLOCK;
  return MS_OK;
}
#endif

int ms_reset_stats(ms_env* h) {
  if (!h) return fail(MS_ERR_INVALID_ARGUMENT, "ms_reset_stats: null handle");
  Counters c0 = {0, 0, (long long)INT64_MAX};
  HIPCHK(hipMemcpyAsync(h->ctr, &c0, sizeof(c0), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemsetAsync(h->S.tally, 0, sizeof(Tally) * (size_t)((h->n + BLK - 1) / BLK), h->stream));
  // c0 lives on this stack frame: the copy must have read it before the call returns
  HIPCHK(hipStreamSynchronize(h->stream));
  return MS_OK;
}

}  // extern "C"
#endif  // MS_KSTEP_TU
