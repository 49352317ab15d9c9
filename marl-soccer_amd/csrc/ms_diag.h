// ms_diag.h — diagnostic hooks of the step kernels (not product behaviour).
//
// STAMP(k) and the ACC_* accumulators compile to nothing unless the library is built with -DMS_STAMPS
// (tools/stamps.py builds libmarlsoccer_stamps.so that way, a separate library the product never
// loads): then every wave records s_memtime / s_memrealtime at the kernel's phase boundaries into
// DevState::stamps. They change no arithmetic and no stored value of the step.
#pragma once

#ifdef MS_STAMPS
// slot k: s_memtime (shader cycles; its counter is per XCD, so cross-wave comparisons hold within
// an XCD only); slot 24 + k: s_memrealtime (the 100-MHz clock every XCD shares: the launch timeline)
#define STAMP(k)                                                                         \
  do {                                                                                   \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                                \
    unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                            \
    const unsigned long long act_ = __ballot(1);                                          \
    if ((int)(threadIdx.x & 63) == __ffsll((long long)act_) - 1 && S.stamps) {            \
      S.stamps[stamp_row * MS_NSTAMP + (k)] = t_;                                        \
      S.stamps[stamp_row * MS_NSTAMP + 24 + (k)] = r_;                                   \
    }                                                                                    \
  } while (0)
// cycles spent inside a region of a divergent loop, accumulated per lane; the wave's figure is
// the maximum over its lanes (the lane that ran the most iterations), written to slot k
#define ACC_DECL(v) unsigned long long v = 0
#define ACC_BEGIN(v) const unsigned long long v##_t0 = __builtin_amdgcn_s_memtime()
#define ACC_END(v) v += __builtin_amdgcn_s_memtime() - v##_t0
#define ACC_INC(v) v++
#define ACC_STORE(v, k)                                                                    \
  do {                                                                                   \
    unsigned long long m_ = v;                                                           \
    for (int o_ = 32; o_ > 0; o_ >>= 1) {                                                \
      const unsigned long long x_ = __shfl_xor(m_, o_);                                  \
      m_ = x_ > m_ ? x_ : m_;                                                            \
    }                                                                                    \
    if ((threadIdx.x & 63) == 0 && S.stamps) S.stamps[stamp_row * MS_NSTAMP + (k)] = m_;       \
  } while (0)
#else
#define STAMP(k) do { } while (0)
#define ACC_DECL(v) do { } while (0)
#define ACC_BEGIN(v) do { } while (0)
#define ACC_END(v) do { } while (0)
#define ACC_INC(v) do { } while (0)
#define ACC_STORE(v, k) do { } while (0)
#endif
#define MS_NSTAMP 48  // [0, 24): cycles and accumulators; [24, 48): real time of stamps 0..23
