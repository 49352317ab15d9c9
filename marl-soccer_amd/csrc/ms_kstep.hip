// ms_kstep.hip — the open-loop K-step kernels of ms_step_n (ms_step_pair_n_kernel,
// ms_step_group_n_kernel) in a translation unit of their own, built with LLVM's machine loop-invariant
// code motion off (build_native.py): each kernel runs the per-step device code of ms_pair.inc /
// ms_group.inc in a K-iteration loop, and hoisting what a step derives from its loop-invariant inputs
// (addresses, masks, Params constants) out of that loop held them across the whole step, which needs
// ~240 of the 256 registers by itself: 44-76 B/lane of scratch with LICM, 0 without.
// The per-step kernels stay in ms_env.hip, built with the default pipeline.
#define MS_KSTEP_TU 1
#include "ms_env.hip"

hipError_t ms_kstep_launch(int G, int param_mode, dim3 grid, hipStream_t st, const DevState& S, const Params& P, int K,
                           const float* actions, float* obs, float* rew, uint8_t* term, uint8_t* trunc, int8_t* goal,
                           int32_t* score, Counters* ctr, int group_solve) {
#define MS_PAIR_N(PM)                                                                                              \
  hipLaunchKernelGGL(ms_step_pair_n_kernel<PM>, grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term, trunc, goal, \
                     score, ctr)
#define MS_GROUP_N(PM, GG)                                                                                           \
  hipLaunchKernelGGL((ms_step_group_n_kernel<PM, GG>), grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term, trunc, \
                     goal, score, ctr, group_solve)
  if (G == 2) {
    if (param_mode == 1) MS_PAIR_N(1);
    else if (param_mode == 2) MS_PAIR_N(2);
    else MS_PAIR_N(0);
#ifndef MS_PAIR_ONLY
  } else if (G == 8) {
    if (param_mode == 1) MS_GROUP_N(1, 8);
    else if (param_mode == 2) MS_GROUP_N(2, 8);
    else MS_GROUP_N(0, 8);
  } else if (G == 16) {
    if (param_mode == 1) MS_GROUP_N(1, 16);
    else if (param_mode == 2) MS_GROUP_N(2, 16);
    else MS_GROUP_N(0, 16);
#endif
  } else {
    return hipErrorInvalidValue;
  }
#undef MS_PAIR_N
#undef MS_GROUP_N
  return hipGetLastError();
}
