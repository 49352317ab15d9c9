// ms_kstep.hip — the open-loop K-step kernels of ms_step_n (ms_step_pair_n_kernel,
// ms_step_group_n_kernel) in a translation unit of their own, built with LLVM's machine loop-invariant
// code motion off (build_native.py): each kernel runs the per-step device code of ms_pair.inc /
// ms_group.inc in a K-iteration loop, and hoisting what a step derives from its loop-invariant inputs
// (addresses, masks, Params constants) out of that loop held them across the whole step, which needs
// ~240 of the 256 registers by itself: 44-76 B/lane of scratch with LICM, 0 without.
// The per-step kernels stay in ms_env.hip, built with the default pipeline.
#define MS_KSTEP_TU 1
#include "ms_env.hip"

hipError_t ms_kstep_launch(int G, bool default_params, dim3 grid, hipStream_t st, const DevState& S, const Params& P, int K,
                           const float* actions, float* obs, float* rew, uint8_t* term, uint8_t* trunc, int8_t* goal,
                           int32_t* score, Counters* ctr, int group_solve) {
  if (G == 2) {
    if (default_params)
      hipLaunchKernelGGL(ms_step_pair_n_kernel<true>, grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term, trunc, goal,
                         score, ctr);
    else
      hipLaunchKernelGGL(ms_step_pair_n_kernel<false>, grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term, trunc,
                         goal, score, ctr);
#ifndef MS_PAIR_ONLY
  } else if (G == 8) {
    if (default_params)
      hipLaunchKernelGGL((ms_step_group_n_kernel<true, 8>), grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term, trunc,
                         goal, score, ctr, group_solve);
    else
      hipLaunchKernelGGL((ms_step_group_n_kernel<false, 8>), grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term,
                         trunc, goal, score, ctr, group_solve);
  } else if (G == 16) {
    if (default_params)
      hipLaunchKernelGGL((ms_step_group_n_kernel<true, 16>), grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term,
                         trunc, goal, score, ctr, group_solve);
    else
      hipLaunchKernelGGL((ms_step_group_n_kernel<false, 16>), grid, dim3(64), 0, st, S, P, K, actions, obs, rew, term,
                         trunc, goal, score, ctr, group_solve);
#endif
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
