#!/usr/bin/env python3
"""Diagnostic (not product): replay test_trajectory_chase_bitexact's scenario with the library
named by MARL_SOCCER_LIB and report the first step where obs/rewards/state leave the fp32 oracle:
which envs, agents, stack slots and frame components, with both values and the env's state
before the step. Used to locate the max-ILP scheduler's mismatch (DESIGN.md §8 "Faults")."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "marl-soccer_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as orc  # noqa: E402
import sim_helpers as sh  # noqa: E402
from marlsoccer import SoccerBatch  # noqa: E402


def main(n=128, steps=1100, seed=19):
    gpu = SoccerBatch(n)
    ref = orc.OracleBatch(n, "f32")
    gpu.reset(seed=seed)
    ref.reset(np.stack([orc.pcg_from_seed(seed + i) for i in range(n)]), 0)
    rng = np.random.default_rng(seed)
    chaser = np.arange(n) % 4
    for t in range(steps):
        st = ref.export_state()
        pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
        act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
        gst = gpu.export_state()
        out = gpu.step(torch.from_numpy(act).to(gpu.device))
        obs, rew, trunc, goal, score, bad = ref.step(act)
        g = out.obs.cpu().numpy()
        bad_obs = np.argwhere(g != obs)
        bad_rew = np.argwhere(out.rew.cpu().numpy() != rew.astype(np.float32))
        if len(bad_obs) or len(bad_rew):
            rep = {"step": t, "obs_mismatch": [[int(e), int(a), int(c) // 22, int(c) % 22, float(g[e, a, c]), float(obs[e, a, c])]
                                               for e, a, c in bad_obs[:20]],
                   "rew_mismatch": [[int(e), int(k)] for e, k in bad_rew[:10]]}
            envs = sorted({int(e) for e, _, _ in bad_obs[:20]})
            for e in envs[:3]:
                rep[f"env{e}_state_before"] = {k: gst[e]["body"][k].tolist() for k in ("px", "py", "vx", "vy", "angle", "w")}
                rep[f"env{e}_hist_empty"] = int(gst[e]["hist_empty"])
                rep[f"env{e}_steps"] = int(gst[e]["steps"])
                rep[f"env{e}_n_arb"] = int(gst[e]["n_arb"])
                rep[f"env{e}_snap_t2"] = gst[e]["snap"][0].tolist()
            print(json.dumps(rep, indent=1))
            return 1
    print("no mismatch")
    return 0


if __name__ == "__main__":
    sys.exit(main())
