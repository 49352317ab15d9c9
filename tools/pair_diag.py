#!/usr/bin/env python3
"""Diagnostic (not product code): step the same envs with two ms_step kernels (lane groups
`--a` and `--b`, e.g. 0 = per-lane, 2 = lane pairs) under the chase policy of the parity tests and
report the first step at which their exported states or outputs differ: which envs, which fields
and bodies, and the env's contact/arbiter counts."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-soccer_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--a", type=int, default=0)
    ap.add_argument("--b", type=int, default=2)
    ap.add_argument("--seed", type=int, default=19)
    args = ap.parse_args()
    import torch
    import marlsoccer as ms
    import oracle as orc
    import sim_helpers as sh

    n = args.envs
    a = ms.SoccerBatch(n)
    b = ms.SoccerBatch(n)
    a.set_lane_group(args.a)
    b.set_lane_group(args.b)
    a.reset(seed=args.seed)
    b.reset(seed=args.seed)
    ref = orc.OracleBatch(n, "f32")
    ref.reset(np.stack([orc.pcg_from_seed(args.seed + i) for i in range(n)]), 0)
    rng = np.random.default_rng(args.seed)
    chaser = np.arange(n) % 4
    report = {"kernels": [a.step_kernel, b.step_kernel]}
    prev_a = a.export_state()
    for t in range(args.steps):
        st = ref.export_state()
        pos = np.stack([st["body"]["px"], st["body"]["py"]], -1)
        act = sh.chase_actions(pos, st["body"]["angle"][:, :4], rng, chaser)
        ref.step(act)
        at = torch.from_numpy(act).to(a.device)
        oa = a.step(at)
        ob = b.step(at)
        ga, gb = a.export_state(), b.export_state()
        bad = {}
        for f in ("px", "py", "vx", "vy", "angle", "w", "vbx", "vby", "wb"):
            d = np.argwhere(ga["body"][f] != gb["body"][f])
            if len(d):
                bad[f"body.{f}"] = d[:8].tolist()
        for f in ("steps", "score_blue", "score_red", "n_arb", "mode", "hist_empty", "pcg_state_lo"):
            d = np.argwhere(ga[f] != gb[f]).ravel()
            if len(d):
                bad[f] = d[:8].tolist()
        d = np.argwhere((ga["snap"] != gb["snap"]).any(-1))
        if len(d):
            bad["snap"] = d[:8].tolist()
        for i in range(n):
            k = int(ga["n_arb"][i])
            for f in ("pair", "count", "idle", "hash", "jn", "jt"):
                if not np.array_equal(ga["arb"][f][i, :k], gb["arb"][f][i, :k]):
                    bad.setdefault(f"arb.{f}", []).append(i)
        oo = (oa.obs != ob.obs).cpu().numpy()
        if oo.any():
            bad["obs"] = np.argwhere(oo)[:12].tolist()
        if bad:
            envs = sorted({int(x[0]) if isinstance(x, list) else int(x) for v in bad.values() for x in v})[:6]
            detail = {}
            for i in envs:
                detail[i] = {
                    "a_body": {f: ga["body"][f][i].tolist() for f in ("px", "py", "vx", "vy", "angle", "w", "vbx", "vby", "wb")},
                    "b_body": {f: gb["body"][f][i].tolist() for f in ("px", "py", "vx", "vy", "angle", "w", "vbx", "vby", "wb")},
                    "prev_n_arb": int(prev_a["n_arb"][i]), "n_arb": [int(ga["n_arb"][i]), int(gb["n_arb"][i])],
                    "a_arb": [(int(ga["arb"]["pair"][i, k]), int(ga["arb"]["count"][i, k]), int(ga["arb"]["idle"][i, k]))
                              for k in range(int(ga["n_arb"][i]))],
                    "b_arb": [(int(gb["arb"]["pair"][i, k]), int(gb["arb"]["count"][i, k]), int(gb["arb"]["idle"][i, k]))
                              for k in range(int(gb["n_arb"][i]))],
                    "prev_arb": [(int(prev_a["arb"]["pair"][i, k]), int(prev_a["arb"]["count"][i, k]),
                                  int(prev_a["arb"]["idle"][i, k])) for k in range(int(prev_a["n_arb"][i]))],
                    "goal": [int(oa.goal[i]), int(ob.goal[i])],
                }
            report.update({"first_step": t, "fields": bad, "detail": detail})
            break
        prev_a = ga
    else:
        report["first_step"] = None
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
