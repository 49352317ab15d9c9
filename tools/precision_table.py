#!/usr/bin/env python3
"""Tabulate the fp32-vs-f64 precision figures of DESIGN.md §4 (CPU only; the GPU kernel is
bit-identical to the fp32 oracle, so the same table holds for it).

    python tools/precision_table.py [--out profiles/r02_precision.json]

One step from every golden-trajectory state: max and 95 % quantile of each quantity's error, the
states above 1e-5 and, for those, the largest ratio of the error to the f64 step's own change
under a one-ulp change of one fp32 input (precision_common.conditioning).
Horizons: from steps 0, 100, 250 of every trajectory, the first step at which each quantity
leaves 1e-5 (121 = never within 120 steps).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import golden_io as gio  # noqa: E402
import oracle as orc  # noqa: E402
import precision_common as pc  # noqa: E402


def main(out=None):
    res = {"tolerance": pc.TOL, "one_step": {}, "horizons": {}}
    for name in gio.TRAJ_NAMES:
        states, actions, cfg = pc.fixture_states(name)
        s32, o32, r32, _ = pc.oracle_one_step(states, actions, cfg, "f32")
        s64, o64, r64, _ = pc.oracle_one_step(states, actions, cfg, "f64")
        errs = pc.step_errors(s32, s64, o32, o64, r32, r64)
        cond = pc.conditioning(name)
        res["one_step"][name] = {"states": int(len(states)),
                                 **{k: {"max": float(e.max()), "q95": float(np.quantile(e, 0.95)),
                                        "states_over_1e-5": int((e > pc.TOL).sum()),
                                        # error / the f64 step's change under a one-ulp input change
                                        "max_ratio_to_one_ulp_sensitivity_over_1e-5": float(
                                            (e[e > pc.TOL] / np.maximum(cond[k][e > pc.TOL], 1e-30)).max())
                                        if (e > pc.TOL).any() else 0.0}
                                    for k, e in errs.items()}}
        fx = gio.load(f"traj_{name}.npz")
        T, n = fx["obs"].shape[:2]
        for t0 in (0, 100, 250):
            st0 = states[t0 * n:(t0 + 1) * n]
            runs = {}
            for prec in ("f32", "f64"):
                b = orc.OracleBatch(n, prec, cfg)
                b.import_state(st0)
                runs[prec] = b

            def make(prec):
                def run(k):
                    obs, rew = runs[prec].step(fx["actions"][t0 + k])[:2]
                    return runs[prec].export_state(), obs, rew
                return run

            res["horizons"][f"{name}@{t0}"] = pc.horizon(make("f32"), make("f64"), 120)
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None)
