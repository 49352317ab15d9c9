#!/usr/bin/env python3
"""Build and time compile-time variants of the step kernel (diagnostic, not product code).

    python tools/variants.py build NAME="-DFOO=1 -DBAR=2" ...   # here: lib/variants/lib_NAME.so
    python tools/variants.py build-ref REV NAME ["-DFOO=1 ..."]  # the step library of git REV
    python tools/variants.py run [--envs N] [--steps K] [--lane-group G] [--max-steps M] NAME ...  # on the GPU box

`run` times each variant with bench.py (MARL_SOCCER_LIB points the loader at the variant) in
child processes, one after another, and prints one line per variant.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "marl-soccer_amd")
# this round's experiment libraries (lib/variants holds older ones and is not shipped: .gpurunignore)
VDIR = os.environ.get("MS_VARIANTS_DIR", os.path.join(PKG, "lib", "exp"))
sys.path.insert(0, PKG)


def build(name, defs, csrc=None):
    """lib_NAME.so from the csrc directory (default: the working tree's) with -D flags `defs`;
    -DMS_PAIR_ONLY: the lane-pair kernels only (no policy kernels), a short build."""
    import build_native
    os.makedirs(VDIR, exist_ok=True)
    out = os.path.join(VDIR, f"lib_{name}.so")
    d = csrc or build_native.CSRC
    names = ["ms_env.hip", "ms_kstep.hip"] if "-DMS_PAIR_ONLY" in defs.split() else ["ms_env.hip", "ms_policy.hip", "ms_kstep.hip"]
    srcs = [os.path.join(d, n) for n in names if os.path.exists(os.path.join(d, n))]  # older revisions: no ms_kstep.hip
    build_native.compile_and_link(out, srcs, extra=defs.split())
    print("built", out)


def main():
    a = sys.argv[1:]
    if a[0] == "build":
        for spec in a[1:]:
            name, _, defs = spec.partition("=")
            build(name, defs)
    elif a[0] == "build-ref":
        # the whole source tree of REV (csrc/ and include/), so that ms_env.hip's includes
        # (ms_device.h, ms_group.inc, marl_soccer.h) are that revision's, not the working tree's
        import shutil
        import tempfile
        rev, name, defs = a[1], a[2], (a[3] if len(a) > 3 else "")
        tmp = tempfile.mkdtemp(prefix="msref_")
        try:
            arc = subprocess.run(["git", "-C", ROOT, "archive", rev, "marl-soccer_amd/csrc", "include"],
                                 check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", tmp], input=arc, check=True)
            build(name, defs, os.path.join(tmp, "marl-soccer_amd", "csrc"))
        finally:
            shutil.rmtree(tmp)
    elif a[0] == "run":
        envs, steps, names, extra = "65536", "1000", [], []
        i = 1
        while i < len(a):
            if a[i] == "--envs":
                envs = a[i + 1]; i += 2
            elif a[i] == "--steps":
                steps = a[i + 1]; i += 2
            elif a[i] in ("--lane-group", "--max-steps", "--warmup"):
                extra += [a[i], a[i + 1]]; i += 2
            else:
                names.append(a[i]); i += 1
        for name in names:
            env = dict(os.environ, MARL_SOCCER_LIB=os.path.join(VDIR, f"lib_{name}.so"))
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-ring-leg", "--fused", "0", "--envs", envs,
                                "--steps", steps, *extra], env=env, capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(name, "FAILED", r.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"{name:16s} {d['roofline']['kernel_ms'] * 1e3:8.2f} us/step  {d['value'] / 1e6:8.1f} M env-steps/s",
                  flush=True)


if __name__ == "__main__":
    main()
