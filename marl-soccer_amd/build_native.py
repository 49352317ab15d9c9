"""Build the HIP library in-tree: marl-soccer_amd/lib/libmarlsoccer.so (gfx950 only).

    python marl-soccer_amd/build_native.py [--force] [--verbose]

hipcc cross-compiles without a GPU. The build is skipped when the .so is newer than
every source.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libmarlsoccer.so")
SOURCES = [os.path.join(CSRC, "ms_env.hip"), os.path.join(CSRC, "ms_policy.hip"), os.path.join(CSRC, "ms_kstep.hip")]
# per-source flags: the K-step kernels (ms_kstep.hip) without LLVM's machine loop-invariant code motion,
# which hoisted per-step values out of their K-step loop and spilled them
UNIT_FLAGS = {"ms_kstep.hip": ["-mllvm", "-disable-machine-licm"]}
DEPS = SOURCES + [os.path.join(CSRC, "ms_device.h"), os.path.join(CSRC, "ms_diag.h"), os.path.join(CSRC, "ms_group.inc"), os.path.join(CSRC, "ms_pair.inc"), os.path.join(ROOT, "include", "marl_soccer.h")]
ARCH = os.environ.get("MS_OFFLOAD_ARCH", "gfx950")
# LLVM's default AMDGPU machine scheduler. The max-ILP strategy (-mllvm
# -amdgpu-sched-strategy=max-ilp, -2.6 % step time in round 1) produced kernels that fault on the
# GPU for several sources whose address arithmetic the bounds-guarded build proves in range
# ("Faults"): it is not used.
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X library cannot be built")


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def unit_flags(src: str) -> list:
    return UNIT_FLAGS.get(os.path.basename(src), [])


def compile_and_link(out: str, sources: list, extra: list = (), verbose: bool = False) -> None:
    """Each source to an object in parallel (hipcc -c, its unit flags), then one shared library."""
    objs, procs = [], []
    for src in sources:
        obj = f"{out}.{os.path.splitext(os.path.basename(src))[0]}.o"
        cmd = [hipcc(), *[f for f in FLAGS if f != "-shared"], *extra, *unit_flags(src), "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    try:
        for p, cmd in procs:
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, cmd)
        cmd = [hipcc(), *FLAGS, "-o", out, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    finally:
        for p, _ in procs:
            if p.poll() is None:
                p.kill()
        for o in objs:
            if os.path.exists(o):
                os.remove(o)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    compile_and_link(tmp, SOURCES, verbose=verbose)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    print(build(a.force, a.verbose))
    sys.exit(0)
