#!/usr/bin/env python3
"""Static instruction mix of one kernel, attributed to source functions (diagnostic, not product code).

    python tools/isa_lines.py [--kernel ms_step_pair_kernelILi1E] [--top 40] [hipcc -D flags...]

Compiles ms_env.hip device-only with -gline-tables-only (same optimisation flags as the product),
walks the kernel's assembly, and counts VALU / LDS / VMEM / SALU instructions by the innermost
source line (.loc) and by the enclosing source function of that line. Loops are listed with their
own counts (a backward branch closes a loop body), so that static counts can be weighted by trip
counts by hand. The SQ counters (tools/gpu.sh sq) give the dynamic totals this splits up.
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "marl-soccer_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))

FUNC_RE = re.compile(r"^(?!\s)(?!#)(?!\}).*?\b([A-Za-z_]\w*)\s*\((?!.*;\s*$)")
SKIP = {"if", "for", "while", "switch", "return", "sizeof", "static_assert", "defined"}


def func_map(path):
    """line -> name of the function whose definition starts at or before it (column-0 heuristics)."""
    names, cur = {}, "?"
    with open(path) as f:
        for i, ln in enumerate(f, 1):
            m = FUNC_RE.match(ln)
            if m and m.group(1) not in SKIP and "=" not in ln.split("(")[0]:
                cur = m.group(1)
            names[i] = cur
    return names


def klass(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="ms_step_pair_kernelILi1E")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--asm", help="an existing .s file instead of compiling")
    args, extra = ap.parse_known_args()
    import build_native

    asm = args.asm or "/tmp/isa_lines.s"
    if not args.asm:
        flags = [f for f in build_native.FLAGS if f not in ("-shared", "-fPIC", "-Wall")]
        cmd = [build_native.hipcc(), *flags, *extra, "--cuda-device-only", "-S", "-gline-tables-only",
               "-o", asm, os.path.join(CSRC, "ms_env.hip")]
        subprocess.run(cmd, check=True, capture_output=True)
    files, fmaps = {}, {}
    body, inside, name = [], False, None
    loc = ("?", 0)
    with open(asm) as f:
        for ln in f:
            m = re.match(r"\s*\.file\s+(\d+)\s+\"([^\"]*)\"\s+\"([^\"]*)\"", ln)
            if m:
                files[m.group(1)] = os.path.join(m.group(2), m.group(3))
                continue
            if not inside:
                if re.match(r"^_Z\w*" + args.kernel + r"\w*:", ln):
                    inside, name = True, ln.split(":")[0]
                continue
            if ln.startswith(".Lfunc_end"):
                break
            m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
            if m:
                loc = (m.group(1), int(m.group(2)))
                continue
            m = re.match(r"^(\.LBB\w+):", ln)
            if m:
                body.append(("label", m.group(1), loc))
                continue
            m = re.match(r"\s+([a-z_][a-z0-9_]*)\b", ln)
            if m and not ln.strip().startswith("."):
                body.append(("inst", m.group(1), loc))
    if not inside:
        sys.exit(f"kernel {args.kernel} not found")

    def where(loc):
        fid, line = loc
        path = files.get(fid, "?")
        base = os.path.basename(path)
        if path not in fmaps:
            fmaps[path] = func_map(path) if os.path.exists(path) else {}
        return base, fmaps[path].get(line, "?"), line

    by_func = collections.defaultdict(collections.Counter)
    by_line = collections.defaultdict(collections.Counter)
    total = collections.Counter()
    for kind, op, loc in body:
        if kind == "label":
            continue
        k = klass(op)
        base, fn, line = where(loc)
        by_func[(base, fn)][k] += 1
        by_line[(base, line, fn)][k] += 1
        total[k] += 1
    print(f"{name}: {dict(total)}")
    print(f"\nby function (static VALU / LDS / VMEM / SALU):")
    for (base, fn), c in sorted(by_func.items(), key=lambda kv: -kv[1]["valu"])[: args.top]:
        print(f"  {c['valu']:6d} {c['lds']:5d} {c['vmem']:5d} {c['salu']:5d}  {base}:{fn}")
    # loops: a branch to an earlier label
    print("\nloops (backward branches): body span, static VALU inside, source functions of the body")
    with open(asm) as f:
        text = f.read()
    start = text.index(name + ":")
    end = text.index(".Lfunc_end", start)
    seg = text[start:end].splitlines()
    lab_idx, idx = {}, 0
    rows = []
    for ln in seg:
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            lab_idx[m.group(1)] = idx
        m = re.match(r"\s+(s_cbranch_\w+|s_branch)\s+(\.LBB\w+)", ln)
        if m and m.group(2) in lab_idx:
            rows.append((lab_idx[m.group(2)], idx))
        if re.match(r"\s+[a-z_]", ln) and not ln.strip().startswith("."):
            idx += 1
    insts = [b for b in body if b[0] == "inst"]
    for a, b in rows:
        c = collections.Counter(klass(x[1]) for x in insts[a:b + 1])
        fns = collections.Counter(where(x[2])[1] for x in insts[a:b + 1])
        print(f"  [{a:6d},{b:6d}] valu {c['valu']:5d} lds {c['lds']:4d} vmem {c['vmem']:3d}  {', '.join(f'{k}:{v}' for k, v in fns.most_common(4))}")


if __name__ == "__main__":
    main()
