#!/usr/bin/env python3
"""Compiler resource usage of the step kernel (the numbers rocprofv3's vgpr/accum_vgpr fields
misreport on gfx950), written to profiles/<tag>_resource_usage.txt.

    python tools/resource_usage.py <tag> [extra hipcc flags...]

Runs the product hipcc command (build_native.FLAGS) device-only with
-Rpass-analysis=kernel-resource-usage and keeps the remarks of every kernel.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def main(tag, extra=()):
    import build_native

    flags = [f for f in build_native.FLAGS if f not in ("-shared",)]
    out = ""
    for src in build_native.SOURCES:
        cmd = [build_native.hipcc(), *flags, *extra, *build_native.unit_flags(src), "-Rpass-analysis=kernel-resource-usage", "--cuda-device-only",
               "-c", "-o", os.devnull, src]
        out += subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    lines = []
    for ln in out.splitlines():
        m = re.search(r"remark:\s+(.*?)\s+\[-Rpass-analysis", ln)
        if m:
            lines.append(m.group(1))
    dst = os.path.join(ROOT, "profiles", f"{tag}_resource_usage.txt")
    with open(dst, "w") as f:
        f.write("# hipcc " + " ".join(flags + list(extra)) + " -Rpass-analysis=kernel-resource-usage\n")
        f.write("\n".join(lines) + "\n")
    print(open(dst).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
