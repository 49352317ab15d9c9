"""The one-residual quotients of the frame arithmetic (ms_device.h div_k / obs_div, MS_DIV_ONESTEP)
equal IEEE n / d for every fp32 numerator of the fast paths' domain, [2^-100, 2^32) of either sign,
for each fixed divisor (1000, pi, the default obs_vmax 200 and obs_wmax 10): tools/div_check.hip
enumerates all of them on the GPU (built by __graft_entry__.build()). The rows over every normal
numerator are information only (the shorter sequence differs where quotients leave the normal
range, which no fast path admits)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "bin", "div_check")


@pytest.mark.gpu
def test_one_residual_division_exhaustive():
    assert os.path.exists(BIN), "tools/bin/div_check missing: run __graft_entry__.build()"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    out = r.stdout
    assert r.returncode == 0, out + r.stderr
    rows = [ln for ln in out.splitlines() if "mismatches" in ln]
    domain = [ln for ln in rows if "(normals)" not in ln]
    assert len(domain) == 4, out
    for ln in domain:
        assert " 0 mismatches" in ln, ln
