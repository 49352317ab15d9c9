"""The reduced-range division / sqrt of ms_device.h (used by the obs encoding) against IEEE.

Compiles tests/native/fastdiv_check.hip with hipcc and runs 2^32 random operand pairs on the
GPU; every result must be bit-identical to the compiler's correctly rounded fp32 division and
sqrtf. The kernel only takes this path for guarded operands, and the GPU parity
suite checks the full step bit for bit as well.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_fast_division_is_ieee_exact():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "fastdiv_check")
        subprocess.run([hipcc, "-O3", "-ffp-contract=off", "--offload-arch=gfx950", "-o", exe,
                        os.path.join(HERE, "native", "fastdiv_check.hip")], check=True, capture_output=True)
        out = subprocess.run([exe, "16"], check=True, capture_output=True, text=True, timeout=300).stdout
    m = re.search(r"samples (\d+) div mismatches (\d+) sqrt mismatches (\d+)", out)
    assert m, out
    executed = re.search(r"samples executed (\d+)", out)
    assert executed and int(executed.group(1)) == int(m.group(1)), out
    assert int(m.group(1)) == 16 << 28
    assert m.group(2) == "0" and m.group(3) == "0", out
