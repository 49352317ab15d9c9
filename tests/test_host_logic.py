"""Host-side logic that needs no GPU: the packed step-output layout, bench.py's regime labels."""
import importlib.util
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 3, 64, 65, 4096])
def test_packed_output_views_tile_the_buffer(n):
    from marlsoccer.batch import OUTPUT_LAYOUT, output_bytes, output_views
    buf = torch.zeros((output_bytes(n),), dtype=torch.uint8)
    v = output_views(buf, n)
    spans = []
    for name, dt, sh in OUTPUT_LAYOUT:
        t = v[name]
        assert t.shape == (n,) + sh and t.dtype == dt
        start = t.data_ptr() - buf.data_ptr()
        assert start % 16 == 0, name  # the kernel's 16-B rew stores, 8-B obs/score stores
        spans.append((start, start + t.numel() * t.element_size()))
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0
    assert spans[-1][1] <= buf.numel()
    # numpy views of a host copy see the same bytes
    v["rew"][:, 0] = torch.arange(n, dtype=torch.float32)
    v["score"][:, 1] = 7
    hv = output_views(buf.numpy(), n)
    np.testing.assert_array_equal(hv["rew"][:, 0], np.arange(n, dtype=np.float32))
    assert (hv["score"][:, 1] == 7).all()


def test_bench_regime_labels():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.regime(1000, 1000, 1000).startswith("steady state")
    assert bench.regime(5, 20, 1000).startswith("first episode only")
    assert bench.regime(900, 200, 1000).startswith("steps 900-1100")
    assert "unbounded" in bench.regime(0, 10, 0)
