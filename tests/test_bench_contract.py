"""bench.py's output contract (the driver parses it at every round end): one JSON line with
BASELINE.json's metric and the fields the task defines, on a short run on one GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_prints_one_contract_line():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "30", "--warmup", "5",
                        "--envs", "4096", "--cpu-envs", "512", "--cpu-seconds", "0.5"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k, t in (("value", float), ("unit", str), ("n_gpus", int), ("steps", int), ("warmup", int),
                 ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str), ("dtype", str),
                 ("data", str), ("config", dict), ("roofline", dict), ("cpu_baseline", dict)):
        assert isinstance(d[k], t), k
    assert d["n_gpus"] == 1 and d["steps"] == 30 and d["warmup"] == 5 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["vs_baseline"] is None and d["dtype"] == "f32" and d["value"] > 0
    assert "workload" in d["config"] and "model" not in d["config"]
    rl = d["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-9 and 0 < rl["frac"] < 1
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert cb["unit"] == "env-steps/s" and cb["sample"]
    assert d["arbiter_overflow"] == 0
    assert d["regime"].startswith("first episode only")  # steps 5-35 of a 1,000-step episode
    # traffic only from a committed PMC pass over the same window of a run with these arguments
    assert rl["traffic"] is None or rl["pmc"]["window"] == "e4096_ms1000_w5_s30"
    assert rl["frac_measured"] is None or abs(rl["frac_measured"] - rl["traffic"] / rl["peak"]) < 1e-9
    cache = rl["cache_entries_per_env_step"]
    assert cache["env_steps_counted"] == 4096 * 30 and cache["read"] >= 0 and cache["written"] >= 0
    assert abs(rl["mean_cached_arbiters"] - 0.5 * (cache["read"] + cache["written"])) < 1e-9
    assert d["ranks_seen"] == 1 and d["config"]["launch"].startswith("lane groups, 8 lanes per env")
    # the K-step leg is in the line at the driver's short window too (its own whole-launch window)
    fs = d["fused_steps"]
    assert fs["K"] == 50 and fs["warmup"] == 50 and fs["steps"] == 200 and fs["value"] > 0
    assert fs["roofline"]["bound"] == "hbm" and 0 < fs["roofline"]["frac"] < 1
    assert abs(fs["roofline"]["frac"] - fs["roofline"]["achieved"] / fs["roofline"]["peak"]) < 1e-9
    # and the frame-ring leg carries its own roofline block
    fr = d["frame_ring"]
    assert fr["R"] == 32 and fr["value"] > 0 and 0 < fr["roofline"]["frac"] < 1
