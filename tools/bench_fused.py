#!/usr/bin/env python3
"""ms_step_n (SoccerBatch.step_n) timing sweep over K and batch size (diagnostic; bench.py's
`fused_steps` leg is the reported number). For each (envs, K): a batch seeded as bench.py's, W warm-up
steps, then T timed steps as T / K calls of step_n, bracketed by HIP events on the env's stream and
by host time; one JSON line per case.

    python tools/bench_fused.py --envs 65536 --k 10 50 250 [--steps 1000] [--warmup 1000] [--max-steps M]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[65536])
    ap.add_argument("--k", type=int, nargs="+", default=[50])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--max-steps", type=int, default=1000)
    a = ap.parse_args()
    import torch
    from marlsoccer import SoccerBatch
    from marlsoccer.batch import OUTPUT_LAYOUT
    cfg = None
    if a.max_steps != 1000:
        from marlsoccer.config import load_config
        cfg = load_config()
        cfg["simulation"]["max_steps"] = a.max_steps
    dev = torch.device("cuda", 0)
    for E in a.envs:
        for K in a.k:
            if a.steps % K or a.warmup % K:
                print(json.dumps({"envs": E, "K": K, "skipped": "steps and warmup must be multiples of K"}))
                continue
            b = SoccerBatch(E, config=cfg)
            b.reset(seed=19)
            gen = torch.Generator(device=dev)
            gen.manual_seed(1000)
            nblk = max(1, min(a.steps // K, int(6 * (1 << 30) // (E * 48 * K))))
            pool = [torch.rand((K, E, 4, 3), device=dev, generator=gen) * 2 - 1 for _ in range(nblk)]
            out = {name: torch.empty((K, E) + sh, dtype=dt, device=dev) for name, dt, sh in OUTPUT_LAYOUT}
            for i in range(a.warmup // K):
                b.step_n(pool[i % nblk], out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(b.stream)
            for i in range(a.steps // K):
                b.step_n(pool[i % nblk], out=out)
            e1.record(b.stream)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            kms = e0.elapsed_time(e1) / a.steps
            print(json.dumps({"envs": E, "K": K, "max_steps": a.max_steps, "kernel": b.step_kernel.replace(
                "_kernel", "_n_kernel") if b.lane_group > 0 else b.step_kernel, "us_per_step": kms * 1e3,
                "env_steps_per_s": E * a.steps / el, "wall_us_per_step": el * 1e6 / a.steps}), flush=True)
            b.close()
            del pool, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
