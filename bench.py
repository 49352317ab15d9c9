#!/usr/bin/env python3
"""Throughput benchmark of the MI355X soccer env step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--allgather]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one env.step of every env resident on a GPU (one ms_step launch): E envs per
GPU (default 65,536 = BASELINE.json configs[2]), weak scaling across ranks (envs are
independent; no collective in the data path). Actions are synthetic uniform(-1, 1) fp32
from torch's device Philox generator, one fresh (E, 4, 3) buffer per step (generated
before the timed region, read from HBM every step). The default timed
window is one whole episode of the steady state: the 1,000 warm-up steps run the first
episode (default random spawn, as SyncMultiAgentVecEnv.reset does), whose end auto-resets
every env with the full-random spawn the vec env uses from then on (marl_vecenv.py:45-51);
the 1,000 timed steps are the second episode including its own auto-reset, so
contact-heavy and contact-free phases are both in the average. (The first episode is ≈10 %
cheaper — fewer agents start against walls — and is not what a training run sees.) Rank 0
prints ONE JSON line. --allgather adds the optional RCCL all-gather of obs (configs[3]).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "marl-soccer_amd"))

METRIC = "env-steps/sec (4 agents × N envs) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# Algorithmic HBM bytes per env-step of ms_step_kernel (DESIGN.md "Roofline"):
# actions, bodies, scalars (steps, score, meta, PCG64 buffered u32), the t-2 obs-history snapshot
# (26 f32; the t-1 snapshot is the body state itself)
ALG_READ = 48 + 176 + 16 + 104
ALG_WRITE = 176 + 16 + 104 + 1056 + 16 + 4 + 4 + 1 + 8  # bodies, scalars, snapshot, obs, rew, term, trunc, goal, score
ARB_BYTES = 20                       # one cached arbiter: header + 4 impulses (read + rewritten)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--max-steps", type=int, default=1000,
                    help="episode length (config.json: 1000; BASELINE configs[4]: 512)")
    ap.add_argument("--action-sets", type=int, default=0,
                    help="distinct device action buffers cycled (0: one per step, capped at --action-gib)")
    ap.add_argument("--action-gib", type=float, default=8.0, help="HBM cap for the action pool")
    ap.add_argument("--allgather", action="store_true", help="RCCL all-gather of obs after every step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-envs", type=int, default=65536)
    ap.add_argument("--cpu-steps", type=int, default=3000)
    return ap.parse_args()


def cpu_baseline(args):
    """The oracle's f64 restatement (reference precision) on this host's cores, bounded."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    n, k = args.cpu_envs, args.cpu_steps
    secs = orc.cpu_baseline(n, k, cores, "f64")
    # also the serial one-env-at-a-time loop on one core
    n1, k1 = 4096, 500
    secs1 = orc.cpu_baseline(n1, k1, 1, "f64")
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except Exception:
        pass
    return {"value": n * k / secs, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"oracle f64 (C restatement of Game.step + Chipmunk) {n} envs x {k} steps, "
                      f"random actions, {cores} threads, {secs:.2f} s wall",
            "single_core": {"value": n1 * k1 / secs1, "sample": f"{n1} envs x {k1} steps, 1 thread, {secs1:.2f} s"},
            "host": {"cpu_count": os.cpu_count(), "model": model}}


def load_pmc_traffic():
    path = os.path.join(ROOT, "profiles", "pmc_step_kernel.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MS_BENCH_SHARED_GPU=1 (rehearsal on a one-GPU box only): every rank on cuda:0, gloo for
    # the barrier and the max-reduce; the driver's multi-GPU runs use one GPU per rank + RCCL
    shared = os.environ.get("MS_BENCH_SHARED_GPU") == "1"
    ordinal = 0 if shared else local
    if world > 1:
        torch.cuda.set_device(ordinal)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", ordinal))
    dev = torch.device("cuda", ordinal if world > 1 else 0)
    torch.cuda.set_device(dev)

    from marlsoccer import SoccerBatch

    E = args.envs
    cfg = None
    if args.max_steps != 1000:
        from marlsoccer.config import load_config
        cfg = load_config()
        cfg["simulation"]["max_steps"] = args.max_steps
    batch = SoccerBatch(E, config=cfg, device=dev.index)
    batch.reset(seed=19 + rank * E)  # env i of rank r seeded 19 + r*E + i (global index)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    want = args.action_sets if args.action_sets > 0 else args.steps + args.warmup
    cap = max(1, int(args.action_gib * (1 << 30) // (E * 48)))
    nsets = max(1, min(want, cap, args.steps + args.warmup))
    actions = [torch.rand((E, 4, 3), device=dev, generator=gen) * 2 - 1 for _ in range(nsets)]
    obs, rew = batch.obs, batch.rew
    term, trunc, goal, score = batch.term, batch.trunc, batch.goal, batch.score
    gathered = None
    if args.allgather and world > 1:
        gathered = torch.empty((world * E, 4, 66), dtype=torch.float32, device=dev)

    launch = batch.launcher(actions, obs, rew, term, trunc, goal, score)

    def one(i):
        launch(i)
        if gathered is not None:
            dist.all_gather_into_tensor(gathered, obs)

    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # The K launches go back to back on the env's stream, bracketed by ONE pair of HIP events:
    # an event record between launches costs ~8 us of wall per step and perturbs the next
    # kernel, so per-launch events would measure a slower loop than the one being timed.
    # kernel_ms = event span / K is therefore the per-launch time including the (small)
    # dispatch gap between consecutive kernels — an upper bound on the kernel duration;
    # profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace) gives the exact one.
    stream = batch.stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        launch(args.warmup + i)
        if gathered is not None:
            dist.all_gather_into_tensor(gathered, obs)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cpu" if shared else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    # With N > 1 ranks and no --allgather: a second, shorter timed loop WITH the whole-batch
    # obs all-gather after every step (BASELINE configs[3]; SURVEY.md 8(e) asks for the rate
    # with and without it). Reported beside `value`, which stays the no-collective rate.
    gather_report = None
    if world > 1 and gathered is None and not shared:
        gbuf = torch.empty((world * E, 4, 66), dtype=torch.float32, device=dev)
        gk = min(200, args.steps)
        for i in range(5):
            launch(i)
            dist.all_gather_into_tensor(gbuf, obs)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for i in range(gk):
            launch(5 + i)
            dist.all_gather_into_tensor(gbuf, obs)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        g_el = float(gt[0])
        gather_report = {"value": world * E * gk / g_el, "unit": "env-steps/s", "steps": gk,
                         "ms_per_step": g_el * 1e3 / gk,
                         "collective": f"RCCL all_gather_into_tensor of obs, {E * 1056 / 1e6:.1f} MB per rank per step"}
        del gbuf

    # cached arbiters per env (the cache bytes of the algorithmic count), sampled mid-episode:
    # 300 more untimed steps, so the sample is not the just-reset state at an episode boundary
    for i in range(300):
        launch(i)
    torch.cuda.synchronize()
    st = batch.export_state()
    mean_arb = float(st["n_arb"].mean())
    stats = batch.stats()
    bytes_per_step = ALG_READ + ALG_WRITE + 2 * ARB_BYTES * mean_arb
    achieved = bytes_per_step * E / (kern_ms * 1e-3) / 1e9
    value = world * E * args.steps / elapsed
    if rank == 0:
        pmc = load_pmc_traffic()
        traffic = None
        pmc_info = None
        if pmc and pmc.get("envs") == E:
            # HBM bytes per launch from the committed rocprofv3 PMC passes, over the live kernel time
            traffic = pmc["hbm_bytes_per_launch"] / (kern_ms * 1e-3) / 1e9
            pmc_info = {"source": f"profiles/{pmc['tag']}_pmc.json", "bytes_per_launch": pmc["hbm_bytes_per_launch"],
                        "alg_bytes_per_launch": bytes_per_step * E}
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: uniform(-1,1) fp32 actions (device Philox, {nsets} distinct (E,4,3) buffers "
                    f"for {args.warmup + args.steps} steps, read from HBM each step); env i seeded 19+i; "
                    "default config.json physics/rewards" + (f", max_steps={args.max_steps}" if args.max_steps != 1000 else ""),
            "config": {"workload": f"{E} parallel envs per MI355X" +
                                   (" (BASELINE.json configs[2])" if E == 65536 and args.max_steps == 1000 else
                                    " (BASELINE.json configs[1])" if E == 4096 and args.max_steps == 1000 else
                                    " (BASELINE.json configs[4] per-GPU shard)" if E == 32768 and args.max_steps == 512
                                    else ""),
                       "envs_per_gpu": E, "global_envs": world * E, "max_steps": args.max_steps,
                       "parallelism": f"env-shard x{world}" + (" + obs all-gather" if gathered is not None else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "ms_step_kernel", "kernel_ms": kern_ms,
                         "kernel_ms_method": "HIP events around the K back-to-back launches / K",
                         "alg_bytes_per_env_step": bytes_per_step,
                         "mean_cached_arbiters": mean_arb,  # sampled mid-episode after the timed window
                         "pmc": pmc_info},
            "arbiter_overflow": stats["arbiter_overflow"],
        }
        if gather_report is not None:
            line["with_obs_allgather"] = gather_report
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args)
            cb["gpu_over_cpu"] = value / cb["value"]
            line["cpu_baseline"] = cb
        print(json.dumps(line), flush=True)
    batch.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
