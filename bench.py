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

# Algorithmic HBM bytes per env-step, SURVEY.md §8(d): B_step = 2,289 + 2·C, where C is the
# warm-start (arbiter) cache read and written per env-step. reads: actions 48, bodies 180,
# episode scalars 16, RNG 40, two prior obs frames 704; writes: bodies 180, scalars 16, RNG 24,
# obs 1,056, rewards 16, term/trunc 8, goal 1. C from this build's layout: 20 B per cached
# arbiter (4-B header + 4 accumulated impulses) × the mean number of cached arbiters per env.
# roofline.achieved uses this figure (the task's definition); the bytes this layout actually
# moves (the t-2 history as a 104-B snapshot instead of two 352-B frames, RNG
# only on respawns) are reported beside it as layout_bytes_per_env_step.
SURVEY_BYTES = 2289
# The frame-ring variant (--frame-ring R) needs neither the prior frames' 704-B read nor their
# 704-B re-write: 881 + 2C, plus the two frames a wrap re-writes every R - 2 steps.
RING_BYTES = SURVEY_BYTES - 704 - 704
ARB_BYTES = 20
LAYOUT_READ = 48 + 176 + 16 + 104
LAYOUT_WRITE = 176 + 16 + 104 + 1056 + 16 + 4 + 4 + 1 + 8  # bodies, scalars, snapshot, obs, rew, term, trunc, goal, score


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; > 1 without a launcher starts torch.distributed.run itself "
                         "(default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--max-steps", type=int, default=1000,
                    help="episode length (config.json: 1000; BASELINE configs[4]: 512)")
    ap.add_argument("--action-sets", type=int, default=0,
                    help="distinct device action buffers cycled (0: one per step, capped at --action-gib)")
    ap.add_argument("--action-gib", type=float, default=8.0, help="HBM cap for the action pool")
    ap.add_argument("--allgather", action="store_true", help="RCCL all-gather of obs after every step")
    ap.add_argument("--frame-ring", type=int, default=0, metavar="R",
                    help="opt-in frame-ring observations (FrameRingBatch, R frames per agent ring); "
                         "default 0: the reference's contiguous (N, 4, 66) stacked obs")
    ap.add_argument("--lane-group", type=int, default=None, metavar="G",
                    help="ms_step kernel (SoccerBatch.set_lane_group): G = 2, 8 or 16 lanes per env, 0 one lane "
                         "per env, -1 automatic; default: the library's (8 lanes while envs x 8 fit the SIMDs, "
                         "else 2)")
    ap.add_argument("--group-solve", type=int, default=0, metavar="M",
                    help="diagnostic: the lane-group kernel's contact-solve schedule (SoccerBatch.set_group_solve): "
                         "0 automatic (default), 1 serial halves, 2 dependency-level rounds")
    ap.add_argument("--generic", choices=("rewards", "physics"), default=None,
                    help="a non-default config: 'rewards' (ball_proximity_multiplier 0.003) runs the default-physics "
                         "kernels with runtime reward multipliers (ms_config_specialised 2), 'physics' "
                         "(action_force_max 150001) the generic kernels with every parameter from the kernel arguments (0)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ring-leg", action="store_true", help="skip the frame-ring leg timed beside the headline")
    ap.add_argument("--fused", type=int, default=50, metavar="K",
                    help="N = 1: time ms_step_n (K steps per call, actions given up front) beside the headline "
                         "(0: skip)")
    ap.add_argument("--cpu-envs", type=int, default=65536)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target wall time of the all-cores CPU baseline (its step count is sized from the "
                         "single-core leg)")
    return ap.parse_args()


def cgroup_cpu_limit():
    """CPUs this process may use per the cgroup CPU quota (None when unlimited or unknown)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2: "<quota> <period>" or "max <period>"
            q, p = f.read().split()[:2]
            return None if q == "max" else max(1, int(int(q) // int(p)))
    except Exception:
        pass
    try:  # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return None if q <= 0 else max(1, q // p)
    except Exception:
        return None


def cpu_baseline(args):
    """The oracle's f64 restatement (reference precision) on every host core this process may
    use (the serial one-env-at-a-time loop on one core, and all cores over env
    shards); bounded to about --cpu-seconds of wall time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_limit()
    cores = max(1, min(affinity, quota) if quota else affinity)
    # the serial one-env-at-a-time loop on one core (marl_vecenv.py:39)
    n1, k1 = 4096, 500
    secs1 = orc.cpu_baseline(n1, k1, 1, "f64")
    rate1 = n1 * k1 / secs1
    n = args.cpu_envs
    k = max(100, int(args.cpu_seconds * rate1 * cores / n))
    secs = orc.cpu_baseline(n, k, cores, "f64")
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except Exception:
        pass
    return {"value": n * k / secs, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"oracle f64 (C restatement of Game.step + Chipmunk) {n} envs x {k} steps, "
                      f"random actions, {cores} threads (every CPU this process may use), {secs:.2f} s wall",
            "single_core": {"value": rate1, "sample": f"{n1} envs x {k1} steps, 1 thread, {secs1:.2f} s"},
            "host": {"cpu_count": os.cpu_count(), "affinity": affinity, "cgroup_cpu_limit": quota, "model": model}}


def ring_kernel_name(batch) -> str:
    """The kernel ms_step_ring launches: the lane-pair frame-ring kernel on the lane-pair launch,
    else the one-lane one."""
    return "ms_step_pair_ring_kernel" if batch.lane_group == 2 else "ms_step_ring_kernel"


def launch_label(lane_group: int) -> str:
    """config.launch: the step kernel's launch shape."""
    if lane_group == 2:
        return "lane pairs, 2 lanes per env (32 envs per wave, 2 waves per SIMD)"
    if lane_group > 2:
        return f"lane groups, {lane_group} lanes per env ({64 // lane_group} envs per wave)"
    return "one lane per env, one wave per 64-env block"


def regime(warmup: int, steps: int, max_steps: int) -> str:
    """Which part of the episode cycle the timed window covers (the cost of a step depends on
    it: DESIGN.md §7)."""
    if max_steps <= 0:
        return f"steps {warmup}-{warmup + steps} of one unbounded episode (default random spawn)"
    first, last = warmup // max_steps, (warmup + steps - 1) // max_steps
    if last == 0:
        return (f"first episode only, steps {warmup}-{warmup + steps} of {max_steps} (default random spawn; "
                "cheaper than the steady state: DESIGN.md §7)")
    if first >= 1 and steps >= max_steps:
        return f"steady state: {steps} steps from step {warmup} (episodes {first + 1}-{last + 1}, full-random respawns)"
    return (f"steps {warmup}-{warmup + steps} (episodes {first + 1}-{last + 1}; episode 1 has the default random "
            "spawn, later ones the full-random respawn)")


def regime_key(envs: int, max_steps: int, warmup: int, steps: int) -> str:
    """Key of a timed window in profiles/pmc_step_kernel.json (tools/pmc_summary.py)."""
    return f"e{envs}_ms{max_steps}_w{warmup}_s{steps}"


def load_pmc_traffic(key: str, kernel: str, name: str = "pmc_step_kernel.json"):
    """The committed rocprofv3 PMC figures of the step kernel over the same timed window
    (dispatches warmup .. warmup + steps of a run with the same arguments), or None — also when
    the profiled launch ran another kernel than this run's (lane groups or pairs). `name`:
    profiles/pmc_step_kernel.json (ms_step) or profiles/pmc_fused_kernel.json (ms_step_n)."""
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            d = json.load(f)
        r = d["regimes"][key]
        if r.get("kernel", d.get("kernel")) != kernel:
            return None
        return dict(r, source=f"profiles/{d['tag']}_pmc.json", tag=d["tag"])
    except Exception:
        return None


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launcher_argv(gpus: int, argv: list, port: int) -> list:
    """The command that runs this bench on `gpus` ranks of one node: torch.distributed.run with
    one process per GPU (the driver's own form), the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def resolve_world(args, argv: list, env=None, run=None):
    """--gpus N against the launcher's WORLD_SIZE. Returns the world size this process runs in, or
    the exit code of a child launch: with N > 1 and no WORLD_SIZE (a plain `python bench.py --gpus
    N`), torch.distributed.run starts N ranks of this script as a CHILD process (no exec: nothing
    here has touched the GPU yet) and its return code is this process's; a launcher whose
    WORLD_SIZE differs from an explicit --gpus is an error, so no N-GPU request can print a
    one-GPU line."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if args.gpus is not None and args.gpus > 1:
            import subprocess
            run = run or subprocess.call
            return {"exit": run(launcher_argv(args.gpus, argv, free_port()))}
        if args.gpus is not None and args.gpus < 1:
            raise SystemExit(f"bench.py: --gpus {args.gpus} must be >= 1")
        return {"world": 1}
    world = int(ws)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    return {"world": world}


def main():
    args = parse()
    how = resolve_world(args, sys.argv[1:])
    if "exit" in how:
        sys.exit(how["exit"])
    import torch
    import torch.distributed as dist

    world = how["world"]
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

    from marlsoccer import FrameRingBatch, SoccerBatch
    from marlsoccer.distributed import all_gather_rows

    E = args.envs
    cfg = None
    if args.max_steps != 1000 or args.generic:
        from marlsoccer.config import load_config
        cfg = load_config()
        cfg["simulation"]["max_steps"] = args.max_steps
        if args.generic == "rewards":
            cfg["rewards"]["ball_proximity_multiplier"] = 0.003
        elif args.generic == "physics":
            cfg["physics"]["action_force_max"] = 150001.0
    ring = args.frame_ring
    if ring and args.allgather:
        raise SystemExit("--frame-ring and --allgather are exclusive")
    batch = (FrameRingBatch(E, ring=ring, config=cfg, device=dev.index) if ring else
             SoccerBatch(E, config=cfg, device=dev.index))
    if args.lane_group is not None and not ring:
        batch.set_lane_group(args.lane_group)
    if args.group_solve and not ring:
        batch.set_group_solve(args.group_solve)
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

    launch = (batch.launcher(actions, rew, term, trunc, goal, score) if ring else
              batch.launcher(actions, obs, rew, term, trunc, goal, score))
    step_kernel = ring_kernel_name(batch) if ring else batch.step_kernel  # the kernel the timed launches run

    nccl = world > 1 and dist.get_backend() == "nccl"

    def gather_into(dst):
        # RCCL all_gather_into_tensor; in the gloo rehearsal the product's all_gather_rows
        # (device tensors staged through host memory)
        if nccl:
            dist.all_gather_into_tensor(dst, obs)
        else:
            dst.copy_(all_gather_rows(obs, world))

    def one(i):
        launch(i)
        if gathered is not None:
            gather_into(gathered)

    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    overflow_warmup = batch.stats()["arbiter_overflow"]
    batch.reset_stats()  # the kernel's cache-entry tally now counts the timed launches only
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
    ev0.record(stream)  # (a marker on the idle stream: the wall clock starts at the first launch)
    t0 = time.perf_counter()
    for i in range(args.steps):
        launch(args.warmup + i)
        if gathered is not None:
            gather_into(gathered)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:  # (one rank: nothing runs between the two, so the first synchronize closes the window)
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    # the arbiter-cache entries the timed launches read and wrote (counted by the kernel)
    stats = batch.stats()

    ranks_seen = 1
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cpu" if shared else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        one = torch.ones(1, dtype=torch.int64, device="cpu" if shared else dev)
        dist.all_reduce(one)  # every rank that took part in the timed window
        ranks_seen = int(one.item())

    # With N > 1 ranks and no --allgather: a second, shorter timed loop WITH the whole-batch
    # obs all-gather after every step (BASELINE configs[3]; SURVEY.md 8(e) asks for the rate
    # with and without it). Reported beside `value`, which stays the no-collective rate.
    # (In the one-GPU gloo rehearsal the same loop runs through the product's all_gather_rows,
    # staged through host memory: it exercises the path, its rate is not RCCL's.)
    gather_report = None
    if world > 1 and gathered is None and not ring:
        gbuf = torch.empty((world * E, 4, 66), dtype=torch.float32, device=dev)
        gk = min(200 if nccl else 20, args.steps)
        for i in range(5):
            launch(i)
            gather_into(gbuf)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for i in range(gk):
            launch(5 + i)
            gather_into(gbuf)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=dev if nccl else "cpu")
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        g_el = float(gt[0])
        gather_report = {"value": world * E * gk / g_el, "unit": "env-steps/s", "steps": gk,
                         "ms_per_step": g_el * 1e3 / gk,
                         "collective": (f"RCCL all_gather_into_tensor of obs, {E * 1056 / 1e6:.1f} MB per rank per step"
                                        if nccl else
                                        f"gloo all_gather of obs staged through host memory (one-GPU rehearsal of "
                                        f"the path, not RCCL's rate), {E * 1056 / 1e6:.1f} MB per rank per step")}
        del gbuf

    # The opt-in frame-ring layout timed beside the headline (N = 1, default run): same envs,
    # seeds, actions and window on a FrameRingBatch with R = 32; reported as `frame_ring`, never
    # as `value` (the reference's API hands back a contiguous stacked obs).
    ring_report = None
    if world == 1 and not ring and not args.no_ring_leg:
        R = 32
        rb = FrameRingBatch(E, ring=R, config=cfg, device=dev.index)
        rb.reset(seed=19)
        rl = rb.launcher(actions, rb.rew, rb.term, rb.trunc, rb.goal, rb.score)
        for i in range(args.warmup):
            rl(i)
        torch.cuda.synchronize()
        rb.reset_stats()
        re0, re1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0 = time.perf_counter()
        re0.record(rb.stream)
        for i in range(args.steps):
            rl(args.warmup + i)
        re1.record(rb.stream)
        torch.cuda.synchronize()
        r_el = time.perf_counter() - r0
        r_kern = re0.elapsed_time(re1) / args.steps
        rst = rb.stats()
        r_kernel = ring_kernel_name(rb)
        rb.close()
        r_arb = 0.5 * (rst["cache_entries_read"] + rst["cache_entries_written"]) / max(1, rst["env_steps"])
        r_bytes = RING_BYTES + 2 * 352 / (R - 2) + 2 * ARB_BYTES * r_arb
        r_ach = r_bytes * E / (r_kern * 1e-3) / 1e9
        ring_report = {"value": E * args.steps / r_el, "unit": "env-steps/s", "ms_per_step": r_el * 1e3 / args.steps,
                       "R": R, "kernel": r_kernel,
                       "roofline": {"bound": "hbm", "achieved": r_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": r_ach / HBM_PEAK_GBS, "traffic": None,
                                    "kernel_ms": r_kern, "alg_bytes_per_env_step": r_bytes,
                                    "alg_bytes_source": "SURVEY.md §8(d) without the prior frames' read and re-write: "
                                                        f"881 + 2 x 352 B / (R - 2) wrap frames (R = {R}) + 2 x 20 B x "
                                                        "mean cached arbiters (counted by the timed launches)"},
                       "obs": f"strided (N, 4, 66) window into a (N, 4, {R}, 22) frame ring, same values as obs"}

    # ms_step_n timed beside the headline (N = 1): the same workload with the actions of K steps handed
    # over per call (an open-loop rollout); with the lane-pair kernel one launch runs the K steps, each
    # wave stepping its envs back to back. Same envs and seeds, its own window (the headline's warm-up
    # and timed steps rounded up to whole K-step launches, at least one warm-up and four timed
    # launches, so that any --steps / --warmup emits it), its own pool of uniform actions (one
    # (E, 4, 3) set per step, read from HBM) and its own (K, E, ...) outputs. Reported as
    # `fused_steps`, never as `value` (the reference's API is one step per call).
    fused_report = None
    K = args.fused
    if world == 1 and not ring and K > 0:
        f_warm = K * max(1, -(-args.warmup // K))
        f_steps = K * max(4, -(-args.steps // K))
        fb = SoccerBatch(E, config=cfg, device=dev.index)
        if args.lane_group is not None:
            fb.set_lane_group(args.lane_group)
        if args.group_solve:
            fb.set_group_solve(args.group_solve)
        fb.reset(seed=19)
        fsets = max(1, min(f_steps // K, int(args.action_gib * (1 << 30) // (E * 48 * K))))
        fpool = [torch.rand((K, E, 4, 3), device=dev, generator=gen) * 2 - 1 for _ in range(fsets)]
        fout = {name: torch.empty((K, E) + sh, dtype=dt, device=dev) for name, dt, sh in
                (("obs", torch.float32, (4, 66)), ("rew", torch.float32, (4,)), ("term", torch.uint8, (4,)),
                 ("trunc", torch.uint8, (4,)), ("goal", torch.int8, ()), ("score", torch.int32, (2,)))}
        for i in range(f_warm // K):
            fb.step_n(fpool[i % fsets], out=fout)
        torch.cuda.synchronize()
        fb.reset_stats()
        fe0, fe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0 = time.perf_counter()
        fe0.record(fb.stream)
        for i in range(f_steps // K):
            fb.step_n(fpool[i % fsets], out=fout)
        fe1.record(fb.stream)
        torch.cuda.synchronize()
        f_el = time.perf_counter() - f0
        f_kern = fe0.elapsed_time(fe1) / f_steps
        fk = {"ms_step_pair_kernel": "ms_step_pair_n_kernel", "ms_step_group_kernel": "ms_step_group_n_kernel"}.get(
            fb.step_kernel, fb.step_kernel)
        fst = fb.stats()
        f_arb = 0.5 * (fst["cache_entries_read"] + fst["cache_entries_written"]) / max(1, fst["env_steps"])
        f_bytes = SURVEY_BYTES + 2 * ARB_BYTES * f_arb
        f_ach = f_bytes * E / (f_kern * 1e-3) / 1e9
        # HBM bytes per env-step of the committed rocprofv3 PMC passes over this kernel and window
        fkey = f"e{E}_ms{args.max_steps}_K{K}_w{f_warm}_s{f_steps}"
        fpm = load_pmc_traffic(fkey, fk, "pmc_fused_kernel.json")
        f_traffic = None if fpm is None else fpm["hbm_bytes_per_launch"] / K / (f_kern * 1e-3) / 1e9
        fused_report = {"value": E * f_steps / f_el, "unit": "env-steps/s", "K": K, "warmup": f_warm,
                        "steps": f_steps, "ms_per_step": f_el * 1e3 / f_steps, "kernel": fk,
                        "kernel_ms_per_step": f_kern,
                        "launches": f_steps // K if fb.lane_group > 0 else f_steps,
                        "regime": regime(f_warm, f_steps, args.max_steps),
                        "roofline": {"bound": "hbm", "achieved": f_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": f_ach / HBM_PEAK_GBS, "traffic": f_traffic,
                                     "frac_measured": None if f_traffic is None else f_traffic / HBM_PEAK_GBS,
                                     "traffic_source": (f"{fpm['source']} window {fkey} (rocprofv3 FETCH_SIZE x 2 + "
                                                        "WRITE_SIZE per launch / K) over this run's kernel time")
                                                       if fpm else f"no committed PMC pass of {fk} for window {fkey}",
                                     "kernel_ms": f_kern, "alg_bytes_per_env_step": f_bytes},
                        "arbiter_overflow": fst["arbiter_overflow"],
                        "actions": f"{fsets} distinct (K, E, 4, 3) uniform(-1,1) blocks",
                        "api": "SoccerBatch.step_n / ms_step_n: K steps with the actions given up front (open loop)"}
        fb.close()
        del fpool, fout

    # arbiter-cache entries per env-step read and written by the timed launches themselves
    # (the kernel's per-block tally, ms_stats): the cache term of the algorithmic byte count
    steps_counted = max(1, stats["env_steps"])
    arb_read = stats["cache_entries_read"] / steps_counted
    arb_written = stats["cache_entries_written"] / steps_counted
    mean_arb = 0.5 * (arb_read + arb_written)
    bytes_per_step = SURVEY_BYTES + 2 * ARB_BYTES * mean_arb
    layout_bytes = LAYOUT_READ + LAYOUT_WRITE + 2 * ARB_BYTES * mean_arb
    if ring:
        bytes_per_step = RING_BYTES + 2 * 352 / (ring - 2) + 2 * ARB_BYTES * mean_arb
        # obs: one frame (+ two on a wrap) instead of three; the t-2 snapshot read only on a wrap
        layout_bytes += (352 + 2 * 352 / (ring - 2)) - 1056 - 104 + 104 / (ring - 2)
    achieved = bytes_per_step * E / (kern_ms * 1e-3) / 1e9
    window = regime(args.warmup, args.steps, args.max_steps)
    value = world * E * args.steps / elapsed
    if rank == 0:
        key = regime_key(E, args.max_steps, args.warmup, args.steps)
        pmc = None if ring else load_pmc_traffic(key, step_kernel)
        traffic = None
        pmc_info = None
        if pmc:
            # HBM bytes per launch measured by rocprofv3 (FETCH_SIZE x 2 + WRITE_SIZE, separate
            # passes) over the same dispatches of a run with these arguments, divided by this
            # run's per-launch time
            pmc_info = {"source": pmc["source"], "window": key, "bytes_per_launch": pmc["hbm_bytes_per_launch"],
                        "read_bytes_per_launch": pmc["hbm_read_bytes_per_launch"],
                        "write_bytes_per_launch": pmc["hbm_write_bytes_per_launch"],
                        "alg_bytes_per_launch": bytes_per_step * E,
                        "layout_bytes_per_launch": layout_bytes * E}
            traffic = pmc["hbm_bytes_per_launch"] / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: uniform(-1,1) fp32 actions (device Philox, {nsets} distinct (E,4,3) buffers "
                    f"for {args.warmup + args.steps} steps, read from HBM each step); env i seeded 19+i; " +
                    ({"rewards": "config.json physics, ball_proximity_multiplier 0.003 (runtime reward multipliers)",
                      "physics": "config.json with action_force_max 150001 (generic kernel)"}.get(args.generic,
                                                                                               "default config.json physics/rewards")) + (f", max_steps={args.max_steps}" if args.max_steps != 1000 else ""),
            "config": {"workload": f"{E} parallel envs per MI355X" +
                                   (" (BASELINE.json configs[2])" if E == 65536 and args.max_steps == 1000 else
                                    " (BASELINE.json configs[1])" if E == 4096 and args.max_steps == 1000 else
                                    " (BASELINE.json configs[4] per-GPU shard)" if E == 32768 and args.max_steps == 512
                                    else ""),
                       "envs_per_gpu": E, "global_envs": world * E, "max_steps": args.max_steps,
                       "parallelism": f"env-shard x{world}" + (" + obs all-gather" if gathered is not None else ""),
                       "launch": launch_label(batch.lane_group if not ring or batch.lane_group == 2 else 0),
                       "specialisation": {1: "default physics and rewards compiled in", 2: "default physics compiled in, "
                                          "runtime reward multipliers", 0: "generic (every parameter from the kernel "
                                          "arguments)"}[batch.specialised],
                       **({"obs_layout": f"frame ring, R = {ring} (opt-in; obs is a strided (N, 4, 66) window)"}
                          if ring else {}),
                       **({"group_solve": {1: "serial halves", 2: "dependency-level rounds"}.get(args.group_solve,
                                                                                            args.group_solve)}
                          if args.group_solve else {})},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         # the HBM bytes rocprofv3 measured (traffic) over the same time: the
                         # fraction of peak the launch really moves
                         "frac_measured": None if traffic is None else traffic / HBM_PEAK_GBS,
                         "kernel": step_kernel, "kernel_ms": kern_ms,
                         "kernel_ms_method": "HIP events around the K back-to-back launches / K",
                         "alg_bytes_per_env_step": bytes_per_step,
                         "alg_bytes_source": ("SURVEY.md §8(d) without the prior frames' read and re-write: 881 + "
                                              f"2 x 352 B / (R - 2) wrap frames (R = {ring}) + 2 x 20 B x mean cached "
                                              "arbiters") if ring else
                                             "SURVEY.md §8(d): 2,289 + 2 x 20 B x mean cached arbiters",
                         "layout_bytes_per_env_step": layout_bytes,
                         "traffic_source": (pmc_info["source"] + f" window {key} (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE "
                                            "per launch, same dispatches of a run with these arguments) over this "
                                            "run's kernel_ms") if traffic is not None else
                                           f"no committed PMC pass of {step_kernel} for window {key}",
                         # counted by the kernel over the timed launches (ms_stats tally)
                         "mean_cached_arbiters": mean_arb,
                         "cache_entries_per_env_step": {"read": arb_read, "written": arb_written,
                                                        "env_steps_counted": stats["env_steps"]},
                         "pmc": pmc_info},
            "regime": window,
            "arbiter_overflow": overflow_warmup + stats["arbiter_overflow"],
        }
        if gather_report is not None:
            line["with_obs_allgather"] = gather_report
        if ring_report is not None:
            line["frame_ring"] = ring_report
        if fused_report is not None:
            line["fused_steps"] = fused_report
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
