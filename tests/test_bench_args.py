"""bench.py's rank logic (CPU): `--gpus N` must mean N ranks. A plain `python bench.py --gpus N`
starts torch.distributed.run with N processes as a child (the driver's own form, 127.0.0.1
rendezvous) and exits with its code; under a launcher, an explicit --gpus that differs from
WORLD_SIZE is an error, so no N-GPU request can print a one-GPU line."""
import argparse
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # top level imports only the standard library
    return mod


def ns(gpus):
    return argparse.Namespace(gpus=gpus)


def test_plain_run_with_gpus_n_starts_n_ranks_as_a_child(bench):
    calls = []

    def fake_run(argv):
        calls.append(argv)
        return 7

    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    how = bench.resolve_world(ns(8), argv, env={}, run=fake_run)
    assert how == {"exit": 7} and len(calls) == 1
    cmd = calls[0]
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # the same bench arguments, --gpus included (checked by every rank)


def test_single_gpu_and_launcher_worlds(bench):
    never = lambda argv: pytest.fail("no child launch expected")  # noqa: E731
    assert bench.resolve_world(ns(None), [], env={}, run=never) == {"world": 1}
    assert bench.resolve_world(ns(1), ["--gpus", "1"], env={}, run=never) == {"world": 1}
    assert bench.resolve_world(ns(2), [], env={"WORLD_SIZE": "2"}, run=never) == {"world": 2}
    assert bench.resolve_world(ns(None), [], env={"WORLD_SIZE": "4"}, run=never) == {"world": 4}


def test_gpus_must_match_the_launcher(bench):
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.resolve_world(ns(8), [], env={"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.resolve_world(ns(0), [], env={})


def test_launch_label_names_the_lane_pair_kernel(bench):
    assert bench.launch_label(2).startswith("lane pairs, 2 lanes per env (32 envs per wave")
    assert bench.launch_label(8) == "lane groups, 8 lanes per env (8 envs per wave)"
    assert bench.launch_label(0).startswith("one lane per env")


def test_bench_source_compiles_without_warnings():
    """bench.py's JSON-line strings are built by implicit concatenation; a missing '+' before a
    parenthesised part turns it into a call that only fails on the GPU box (SyntaxWarning here)."""
    import warnings
    with open(os.path.join(ROOT, "bench.py")) as f:
        src = f.read()
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        compile(src, "bench.py", "exec")
