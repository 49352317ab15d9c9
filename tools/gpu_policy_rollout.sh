#!/bin/bash
OUT=gpurun_out/r03o; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_policy.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_policy.log 2>&1; rc=$?
tail -3 $OUT/pytest_policy.log
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAIL" $OUT/pytest_policy.log | head -60; exit $rc; }
timeout -k 10 300 python tools/bench_policy.py --envs 65536 --iters 30 > $OUT/bench_policy.jsonl 2> $OUT/bench_policy.err || { tail -5 $OUT/bench_policy.err; exit 1; }
grep ms_policy $OUT/bench_policy.jsonl
timeout -k 10 200 python tools/bench_rollout.py --envs 65536 --steps 64 --graph > $OUT/rollout_graph.json 2> $OUT/rollout.err || { tail -5 $OUT/rollout.err; exit 1; }
cat $OUT/rollout_graph.json
timeout -k 10 200 python tools/bench_rollout.py --envs 65536 --steps 64 --graph --policy torch > $OUT/rollout_graph_torch.json 2>> $OUT/rollout.err || { tail -5 $OUT/rollout.err; exit 1; }
cat $OUT/rollout_graph_torch.json
