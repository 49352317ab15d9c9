#!/bin/bash
OUT=gpurun_out/r03h; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_policy.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_policy.log 2>&1; rc=$?
tail -4 $OUT/pytest_policy.log
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAIL" $OUT/pytest_policy.log | head -60; exit $rc; }
for P in fused torch; do
  timeout -k 10 200 python tools/bench_rollout.py --envs 65536 --steps 64 --graph --policy $P > $OUT/rollout_graph_$P.json 2> $OUT/rollout_$P.err || { tail -5 $OUT/rollout_$P.err; exit 1; }
  cat $OUT/rollout_graph_$P.json
  timeout -k 10 200 python tools/bench_rollout.py --envs 65536 --steps 64 --policy $P > $OUT/rollout_eager_$P.json 2>> $OUT/rollout_$P.err || { tail -5 $OUT/rollout_$P.err; exit 1; }
  cat $OUT/rollout_eager_$P.json
done
