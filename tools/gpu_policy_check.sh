#!/bin/bash
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_policy.py -x -v --timeout 200 --timeout-method thread -k fused > $OUT/pytest_policy.log 2>&1; rc=$?
tail -15 $OUT/pytest_policy.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_policy.py --envs 65536 --iters 20 > $OUT/bench_policy.jsonl 2> $OUT/bench_policy.err || { tail -5 $OUT/bench_policy.err; exit 1; }
cat $OUT/bench_policy.jsonl
