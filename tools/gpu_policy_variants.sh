#!/bin/bash
# Policy-kernel build variants (A-operand prefetch depth, chunk of output tiles), timed by
# tools/bench_policy.py's ms_policy_forward leg.
OUT=gpurun_out/r03g; mkdir -p $OUT
for L in marl-soccer_amd/lib/libpolv_*.so; do
  V=$(basename $L .so)
  MARL_SOCCER_LIB=$PWD/$L timeout -k 10 200 python tools/bench_policy.py --envs 65536 --iters 30 > $OUT/$V.jsonl 2> $OUT/$V.err || { tail -3 $OUT/$V.err; exit 1; }
  echo "$V $(grep '"ms_policy_forward"' $OUT/$V.jsonl)"
done
