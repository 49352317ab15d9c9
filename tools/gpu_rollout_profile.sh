#!/bin/bash
OUT=gpurun_out/r03n; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python tools/bench_rollout.py --envs 65536 --steps 64 --graph > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
head -30 $OUT/trace/run_kernel_stats.csv
