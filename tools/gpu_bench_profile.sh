#!/bin/bash
# Runs on the GPU box (via gpurun): bench line + rocprofv3 kernel-trace stats + PMC passes.
# Usage: tools/gpu_bench_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --no-cpu-baseline "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 200 --warmup 1000 --no-cpu-baseline "$@" > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 200 --warmup 1000 --no-cpu-baseline "$@" > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
