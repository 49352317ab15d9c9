#!/bin/bash
# Runs on the GPU box (via gpurun): bench line + rocprofv3 kernel-trace stats + PMC passes.
# Usage: tools/gpu_bench_profile.sh <tag> [bench args...]
# PMC: FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md), each over two timed
# windows of bench.py: the driver's (--warmup 5 --steps 20, first episode) and the steady state
# (--warmup 1000 --steps 1000, the default bench window); tools/pmc_summary.py keeps the window's dispatches only.
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --no-cpu-baseline "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
for WS in "5 20" "1000 1000"; do
  set -- $WS
  W=$1; S=$2
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_${C}_w${W}_s${S} -o run -- python bench.py --warmup $W --steps $S --no-cpu-baseline --no-ring-leg > $OUT/pmc_${C}_w${W}_s${S}.log 2>&1 || { echo "pmc $C w$W s$S failed"; tail -20 $OUT/pmc_${C}_w${W}_s${S}.log; exit 1; }
  done
done
find $OUT -name "*.csv" | head -20
