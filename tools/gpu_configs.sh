#!/bin/bash
# The BASELINE configurations' per-GPU batch sizes on one GPU (bench.py's protocol, steady-state
# window unless noted) and the driver's short window; one JSON line each under gpurun_out/<tag>/.
# Usage: tools/gpu_configs.sh <tag>
set -o pipefail
TAG=${1:-r03_configs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
    || { echo "bench $name failed"; tail -20 $OUT/bench_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us', round(d['value']/1e6,1), 'M/s', 'frac', round(d['roofline']['frac'],3), 'ring', d.get('frame_ring',{}).get('ms_per_step'))" $OUT/bench_$name.json $name
}
run driver_window --steps 20 --warmup 5
run 4096 --envs 4096
run 8192 --envs 8192
run 32768_ms512 --envs 32768 --max-steps 512
run 131072 --envs 131072
run 262144_ms512 --envs 262144 --max-steps 512 --steps 512 --warmup 512
