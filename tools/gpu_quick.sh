#!/bin/bash
# Runs on the GPU box: GPU parity tests of the step kernels, then the bench at the given batch sizes
# (steady-state window). Usage: tools/gpu_quick.sh <tag> [envs...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
tail -1 $O/pytest.log
for N in ${@:-8192}; do
  timeout -k 10 200 python bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --no-ring-leg --envs $N > $O/bench_$N.json 2> $O/bench_$N.err || { tail $O/bench_$N.err; exit 13; }
  python -c "import json; d=json.load(open('$O/bench_$N.json')); print($N, round(d['ms_per_step']*1e3, 2), 'us', round(d['value']/1e6, 1), 'M/s', d['config']['launch'])"
done
