#!/bin/bash
# Runs on the GPU box (via gpurun): the lane-group kernel's parity tests (and every GPU parity test
# of small batches, which take the lane-group launch by default), benches at 4,096 and 8,192 envs
# and the per-phase stamps of the 8,192-env shard. Usage: tools/gpu_group_check.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --no-ring-leg"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 12; }
tail -2 $O/pytest.log
for N in 4096 8192; do
  timeout -k 10 120 $B --envs $N > $O/bench_$N.json 2> $O/bench_$N.err || { tail $O/bench_$N.err; exit 13; }
  python -c "import json; d=json.load(open('$O/bench_$N.json')); print($N, round(d['ms_per_step']*1e3, 2), 'us', d['config']['launch'])"
done
timeout -k 10 180 python tools/stamps.py --envs 8192 --steps 300 --warmup 1000 --every 10 --lane-group 8 --out $O/stamps_8192_g8.json > $O/stamps_8192_g8.log 2>&1 || { tail $O/stamps_8192_g8.log; exit 14; }
python -c "import json; d=json.load(open('$O/stamps_8192_g8.json')); print(d['worst_wave_cycles_mean'], d['worst_wave_phases_mean'])"
