#!/bin/bash
# Runs on the GPU box: per-phase stamps of the lane-group kernel (tools/stamps.py; build the stamps
# library here first with `python tools/stamps.py --build`). Usage: tools/gpu_group_stamps.sh <tag> [envs...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
for N in ${@:-8192}; do
  timeout -k 10 180 python tools/stamps.py --envs $N --steps 300 --warmup 1000 --every 10 --out $O/stamps_$N.json > $O/stamps_$N.log 2>&1 || { tail $O/stamps_$N.log; exit 14; }
  python -c "import json; d=json.load(open('$O/stamps_$N.json')); print($N, d['launch'], 'worst', round(d['worst_wave_cycles_mean']), {k: round(v) for k, v in d['worst_wave_phases_mean'].items()}, 'maxc', d['worst_wave_max_contacts'])"
done
