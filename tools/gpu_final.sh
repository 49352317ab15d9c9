#!/bin/bash
# Runs on the GPU box: the whole GPU suite, smoke(), the default bench line, the BASELINE configs
# (tools/gpu_configs.sh) and the lane-group stamps at 8,192 / 4,096 envs. Stops at the first
# failing step. Usage: tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-r03final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash tools/gpu_configs.sh ${TAG}_configs || exit 1
bash tools/gpu_group_stamps.sh ${TAG}_stamps 8192 4096 || exit 1
