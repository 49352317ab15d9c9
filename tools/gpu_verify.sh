#!/bin/bash
# Runs on the GPU box (via gpurun): the GPU test suite, smoke(), then the bench line and the
# rocprofv3 summaries of tools/gpu_bench_profile.sh. Stops at the first failing step.
# Usage: tools/gpu_verify.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/gpu_bench_profile.sh "$@"
