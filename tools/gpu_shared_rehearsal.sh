#!/bin/bash
# Multi-rank bench.py on ONE GPU (MS_BENCH_SHARED_GPU=1: every rank on cuda:0, gloo for the
# barrier, the max-reduce and the obs all-gather leg); a rehearsal of the driver's N-GPU runs.
# Usage: tools/gpu_shared_rehearsal.sh <tag>
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export MS_BENCH_SHARED_GPU=1
for E in 8192 65536; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --envs $E --steps 200 --warmup 50 > $OUT/bench_shared2_e$E.json 2> $OUT/bench_shared2_e$E.err \
    || { echo "shared bench E=$E failed"; tail -20 $OUT/bench_shared2_e$E.err; exit 1; }
  cat $OUT/bench_shared2_e$E.json
done
