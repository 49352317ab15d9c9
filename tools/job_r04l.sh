# r04l: the lane-group K-step launch (ms_step_group_n_kernel): step_n tests (all launch shapes),
# lane-group parity, open-loop rates at the small batches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_step_n.py > $O/pytest_step_n.log 2>&1 || { tail -30 $O/pytest_step_n.log; exit 1; }
tail -2 $O/pytest_step_n.log
bash tools/gpu.sh multi "parity r04l lanes8+or+lanes16+or+group+or+lane-group" || exit 1
timeout -k 10 300 python tools/bench_fused.py --envs 4096 8192 --k 10 50 250 > $O/fused_small.jsonl 2> $O/fused_small.err || { tail -5 $O/fused_small.err; exit 1; }
cat $O/fused_small.jsonl
bash tools/gpu.sh multi "bench1 r04l 4096 --envs 4096" "bench1 r04l 65536 --envs 65536" && python -c "
import json
for n in ('4096', '65536'):
    d = json.loads(open(f'gpurun_out/r04l/bench_{n}.json').read().strip().splitlines()[-1]); print(n, d['fused_steps'])"
