set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
B="python bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --no-ring-leg"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lane_group" > $O/pytest.log 2>&1 || exit 12
for N in 4096 8192; do for G in 0 8 16; do
  timeout -k 10 120 $B --envs $N --lane-group $G > $O/bench_${N}_g$G.json 2> $O/bench_${N}_g$G.err || exit 13
done; done
timeout -k 10 180 python tools/stamps.py --envs 8192 --steps 300 --warmup 1000 --every 10 --lane-group 8 --out $O/stamps_8192_g8.json > $O/stamps_8192_g8.log 2>&1 || exit 14
timeout -k 10 180 python tools/stamps.py --envs 8192 --steps 300 --warmup 1000 --every 10 --lane-group 0 --out $O/stamps_8192_g0.json > $O/stamps_8192_g0.log 2>&1 || exit 15
