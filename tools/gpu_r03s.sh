set -o pipefail
mkdir -p gpurun_out/r03s
B="python bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --no-ring-leg"
timeout -k 10 120 $B --envs 8192 --lane-group 8 > gpurun_out/r03s/bench_8192_g8.json 2> gpurun_out/r03s/bench_8192_g8.err || exit 11
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lane_group or corner or fallback" > gpurun_out/r03s/pytest.log 2>&1 || exit 12
for N in 4096 8192; do for G in 0 8 16; do
  timeout -k 10 120 $B --envs $N --lane-group $G > gpurun_out/r03s/bench_${N}_g$G.json 2> gpurun_out/r03s/bench_${N}_g$G.err || exit 13
done; done
