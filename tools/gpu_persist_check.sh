mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03c/pytest_parity.log 2>&1 || { tail -30 gpurun_out/r03c/pytest_parity.log; exit 1; }
tail -2 gpurun_out/r03c/pytest_parity.log
for E in 65536 131072 262144; do for W in 0 -1; do
  MS=1000; [ $E = 262144 ] && MS=512
  timeout -k 10 300 python bench.py --envs $E --max-steps $MS --persistent $W --no-cpu-baseline --no-ring-leg > gpurun_out/r03c/bench_${E}_p${W}.json 2> gpurun_out/r03c/bench_${E}_p${W}.err || { tail -5 gpurun_out/r03c/bench_${E}_p${W}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03c/bench_${E}_p${W}.json')); print($E, $W, round(d['value']/1e9,4), round(d['ms_per_step']*1e3,2), d['config']['launch'])"
done; done
