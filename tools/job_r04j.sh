# r04j: the r04f lane-pair kernel (early obs stores reverted) + the fused K-step launch: whole GPU
# suite + smoke, per-call A/B against r04f, default bench line (with its fused_steps leg), profile
bash tools/gpu.sh multi "suite r04j" && timeout -k 10 400 python tools/variants.py run --envs 65536 f cur f cur > gpurun_out/r04j/variants.txt 2>&1; cat gpurun_out/r04j/variants.txt; bash tools/gpu.sh multi "profile r04j" && python -c "import json; d=json.loads(open('gpurun_out/r04j/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'], d.get('fused_steps'))"
