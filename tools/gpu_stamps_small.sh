#!/bin/bash
# stamps of small shards (latency floor): 8,192 and 4,096 envs, steady state
OUT=gpurun_out/r03p; mkdir -p $OUT
for n in 8192 4096; do
  timeout -k 10 240 python tools/stamps.py --envs $n --steps 300 --every 10 --warmup 1000 --out $OUT/stamps_${n}_steady.json > $OUT/stamps_$n.log 2>&1 || { tail -5 $OUT/stamps_$n.log; exit 1; }
done
python - <<'PY'
import json
for n in (8192, 4096):
    r = json.load(open(f"gpurun_out/r03p/stamps_{n}_steady.json"))
    print(n, round(r["wave_cycles_mean"]), round(r["wave_cycles_slowest5pct"]), round(r["launch_span_cycles"]))
    for k, v in r["phases"].items():
        print("  ", k, v["mean"], v["slow5"], r["worst_wave_phases_mean"].get(k))
PY
