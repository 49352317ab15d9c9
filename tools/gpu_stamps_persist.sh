#!/bin/bash
# Wave timelines (tools/stamps.py) of the step kernel: one wave per block vs the persistent launch.
OUT=gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 300 python tools/stamps.py --envs 65536 --warmup 1000 --steps 200 --every 10 --persistent 0 --out $OUT/stamps_65536_steady.json > $OUT/s1.log 2>&1 || { tail -20 $OUT/s1.log; exit 1; }
timeout -k 10 300 python tools/stamps.py --envs 262144 --warmup 1000 --steps 200 --every 10 --persistent 0 --out $OUT/stamps_262144_perblock.json > $OUT/s2.log 2>&1 || { tail -20 $OUT/s2.log; exit 1; }
timeout -k 10 300 python tools/stamps.py --envs 262144 --warmup 1000 --steps 200 --every 10 --persistent -1 --out $OUT/stamps_262144_persistent.json > $OUT/s3.log 2>&1 || { tail -20 $OUT/s3.log; exit 1; }
for f in $OUT/stamps_*.json; do python -c "
import json,sys; d=json.load(open('$f')); print('$f', d['launch'], 'mean', round(d['wave_cycles_mean']), 'slow5', round(d['wave_cycles_slowest5pct']), 'span', round(d['launch_span_cycles'])); print({k:v['mean'] for k,v in d['phases'].items()})"; done
