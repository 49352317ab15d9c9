#!/bin/bash
# A/B of lib/exp variants: generic physics (PM 0) steady window with its K-step leg, and the driver's window
# with the K-step leg (default config)
O=gpurun_out/$1; shift; mkdir -p $O  # ENVS=N: another batch size (default 65,536)
for r in 1 2; do
  for V in "$@"; do
    MARL_SOCCER_LIB=marl-soccer_amd/lib/exp/lib_$V.so timeout -k 10 300 python bench.py --envs ${ENVS:-65536} --generic physics --no-cpu-baseline --no-ring-leg --fused 50 > $O/gphys_$V.json 2>$O/gphys_$V.err || { tail $O/gphys_$V.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); f=d.get('fused_steps') or {}; print(sys.argv[2], 'generic physics', round(d['roofline']['kernel_ms']*1e3,2), 'us; fused', f.get('ms_per_step') and round(f['ms_per_step']*1e3,2), 'us')" $O/gphys_$V.json $V
    MARL_SOCCER_LIB=marl-soccer_amd/lib/exp/lib_$V.so timeout -k 10 300 python bench.py --envs ${ENVS:-65536} --no-cpu-baseline --no-ring-leg --fused 50 --steps 20 --warmup 5 > $O/fused_$V.json 2>$O/fused_$V.err || { tail $O/fused_$V.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); f=d.get('fused_steps') or {}; print(sys.argv[2], 'driver', round(d['roofline']['kernel_ms']*1e3,2), 'us; fused', f.get('ms_per_step') and round(f['ms_per_step']*1e3,2), 'us')" $O/fused_$V.json $V
  done
done
