#!/bin/bash
# The lane-group kernel's contact-solve modes (bench.py --group-solve: 0 automatic, 1 serial halves,
# 2 rounds) at 4,096 and 8,192 envs, steady window, for the product library or lib/exp variants:
#   bash tools/group_solve_ab.sh TAG [variant ...]
O=gpurun_out/$1; shift; mkdir -p $O
VS=${@:-product}
for r in 1 2; do for V in $VS; do for N in 4096 8192; do for M in 0 1 2; do
  if [ $M = 1 ] && [ "$V" != product ] && [ "$V" != base ]; then continue; fi
  if [ "$V" = product ]; then unset MARL_SOCCER_LIB; else export MARL_SOCCER_LIB=marl-soccer_amd/lib/exp/lib_$V.so; fi
  timeout -k 10 200 python bench.py --envs $N --group-solve $M --no-cpu-baseline --no-ring-leg --fused 0 > $O/b_${V}_${N}_${M}.json 2> $O/b_${V}_${N}_${M}.err || { tail $O/b_${V}_${N}_${M}.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['roofline']['kernel_ms']*1e3,2), 'us')" $O/b_${V}_${N}_${M}.json $V $N $M | tee -a $O/summary.txt
done; done; done; done
