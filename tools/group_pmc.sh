#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over the lane-group kernel (steady window) at the given batch sizes
# (run on the GPU box from the repo root; summarised by tools/ring_pmc.py-style medians in the log)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for N in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/gpmc_${N}_$C -o run -- python bench.py --envs $N --warmup 1000 --steps 200 --no-cpu-baseline --no-ring-leg --fused 0 > $O/gpmc_${N}_$C.log 2>&1 \
      || { echo "group pmc $N $C failed"; tail -5 $O/gpmc_${N}_$C.log; exit 1; }
  done
  python3 - "$O" "$N" <<'PY'
import csv, statistics, sys, json
o, n = sys.argv[1], int(sys.argv[2])
def med(c):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{o}/gpmc_{n}_{c}/run_counter_collection.csv")) if "ms_step_group_kernel<" in r["Kernel_Name"]]
    return statistics.median(v[-200:]), len(v)
(f, nf), (w, nw) = med("FETCH_SIZE"), med("WRITE_SIZE")
out = {"envs": n, "kernel": "ms_step_group_kernel", "launches": [nf, nw], "hbm_read_bytes_per_env_step": 2 * f * 1024 / n,
       "hbm_write_bytes_per_env_step": w * 1024 / n, "correction": "read = 2 x FETCH_SIZE KiB (gfx950), write = WRITE_SIZE KiB; medians of the last 200 launches"}
out["hbm_bytes_per_env_step"] = out["hbm_read_bytes_per_env_step"] + out["hbm_write_bytes_per_env_step"]
json.dump(out, open(f"{o}/group_pmc_{n}.json", "w"), indent=1)
print(json.dumps(out))
PY
done
