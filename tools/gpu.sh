#!/bin/bash
# One runner for every GPU-box job (run through gpurun from the repo root). Each step runs under
# its own time limit; the first failing step ends the call (no GPU step after a failure).
#
#   tools/gpu.sh suite    <tag>                 whole `pytest -m gpu` suite + smoke()
#   tools/gpu.sh parity   <tag> [pytest -k expr] tests/test_gpu_parity.py (optionally filtered)
#   tools/gpu.sh bench    <tag> [envs...]       steady-state bench line per batch size (no CPU leg)
#   tools/gpu.sh profile  <tag> [bench args]    bench line + rocprofv3 kernel-trace stats + FETCH/WRITE PMC
#                                               passes over the driver's and the default window
#   tools/gpu.sh configs  <tag>                 the BASELINE configs' per-GPU batch sizes
#   tools/gpu.sh sq       <tag> <envs> [bench args]  SQ counter passes (steady window: warm-up 1000, 100 steps)
#   tools/gpu.sh sqfused  <tag> <envs> <K>      SQ counter passes over the K-step launch (10 timed launches)
#   tools/gpu.sh fused    <tag> <envs> <K>       K-step launch sweep (tools/bench_fused.py; "+" joins values)
#   tools/gpu.sh pmcfused <tag> <envs> <K>      FETCH/WRITE PMC passes + kernel trace over the K-step launch
#   tools/gpu.sh stamps   <tag> [G=lanes] <envs...>  per-phase wave stamps (tools/stamps.py; stamps library prebuilt)
#   tools/gpu.sh rehearse <tag>                 plain `bench.py --gpus 2` (it starts torchrun itself), both ranks on cuda:0 (gloo)
#   tools/gpu.sh driver   <tag>                 the driver's own `bench.py --gpus 1 --steps 20 --warmup 5` line
#   tools/gpu.sh ringpmc  <tag>                 FETCH/WRITE PMC + kernel trace of the frame-ring leg (lane-pair ring kernel)
#   tools/gpu.sh groupprof <tag>                lane-group kernel at 4,096 / 8,192 envs: kernel trace + stamps (lib/exp/lib_stg.so)
#   tools/gpu.sh policy   <tag>                 policy/rollout GPU tests + bench_policy + graph rollouts
#
# Several jobs in one call: tools/gpu.sh multi "suite r04a" "sq r04a_sq 65536" ...
set -o pipefail
export TMPDIR=/tmp
job=$1; shift

suite() {
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; return 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; return 1; }
  cat $O/smoke.log
}

parity() {
  local O=gpurun_out/$1; shift; mkdir -p $O
  local K=()
  [ -n "$1" ] && K=(-k "${1//+/ }")  # "+" stands for a space in the -k expression
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py "${K[@]}" > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; return 1; }
  tail -1 $O/pytest.log
}

ptest() {  # tag test-file: one GPU test file
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$2" > $O/pytest_$(basename $2 .py).log 2>&1 \
    || { tail -40 $O/pytest_$(basename $2 .py).log; return 1; }
  tail -1 $O/pytest_$(basename $2 .py).log
}

bench1() {  # tag name bench-args...
  local O=gpurun_out/$1 name=$2; shift 2; mkdir -p $O
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-ring-leg "$@" > $O/bench_$name.json 2> $O/bench_$name.err \
    || { echo "bench $name failed"; tail -20 $O/bench_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,2), 'us', round(d['value']/1e6,1), 'M/s frac', round(r['frac'],3), r.get('kernel'), d['config'].get('launch'))" $O/bench_$name.json $name
}

bench() {
  local T=$1; shift
  for N in ${@:-65536}; do bench1 $T $N --envs $N || return 1; done
}

configs() {
  local T=$1
  bench1 $T driver_window --steps 20 --warmup 5 || return 1
  bench1 $T 4096 --envs 4096 || return 1
  bench1 $T 8192 --envs 8192 || return 1
  bench1 $T 16384 --envs 16384 || return 1
  bench1 $T 32768_ms512 --envs 32768 --max-steps 512 || return 1
  bench1 $T 65536 --envs 65536 || return 1
  bench1 $T 131072 --envs 131072 || return 1
  bench1 $T 262144_ms512 --envs 262144 --max-steps 512 --steps 512 --warmup 512 || return 1
}

profile() {
  local T=$1; shift
  local O=gpurun_out/$T; mkdir -p $O
  timeout -k 10 300 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; return 1; }
  cat $O/bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --no-cpu-baseline "$@" > $O/trace.log 2>&1 \
    || { echo "trace failed"; tail -20 $O/trace.log; return 1; }
  local WS W S C
  for WS in "5 20" "1000 1000"; do
    read W S <<< "$WS"
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${C}_w${W}_s${S} -o run -- python bench.py --warmup $W --steps $S --no-cpu-baseline --no-ring-leg "$@" > $O/pmc_${C}_w${W}_s${S}.log 2>&1 \
        || { echo "pmc $C w$W s$S failed"; tail -20 $O/pmc_${C}_w${W}_s${S}.log; return 1; }
    done
  done
}

sq() {  # tag envs bench-args...
  local T=$1 N=$2; shift 2
  local O=gpurun_out/$T/sq_$N; mkdir -p $O
  local P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  local P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
  local P3="SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS"
  local i=0 P
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python bench.py --envs $N --warmup 1000 --steps 100 --no-cpu-baseline --no-ring-leg --fused 0 "$@" > $O/p$i.log 2>&1 \
      || { echo "sq pass $i failed"; tail -5 $O/p$i.log; return 1; }
  done
  python tools/sq_summary.py $O --last 100 --json $O/summary.json | tee $O/summary.txt
  rm -rf $O/p1 $O/p2 $O/p3  # the raw per-dispatch CSVs exceed gpurun's 64-MiB copy-back
}

vsq() {  # tag envs name...: one SQ pass (instruction mix) over each lib/exp variant's step kernel, steady window
  local T=$1 N=$2; shift 2
  local P="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"
  local v
  for v in "$@"; do
    local O=gpurun_out/$T/vsq_${v}_$N; mkdir -p $O
    MARL_SOCCER_LIB=marl-soccer_amd/lib/exp/lib_$v.so timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p1 -o run -- python bench.py --envs $N --warmup 1000 --steps 100 --no-cpu-baseline --no-ring-leg --fused 0 > $O/p1.log 2>&1 \
      || { echo "vsq $v failed"; tail -5 $O/p1.log; return 1; }
    echo "--- $v"; python tools/sq_summary.py $O --last 100 --json $O/summary.json | tee $O/summary.txt
    rm -rf $O/p1
  done
}

fused() {  # tag envs K ("+" joins several: 4096+65536 10+50): tools/bench_fused.py sweep, steady window
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 400 python tools/bench_fused.py --envs ${2//+/ } --k ${3//+/ } >> $O/fused.jsonl 2>> $O/fused.err || { tail -5 $O/fused.err; return 1; }
  cat $O/fused.jsonl
}

pmcfused() {  # tag envs K: FETCH_SIZE / WRITE_SIZE passes and a kernel-trace run over the K-step launch
  local T=$1 N=$2 K=$3 C
  local O=gpurun_out/$T; mkdir -p $O
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_fused_$C -o run -- python tools/bench_fused.py --envs $N --k $K > $O/pmc_fused_$C.log 2>&1 \
      || { echo "pmc $C failed"; tail -5 $O/pmc_fused_$C.log; return 1; }
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_fused -o run -- python tools/bench_fused.py --envs $N --k $K > $O/trace_fused.log 2>&1 \
    || { echo "trace failed"; tail -5 $O/trace_fused.log; return 1; }
}

sqfused() {  # tag envs K: the SQ passes over the open-loop K-step launch (tools/bench_fused.py)
  local T=$1 N=$2 K=$3
  local O=gpurun_out/$T/sqfused_$N; mkdir -p $O
  local P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  local P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH"
  local P3="SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INSTS"
  local i=0 P
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python tools/bench_fused.py --envs $N --k $K --steps $((10 * K)) --warmup $((10 * K)) > $O/p$i.log 2>&1 \
      || { echo "sqfused pass $i failed"; tail -5 $O/p$i.log; return 1; }
  done
  python tools/sq_summary.py $O --last 10 --json $O/summary.json | tee $O/summary.txt
  rm -rf $O/p1 $O/p2 $O/p3
}

stamps() {  # tag [G=lanes] envs...
  local T=$1; shift
  local O=gpurun_out/$T; mkdir -p $O
  local LG=()
  case "$1" in G=*) LG=(--lane-group ${1#G=}); shift;; esac
  for N in "$@"; do
    timeout -k 10 240 python tools/stamps.py --envs $N --steps 300 --warmup 1000 --every 10 "${LG[@]}" --out $O/stamps_$N.json > $O/stamps_$N.log 2>&1 || { tail $O/stamps_$N.log; return 1; }
    python -c "import json; d=json.load(open('$O/stamps_$N.json')); print($N, d['launch'], 'mean', round(d['wave_cycles_mean']), 'worst', round(d.get('worst_wave_cycles_mean', 0)), {k: round(v['mean']) for k, v in d['phases'].items()})"
  done
}

rehearse() {  # bench.py --gpus 2 through the PLAIN entry (bench.py starts torch.distributed.run itself), both ranks on cuda:0 (gloo)
  local O=gpurun_out/$1; mkdir -p $O
  local E
  for E in 8192 65536; do
    MS_BENCH_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --envs $E --steps 200 --warmup 50 > $O/bench_shared2_e$E.json 2> $O/bench_shared2_e$E.err \
      || { echo "shared bench E=$E failed"; tail -20 $O/bench_shared2_e$E.err; return 1; }
    cat $O/bench_shared2_e$E.json
  done
}

vrun() {  # tag name...: time lib/exp variants (tools/variants.py run), steady window then the driver's window, twice
  local O=gpurun_out/$1; shift; mkdir -p $O
  local r
  for r in 1 2; do
    timeout -k 10 600 python tools/variants.py run --envs 65536 "$@" >> $O/variants.txt 2>&1 || { tail -20 $O/variants.txt; return 1; }
    timeout -k 10 600 python tools/variants.py run --envs 65536 --steps 20 --warmup 5 "$@" >> $O/variants_driver.txt 2>&1 || { tail -20 $O/variants_driver.txt; return 1; }
  done
  cat $O/variants.txt $O/variants_driver.txt
}

vrunn() {  # tag envs name...: vrun at another batch size (steady window, twice)
  local O=gpurun_out/$1 N=$2; shift 2; mkdir -p $O
  local r
  for r in 1 2; do
    timeout -k 10 600 python tools/variants.py run --envs $N "$@" >> $O/variants_$N.txt 2>&1 || { tail -20 $O/variants_$N.txt; return 1; }
  done
  cat $O/variants_$N.txt
}

vstamps() {  # tag lib-name envs: per-phase stamps of a -DMS_STAMPS lib/exp variant
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 240 python tools/stamps.py --fine --lib marl-soccer_amd/lib/exp/lib_$2.so --envs $3 --steps 300 --warmup 1000 --every 10 --out $O/stamps_$2_$3.json > $O/stamps_$2_$3.log 2>&1 || { tail $O/stamps_$2_$3.log; return 1; }
  python -c "import json; d=json.load(open('$O/stamps_$2_$3.json')); print('$2', $3, 'mean', round(d['wave_cycles_mean']), 'slow5', round(d['wave_cycles_slowest5pct']), 'worst', round(d.get('worst_wave_cycles_mean', 0)), {k: round(v['mean']) for k, v in d['phases'].items()}); t=d['timeline']; print({k: v for k, v in t.items() if k != 'waves_in_phase_per_us_bin'})"
}

vstampsd() {  # tag lib-name envs: the same over the driver's window (warm-up 5, 20 steps, every launch)
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 240 python tools/stamps.py --fine --lib marl-soccer_amd/lib/exp/lib_$2.so --envs $3 --steps 20 --warmup 5 --every 1 --out $O/stampsd_$2_$3.json > $O/stampsd_$2_$3.log 2>&1 || { tail $O/stampsd_$2_$3.log; return 1; }
  python -c "import json; d=json.load(open('$O/stampsd_$2_$3.json')); print('$2', $3, 'mean', round(d['wave_cycles_mean']), 'slow5', round(d['wave_cycles_slowest5pct']), 'worst', round(d.get('worst_wave_cycles_mean', 0)), {k: round(v['mean']) for k, v in d['phases'].items()}); t=d['timeline']; print({k: v for k, v in t.items() if k != 'waves_in_phase_per_us_bin'})"
}

tcc() {  # tag lib-name: HBM request-size split of the lane-pair step kernel (tools/tcc_split.py), steady window
  local T=$1 V=$2 i=0 P
  local O=gpurun_out/$T/tcc_$V; mkdir -p $O
  local LIB=marl-soccer_amd/lib/exp/lib_$V.so
  [ "$V" = product ] && LIB=marl-soccer_amd/lib/libmarlsoccer.so
  for P in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum"; do
    i=$((i+1))
    MARL_SOCCER_LIB=$LIB timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python bench.py --envs 65536 --warmup 1000 --steps 200 --no-cpu-baseline --no-ring-leg --fused 0 > $O/p$i.log 2>&1 \
      || { echo "tcc pass $i failed"; tail -5 $O/p$i.log; return 1; }
  done
  python tools/tcc_split.py $O ms_step_pair_kernel 65536 200 | tee $O/summary.json
  rm -rf $O/p1 $O/p2  # the raw per-dispatch CSVs exceed gpurun's 64-MiB copy-back
}

ringpmc() {  # tag: FETCH/WRITE passes and a kernel trace over a driver-window bench run WITH its frame-ring leg
  local O=gpurun_out/$1; mkdir -p $O
  local C
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/ring_$C -o run -- python bench.py --warmup 5 --steps 20 --no-cpu-baseline --fused 0 > $O/ring_$C.log 2>&1 \
      || { echo "ring pmc $C failed"; tail -5 $O/ring_$C.log; return 1; }
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ring_trace -o run -- python bench.py --warmup 5 --steps 20 --no-cpu-baseline --fused 0 > $O/ring_trace.log 2>&1 \
    || { echo "ring trace failed"; tail -5 $O/ring_trace.log; return 1; }
  python tools/ring_pmc.py $O 65536 | tee $O/ring_summary.json
}

groupprof() {  # tag: the lane-group kernel at 4,096 and 8,192 envs: kernel trace (per-step and K-step), stamps (lib_stg)
  local O=gpurun_out/$1; mkdir -p $O
  local N
  for N in 4096 8192; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gtrace_$N -o run -- python bench.py --envs $N --no-cpu-baseline --no-ring-leg --fused 50 > $O/gtrace_$N.log 2>&1 \
      || { echo "group trace $N failed"; tail -5 $O/gtrace_$N.log; return 1; }
    grep -h "group" $O/gtrace_$N/run_kernel_stats.csv | cut -c1-60,160-260
    timeout -k 10 240 python tools/stamps.py --lib marl-soccer_amd/lib/exp/lib_stg.so --envs $N --steps 300 --warmup 1000 --every 10 --out $O/gstamps_$N.json > $O/gstamps_$N.log 2>&1 \
      || { echo "group stamps $N failed"; tail -5 $O/gstamps_$N.log; return 1; }
    python -c "import json; d=json.load(open('$O/gstamps_$N.json')); print($N, d['launch'], 'mean', round(d['wave_cycles_mean']), 'worst', round(d.get('worst_wave_cycles_mean', 0)), {k: round(v['mean']) for k, v in d['phases'].items() if v['mean']}); t=d['timeline']; print({k: v for k, v in t.items() if k != 'waves_in_phase_per_us_bin'})"
  done
}

driver() {  # the driver's own bench command, N = 1 (BENCH_rNN.json)
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
    || { echo "driver bench failed"; tail -20 $O/bench_driver.err; return 1; }
  cat $O/bench_driver.json
}

policy() {
  local O=gpurun_out/$1; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_policy.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_policy.log 2>&1 \
    || { tail -40 $O/pytest_policy.log; return 1; }
  tail -1 $O/pytest_policy.log
  timeout -k 10 300 python tools/bench_policy.py --envs 65536 --iters 30 > $O/bench_policy.jsonl 2> $O/bench_policy.err || { tail -5 $O/bench_policy.err; return 1; }
  timeout -k 10 200 python tools/bench_rollout.py --envs 65536 --steps 64 --graph > $O/rollout_graph.json 2> $O/rollout.err || { tail -5 $O/rollout.err; return 1; }
  cat $O/rollout_graph.json
}

if [ "$job" = multi ]; then
  for spec in "$@"; do
    echo "=== $spec"
    read -r -a a <<< "$spec"
    "${a[@]}" || exit 1
  done
else
  $job "$@" || exit 1
fi
