# r04k: ms_step_n sweep over K and batch size; FETCH/WRITE PMC passes over the fused kernel; configs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python tools/bench_fused.py --envs 65536 --k 10 25 50 100 250 > $O/fused_k.jsonl 2> $O/fused_k.err || { tail -5 $O/fused_k.err; exit 1; }
cat $O/fused_k.jsonl
timeout -k 10 300 python tools/bench_fused.py --envs 16384 32768 131072 --k 50 > $O/fused_n.jsonl 2> $O/fused_n.err || { tail -5 $O/fused_n.err; exit 1; }
timeout -k 10 200 python tools/bench_fused.py --envs 32768 --k 64 --max-steps 512 --steps 1024 --warmup 1024 >> $O/fused_n.jsonl 2>> $O/fused_n.err || { tail -5 $O/fused_n.err; exit 1; }
timeout -k 10 300 python tools/bench_fused.py --envs 262144 --k 32 --max-steps 512 --steps 512 --warmup 512 >> $O/fused_n.jsonl 2>> $O/fused_n.err || { tail -5 $O/fused_n.err; exit 1; }
cat $O/fused_n.jsonl
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_fused_$C -o run -- python tools/bench_fused.py --envs 65536 --k 50 --steps 1000 --warmup 1000 > $O/pmc_fused_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $O/pmc_fused_$C.log; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_fused -o run -- python tools/bench_fused.py --envs 65536 --k 50 > $O/trace_fused.log 2>&1 || { echo "trace failed"; tail -5 $O/trace_fused.log; exit 1; }
bash tools/gpu.sh configs r04k
