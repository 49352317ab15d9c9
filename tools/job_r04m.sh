# r04m: solver with next-slot record prefetch + forwarding (MS_PAIR_FWD=1) vs the product solver
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
MARL_SOCCER_LIB=$PWD/marl-soccer_amd/lib/variants/lib_fwd.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lane-pair or lanes2 or lane_pair" > $O/pytest_fwd.log 2>&1 || { tail -30 $O/pytest_fwd.log; exit 1; }
tail -1 $O/pytest_fwd.log
timeout -k 10 500 python tools/variants.py run --envs 65536 cur fwd cur fwd > $O/variants.txt 2>&1; cat $O/variants.txt
timeout -k 10 300 python tools/variants.py run --envs 32768 --max-steps 512 cur fwd > $O/variants_32768.txt 2>&1; cat $O/variants_32768.txt
