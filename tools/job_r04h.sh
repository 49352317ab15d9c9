# r04h: lane pairs with round-aligned shared static-agent windows and the late loads ahead of the
# cache-write stores: parity subset, A/B timing against the r04f build, stamps; configs; rehearsal
bash tools/gpu.sh multi "parity r04h lane-pair+or+lanes2+or+2lanes+or+ragged+or+lane_pair+or+corner+or+config" && timeout -k 10 400 python tools/variants.py run --envs 65536 prev cur prev cur > gpurun_out/r04h/variants.txt 2>&1; cat gpurun_out/r04h/variants.txt; bash tools/gpu.sh multi "stamps r04h G=2 65536" "configs r04h" "rehearse r04h_multirank"
