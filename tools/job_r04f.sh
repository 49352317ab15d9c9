# r04f: the lane-pair kernel (shared static-agent tests): its parity subset, profile at 65,536 envs
# (bench line, rocprofv3 stats, PMC of both windows), SQ counters and per-phase stamps
bash tools/gpu.sh multi "parity r04f lane-pair+or+lanes2+or+2lanes+or+ragged+or+lane_pair" "profile r04f --lane-group 2" "sq r04f 65536 --lane-group 2" "stamps r04f G=2 65536 32768"
