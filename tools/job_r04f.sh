# r04f: the lane-pair kernel's profile at 65,536 envs (bench line, rocprofv3 stats, PMC of both
# windows), its SQ counters and per-phase stamps
bash tools/gpu.sh multi "profile r04f --lane-group 2" "sq r04f 65536 --lane-group 2" "stamps r04f G=2 65536 32768"
