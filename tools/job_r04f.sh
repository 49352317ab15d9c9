# r04f: the whole GPU suite on the lane-pair default; the default bench line's profile at 65,536 envs
# (rocprofv3 stats, PMC of both windows); the lane-pair kernel's SQ counters and per-phase stamps;
# wave-priority variants
bash tools/gpu.sh multi "suite r04f" "profile r04f" "sq r04f 65536" "stamps r04f G=2 65536 32768" && timeout -k 10 300 python tools/variants.py run --envs 65536 pbase prio1 prio2 > gpurun_out/r04f/variants.txt 2>&1; cat gpurun_out/r04f/variants.txt
