# r04g: the BASELINE configs' batch sizes on the default launch, the two-rank rehearsal of the
# driver's N-GPU bench on the lane-pair default, and wave-priority variants at 65,536 envs
bash tools/gpu.sh multi "configs r04g" "rehearse r04g_multirank" && timeout -k 10 400 python tools/variants.py run --envs 65536 pbase prio1 prio2 > gpurun_out/r04g/variants.txt 2>&1; cat gpurun_out/r04g/variants.txt
