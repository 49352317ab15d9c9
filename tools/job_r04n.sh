# r04n (final tree): whole GPU suite + smoke, default bench line + rocprofv3 stats + PMC, two-rank
# rehearsal, SQ passes over the K-step launch
bash tools/gpu.sh multi "suite r04n" "profile r04n" "rehearse r04n_multirank" "sqfused r04n 65536 50"
