import json, sys, glob, os
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "bench_*.json"))):
    try:
        j = json.load(open(f)); print(os.path.basename(f), round(j["ms_per_step"] * 1000, 2), "us", round(j["value"] / 1e6, 1), "M/s")
    except Exception as e:
        print(f, "ERR", e)
for f in sorted(glob.glob(os.path.join(d, "stamps_*.json"))):
    j = json.load(open(f))
    print(os.path.basename(f), "mean", round(j["wave_cycles_mean"]), "slow5", round(j["wave_cycles_slowest5pct"]), "worst", round(j["worst_wave_cycles_mean"]))
    print("  worst", {k: round(v) for k, v in j["worst_wave_phases_mean"].items()})
    print("  slow5", {k: round(v["slow5"]) for k, v in j["phases"].items()})
