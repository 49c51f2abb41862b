"""Join tools/gpu_layer_counters.sh's PMC passes with the kernel-trace stats of
the same serial bench: per layer kernel the counters (per-dispatch means), MFMA
busy fraction, VALU / MFMA instruction ratio and HBM bytes / bandwidth."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
ctr = json.load(open(os.path.join(d, "summary.json")))
stats = {}
for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        stats[r["Name"]] = float(r["AverageNs"]) / 1e3
out = {"source": "rocprofv3 --pmc, 3 separate passes (SQ/GRBM group, FETCH_SIZE, WRITE_SIZE), "
                 "--kernel-include-regex layer kernels, bench.py --steps 2 --warmup 1 --serial "
                 "--no-f32-exact (cy-mmpde, B=16, n=40336); durations from a --kernel-trace --stats "
                 "pass of bench.py --steps 10 --warmup 3 --serial; tools/gpu_layer_counters.sh",
       "derived_definitions": {
           "mfma_busy_frac": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)",
           "valu_per_mfma": "SQ_INSTS_VALU / SQ_INSTS_MFMA (instructions, per dispatch)",
           "hbm_bytes": "2*FETCH_SIZE + WRITE_SIZE (KiB x 1024; gfx950 FETCH_SIZE half-count correction)",
           "hbm_GBps": "hbm_bytes / mean kernel duration"},
       "kernels": {}}
for k, c in ctr.items():
    e = {"counters": c}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
        e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)
    if c.get("SQ_INSTS_MFMA"):
        e["valu_per_mfma"] = c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    dur = next((v for n, v in stats.items() if n == k or n.startswith(k[:60])), None)
    if dur:
        e["duration_us"] = dur
        if "hbm_bytes_per_launch" in e:
            e["hbm_GBps"] = e["hbm_bytes_per_launch"] / (dur * 1e3)
            e["hbm_frac_of_8TBps"] = e["hbm_GBps"] / 8000
    out["kernels"][k] = e
json.dump(out, open(os.path.join(d, "layer_counters.json"), "w"), indent=1)
for k, e in out["kernels"].items():
    print(k[:70], {x: round(v, 3) for x, v in e.items() if isinstance(v, float)})
