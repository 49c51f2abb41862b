#!/usr/bin/env python
"""Summarise the two rocprofv3 --pmc passes written by tools/gpu_pmc.sh.

Per kernel name: mean FETCH_SIZE and WRITE_SIZE per dispatch (rocprofv3
reports both in KiB), and the corrected HBM bytes per launch
    hbm = 2 * FETCH_SIZE + WRITE_SIZE
(MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE tallies 128-B requests at
64 B, i.e. reads exactly half of a wide coalesced read; WRITE_SIZE is exact
for 16-B-per-lane stores).  Writes gpurun_out/pmc/<name>.json; copy it to
profiles/ to have bench.py report it as roofline.traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def summarise(d):
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        rec = {"dispatches": max(len(f), len(w)), "fetch_kib": fk, "write_kib": wk}
        if fk is not None and wk is not None:
            rec["hbm_bytes_per_launch"] = (2.0 * fk + wk) * 1024.0
            rec["hbm_bytes_per_launch_uncorrected"] = (fk + wk) * 1024.0
        out[k] = rec
    return out


def main():
    """pmc_summary.py OUT_NAME WORKLOAD NODES MODE=DIR [MODE=DIR ...]: one
    record per arithmetic mode (bench.py --edge-gemm), as bench.py reads it for
    roofline.traffic: {"workload", "nodes", "modes": {mode: {"hbm_bytes_per_launch",
    "per_kernel"}}}.  Kernels of several template variants are averaged by
    dispatch count."""
    name, workload, nodes = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rec = {"workload": workload, "nodes": nodes,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                     "tools/gpu_pmc.sh; per-dispatch means; hbm = 2*FETCH_SIZE + WRITE_SIZE "
                     "(gfx950 FETCH_SIZE half-count correction, MI355X_MICROARCH.md HBM)",
           "modes": {}}
    for arg in sys.argv[4:]:
        mode, d = arg.split("=", 1)
        per = summarise(d)
        tot = sum(v["hbm_bytes_per_launch"] * v["dispatches"] for v in per.values()
                  if "hbm_bytes_per_launch" in v)
        cnt = sum(v["dispatches"] for v in per.values() if "hbm_bytes_per_launch" in v)
        rec["modes"][mode] = {"hbm_bytes_per_launch": tot / max(cnt, 1), "per_kernel": per}
    os.makedirs("gpurun_out/pmc", exist_ok=True)
    with open(os.path.join("gpurun_out/pmc", name + ".json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps({m: v["hbm_bytes_per_launch"] for m, v in rec["modes"].items()}))


if __name__ == "__main__":
    main()
