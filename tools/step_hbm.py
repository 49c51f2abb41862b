#!/usr/bin/env python
"""HBM bytes per step of a whole bench run (every kernel), from the two rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE) written by tools/gpu_configs.sh.

    step_hbm.py OUT_JSON WORKLOAD NODES EDGE_LAUNCHES_PER_STEP DIR

Per kernel: summed FETCH/WRITE (KiB) over all dispatches; bytes =
2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE half-count correction,
MI355X_MICROARCH.md HBM).  Steps = edge-stage dispatches / edge launches per
step (one-time setup kernels are included in the total: an upper bound).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def sums(d, counter):
    tot = defaultdict(float)
    disp = defaultdict(int)
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            tot[row["Kernel_Name"]] += float(row["Counter_Value"])
            disp[row["Kernel_Name"]] += 1
    return tot, disp


def main():
    out, workload, nodes, per_step, d = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    fetch, disp = sums(d, "FETCH_SIZE")
    write, _ = sums(d, "WRITE_SIZE")
    edge = sum(v for k, v in disp.items() if "gnn_edge" in k)
    steps = edge / per_step
    kern = {}
    total = 0.0
    for k in set(fetch) | set(write):
        b = (2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024.0
        kern[k[:90]] = {"dispatches": disp.get(k, 0), "hbm_bytes_per_step": b / steps}
        total += b
    rec = {"workload": workload, "nodes": nodes, "steps_profiled": steps,
           "hbm_bytes_per_step": total / steps,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over the "
                     "whole bench run, tools/gpu_configs.sh; bytes = 2*FETCH_SIZE + WRITE_SIZE",
           "per_kernel": dict(sorted(kern.items(), key=lambda kv: -kv[1]["hbm_bytes_per_step"]))}
    with open(out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps({"hbm_bytes_per_step": rec["hbm_bytes_per_step"], "steps": steps}))


if __name__ == "__main__":
    main()
