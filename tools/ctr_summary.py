#!/usr/bin/env python
"""Per-kernel mean of every counter found under a tools/gpu_counters.sh output dir."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    with open(os.path.join(d, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, cs in out.items():
        print(k[:100])
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {v:.6g}")


if __name__ == "__main__":
    main()
