"""Median duration per (kernel, grid) from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if pat in r["Kernel_Name"]:
        key = (r["Kernel_Name"][:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    v.sort()
    print(k, len(v), "median %.1f us" % v[len(v) // 2])
