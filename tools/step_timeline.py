"""One step of a rocprofv3 kernel trace as a timeline (profiling aid): start, end and
duration of every kernel relative to the step's start, with its stream, e.g. to see how
long the moving-mesh chain's small kernels wait behind the fixed-grid GNN's launches.
    python3 tools/step_timeline.py <run_kernel_trace.csv> [skip] [back]
(a step ends with its interpolation kernel; skip: steps at the end left out, e.g.
bench.py's traced pass (13 with --steps 10 --warmup 3); back: which step before those)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
            for r in rows)
ends = [e for s, e, n, _ in ev if "itp_interp" in n]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 13
back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
t0, t1 = ends[-skip - back - 1], ends[-skip - back]
print("   start      end      dur stream kernel (us from the previous step's end)")
for s, e, n, st in ev:
    if t0 - 1000 <= s < t1:
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} s{st}  {short}")
