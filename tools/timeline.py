"""Concurrency of a rocprofv3 kernel trace (profiling aid): for the last N steps of a
bench run (non-serial, three streams), the time each kernel runs with no other kernel
beside it, summed per kernel name, and the idle gaps.
    python3 tools/timeline.py <run_kernel_trace.csv> [steps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
# the last `steps` steps: cut at the gnn head launches (2 per step)
heads = [s for s, e, n in ev if "head_kernel" in n]
t0 = heads[-2 * steps - 1] if len(heads) > 2 * steps else ev[0][0]
ev = [x for x in ev if x[0] >= t0]
pts = sorted({t for s, e, _ in ev for t in (s, e)})
alone = defaultdict(float)
busy = idle = 0.0
for a, b in zip(pts, pts[1:]):
    act = [n for s, e, n in ev if s <= a and e >= b]
    d = (b - a) / 1e3
    if not act:
        idle += d
    else:
        busy += d
        if len(act) == 1:
            alone[act[0][:60]] += d
span = (pts[-1] - pts[0]) / 1e3
print(f"span {span:.1f} us over ~{steps} steps: busy {busy:.1f}, idle {idle:.1f}")
for n, d in sorted(alone.items(), key=lambda x: -x[1])[:15]:
    print(f"{d / steps:8.1f} us/step alone  {n}")
