"""Compare two rocprofv3 kernel traces of the same bench workload (profiling aid),
e.g. the eager step against hipGraph replay: per step, the span, the GPU's busy
and idle time, the summed kernel durations (concurrent kernels counted once
each), and the kernels whose mean duration differs most.
    python3 tools/trace_compare.py <A_kernel_trace.csv> <B_kernel_trace.csv> [steps] [itp per step] [skip]
(the step boundary is the end of its last interpolation kernel: 1 per cylinder step,
2 per Burgers step); skip: steps at the end left out, e.g. bench.py's traced pass
(warmup + steps of its own) to compare the timed passes)"""
import csv
import sys
from collections import defaultdict


def load(path, steps, per_step, skip):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # the last `steps` steps: cut at the interpolation kernel that ends each step
    ends = [e for s, e, n in ev if "itp_interp" in n]
    ends = ends[per_step - 1::per_step]
    ends = ends[:len(ends) - skip]
    t0, t1 = ends[-steps - 1], ends[-1]
    ev = [x for x in ev if x[0] >= t0 and x[1] <= t1]
    pts = sorted({t for s, e, _ in ev for t in (s, e)})
    busy = 0.0
    for a, b in zip(pts, pts[1:]):
        if any(s <= a and e >= b for s, e, _ in ev):
            busy += (b - a) / 1e3
    dur = defaultdict(list)
    for s, e, n in ev:
        short = n.replace("void ", "").replace("(anonymous namespace)::", "")
        dur[short.split("(")[0][:70]].append((e - s) / 1e3)
    span = (t1 - t0) / 1e3
    return span / steps, busy / steps, sum(sum(v) for v in dur.values()) / steps, dur


def main():
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    per_step = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    skip = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    a = load(sys.argv[1], steps, per_step, skip)
    b = load(sys.argv[2], steps, per_step, skip)
    for tag, (span, busy, ksum, _) in (("A", a), ("B", b)):
        print(f"{tag}: step span {span:8.1f} us  busy {busy:8.1f}  idle {span - busy:7.1f}  "
              f"kernel time {ksum:8.1f}  (overlap {ksum - busy:6.1f})")
    rows = []
    for n in set(a[3]) | set(b[3]):
        va, vb = a[3].get(n, []), b[3].get(n, [])
        ma = sum(va) / len(va) if va else 0.0
        mb = sum(vb) / len(vb) if vb else 0.0
        rows.append((sum(vb) / steps - sum(va) / steps, n, len(va) // steps, len(vb) // steps, ma, mb))
    print("kernel (per step: B - A total us, calls A/B, mean A/B us)")
    for d, n, ca, cb, ma, mb in sorted(rows, key=lambda r: -abs(r[0]))[:20]:
        print(f"  {d:+8.1f}  {ca:3d}/{cb:3d}  {ma:8.2f} {mb:8.2f}  {n}")


if __name__ == "__main__":
    main()
