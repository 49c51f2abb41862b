"""Per-step kernel time by kernel from a rocprofv3 kernel trace of bench.py
--serial (profiling aid): steps are cut at each launch of the step's first
kernel (dmm_embed_kernel, or gnn_embed_kernel without a DMM); the last
--steps steps are averaged, so setup-time launches do not count.

    python tools/step_breakdown.py run_kernel_trace.csv [--steps 20]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    names = [short(r["Kernel_Name"]) for r in rows]
    first = "dmm_embed_kernel" if any("dmm_embed_kernel" in n for n in names) else "gnn_embed_kernel"
    starts = [i for i, n in enumerate(names) if first in n]
    if first == "gnn_embed_kernel":
        starts = starts[::1]
    sel = starts[-a.steps - 1:]
    per = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for s0, s1 in zip(sel[:-1], sel[1:]):
        for i in range(s0, s1):
            r = rows[i]
            per[names[i]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[names[i]] += 1
    nst = len(sel) - 1
    tot = sum(per.values()) / nst
    wall = (int(rows[sel[-1]]["Start_Timestamp"]) - int(rows[sel[0]]["Start_Timestamp"])) / 1e3 / nst
    print(f"{nst} steps: kernel sum {tot:.1f} us/step, wall {wall:.1f} us/step")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"{v / nst:8.1f} us/step  {cnt[k] / nst:5.2f}/step  avg {v / cnt[k]:7.1f}  {k}")


if __name__ == "__main__":
    main()
