#!/bin/bash
# SQ instruction-mix / wait counters of the kernels matching $1 (one rocprofv3
# --pmc pass, 8 SQ counters, kernel-trace only) over a short bench run.
set -u
export TMPDIR=/tmp
REGEX=${1:-knn_kernel}
OUT=gpurun_out/sq
mkdir -p "$OUT"
timeout -k 10 ${SQ_TIMEOUT:-240} rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM --kernel-include-regex "$REGEX" \
    --output-format csv -d "$OUT" -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-f32-exact > "$OUT/bench.log" 2>&1
rc=$?
echo "pmc rc=$rc"
[ $rc -eq 0 ] || { tail -20 "$OUT/bench.log"; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    n = max(cnt[(k, "SQ_WAVES")], 1)
    print(k, {c: round(v / n) for c, v in sorted(d.items())})
PY
