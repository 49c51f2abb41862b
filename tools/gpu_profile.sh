#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC here; counters
# are collected in separate passes by tools/gpu_pmc.sh).
set -u
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 bench.py ${PROF_BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline} --serial > "$OUT/bench_under_prof.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$OUT" -name '*kernel_stats.csv' | head -3
exit $rc
