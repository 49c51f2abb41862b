#!/bin/bash
# GPU tests, then a short bench line (no CPU baseline / f32 pass): the quick
# check after a kernel change.  Output under gpurun_out/quick.
set -u
mkdir -p gpurun_out/quick
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/quick/tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-f32-exact ${QUICK_BENCH_ARGS:-} \
    > gpurun_out/quick/bench.log 2>&1
rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/quick/bench.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print("value %.4g ms/step %.4f edge_us %.1f node_us %.1f frac %.4f" % (
            d["value"], d["ms_per_step"], 1e3 * d["roofline"]["launch_ms"], 1e3 * d["node_stage_ms"],
            d["roofline"]["frac"]))
PY
exit $rc
