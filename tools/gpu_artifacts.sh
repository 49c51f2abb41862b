#!/bin/bash
# Round artifacts in one GPU call: GPU tests, the default bench line (with the
# CPU baseline), a rocprofv3 kernel-trace --stats run, and the edge-kernel HBM
# traffic passes.  Everything lands under gpurun_out/art, gpurun_out/prof and
# gpurun_out/pmc; copy what is judged into profiles/.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/art
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/art/gpu_tests.log 2>&1 || { tail -30 gpurun_out/art/gpu_tests.log; exit 1; }
tail -2 gpurun_out/art/gpu_tests.log
# the edge kernel's HBM traffic first: bench.py reports it as roofline.traffic
PMC_NAME=edge_pmc_r02 timeout -k 10 900 bash tools/gpu_pmc.sh || exit 1
cp gpurun_out/pmc/edge_pmc_r02.json profiles/edge_pmc_r02.json
timeout -k 10 400 python -u bench.py > gpurun_out/art/bench.log 2>&1 || { tail -30 gpurun_out/art/bench.log; exit 1; }
grep '^{' gpurun_out/art/bench.log | tail -1 > gpurun_out/art/bench.json
echo "bench ok"
PROF_BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline" timeout -k 10 420 bash tools/gpu_profile.sh || exit 1
echo "artifacts ok"
