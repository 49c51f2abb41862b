#!/bin/bash
# Edge split placement A/B (wave_diag, bench) + GNN parity tests on the new default.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 bash tools/ubench/ab_run.sh || exit 1
timeout -k 10 500 bash tools/gpu_ab.sh || exit 1
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_precision.py tests/test_gpu_eval.py > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab/tests.log
