#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
T="tests/test_gpu_eval.py::test_timestep_losses_vs_oracle"
for v in "" "MMPDE_NO_DMM_CHAIN=1" "MMPDE_NO_RES_CHAIN=1" "MMPDE_NO_DMM_CHAIN=1 MMPDE_NO_RES_CHAIN=1"; do
  env $v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$T" > $O/t.log 2>&1
  rc=$?; echo "[$v] rc=$rc $(grep -E 'passed|failed' $O/t.log | tail -1)"
  [ $rc -le 1 ] || exit $rc
done
