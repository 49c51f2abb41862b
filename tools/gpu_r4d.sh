#!/bin/bash
# Round 4: node-stage variant A/B (node_phases_<v>), kNN policy + training tests, kNN timing.
set -u
O=gpurun_out/r4d
mkdir -p $O
for rep in 1 2; do
  for v in base ldsbar rows proj2 rowsbar; do
    timeout -k 10 120 tools/ubench/node_phases_$v 16 > $O/$v.$rep.log 2>&1 || { echo "$v failed"; cat $O/$v.$rep.log; exit 3; }
    echo "== $v rep $rep: $(grep -E 'node kernel|hash' $O/$v.$rep.log | tr -s ' ' | tr '\n' ' ')"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn_policy.py tests/test_gpu_train.py tests/test_gpu_knn_ties.py \
    -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/knn_cand_time.py 16 0.004 0.02 > $O/knn_cand_time.log 2>&1; echo "knn rc=$?"; grep -E "policy|rollout" $O/knn_cand_time.log
timeout -k 10 300 python -u tools/train_bench.py --edge-gemm f16x3 > $O/train_f16x3.json 2>&1; echo "train rc=$?"; tail -2 $O/train_f16x3.json
