#!/bin/bash
# Round 4: tie-count tests, the kNN table policy timing, node-stage phases.
set -u
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn_ties.py tests/test_gpu_eval.py -k "ties or rccl" -q -v \
    --timeout 200 --timeout-method thread > $O/ties_tests.log 2>&1
rc=$?; echo "ties pytest rc=$rc"; tail -12 $O/ties_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 tools/ubench/node_phases 16 > $O/node_phases.log 2>&1; echo "node_phases rc=$?"; cat $O/node_phases.log
timeout -k 10 300 python -u tools/knn_cand_time.py 16 0.004 0.01 0.02 > $O/knn_cand_time.log 2>&1; echo "knn rc=$?"; cat $O/knn_cand_time.log
