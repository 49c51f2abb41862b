#!/bin/bash
# Skinny linears with 16-byte loads: dense / DMM / ItpNet parity tests, serial kernel trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_dense.py \
    tests/test_gpu_dmm_api.py tests/test_gpu_parity.py -k "skinny or dmm or itp or res_cut or full_size or mesh" \
    > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > $O/stats.log 2>&1 || exit 1
python3 tools/step_breakdown.py $O/stats/run_kernel_trace.csv | head -8
python3 - <<'PY'
import csv, collections
rows = sorted(csv.DictReader(open('gpurun_out/r3n/stats/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
d = collections.defaultdict(list)
for r in rows[-1500:]:
    if 'linear_skinny' in r['Kernel_Name']:
        d[(r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    print('skinny grid', k, 'n', len(v), 'avg %.2f us' % (sum(v) / len(v)))
PY
