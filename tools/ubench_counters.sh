#!/bin/bash
# PMC passes over tools/ubench/fused_ubench (per-phase variants of the fused
# layer kernel).  Usage: tools/ubench_counters.sh "GRP1" "GRP2" ...
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/uctr}
mkdir -p "$OUT"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- \
      ${UBENCH:-tools/ubench/fused_ubench 16} > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "pmc group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/g$i.log"; exit $rc; fi
done
python3 tools/ctr_summary.py "$OUT"
