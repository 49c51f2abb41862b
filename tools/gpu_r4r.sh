#!/bin/bash
# Round 4: wave-uniform lane broadcasts in the kNN kernels as v_readlane (new)
# against HEAD (old): serial-bench kernel stats with either library, then the
# kNN GPU tests (bit-exact against the oracle) with the new one.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
LIB=mm-pde_amd/mmpde_amd/lib/libmmpde_hip.so
for rep in 1 2; do
  for v in old new; do
    cp tools/ubench/libab/$v/libmmpde_hip.so $LIB || exit 4
    rm -rf /tmp/r4r_$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4r_$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial > $O/b_$v.$rep.json 2>&1 || { tail $O/b_$v.$rep.json; exit 3; }
    f=$(find /tmp/r4r_$v -name '*kernel_stats.csv' | head -1)
    cp $f $O/stats_$v.$rep.csv
    python3 - "$f" "$v" "$rep" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if "knn" in r["Name"]]
print(sys.argv[2], sys.argv[3], " | ".join("%s %.2f" % (r["Name"].split("(")[0].split("::")[-1][:30], float(r["AverageNs"]) / 1e3) for r in sel))
PY
  done
done
cp tools/ubench/libab/new/libmmpde_hip.so $LIB
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "knn" > $O/knn_tests.log 2>&1; echo "pytest rc=$?"; tail -2 $O/knn_tests.log
