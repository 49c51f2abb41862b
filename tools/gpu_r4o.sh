#!/bin/bash
# Round 4: DPP / permlane butterflies in the DMM GNN, mesh VJP, phi and kNN
# cells kernels (new) against HEAD (old): the reduction check (bitwise), then
# serial-bench kernel stats with either library, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 60 tools/ubench/dpp_check || exit 1
LIB=mm-pde_amd/mmpde_amd/lib/libmmpde_hip.so
for rep in 1 2; do
  for v in old new; do
    cp tools/ubench/libab/$v/libmmpde_hip.so $LIB || exit 4
    rm -rf /tmp/r4o_$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4o_$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial > $O/b_$v.$rep.json 2>&1 || { tail $O/b_$v.$rep.json; exit 3; }
    f=$(find /tmp/r4o_$v -name '*kernel_stats.csv' | head -1)
    cp $f $O/stats_$v.$rep.csv
    python3 - "$f" "$v" "$rep" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if any(k in r["Name"] for k in ("mesh_vjp", "dmm_gnn", "knn_cells", "phi_kernel", "gnn_edge_wave"))]
print(sys.argv[2], sys.argv[3], " | ".join("%s %.2f" % (r["Name"].split("(")[0].split("::")[-1][:24], float(r["AverageNs"]) / 1e3) for r in sel))
PY
  done
done
cp tools/ubench/libab/new/libmmpde_hip.so $LIB
