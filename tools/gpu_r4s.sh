#!/bin/bash
# Round 4: the Conv1d head on eight waves (new) against HEAD (old): GNN forward
# outputs compared bit for bit, then serial-bench kernel stats, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
LIB=mm-pde_amd/mmpde_amd/lib/libmmpde_hip.so
for v in old new; do
  cp tools/ubench/libab/$v/libmmpde_hip.so $LIB || exit 4
  timeout -k 10 300 python3 tools/gnn_out_dump.py $O/out_$v.pt > $O/dump_$v.log 2>&1 || { tail $O/dump_$v.log; exit 2; }
done
python3 -c "
import torch
a = torch.load('$O/out_old.pt', weights_only=True); b = torch.load('$O/out_new.pt', weights_only=True)
print('bitwise equal:', {k: torch.equal(a[k], b[k]) for k in a})"
for rep in 1 2; do
  for v in old new; do
    cp tools/ubench/libab/$v/libmmpde_hip.so $LIB || exit 4
    rm -rf /tmp/r4s_$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4s_$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial > $O/b_$v.$rep.json 2>&1 || { tail $O/b_$v.$rep.json; exit 3; }
    f=$(find /tmp/r4s_$v -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" "$rep" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if "head_kernel" in r["Name"] or "gnn_edge_wave" in r["Name"]]
print(sys.argv[2], sys.argv[3], " | ".join("%s %.2f" % (r["Name"].split("(")[0].split("::")[-1][:24], float(r["AverageNs"]) / 1e3) for r in sel))
PY
  done
done
cp tools/ubench/libab/new/libmmpde_hip.so $LIB
