#!/bin/bash
# Launch forms and batch sizes of the default bench: plain python, torch.distributed.run with one
# rank (the driver's N = 1 form), and cy-mmpde at 8 and 4 trajectories (configs[4]'s 8-GPU end
# point of 64 trajectories runs 8 per rank); host issue time per step beside each pass.
set -u
O=gpurun_out/gap; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-f32-exact > $O/plain.json 2> $O/plain.err || exit 3
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --no-cpu-baseline --no-f32-exact > $O/trun.json 2> $O/trun.err || exit 4
for b in 8 4; do timeout -k 10 300 python -u bench.py --steps 20 --batch $b --no-cpu-baseline --no-f32-exact > $O/b$b.json 2> $O/b$b.err || exit 5; done
python - <<'PY'
import json
for f in ("plain", "trun", "b8", "b4"):
    r = json.loads(open(f"gpurun_out/gap/{f}.json").read().strip().splitlines()[-1])
    ro = r["roofline"]
    print(f, "value %.3fM ms %.3f host %.3f | traced %.3f host %.3f | edge %.1f us frac %.3f node %.1f" % (r["value"]/1e6, r["ms_per_step"], r["host_issue_ms_per_step"], ro["traced_pass_ms_per_step"], ro["traced_pass_host_ms_per_step"], ro["launch_ms"]*1e3, ro["frac"], r["node_stage_ms"]*1e3))
PY
