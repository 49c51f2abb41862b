set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|Error|error" gpurun_out/t2.log | tail -5
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b2.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/b2.log | cut -c 1-200; grep -o '"launch_ms[^,]*\|"node_stage_ms[^,]*\|"f32_exact[^}]*' gpurun_out/b2.log
PROF_BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-f32-exact" timeout -k 10 300 bash tools/gpu_profile.sh
