set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/t2.log | tail -5
[ $rc -eq 0 ] || exit $rc
PROF_BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-f32-exact" timeout -k 10 300 bash tools/gpu_profile.sh; grep -o '"value": [0-9.]*' gpurun_out/prof/bench_under_prof.log
