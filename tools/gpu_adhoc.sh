set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_ARGS="--timeout 120 --timeout-method thread" bash tools/gpu_check.sh || exit 1
PROF_BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-f32-exact" timeout -k 10 300 bash tools/gpu_profile.sh || exit 1
timeout -k 10 900 bash tools/gpu_pmc.sh
