set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t2.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact > gpurun_out/b2.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/b2.log | cut -c1-300
