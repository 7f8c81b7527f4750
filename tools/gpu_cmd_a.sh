set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2a/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2a/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2a/prof_bench.log 2>&1 || exit $?
