#!/bin/bash
# GPU session: parity tests, then a rocprofv3 kernel trace of a short bench,
# then bench variants. Every GPU step has its own limit; stop at first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r1b}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -x -q -m gpu > gpurun_out/$TAG/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o bench \
    -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/$TAG/prof_bench.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-"--cudnn-benchmark 1" "--evaluator nn-plain"}; do :; done
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --cudnn-benchmark 1 > gpurun_out/$TAG/bench_find.log 2>&1
rc=$?; echo "bench find rc=$rc"; tail -1 gpurun_out/$TAG/bench_find.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --evaluator nn-plain > gpurun_out/$TAG/bench_plain.log 2>&1
rc=$?; echo "bench plain rc=$rc"; tail -1 gpurun_out/$TAG/bench_plain.log | cut -c1-400
exit $rc
