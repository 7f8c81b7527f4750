#!/bin/bash
# GPU session: parity tests, default bench (with CPU baseline), then the same
# bench under rocprofv3 --kernel-trace --stats. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r1c}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -q -m gpu > gpurun_out/$TAG/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o bench \
    -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/$TAG/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/$TAG/prof_bench.log | cut -c1-300
exit $rc
