#!/bin/bash
# Round-2 GPU session: every -m gpu test (verbose, per-test timeout), smoke,
# the default bench (variants + CPU baselines), then the same bench under
# rocprofv3 --kernel-trace --stats. Each GPU step has its own time limit and
# the session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out/$TAG
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
      > gpurun_out/$TAG/gputests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/$TAG/gputests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/$TAG/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
if [ -z "${SKIP_PROF:-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o bench \
      -- python3 bench.py --no-cpu-baseline --no-variants --no-isolated ${BENCH_ARGS:-} > gpurun_out/$TAG/prof_bench.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/$TAG/prof_bench.log | cut -c1-300
fi
exit $rc
