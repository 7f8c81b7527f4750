#!/bin/bash
# One GPU session: parity tests -> smoke -> short bench. Each GPU step has its
# own time limit; a crash/timeout (exit >= 2 from pytest, anything nonzero from
# the rest) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 ${T_TEST:-600} python -m pytest tests/test_engine_gpu.py -x -q -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 ${T_SMOKE:-240} python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${T_BENCH:-300} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-seconds 5} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.log
exit $rc
