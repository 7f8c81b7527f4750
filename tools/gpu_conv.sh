#!/bin/bash
# GPU session for conv-kernel work: the network/conv parity tests, then variant timings
# and phase stamps (tools/diag). Each step has its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-conv}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
    -k "${TESTK:-winograd or split or fused or network or batch}" > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/diag/wino3h_modes.py ${BOARDS:-1344 2688 16384} > gpurun_out/$TAG/modes.log 2>&1
rc=$?; echo "modes rc=$rc"; grep boards gpurun_out/$TAG/modes.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${STAMPS:-}" ]; then
  MODES=$STAMPS timeout -k 10 240 python -u tools/diag/wino3h_stamps.py 1344 > gpurun_out/$TAG/stamps.log 2>&1
  rc=$?; echo "stamps rc=$rc"; grep "mode\|chunk 5\|chunk 7" gpurun_out/$TAG/stamps.log
fi
exit $rc
