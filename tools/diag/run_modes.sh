#!/bin/bash
# GPU diag session: conv variant timings (wino3h_modes.py) and phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=${1:-modes}
mkdir -p gpurun_out/$TAG
timeout -k 10 240 python -u tools/diag/wino3h_modes.py ${BOARDS:-1344 2688 16384} > gpurun_out/$TAG/modes.log 2>&1
rc=$?; echo "modes rc=$rc"; cat gpurun_out/$TAG/modes.log | tail -5
[ $rc -eq 0 ] || exit $rc
if [ -n "${STAMPS:-}" ]; then
  MODES=$STAMPS timeout -k 10 240 python -u tools/diag/wino3h_stamps.py 1344 > gpurun_out/$TAG/stamps.log 2>&1
  rc=$?; echo "stamps rc=$rc"; cat gpurun_out/$TAG/stamps.log | tail -30
fi
exit $rc
