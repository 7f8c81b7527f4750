#!/bin/bash
# GPU session: selected parity tests, then bench variants (no rocprof). Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-q}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -q -m gpu ${TESTS:-} > gpurun_out/$TAG/gputests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/gputests.log
[ $rc -le 1 ] || exit $rc
i=0
IFS=';' read -ra VARS <<< "${BENCHES:---no-cpu-baseline}"
for v in "${VARS[@]}"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py $v > gpurun_out/$TAG/bench$i.log 2>&1
  rc=$?; echo "bench[$v] rc=$rc"; tail -1 gpurun_out/$TAG/bench$i.log | cut -c1-120
  [ $rc -eq 0 ] || exit $rc
done
exit 0
