#!/bin/bash
# Bench at several lane counts (no variants, no CPU baseline), alternating with the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-lanes}
mkdir -p gpurun_out/$TAG
for L in ${LANES:-2 3 2 3}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --lanes $L ${BENCH_ARGS:-} \
      > gpurun_out/$TAG/bench_L$L.log 2>&1
  rc=$?
  echo "lanes=$L rc=$rc $(tail -1 gpurun_out/$TAG/bench_L$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["rounds_per_step"])' 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
