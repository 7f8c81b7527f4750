#!/bin/bash
# A/B of an environment knob on the bench (no variants, no CPU baseline), alternating
# A B A B so box drift shows. usage: KNOB=UTTT_WINO_GRID A=0 B=1 tools/gpu_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-ab}
mkdir -p gpurun_out/$TAG
for i in 1 2; do
  for v in "$A" "$B"; do
    env "$KNOB=$v" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants ${BENCH_ARGS:-} \
        > gpurun_out/$TAG/bench_${v}_$i.log 2>&1
    rc=$?
    echo "$KNOB=$v run $i rc=$rc $(tail -1 gpurun_out/$TAG/bench_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"])' 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
