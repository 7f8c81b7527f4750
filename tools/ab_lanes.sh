#!/bin/bash
# Headline A/B of the lane count (concurrent engines per GPU, each on its own stream).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-lanes}
mkdir -p $OUT
i=0
for l in ${LANES:-2 4 2 4}; do
  i=$((i + 1))
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 \
    --lanes $l > $OUT/head_${i}_l$l.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('lanes', sys.argv[2], d['value'])" $OUT/head_${i}_l$l.log $l
done
