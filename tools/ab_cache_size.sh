#!/bin/bash
# Headline A/B of the evaluation cache size (--cache-log2): short bench runs alternating sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-cache}
mkdir -p $OUT
i=0
for c in ${SIZES:-23 25 23 25}; do
  i=$((i + 1))
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 \
    --cache-log2 $c > $OUT/head_${i}_c$c.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['nn']['rows_evaluated'])" $OUT/head_${i}_c$c.log $c
done
