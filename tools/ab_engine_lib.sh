#!/bin/bash
# Tree-only A/B of an alternative engine library (AB_LIB, e.g. the previous commit's build) against the
# in-tree one, interleaved; each run is the bench's tree-only configuration (hash evaluator, one lane).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_lib}
mkdir -p $OUT
i=0
for v in ${ORDER:-new old new old new old}; do
  i=$((i + 1))
  if [ $v = old ]; then lib=$AB_LIB; else lib=""; fi
  UTTT_ENGINE_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 20 \
    --warmup 4 --evaluator hash --lanes 1 --age 100 > $OUT/tree_${v}_$i.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d.get('breakdown_ms'))" $OUT/tree_${v}_$i.log $v
done
