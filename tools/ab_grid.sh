#!/bin/bash
# A/B of the conv's persistent grid (UTTT_WINO3H_GRID = workgroups per CU per launch) on the headline:
# short bench runs alternating the settings; each run under its own time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-grid}
mkdir -p $OUT
i=0
for g in ${GRIDS:-1 0.5 1 0.5}; do
  i=$((i + 1))
  UTTT_WINO3H_GRID=$g timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 \
    --warmup 4 ${BENCH_ARGS:-} > $OUT/head_${i}_g$g.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_us'], d['nn']['frac'])" $OUT/head_${i}_g$g.log $g
done
