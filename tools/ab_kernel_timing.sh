#!/bin/bash
# The bench's per-dispatch timing events (engine dispatch events, evaluator and tower events) on and off,
# alternating, tree-only and headline; each run under its own time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-timing}
mkdir -p $OUT
for i in 1 2; do
  for t in 1 0; do
    UTTT_BENCH_KERNEL_TIMING=$t timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 \
      --warmup 4 > $OUT/head_t${t}_$i.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['value'])" $OUT/head_t${t}_$i.log
  done
done
