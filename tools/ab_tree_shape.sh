#!/bin/bash
# Tree-only shape A/B (round 5): round look-ahead depth and lanes with the fused hash rounds; 30-step runs
# alternating the settings; each run under its own time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-shape}
mkdir -p $OUT
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 30 --warmup 4 \
    --evaluator hash --age 100 ${LANES_ARG:-} > $OUT/$name.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'])" $OUT/$name.log $name
}
for i in 1 2 3; do
  LANES_ARG="--lanes 1" run la2_l1_$i UTTT_ROUND_LOOKAHEAD=2
  LANES_ARG="--lanes 1" run la3_l1_$i UTTT_ROUND_LOOKAHEAD=3
  LANES_ARG="--lanes 2" run la2_l2_$i UTTT_ROUND_LOOKAHEAD=2
done
