#!/bin/bash
# Round 6: tree-only (hash evaluator, one lane) against the select budget (in-place completions per tree and
# launch, UTTT_SELECT_BUDGET; results are unchanged by it), interleaved.
set -u
OUT=gpurun_out/${1:-budget}
mkdir -p $OUT
for rep in 1 2; do
  for b in 8 4 12 16 32; do
    f=$OUT/t_b${b}_$rep.log
    UTTT_SELECT_BUDGET=$b timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "budget=$b $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
