#!/bin/bash
# Round 6: tree-only (hash evaluator, one lane) rounds per host call x rounds in flight, short bench runs
# on one box, interleaved. Output: gpurun_out/$1/
set -u
OUT=gpurun_out/${1:-treeab}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "1 3" "2 3" "2 4" "4 2" "1 4"; do
    set -- $cfg
    f=$OUT/t_r$1_d$2_$rep.log
    UTTT_ROUND_BATCH=$1 UTTT_ROUND_LOOKAHEAD=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "batch=$1 depth=$2 $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
