#!/bin/bash
# Round 6: tree-only (hash evaluator, one lane) host polling: spin (default) vs the 20-us sleep, interleaved.
set -u
OUT=gpurun_out/${1:-treeab2}
mkdir -p $OUT
for rep in 1 2 3; do
  for ps in 0 1; do
    f=$OUT/t_sleep${ps}_$rep.log
    UTTT_POLL_SLEEP=$ps timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "sleep=$ps $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
