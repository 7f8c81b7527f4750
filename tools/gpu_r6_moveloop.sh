#!/bin/bash
# Round 6: tree-only (hash evaluator, one lane): each move's round loop in one C call (default) against the
# Python round loop (UTTT_MOVE_LOOP=0), interleaved.
set -u
OUT=gpurun_out/${1:-moveloop}
mkdir -p $OUT
for rep in 1 2 3; do
  for m in 1 0; do
    f=$OUT/t_loop${m}_$rep.log
    UTTT_MOVE_LOOP=$m timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "loop=$m $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
