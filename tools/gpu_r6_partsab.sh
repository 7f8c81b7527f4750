#!/bin/bash
# Round 6: tree-only (hash evaluator, one lane, the C move loop): per-block count words summed by the host
# (default) against the last-block publish into the ring slot (UTTT_ROUND_PARTS=0), interleaved.
set -u
OUT=gpurun_out/${1:-partsab}
mkdir -p $OUT
for rep in 1 2 3; do
  for m in 1 0; do
    f=$OUT/t_parts${m}_$rep.log
    UTTT_ROUND_PARTS=$m timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "parts=$m $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
