#!/bin/bash
# Round 6: tree-only (hash evaluator, one lane) against the hash rounds in flight per lane
# (UTTT_ROUND_LOOKAHEAD), interleaved.
set -u
OUT=gpurun_out/${1:-lookahead}
mkdir -p $OUT
for rep in 1 2; do
  for d in 3 4 5 6; do
    f=$OUT/t_d${d}_$rep.log
    UTTT_ROUND_LOOKAHEAD=$d timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "depth=$d $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
