#!/bin/bash
# Round 6: refilled slots' keys seeded on the engine's side stream (default) vs in place by k_archive
# (UTTT_SEED_STREAM=0), interleaved: tree-only (one lane) and the headline (two lanes).
set -u
OUT=gpurun_out/${1:-seedab}
mkdir -p $OUT
for rep in 1 2 3; do
  for m in 1 0; do
    f=$OUT/t_seed${m}_$rep.log
    UTTT_SEED_STREAM=$m timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "tree seed_stream=$m $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
    f=$OUT/h_seed${m}_$rep.log
    UTTT_SEED_STREAM=$m timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        > $f 2>&1 || exit 1
    echo "head seed_stream=$m $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
