#!/bin/bash
# Round 6: the in-tree engine library against a previous build (build_ab/libuttt_engine_old.so, built from
# the parent commit's engine.hip), interleaved, REPS rounds: tree-only (hash evaluator, one lane) and, with
# HEAD=1, the headline (two lanes, fused network); TREE=0 skips the tree-only runs.
set -u
OUT=gpurun_out/${1:-libab}
REPS=${REPS:-3}
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in new old; do
    lib=""
    [ $v = old ] && lib=$PWD/build_ab/libuttt_engine_old.so
    if [ "${TREE:-1}" = 1 ]; then
      f=$OUT/t_${v}_$rep.log
      UTTT_ENGINE_LIB=$lib timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
          --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
      echo "tree $v $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
    fi
    if [ "${HEAD:-0}" = 1 ]; then
      f=$OUT/h_${v}_$rep.log
      UTTT_ENGINE_LIB=$lib timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
          > $f 2>&1 || exit 1
      echo "head $v $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
    fi
  done
done
