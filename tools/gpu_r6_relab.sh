#!/bin/bash
# Round 6: host hand-offs (k_scan / k_round1 count tags) with a system-scope release store (build_ab/,
# the previous build) vs stores drained by vmcnt(0) then a relaxed tag (in-tree build), interleaved:
# headline (two lanes, fused network) and tree-only (hash evaluator, one lane).
set -u
OUT=gpurun_out/${1:-relab}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in new rel; do
    lib=""
    [ $v = rel ] && lib=$PWD/build_ab/libuttt_engine_rel.so
    f=$OUT/h_${v}_$rep.log
    UTTT_ENGINE_LIB=$lib timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        > $f 2>&1 || exit 1
    echo "head $v $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
    f=$OUT/t_${v}_$rep.log
    UTTT_ENGINE_LIB=$lib timeout -k 10 170 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        --evaluator hash --lanes 1 --age 100 --steps 60 > $f 2>&1 || exit 1
    echo "tree $v $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
