#!/bin/bash
# Round 6: the headline with the tree kernels at the highest wave priority (in-tree) against without
# (build_ab/libuttt_engine_old.so built with -DUTTT_TREE_PRIO=0): value and the select's per-trip latency.
set -u
OUT=gpurun_out/${1:-prioab}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in new old; do
    lib=""
    [ $v = old ] && lib=$PWD/build_ab/libuttt_engine_old.so
    f=$OUT/h_${v}_$rep.log
    UTTT_ENGINE_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-variants --no-isolated \
        > $f 2>&1 || exit 1
    echo "head $v $rep $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"us_per_trip_of_slowest_tree": [0-9.]*' $f | head -1)"
  done
done
