#!/bin/bash
# Round 6: the persistent dataflow tower (UTTT_NN_TOWER=dataflow) with fewer workgroups than CUs
# (UTTT_TOWER_CUS: the rest left to the other lane's kernels) against the per-conv launches, headline
# config, short bench runs on one box, interleaved. Output: gpurun_out/$1/
set -u
OUT=gpurun_out/${1:-sweep3}
mkdir -p $OUT
for rep in 1 2; do
  for c in layers 256 248 240 224; do
    if [ $c = layers ]; then env="UTTT_NN_TOWER=layers"; else env="UTTT_NN_TOWER=dataflow UTTT_TOWER_CUS=$c"; fi
    f=$OUT/b_${c}_$rep.log
    env $env timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 30 > $f 2>&1 || exit 1
    echo "$c $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
