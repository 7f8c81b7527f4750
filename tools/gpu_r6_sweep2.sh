#!/bin/bash
# Round 6: lanes x items-per-workgroup for the dataflow tower against the per-conv launches, short bench
# runs on one box, interleaved: the headline config (4,096 games) and the cycle's one-lane shape (512 games).
# Output: gpurun_out/$1/
set -u
OUT=gpurun_out/${1:-sweep2}
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "layers 2 4096" "0 2 4096" "0 1 4096" "12 2 4096" "24 2 4096" "layers 1 512" "0 1 512" "12 1 512"; do
    set -- $cfg
    k=$1; lanes=$2; g=$3
    if [ $k = layers ]; then env="UTTT_NN_TOWER=layers"; else env="UTTT_TOWER_ITEMS=$k"; fi
    f=$OUT/b_${k}_l${lanes}_g${g}_$rep.log
    env $env timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 30 --lanes $lanes --games $g > $f 2>&1 || exit 1
    echo "$k lanes=$lanes games=$g $rep $(grep -o '"value": [0-9.]*' $f | head -1)"
  done
done
