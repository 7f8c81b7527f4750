#!/bin/bash
# Round 6: the dataflow tower's items-per-workgroup cap (UTTT_TOWER_ITEMS) against the per-conv launches,
# headline config, short bench runs on one box, interleaved. Output: gpurun_out/$1/
set -u
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_engine_gpu.py -k "dataflow or fused_hash_rounds" > $OUT/t0.log 2>&1 || exit 1
for rep in 1 2; do
  for k in layers 0 3 6 12; do
    if [ $k = layers ]; then env="UTTT_NN_TOWER=layers"; else env="UTTT_TOWER_ITEMS=$k"; fi
    env $env timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 30 > $OUT/b_${k}_$rep.log 2>&1 || exit 1
    echo "$k $rep $(grep -o '"value": [0-9.]*' $OUT/b_${k}_$rep.log | head -1)"
  done
done
