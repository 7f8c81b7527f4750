set -u
OUT=gpurun_out/${TAG:-t6c}
mkdir -p $OUT
for i in 1 2 3 4; do
  for f in 1 0; do
    UTTT_FUSED_ROUNDS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 30 --warmup 4 \
      --evaluator hash --lanes 1 --age 100 > $OUT/tree_f${f}_$i.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['roofline_select']['event_avg_launch_us'])" $OUT/tree_f${f}_$i.log
  done
done
