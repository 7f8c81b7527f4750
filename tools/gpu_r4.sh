#!/bin/bash
# Round-4 GPU session. quick: headline + tree-only short bench lines. STEPS (default "tests smoke train cycle bench") picks the steps, in this order:
#   tests  every -m gpu test (verbose, per-test timeout)     smoke  __graft_entry__.smoke()
#   train  tools/bench_train.py (eager / HIP graph / graph + channels-last)
#   cycle  tools/bench_cycle.py (BASELINE configs[4] on one GPU)
#   hist   tools/bench_history.py (.history path at C4 scale)   vars  conv pipeline variants (diag lib)
#   pmcconv conv HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
#   ab     launch-shape A/B (grid policy, lanes, cache size)   bench  bench.py (headline, variants, CPU baselines)     prof  bench under rocprofv3 --kernel-trace --stats
# Each GPU step has its own time limit; the session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
STEPS=${STEPS:-"tests smoke train cycle bench"}
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread ${PYTEST_K:-} \
               > $OUT/gputests.log 2>&1 ;;
    smoke) timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    train) timeout -k 10 400 python -u tools/bench_train.py ${TRAIN_ARGS:-} > $OUT/train.log 2>&1 ;;
    cycle) timeout -k 10 900 python -u tools/bench_cycle.py --out $OUT/cycle.json ${CYCLE_ARGS:-} > $OUT/cycle.log 2>&1 ;;
    cycle16) UTTT_TRAIN_PRECISION=f16 timeout -k 10 900 python -u tools/bench_cycle.py --out $OUT/cycle_f16.json ${CYCLE_ARGS:-} > $OUT/cycle_f16.log 2>&1 ;;
    hist)  timeout -k 10 300 python -u tools/bench_history.py > $OUT/history.log 2>&1 ;;
    pmctree) PMC_OUT=$OUT/pmc_tree PMC_AGE=100 PMC_BENCH_ARGS="--evaluator hash --lanes 1" timeout -k 10 900 bash tools/pmc_select.sh \
               > $OUT/pmc_tree.log 2>&1 && \
             python tools/pmc_summary.py $OUT/pmc_tree $OUT/pmc_tree/p1.log $OUT/pmc_select_tree.json k_select >> $OUT/pmc_tree.log && \
             python tools/pmc_summary.py $OUT/pmc_tree $OUT/pmc_tree/p1.log $OUT/pmc_apply_tree.json k_apply >> $OUT/pmc_tree.log && \
             rm -rf $OUT/pmc_tree/p1 $OUT/pmc_tree/p2 $OUT/pmc_tree/p3 ;;  # raw CSVs: gpurun copies back <= 64 MiB
    pmcsel) PMC_OUT=$OUT/pmc_sel timeout -k 10 900 bash tools/pmc_select.sh > $OUT/pmc_select.log 2>&1 && \
             python tools/pmc_summary.py $OUT/pmc_sel $OUT/pmc_sel/p1.log $OUT/pmc_select.json k_select >> $OUT/pmc_select.log && \
             python tools/pmc_summary.py $OUT/pmc_sel $OUT/pmc_sel/p1.log $OUT/pmc_apply.json k_apply >> $OUT/pmc_select.log && \
             rm -rf $OUT/pmc_sel/p1 $OUT/pmc_sel/p2 $OUT/pmc_sel/p3 ;;
    pmcconv) timeout -k 10 600 bash tools/pmc_conv.sh > $OUT/pmc_conv.log 2>&1 && \
             python tools/pmc_conv_summary.py gpurun_out/pmc_conv ${N:-1344} $OUT/pmc_conv.json >> $OUT/pmc_conv.log 2>&1 ;;
    pmcl2) timeout -k 10 1000 bash tools/pmc_l2.sh > $OUT/pmc_l2.log 2>&1 && \
           python tools/pmc_l2_summary.py gpurun_out/pmc_l2 ${NB:-1381} $OUT/pmc_l2.json >> $OUT/pmc_l2.log 2>&1 ;;
    pmcsq) timeout -k 10 600 bash tools/pmc_sq.sh > $OUT/pmc_sq.log 2>&1 ;;
    tprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tprof -o train \
               -- python3 tools/bench_train.py --variants ${TPROF_VARIANT:-graph_f16} --epochs 1 --samples 8192 --cpu-steps 0 \
               > $OUT/tprof.log 2>&1 ;;
    dups)  timeout -k 10 300 python -u tools/diag/round_duplicates.py ${DUPS_ARGS:-} > $OUT/round_duplicates.log 2>&1 ;;
    selcyc) timeout -k 10 300 python -u tools/diag/select_cycles.py ${SELCYC_ARGS:-} > $OUT/select_cycles.log 2>&1 ;;
    pretouch) for m in 0 1 2 3; do  # k_select's first root load: TLB or line? (engine.hip g_sel_pretouch)
                timeout -k 10 300 python -u tools/diag/select_cycles.py 100 10 $m > $OUT/pretouch_$m.log 2>&1 || exit $?
              done ;;
    stamps) timeout -k 10 300 python -u tools/diag/wino3h_stamps.py 1344 16384 > $OUT/stamps.log 2>&1 ;;
    lat)   timeout -k 10 300 python -u tools/diag/latency_single.py > $OUT/latency.log 2>&1 ;;
    vsmall) VARIANTS= timeout -k 10 300 python -u tools/diag/wino3h_variants.py 250 500 1000 > $OUT/variants_small.log 2>&1 ;;
    tcomp) timeout -k 10 600 python -u tools/diag/train_compare.py > $OUT/train_compare.log 2>&1 ;;
    tcheck) timeout -k 10 300 python -u tools/diag/train_graph_check.py > $OUT/train_check.log 2>&1 ;;
    heads) timeout -k 10 300 python -u tools/diag/heads_bits.py > $OUT/heads_bits.log 2>&1 ;;
    vars)  timeout -k 10 300 python -u tools/diag/wino3h_variants.py ${VAR_BOARDS:-1344 2688 16384} > $OUT/variants.log 2>&1 ;;
    ab)    # A/B of launch shapes on the headline workload (short runs, one JSON line each)
           cfgs=("base:" "grid0:UTTT_WINO3H_GRID=0" "grid2:UTTT_WINO3H_GRID=2" "lanes1:--lanes 1"
                 "lanes1_grid0:UTTT_WINO3H_GRID=0 --lanes 1" "lanes4_grid0:UTTT_WINO3H_GRID=0 --lanes 4" "cache25:--cache-log2 25")
           [ -n "${AB_CFGS:-}" ] && IFS=';' read -ra cfgs <<< "$AB_CFGS"
           for cfg in "${cfgs[@]}"; do
             name=${cfg%%:*}; rest=${cfg#*:}; envs=""; args=""
             for w in $rest; do case $w in UTTT_*=*) envs="$envs $w" ;; *) args="$args $w" ;; esac; done
             env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps ${AB_STEPS:-10} --warmup 4 $args \
               > $OUT/ab_$name.log 2>&1 || exit $?
             echo "$name $(tail -1 $OUT/ab_$name.log | cut -c1-260)" >> $OUT/ab.log
           done ;;
    abl)   # same-box A/B of the engine library: the in-tree build against libuttt_engine_base.so (a build of
           # the previous engine.hip), alternating base / new, headline workload and tree-only
           for i in 1 2; do
             for lib in base new; do
               envs=""; [ $lib = base ] && envs="UTTT_ENGINE_LIB=$PWD/ultimate-tictactoe-alphazero_amd/libuttt_engine_base.so"
               for ev in ${ABL_EVS:-fused hash}; do
                 env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps ${AB_STEPS:-10} --warmup 4 \
                   --evaluator $ev ${ABL_ARGS:-} > $OUT/abl_${lib}_${ev}_$i.log 2>&1 || exit $?
                 echo "$lib $ev $i $(tail -1 $OUT/abl_${lib}_${ev}_$i.log | cut -c1-200)" >> $OUT/abl.log
               done
             done
           done ;;
    smallpf) timeout -k 10 300 python -u tools/diag/conv_small_pf.py > $OUT/conv_small_pf.log 2>&1 ;;
    split) timeout -k 10 300 python -u tools/diag/conv_split_time.py ${SPLIT_BOARDS:-} > $OUT/conv_split.log 2>&1 ;;
    chase) # dependent-load latency (k_select's latency-model unit); the bench reads profiles/r*/chase.json
           timeout -k 10 180 tools/diag/chase 200 > $OUT/chase.json && cp $OUT/chase.json profiles/r4/chase.json ;;
    bench) timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 ;;
    quick) # headline and tree-only, short runs (no variants / CPU baselines / isolated conv)
           timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 \
             > $OUT/quick_head.log 2>&1 && \
           timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 \
             --evaluator hash --lanes 1 --age 100 > $OUT/quick_tree.log 2>&1 ;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench \
               -- python3 bench.py --no-cpu-baseline --no-variants --no-isolated ${BENCH_ARGS:-} > $OUT/prof_bench.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "== $s rc=$rc"
  log=$(ls -t $OUT/*.log | head -1)
  tail -3 "$log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
exit 0
