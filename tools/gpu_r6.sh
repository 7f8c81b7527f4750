#!/bin/bash
# Round-6 GPU session (tools/gpu_r5.sh plus the dataflow tower steps). STEPS picks the steps, in this order; each GPU step has its own time limit and the
# session stops at the first failure (no retries).
#   tests  every -m gpu test (verbose, per-test timeout)      smoke  __graft_entry__.smoke()
#   ring   tools/diag/lds_ring: the conv's point-GEMM loop with U by vector loads vs a per-wave LDS-DMA ring
#   fcal   FETCH_SIZE calibration on k_select's load shapes (tools/diag/fetch_cal under two rocprofv3 --pmc passes)
#   tprof  tree-only bench (hash evaluator, one lane) under rocprofv3 --kernel-trace --stats + prof_summary
#   hprof  the headline bench under rocprofv3 --kernel-trace --stats + prof_summary
#   pmcsel / pmctree  k_select / k_apply PMC traffic (headline / tree-only population, unfused)   pmcround  k_round (fused)
#   quick  headline + tree-only short bench lines    bench  bench.py (full: variants, isolated conv, CPU baselines)
#   train  tools/bench_train.py   dptrain  tools/bench_train_dp.py (one nccl rank: eager DDP+SyncBN vs graphed DP step)
#   vars   conv variants (diag lib)   modes  conv MODE ablations (tools/diag/wino3h_modes.py)
#   f16    the conv's f16 mode: errors, timing, headline line   lat  single-tree latency (Option A)   cycle  configs[4] on one GPU
#   tower  the dataflow tower against the per-conv launches, isolated, interleaved (tools/diag/tower_ab.py)
#   pmctower  the dataflow tower's HBM traffic (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_conv.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
STEPS=${STEPS:-"tests smoke quick"}
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread ${PYTEST_K:-} \
               > $OUT/gputests.log 2>&1 ;;
    smoke) timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    ring)  timeout -k 10 120 tools/diag/lds_ring ${RING_CHUNKS:-64} > $OUT/lds_ring.json 2> $OUT/lds_ring.log ;;
    gemm)  timeout -k 10 180 tools/diag/gemm_phase ${GEMM_CHUNKS:-64} > $OUT/gemm_phase.json 2> $OUT/gemm_phase.log ;;
    counters) timeout -k 10 120 rocprofv3 -L > $OUT/counters_all.txt 2> $OUT/counters.log; \
           grep -E "TCC_EA0_RD|TCC_REQ|TCC_READ|TCC_BUBBLE|TCC_EA0_WR" $OUT/counters_all.txt > $OUT/counters_tcc.txt; true ;;
    fcal)  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fcal1 -o f \
               -- tools/diag/fetch_cal > $OUT/fetch_cal.json 2> $OUT/fcal1.log && \
           timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv \
               -d $OUT/fcal2 -o f -- tools/diag/fetch_cal > $OUT/fetch_cal2.json 2> $OUT/fcal2.log && \
           python3 tools/diag/fetch_cal_summary.py $OUT/fetch_cal.json $(ls $OUT/fcal1/*/f_counter_collection.csv $OUT/fcal1/f_counter_collection.csv 2>/dev/null | head -1) \
               $(ls $OUT/fcal2/*/f_counter_collection.csv $OUT/fcal2/f_counter_collection.csv 2>/dev/null | head -1) \
               $OUT/fetch_cal_summary.json > $OUT/fcal.log 2>&1 ;;
    tprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tprof -o bench \
               -- python3 bench.py --no-cpu-baseline --no-variants --no-isolated --evaluator hash --lanes 1 --age 100 \
               --steps 20 --warmup 3 > $OUT/tprof_bench.log 2>&1 && \
           python3 tools/prof_summary.py $(ls $OUT/tprof/*/bench_kernel_trace.csv $OUT/tprof/bench_kernel_trace.csv 2>/dev/null | head -1) \
               $OUT/tprof_bench.log $OUT/prof_tree_only.md > $OUT/tprof_summary.log 2>&1 && \
           { cp $(ls $OUT/tprof/*/bench_kernel_stats.csv $OUT/tprof/bench_kernel_stats.csv 2>/dev/null | head -1) \
               $OUT/tprof_kernel_stats.csv 2>/dev/null; rm -rf $OUT/tprof; true; } ;;
    hprof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/hprof -o bench \
               -- python3 bench.py --no-cpu-baseline --no-variants --no-isolated ${BENCH_ARGS:-} > $OUT/hprof_bench.log 2>&1 && \
           python3 tools/prof_summary.py $(ls $OUT/hprof/*/bench_kernel_trace.csv $OUT/hprof/bench_kernel_trace.csv 2>/dev/null | head -1) \
               $OUT/hprof_bench.log $OUT/prof_headline.md > $OUT/hprof_summary.log 2>&1 && \
           { cp $(ls $OUT/hprof/*/bench_kernel_stats.csv $OUT/hprof/bench_kernel_stats.csv 2>/dev/null | head -1) \
               $OUT/hprof_kernel_stats.csv 2>/dev/null; rm -rf $OUT/hprof; true; } ;;
    pmctree) UTTT_FUSED_ROUNDS=0 PMC_OUT=$OUT/pmc_tree PMC_AGE=100 PMC_BENCH_ARGS="--evaluator hash --lanes 1" timeout -k 10 900 bash tools/pmc_select.sh \
               > $OUT/pmc_tree.log 2>&1 && \
             python tools/pmc_summary.py $OUT/pmc_tree $OUT/pmc_tree/p1.log $OUT/pmc_select_tree.json k_select >> $OUT/pmc_tree.log && \
             python tools/pmc_summary.py $OUT/pmc_tree $OUT/pmc_tree/p1.log $OUT/pmc_apply_tree.json k_apply >> $OUT/pmc_tree.log && \
             rm -rf $OUT/pmc_tree/p1 $OUT/pmc_tree/p2 $OUT/pmc_tree/p3 ;;
    pmcround) PMC_OUT=$OUT/pmc_round PMC_AGE=100 PMC_BENCH_ARGS="--evaluator hash --lanes 1" timeout -k 10 900 bash tools/pmc_select.sh \
               > $OUT/pmc_round.log 2>&1 && \
             python tools/pmc_summary.py $OUT/pmc_round $OUT/pmc_round/p1.log $OUT/pmc_round_tree.json k_round >> $OUT/pmc_round.log && \
             rm -rf $OUT/pmc_round/p1 $OUT/pmc_round/p2 $OUT/pmc_round/p3 ;;
    pmcsel) PMC_OUT=$OUT/pmc_sel timeout -k 10 900 bash tools/pmc_select.sh > $OUT/pmc_select.log 2>&1 && \
             python tools/pmc_summary.py $OUT/pmc_sel $OUT/pmc_sel/p1.log $OUT/pmc_select.json k_select >> $OUT/pmc_select.log && \
             python tools/pmc_summary.py $OUT/pmc_sel $OUT/pmc_sel/p1.log $OUT/pmc_apply.json k_apply >> $OUT/pmc_select.log && \
             rm -rf $OUT/pmc_sel/p1 $OUT/pmc_sel/p2 $OUT/pmc_sel/p3 ;;
    quick) timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 ${BENCH_ARGS:-} \
             > $OUT/quick_head.log 2>&1 && \
           timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 \
             --evaluator hash --lanes 1 --age 100 > $OUT/quick_tree.log 2>&1 ;;
    bench) timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 ;;
    train) timeout -k 10 400 python -u tools/bench_train.py ${TRAIN_ARGS:-} > $OUT/train.log 2>&1 ;;
    dptrain) timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
               --master-port 29531 tools/bench_train_dp.py --out $OUT/train_dp.json ${DPTRAIN_ARGS:-} > $OUT/train_dp.log 2>&1 ;;
    vars)  timeout -k 10 400 python -u tools/diag/wino3h_variants.py ${VAR_BOARDS:-1344 2688 16384} > $OUT/variants.log 2>&1 ;;
    modes) MODES=${MODES:-0,8,1048576,1048584} timeout -k 10 300 python -u tools/diag/wino3h_modes.py ${MODE_BOARDS:-1344 16384} \
             > $OUT/modes.log 2>&1 ;;
    f16)   timeout -k 10 300 python -u tools/diag/f16_mode_check.py > $OUT/f16_check.log 2>&1 && \
           timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-variants --no-isolated --steps 10 --warmup 4 \
             --evaluator fused_f16 > $OUT/quick_f16.log 2>&1 ;;
    lat)   timeout -k 10 300 python -u tools/diag/latency_single.py > $OUT/latency.log 2>&1 ;;
    cycle) timeout -k 10 900 python -u tools/bench_cycle.py --out $OUT/cycle.json ${CYCLE_ARGS:-} > $OUT/cycle.log 2>&1 ;;
    tower) timeout -k 10 300 python -u tools/diag/tower_ab.py $OUT/tower_ab.json ${TOWER_BOARDS:-1370,2740,4096,16384} 4 10 \
             > $OUT/tower_ab.log 2>&1 ;;
    pmctower) UTTT_NN_TOWER=dataflow timeout -k 10 600 bash tools/pmc_conv.sh > $OUT/pmc_tower.log 2>&1 && \
             python3 tools/pmc_conv_summary.py gpurun_out/pmc_conv 1344 $OUT/pmc_tower.json k_wino3t_tower 32 >> $OUT/pmc_tower.log && \
             rm -rf gpurun_out/pmc_conv/p1 gpurun_out/pmc_conv/p2 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "== $s rc=$rc"
  log=$(ls -t $OUT/*.log | head -1)
  tail -3 "$log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
exit 0
