#!/bin/bash
# L2 behaviour of k_wino3h_conv in the headline bench (two lanes' convs overlapping) against one
# lane's forward alone (tools/diag/nn_forward_only.py at 1,344 boards): TCC hit / miss counts, and
# FETCH_SIZE in the bench, one rocprofv3 pass each (kernel trace only). Summarised by
# tools/pmc_l2_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_l2
mkdir -p $OUT
run() {  # name counters cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $OUT/$name -o t -- "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "pass $name ($ctr) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/$name.log; exit $rc; }
}
BENCH="python3 bench.py --no-cpu-baseline --no-variants --no-isolated --steps 6 --warmup 2 --age 40"
run bench_hit "TCC_HIT_sum TCC_MISS_sum" $BENCH
run fwd_hit "TCC_HIT_sum TCC_MISS_sum" python3 tools/diag/nn_forward_only.py 1344 12
run bench_fetch "FETCH_SIZE" $BENCH
exit 0
