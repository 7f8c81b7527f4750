#!/bin/bash
# HBM traffic of k_select and k_apply from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (kernel trace only) over a short bench run whose population is aged like the bench's
# (--age 300, PMC_AGE to change), so the traffic and the algorithmic bytes (the same run's bench line,
# p1.log) describe one population.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_sel}
mkdir -p $OUT
i=0
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/p$i -o t \
      -- python3 bench.py --no-cpu-baseline --no-variants --no-isolated --steps 6 --warmup 2 --age ${PMC_AGE:-300} ${PMC_BENCH_ARGS:-} \
      > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($c) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
exit 0
