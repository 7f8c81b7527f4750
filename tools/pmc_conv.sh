#!/bin/bash
# HBM traffic of k_wino3h_conv from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (kernel trace only) over tools/diag/nn_forward_only.py (1344 positions,
# a lane's batch at the bench config). Summarised by tools/pmc_conv_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_conv
N=${N:-1344}
mkdir -p $OUT
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/p$i -o t \
      -- python3 tools/diag/nn_forward_only.py $N 12 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($c) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
exit 0
