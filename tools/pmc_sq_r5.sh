#!/bin/bash
# VERDICT r4 item 2's counters: the same four SQ passes as tools/pmc_sq.sh (kernel trace only, <= 8 SQ
# counters per pass, each pass under its own KILL timeout), over
#   conv: the product conv at N boards, split-f16 and the f16 mode (half the U bytes per set), one
#         process (tools/diag/conv_once.py), and
#   ring: tools/diag/lds_ring, the point-GEMM loop with U by vector loads (k_ring<0>) and by a
#         per-wave LDS-DMA ring (k_ring<1>).
# Stops at the first pass that does not exit 0. Summarised by tools/pmc_sq_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_r5
N=${N:-16384}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1
echo "list rc=$?"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_MFMA"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_MFMA_F16"
  "SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_INST_VMEM SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32"
)
for tgt in conv ring; do
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    sel=""
    for c in $p; do grep -qw "$c" $OUT/list.txt && sel="$sel $c"; done
    echo "$tgt pass $i:$sel"
    [ -n "$sel" ] || continue
    if [ $tgt = conv ]; then
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $sel --output-format csv -d $OUT/$tgt/p$i -o t \
          -- python3 tools/diag/conv_once.py $N 3 > $OUT/$tgt.p$i.log 2>&1
    else
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $sel --output-format csv -d $OUT/$tgt/p$i -o t \
          -- tools/diag/lds_ring ${RING_CHUNKS:-64} > $OUT/$tgt.p$i.log 2>&1
    fi
    rc=$?
    echo "$tgt pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
