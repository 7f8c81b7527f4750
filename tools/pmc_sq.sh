#!/bin/bash
# Where k_wino3h_conv's cycles go: SQ counters in separate rocprofv3 passes (kernel trace only,
# <= 8 SQ counters per pass, each pass under its own KILL timeout) over the product launch at
# N boards (tools/diag/wino3h_variants.py, no variants, one round). Counter names are taken from
# `rocprofv3 -L` on the box; names it does not list are dropped. Summarised by tools/pmc_sq_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq
N=${N:-16384}
export VARIANTS= ROUNDS=1
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1
echo "list rc=$?"
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_MFMA"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_MFMA_F16"
  "SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_INST_VMEM SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  sel=""
  for c in $p; do grep -qw "$c" $OUT/list.txt && sel="$sel $c"; done
  echo "pass $i:$sel"
  [ -n "$sel" ] || continue
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $sel --output-format csv -d $OUT/p$i -o t \
      -- python3 tools/diag/wino3h_variants.py $N > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
