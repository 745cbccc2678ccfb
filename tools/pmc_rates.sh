#!/bin/bash
# PMC passes over the instruction-rate probe (tools/ubench/rates): what the
# SQ VALU counters read for instruction classes of known issue cost.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_rates}
mkdir -p $OUT
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE SQ_WAVES" "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- tools/ubench/rates > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
echo "pmc rates done"
