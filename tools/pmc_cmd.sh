#!/bin/bash
# SQ counters of every kernel a command launches, one rocprofv3 --pmc pass per
# group (no trace domains mixed in): wave time split (issue / wait / stall),
# VALU and LDS instruction counts.  Summarise with tools/pmc_cmd_summary.py.
#   tools/pmc_cmd.sh TAG python3 tools/time_lde.py 19,8
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/p$i -o run -- "$@" > gpurun_out/$TAG/p$i.log 2>&1 || { tail -20 gpurun_out/$TAG/p$i.log; exit 1; }
done
echo "pmc $TAG done"
