#!/bin/bash
# VALU / LDS counters for every kernel of one 2^19 prove (tools/time_prove.py),
# one rocprofv3 --pmc pass per counter group (no trace domains mixed in).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-valu}
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/p$i -o run -- python3 tools/time_prove.py 19 > gpurun_out/$TAG.p$i.log 2>&1 || { tail -20 gpurun_out/$TAG.p$i.log; exit 1; }
done
echo "pmc valu done"
