#!/bin/bash
# The PMC passes bench.py's roofline reads, and nothing else: FETCH_SIZE /
# WRITE_SIZE of the 2^19 x 8 coset LDE (tools/pmc_round.sh's first three
# passes) and the VALU / LDS groups of one 2^19 prove (tools/pmc_valu.sh).
# The library's stamp (liblsp_hip.so.src, written by build.py at link time) is
# copied into the run directory; summarize afterwards here (the summaries take
# the run's stamp, so the profile names the build that ran on the box):
#   python tools/pmc_traffic.py gpurun_out/$TAG/fetch/lde_counter_collection.csv \
#       gpurun_out/$TAG/write/lde_counter_collection.csv 524288 8 > profiles/${TAG}_lde_traffic.json
#   python tools/pmc_valu_summary.py gpurun_out/$TAG/valu profiles/${TAG}_valu_pmc.json
#   python tools/pmc_valu_summary.py gpurun_out/$TAG/valu_wide profiles/${TAG}_valu_pmc_wide.json
# (the last: the same VALU group over one wide-AIR 2^20 prove, BASELINE configs[2],
# which bench.py's wide_c3 leg reads)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-stamp}
mkdir -p gpurun_out/$TAG
cp linea_stark_prover_amd/_lib/liblsp_hip.so.src gpurun_out/$TAG/lib_src_sha16.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/kt -o lde -- python3 tools/lde_probe.py 19 3 > gpurun_out/$TAG.kt.log 2>&1 || { tail -20 gpurun_out/$TAG.kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/fetch -o lde -- python3 tools/lde_probe.py 19 3 > gpurun_out/$TAG.fetch.log 2>&1 || { tail -20 gpurun_out/$TAG.fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/write -o lde -- python3 tools/lde_probe.py 19 3 > gpurun_out/$TAG.write.log 2>&1 || { tail -20 gpurun_out/$TAG.write.log; exit 1; }
echo "lde pmc done"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/valu/p$i -o run -- python3 tools/time_prove.py 19 > gpurun_out/$TAG.p$i.log 2>&1 || { tail -20 gpurun_out/$TAG.p$i.log; exit 1; }
done
echo "valu pmc done"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/valu_wide/p1 -o run -- python3 tools/time_prove.py w20 > gpurun_out/$TAG.w1.log 2>&1 || { tail -20 gpurun_out/$TAG.w1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d gpurun_out/$TAG/valu_wide/p2 -o run -- python3 tools/time_prove.py w20 > gpurun_out/$TAG.w2.log 2>&1 || { tail -20 gpurun_out/$TAG.w2.log; exit 1; }
echo "wide valu pmc done"
