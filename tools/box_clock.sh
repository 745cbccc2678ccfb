#!/bin/bash
# Box-to-box variance probe: a short bench (prove time on this box) and, on the
# same box, one PMC pass whose GRBM_GUI_ACTIVE gives each kernel's mean clock
# (tools/pmc_valu_summary.py), so a slow box can be told apart from a slow build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-clock}
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --inflight 0 --shard-leg none --batch-leg none --no-host-trace-leg > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/p1 -o run -- python3 tools/time_prove.py 19 > gpurun_out/$TAG.p1.log 2>&1 || { tail -20 gpurun_out/$TAG.p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d gpurun_out/$TAG/p2 -o run -- python3 tools/time_prove.py 19 > gpurun_out/$TAG.p2.log 2>&1 || { tail -20 gpurun_out/$TAG.p2.log; exit 1; }
echo "box clock done"
