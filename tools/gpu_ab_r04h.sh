#!/bin/bash
# r04h: the two host-side changes of round 4 as runtime switches, same library,
# --swap (the switch moves between the two contexts halfway: their own bias cancels)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh r04h tests:test_gpu_parity.py || exit 1
for sw in LSP_QUERY_POOL=0 LSP_HOST_LEVELS=r3; do
  timeout -k 10 300 python tools/ab_inproc.py _ab/new.so _ab/new.so --pairs 80 --swap --env-b $sw > gpurun_out/ab_${sw%%=*}_r04h.txt 2>&1 || { tail -20 gpurun_out/ab_${sw%%=*}_r04h.txt; exit 1; }
  cat gpurun_out/ab_${sw%%=*}_r04h.txt
done
bash tools/gpu.sh r04h prof || exit 1
f=$(ls gpurun_out/prof_r04h/*kernel_trace.csv | head -1)
python tools/trace_gaps.py $f > gpurun_out/trace_gaps_r04h.txt && cat gpurun_out/trace_gaps_r04h.txt
