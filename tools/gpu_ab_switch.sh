#!/bin/bash
# Same-box A/B of one runtime switch of the round-4 library, --swap (the switch
# moves between the two contexts halfway, so their own bias cancels), after
# the parity tests of that library:
#   bash tools/gpu_ab_switch.sh TAG VAR=VAL [pairs]
# r04i: LSP_RECYCLE=0 (proof memory recycling off); r04j: LSP_GATHER_ZEROCOPY=0.
# Copy the library under test to _ab/new.so first.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:?tag}; sw=${2:?VAR=VAL}; pairs=${3:-80}
bash tools/gpu.sh $TAG tests:test_gpu_parity.py,test_proof_view.py || exit 1
out=gpurun_out/ab_${sw%%=*}_$TAG.txt
timeout -k 10 300 python tools/ab_inproc.py _ab/new.so _ab/new.so --pairs $pairs --swap --env-b $sw > $out 2>&1 || { tail -20 $out; exit 1; }
cat $out
timeout -k 10 200 python tools/time_step_parts.py 19 30 > gpurun_out/parts_$TAG.log 2>&1 && tail -3 gpurun_out/parts_$TAG.log
