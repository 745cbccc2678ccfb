#!/bin/bash
# Same-box A/B of runtime switches of the round-4 library, each on its own,
# --swap (the switch moves between the two contexts halfway, so their own
# bias cancels), after the parity tests of that library:
#   bash tools/gpu_ab_switch.sh TAG VAR=VAL[,VAR2=VAL2] [VAR=VAL ...]
# r04i: LSP_RECYCLE=0 (proof memory recycling off); r04j: LSP_GATHER_ZEROCOPY=0;
# r04k: the host/GPU boundaries (LSP_HOST_TREE_TOP, LSP_FRI_HOST_TAIL).
# Copy the library under test to _ab/new.so first.  PAIRS (env) pairs per switch, default 80.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:?tag}
shift
bash tools/gpu.sh $TAG tests:test_gpu_parity.py,test_proof_view.py || exit 1
for sw in "$@"; do
  name=$(echo "${sw}" | tr ',=' '__')
  out=gpurun_out/ab_${name}_$TAG.txt
  timeout -k 10 300 python tools/ab_inproc.py _ab/new.so _ab/new.so --pairs ${PAIRS:-80} --swap --env-b $sw > $out 2>&1 \
    || { tail -20 $out; exit 1; }
  tail -3 $out
done
timeout -k 10 200 python tools/time_step_parts.py 19 30 > gpurun_out/parts_$TAG.log 2>&1 && tail -3 gpurun_out/parts_$TAG.log
