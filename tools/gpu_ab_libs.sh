#!/bin/bash
# Same-box A/B of library builds (replaces round 4's single-use gpu_ab_r04f/g/h.sh):
#
#   bash tools/gpu_ab_libs.sh TAG A:B [A:B ...]
#
# A and B name libraries under _ab/ (copy them there first: _ab/base.so,
# _ab/new.so, ...).  Every pair runs tools/ab_inproc.py (both libraries in one
# process, proofs alternating, the same trace) after the parity tests of the
# library under test (_ab/new.so is what the in-tree build produced).
# PAIRS (env) proofs per side, default 40; TESTS (env) the GPU test files to run
# first, default test_gpu_parity.py; TESTS=none skips them.  AB_ARGS (env): more
# tools/ab_inproc.py arguments (e.g. --r3-abi a when A is a round-3 build).
# Runtime switches of one library: tools/gpu_ab_switch.sh.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:?usage: tools/gpu_ab_libs.sh TAG A:B [A:B ...]}
shift
if [ "${TESTS:-test_gpu_parity.py}" != none ]; then
  bash tools/gpu.sh $TAG tests:${TESTS:-test_gpu_parity.py} || exit 1
fi
for pair in "$@"; do
  a=${pair%%:*}
  b=${pair##*:}
  out=gpurun_out/ab_${a}_${b}_$TAG.txt
  timeout -k 10 300 python tools/ab_inproc.py _ab/$a.so _ab/$b.so --pairs ${PAIRS:-40} ${AB_ARGS:-} > $out 2>&1 \
    || { tail -20 $out; exit 1; }
  cat $out
done
