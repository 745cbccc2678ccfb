#!/bin/bash
# same-box A/B of LDE timings over variant libraries built by tools/variant_lib.py
# usage: [ABDIR=_ab] tools/ab_lde_variants.sh "base v1 v2" [rounds] [shapes...]  (ABDIR: where the .so files are; abl/ does not travel to the GPU box)
set -o pipefail
VS=$1; N=${2:-2}; shift 2; SH=${@:-19,8 19,4 22,8}
for i in $(seq $N); do
  for v in $VS; do
    echo "== $v"; LSP_LIB=${ABDIR:-abl}/$v.so LSP_LIB_OLDER=1 timeout -k 10 120 python tools/time_lde.py $SH || exit 1
  done
done
