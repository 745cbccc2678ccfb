#!/bin/bash
# same-box A/B of LDE timings over variant libraries built by tools/variant_lib.py
# usage: tools/ab_lde_variants.sh "base v1 v2" [rounds] [shapes...]
set -o pipefail
VS=$1; N=${2:-2}; shift 2; SH=${@:-19,8 19,4 22,8}
for i in $(seq $N); do
  for v in $VS; do
    echo "== $v"; LSP_LIB=abl/$v.so timeout -k 10 120 python tools/time_lde.py $SH || exit 1
  done
done
