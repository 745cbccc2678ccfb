#!/bin/bash
# same-box A/B of variant libraries (tools/variant_lib.py): alternating 2^LG
# prove timings with the hashing-dominated phases
# usage: tools/ab_prove.sh "base v1 ..." [rounds] [log_n]
set -o pipefail
VS=$1; N=${2:-3}; LG=${3:-19}
for i in $(seq $N); do
  for v in $VS; do
    out=$(LSP_LIB=abl/$v.so timeout -k 10 180 python tools/time_prove.py $LG 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "$v $(echo "$out" | grep "log_n=$LG" | cut -d' ' -f3,5) $(echo "$out" | grep -E "  merkle tree |commit to quotient|commit phase|reduce rows" | awk '{printf "%s=%s ", $1, $(NF-1)}')"
  done
done
