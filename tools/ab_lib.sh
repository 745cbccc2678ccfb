#!/bin/bash
# same-box A/B of two builds of liblsp_hip.so: alternating 2^19 prove timings
# usage: tools/ab_lib.sh libA.so libB.so [rounds] [log_n]
set -o pipefail
A=$1; B=$2; N=${3:-3}; LG=${4:-19}
for i in $(seq $N); do
  for lib in $A $B; do
    r=$(LSP_LIB=$lib timeout -k 10 120 python tools/time_prove.py $LG 2>&1 | grep "log_n=$LG") || exit 1
    echo "$(basename $lib) $r"
  done
done
