#!/bin/bash
# same-box A/B of two library builds on one phase of the 2^19 prove (tools/time_prove.py timings)
# usage: tools/ab_phase.sh libA.so libB.so "phase name" [rounds]
set -o pipefail
A=$1; B=$2; PH=$3; N=${4:-3}
for i in $(seq $N); do
  for lib in $A $B; do
    r=$(LSP_LIB=$lib timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep -E "log_n=19|  $PH  " | tr -s ' ' | tr '\n' ' ') || exit 1
    echo "$(basename $lib) $r"
  done
done
