#!/bin/bash
# A/B of an environment switch on one box: alternating 2^19 prove timings
# usage: tools/ab_env.sh VAR valA valB [rounds]
set -o pipefail
V=$1; A=$2; B=$3; N=${4:-3}
for i in $(seq $N); do
  for val in $A $B; do
    r=$(env $V=$val timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep "log_n=19") || exit 1
    echo "$V=$val $r"
  done
done
