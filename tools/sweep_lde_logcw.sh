#!/bin/bash
# LDE time per minimum column chunk (LSP_NTT_LOGCW) at the given shapes
# usage: tools/sweep_lde_logcw.sh "20,184 19,64" [rounds] [logcw values]
set -o pipefail
SH=${1:-"20,184 19,64"}; N=${2:-2}; CWS=${3:-"0 1 2 3"}
for i in $(seq $N); do
for cw in $CWS; do
  r=$(LSP_NTT_LOGCW=$cw timeout -k 10 200 python tools/time_lde.py $SH 2>&1 | grep "lde 2" | tr '\n' ' ') || exit 1
  echo "LOGCW=$cw $r"
done
done
