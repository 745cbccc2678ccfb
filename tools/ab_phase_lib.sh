#!/bin/bash
# same-box A/B of one prove phase over library builds (tools/time_prove.py 19)
# usage: tools/ab_phase_lib.sh "abl/a.so abl/b.so" "phase name" [rounds]
set -o pipefail
LIBS=$1; PH=$2; N=${3:-3}
for i in $(seq $N); do
  for lib in $LIBS; do
    r=$(LSP_LIB=$lib timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep -E "log_n=19|$PH" | tr '\n' ' ') || exit 1
    echo "$(basename $lib) $r"
  done
done
