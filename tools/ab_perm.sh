#!/bin/bash
# same-box A/B of Poseidon2 variants: register-resident permutation rate and
# 2^19 prove time (tools/perm_rate.py), alternating over the given libraries
# usage: tools/ab_perm.sh "abl/a.so abl/b.so ..." [rounds]
set -o pipefail
LIBS=$1; N=${2:-3}
for i in $(seq $N); do
  for lib in $LIBS; do
    r=$(LSP_LIB=$lib timeout -k 10 120 python tools/perm_rate.py 2>&1 | tr '\n' ' ') || exit 1
    echo "$(basename $lib) $r"
  done
done
