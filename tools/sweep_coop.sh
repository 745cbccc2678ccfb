#!/bin/bash
# prove time at 2^19 vs the quad-cooperative Merkle-level block size and width cutoff
set -o pipefail
for cfg in "64 16384" "256 16384" "128 16384" "64 8192" "256 32768"; do
  set -- $cfg
  r=$(LSP_COOP_BS=$1 LSP_COOP_MAX=$2 timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep "log_n=19") || exit 1
  echo "bs=$1 max=$2 $r"
done
