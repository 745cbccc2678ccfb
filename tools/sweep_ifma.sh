#!/bin/bash
# 2^19 prove time vs host IFMA on/off and the host tree-top threshold
set -o pipefail
for rep in 1 2; do
for cfg in "0 256" "1 256" "1 1024" "1 2048" "1 4096"; do
  set -- $cfg
  r=$(LSP_HOST_IFMA=$1 LSP_HOST_TREE_TOP=$2 LSP_TIME_TOPS=1 timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep -E "log_n=19|tree tops" | tr '\n' ' ') || exit 1
  echo "ifma=$1 top=$2 $r"
done
done
