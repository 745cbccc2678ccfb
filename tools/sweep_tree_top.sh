#!/bin/bash
# prove time at 2^19 vs the host tree-top threshold and host threads
set -o pipefail
for top in 128 256 512; do
  for th in 8 16; do
    r=$(LSP_HOST_TREE_TOP=$top LSP_HOST_THREADS=$th timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep "log_n=19") || exit 1
    echo "top=$top threads=$th $r"
  done
done
