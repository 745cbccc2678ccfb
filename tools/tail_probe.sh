#!/bin/bash
# The FRI host tail's boundary (LSP_FRI_HOST_TAIL = 2048, 1024, 512, 4096 leaves): per-round
# host times (LSP_TIME_TOPS=1) and the 2^19 prove time for each.
set -o pipefail
mkdir -p gpurun_out
for t in 2048 1024 512 4096; do
  echo "== LSP_FRI_HOST_TAIL=$t"
  LSP_FRI_HOST_TAIL=$t LSP_TIME_TOPS=1 timeout -k 10 120 python tools/time_prove.py 19 > gpurun_out/tail_$t.log 2>&1 || exit 1
  grep -E "log_n=19|fri tail|commit phase|FRI prover" gpurun_out/tail_$t.log | tail -30
done
