#!/bin/bash
# Same-box A/B of the host tree tops: ab/lib_prev.so against the in-tree library, alternating,
# with LSP_TIME_TOPS=1 (per-tree host levels, query-phase parts) at 2^19.
set -o pipefail
for i in 1 2 3; do
  for lib in ab/lib_prev.so linea_stark_prover_amd/_lib/liblsp_hip.so; do
    r=$(LSP_LIB=$lib LSP_TIME_TOPS=1 timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep -E "log_n=19|tree tops|\[query\]" | tail -3 | tr '\n' ' ') || exit 1
    echo "$(basename $lib) $r"
  done
done
