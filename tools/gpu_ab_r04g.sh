#!/bin/bash
# r04g: which host-side change moved the 2^19 proof: base (c9ef633) -> v1 (parallel query
# assembly + serialization, f709aaa) -> new (+ per-thread host subtrees, block-k0 twist table)
set -o pipefail
mkdir -p gpurun_out
for pair in "base v1" "v1 new" "new base"; do
  set -- $pair
  timeout -k 10 300 python tools/ab_inproc.py _ab/$1.so _ab/$2.so --pairs 40 > gpurun_out/ab_$1_$2_r04g.txt 2>&1 || { tail -20 gpurun_out/ab_$1_$2_r04g.txt; exit 1; }
  cat gpurun_out/ab_$1_$2_r04g.txt
done
