#!/bin/bash
# r03c4: the chained-twist library on the other BASELINE shapes -- the wide
# AIR (C3, 2^20 rows) and the LDE shapes of the wide plan, same-box A/B of
# LSP_NTT_CHAIN on the wide LDE
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --air wide --log-n 20 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_wide_r03c4.json 2> gpurun_out/bench_wide_r03c4.err || { tail -20 gpurun_out/bench_wide_r03c4.err; exit 1; }
cut -c1-400 gpurun_out/bench_wide_r03c4.json
for i in 1 2; do
  for v in 0 1; do
    echo "LSP_NTT_CHAIN=$v" >> gpurun_out/chain_lde_wide_r03c4.txt
    LSP_NTT_CHAIN=$v timeout -k 10 200 python tools/time_lde.py 20,184 19,64 19,14 >> gpurun_out/chain_lde_wide_r03c4.txt 2>&1 || exit 1
  done
done
cat gpurun_out/chain_lde_wide_r03c4.txt
