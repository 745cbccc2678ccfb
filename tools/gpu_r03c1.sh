#!/bin/bash
# r03c1: chained coset twist in the fused LDE pass -- LDE / DFT / proof parity
# (one GPU, virtual-rank shards), then a same-box A/B of LSP_NTT_CHAIN (LDE
# shapes and whole 2^19 proofs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dft.py tests/test_gpu_fullsize.py \
  tests/test_gpu_shard.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/chain_tests_r03c1.log 2>&1 || { tail -30 gpurun_out/chain_tests_r03c1.log; exit 1; }
tail -3 gpurun_out/chain_tests_r03c1.log
for i in 1 2 3; do
  for v in 0 1; do
    echo "LSP_NTT_CHAIN=$v" >> gpurun_out/chain_lde_r03c1.txt
    LSP_NTT_CHAIN=$v timeout -k 10 120 python tools/time_lde.py 19,8 19,4 22,8 >> gpurun_out/chain_lde_r03c1.txt 2>&1 || exit 1
  done
done
cat gpurun_out/chain_lde_r03c1.txt
timeout -k 10 400 bash tools/ab_env.sh LSP_NTT_CHAIN 0 1 3 | tee gpurun_out/chain_prove_r03c1.txt
