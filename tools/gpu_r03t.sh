#!/bin/bash
# r03t: A/A bias of two contexts, then switch A/Bs with the context swap
set -o pipefail
mkdir -p gpurun_out
L=linea_stark_prover_amd/_lib/liblsp_hip.so
echo "== A/A" >> gpurun_out/ab_r03t.txt
timeout -k 10 300 python tools/ab_inproc.py $L $L --pairs 60 >> gpurun_out/ab_r03t.txt 2>&1 || { cat gpurun_out/ab_r03t.txt; exit 1; }
for kv in LSP_PHASE_EVENTS=0 LSP_HOST_TREE_TOP=2048,LSP_FRI_HOST_TAIL=1024; do
  echo "== $kv (swap)" >> gpurun_out/ab_r03t.txt
  timeout -k 10 300 python tools/ab_inproc.py $L $L --pairs 100 --swap --env-b $kv >> gpurun_out/ab_r03t.txt 2>&1 || { cat gpurun_out/ab_r03t.txt; exit 1; }
done
cat gpurun_out/ab_r03t.txt
