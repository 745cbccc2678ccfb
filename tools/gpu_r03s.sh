#!/bin/bash
# r03s: same-process A/Bs of the per-proof knobs (tools/ab_inproc.py): the
# host/GPU boundary of the FRI tail and of the tree tops
set -o pipefail
mkdir -p gpurun_out
L=linea_stark_prover_amd/_lib/liblsp_hip.so
for kv in LSP_PHASE_EVENTS=0 LSP_PHASE_EVENTS=0; do
  echo "== $kv" >> gpurun_out/ab_knobs_r03s.txt
  timeout -k 10 300 python tools/ab_inproc.py $L $L --pairs 80 --env-b $kv >> gpurun_out/ab_knobs_r03s.txt 2>&1 || { cat gpurun_out/ab_knobs_r03s.txt; exit 1; }
done
cat gpurun_out/ab_knobs_r03s.txt
