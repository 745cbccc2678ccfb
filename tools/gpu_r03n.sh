#!/bin/bash
# r03n: in-process A/Bs (tools/ab_inproc.py): the previous build against
# this one (openings from host copies), and phase events on/off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_inproc.py abl/r03m_base.so linea_stark_prover_amd/_lib/liblsp_hip.so --pairs 40 > gpurun_out/ab_inproc_r03n.txt 2>&1 || { cat gpurun_out/ab_inproc_r03n.txt; exit 1; }
timeout -k 10 300 python tools/ab_inproc.py linea_stark_prover_amd/_lib/liblsp_hip.so linea_stark_prover_amd/_lib/liblsp_hip.so --pairs 40 --env-b LSP_PHASE_EVENTS=0 >> gpurun_out/ab_inproc_r03n.txt 2>&1 || { cat gpurun_out/ab_inproc_r03n.txt; exit 1; }
cat gpurun_out/ab_inproc_r03n.txt
