#!/bin/bash
# r03m: openings from the host copies of host-made layers (no top uploads):
# the proof suites that exercise the query openings, then a same-box A/B of
# the library against the previous build, and of the phase events.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_fullsize.py tests/test_linear_layers.py > gpurun_out/tests_r03m.log 2>&1 || { tail -30 gpurun_out/tests_r03m.log; exit 1; }
tail -2 gpurun_out/tests_r03m.log
export LSP_TP_REPS=15
for i in 1 2 3 4; do
  for lib in abl/r03m_base.so linea_stark_prover_amd/_lib/liblsp_hip.so; do
    r=$(LSP_LIB=$lib timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep "log_n=19") || exit 1
    echo "$(basename $lib) $r" | tee -a gpurun_out/ab_r03m.txt
  done
done
for i in 1 2 3 4; do
  for v in 1 0; do
    r=$(LSP_PHASE_EVENTS=$v timeout -k 10 120 python tools/time_prove.py 19 2>&1 | grep "log_n=19") || exit 1
    echo "LSP_PHASE_EVENTS=$v $r" | tee -a gpurun_out/ab_r03m.txt
  done
done
