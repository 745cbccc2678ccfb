#!/bin/bash
# r03j: single-wave MAD latency probe, NTT parity after the trivial-end
# groups change, same-box LDE A/B (abl/base.so vs the tree's library), then
# the stamped PMC passes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "coset_lde or prove_bit_exact" tests/test_gpu_fullsize.py > gpurun_out/ntt_tests_r03j.log 2>&1 || { tail -30 gpurun_out/ntt_tests_r03j.log; exit 1; }
tail -2 gpurun_out/ntt_tests_r03j.log
for i in 1 2 3; do
  for lib in abl/base.so linea_stark_prover_amd/_lib/liblsp_hip.so; do
    echo "== $lib" >> gpurun_out/lde_ab_r03j.txt
    LSP_LIB=$lib timeout -k 10 120 python tools/time_lde.py 19,8 19,4 22,8 >> gpurun_out/lde_ab_r03j.txt 2>&1 || { tail -20 gpurun_out/lde_ab_r03j.txt; exit 1; }
  done
done
cat gpurun_out/lde_ab_r03j.txt
bash tools/pmc_stamp.sh r03j
LSP_TIME_TOPS=1 timeout -k 10 120 python tools/time_prove.py 19 > gpurun_out/time_tops_r03j.txt 2>&1 || { tail -20 gpurun_out/time_tops_r03j.txt; exit 1; }
tail -5 gpurun_out/time_tops_r03j.txt
