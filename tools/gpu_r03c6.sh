#!/bin/bash
# r03c6: query assembly straight from the pinned download (one rank) -- proof
# parity (whole proofs, shards, proof views), then a same-process A/B against
# the previous build (_ab/base.so) and the host-side query timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py \
  tests/test_proof_view.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/query_tests_r03c6.log 2>&1 || { tail -30 gpurun_out/query_tests_r03c6.log; exit 1; }
tail -2 gpurun_out/query_tests_r03c6.log
LSP_TIME_TOPS=1 LSP_TP_REPS=3 timeout -k 10 200 python tools/time_prove.py 19 2>&1 | grep -E "query|log_n" > gpurun_out/query_tops_r03c6.txt || exit 1
cat gpurun_out/query_tops_r03c6.txt
timeout -k 10 400 python tools/ab_inproc.py _ab/base.so linea_stark_prover_amd/_lib/liblsp_hip.so --pairs 80 > gpurun_out/ab_query_r03c6.txt 2>&1 || { tail -20 gpurun_out/ab_query_r03c6.txt; exit 1; }
tail -8 gpurun_out/ab_query_r03c6.txt
