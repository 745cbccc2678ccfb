#!/bin/bash
# r03l: sharded proofs over more ranks than cosets (G = 16, 32 virtual
# ranks), the existing shard suite, and prove's argument validation.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shard.py tests/test_gpu_parity.py::test_prove_rejects_bad_arguments > gpurun_out/shard_tests_r03l.log 2>&1 || { tail -40 gpurun_out/shard_tests_r03l.log; exit 1; }
tail -3 gpurun_out/shard_tests_r03l.log
