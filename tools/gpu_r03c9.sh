#!/bin/bash
# r03c9: the round's final tree -- every GPU test and smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r03c9.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r03c9.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r03c9.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03c9.log 2>&1 || { cat gpurun_out/smoke_r03c9.log; exit 1; }
cat gpurun_out/smoke_r03c9.log
