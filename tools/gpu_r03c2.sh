#!/bin/bash
# r03c2: the round's final library (chained coset twist) -- every GPU test,
# smoke, the default bench line, then the rocprofv3 kernel trace of the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03c2
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_$TAG.json
