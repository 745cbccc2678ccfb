#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-w}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 900 python bench.py --air wide --log-n 20 --steps 2 --warmup 1 > gpurun_out/bench_wide_$TAG.json 2> gpurun_out/bench_wide_$TAG.err || { tail -20 gpurun_out/bench_wide_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_wide_$TAG.json
python -c "import json; d=json.load(open('gpurun_out/bench_wide_$TAG.json')); print(d['phases_ms'])"
