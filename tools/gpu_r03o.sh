#!/bin/bash
# r03o: phase-timing selection (test), then the bench main line timing only
# the roofline phases
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_knobs.py::test_phase_timing_selection tests/test_replicas.py > gpurun_out/tests_r03o.log 2>&1 || { tail -30 gpurun_out/tests_r03o.log; exit 1; }
tail -2 gpurun_out/tests_r03o.log
timeout -k 10 300 python bench.py --no-cpu-baseline --shape-leg none --batch-leg none --shard-leg none --inflight 0 --no-host-trace-leg > gpurun_out/bench_r03o.json 2> gpurun_out/bench_r03o.err || { tail -20 gpurun_out/bench_r03o.err; exit 1; }
cut -c1-400 gpurun_out/bench_r03o.json
