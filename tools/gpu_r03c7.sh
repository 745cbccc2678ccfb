#!/bin/bash
# r03c7: the bench.log-shape leg with bench.log's 29 proof-of-work bits (GPU grind)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --inflight 0 --shard-leg none --batch-leg none --no-host-trace-leg --shape-pow-bits 29 > gpurun_out/bench_pow_r03c7.json 2> gpurun_out/bench_pow_r03c7.err || { tail -20 gpurun_out/bench_pow_r03c7.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_pow_r03c7.json')); print(d['ms_per_step']); s=d['shape_bench_log']; print(s['prove_time_s'], s.get('proof_of_work_bits')); print(json.dumps(s.get('with_pow')))"
