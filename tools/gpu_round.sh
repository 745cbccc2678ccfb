#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
echo "=== tests"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
echo "=== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
echo "=== bench"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { cat gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
echo "=== rocprof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --inflight 0 --shard-leg none --batch-leg none --shape-leg none --no-host-trace-leg > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail -20 gpurun_out/prof_$TAG.err; exit 1; }
echo done
echo "=== pmc (stamped with this library)"
bash tools/pmc_stamp.sh pmc_$TAG || exit 1
echo pmc done
