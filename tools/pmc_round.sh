#!/bin/bash
# PMC passes for the roofline kernel (coset LDE) + a 2^22 bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/kt -o lde -- python3 tools/lde_probe.py 19 3 > gpurun_out/$TAG.kt.log 2>&1 || { tail -20 gpurun_out/$TAG.kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/fetch -o lde -- python3 tools/lde_probe.py 19 3 > gpurun_out/$TAG.fetch.log 2>&1 || { tail -20 gpurun_out/$TAG.fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/write -o lde -- python3 tools/lde_probe.py 19 3 > gpurun_out/$TAG.write.log 2>&1 || { tail -20 gpurun_out/$TAG.write.log; exit 1; }
echo "pmc done"
timeout -k 10 600 python bench.py --log-n 22 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench22_$TAG.json 2> gpurun_out/bench22_$TAG.err || { tail -20 gpurun_out/bench22_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/bench22_$TAG.json
timeout -k 10 900 python bench.py --air wide --log-n 20 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_wide_$TAG.json 2> gpurun_out/bench_wide_$TAG.err || { tail -20 gpurun_out/bench_wide_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_wide_$TAG.json
