#!/bin/bash
# r03c3: the final library's profiles -- host tree-top timings of one 2^19
# prove (LSP_TIME_TOPS=1), the rocprofv3 kernel trace of the bench command, and
# the stamped PMC passes bench.py's roofline fields read
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03c3
LSP_TIME_TOPS=1 LSP_TP_REPS=3 timeout -k 10 200 python tools/time_prove.py 19 > gpurun_out/tops_$TAG.txt 2>&1 || { tail -20 gpurun_out/tops_$TAG.txt; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --inflight 0 --shard-leg none --batch-leg none --shape-leg none --no-host-trace-leg > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail -20 gpurun_out/prof_$TAG.err; exit 1; }
echo "rocprof done"
bash tools/pmc_stamp.sh pmc_$TAG || exit 1
echo "pmc done"
