#!/bin/bash
# Round-3 GPU session: the gpu_round.sh steps, then F1 witness timing at 2^20
# and the configs[3] one-rank rehearsal at 2^26 (ranks 0 and 7 of 8).
set -o pipefail
TAG=${1:-r03}
bash tools/gpu_round.sh $TAG || exit 1
echo "=== witness 2^20"
timeout -k 10 300 python tools/time_witness.py 20 > gpurun_out/witness_$TAG.log 2>&1 || { tail -20 gpurun_out/witness_$TAG.log; exit 1; }
tail -5 gpurun_out/witness_$TAG.log
echo "=== rank rehearsal 2^26"
timeout -k 10 600 python tools/rank_rehearsal.py --log-n 26 --ranks 0,7 --steps 2 > gpurun_out/rehearsal_$TAG.jsonl 2> gpurun_out/rehearsal_$TAG.err || { tail -20 gpurun_out/rehearsal_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/rehearsal_$TAG.jsonl
echo done
