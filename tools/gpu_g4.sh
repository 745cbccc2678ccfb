#!/bin/bash
# Round-3 GPU session: the column-split inverse NTT of sharded proofs (tests,
# 2^24 over 8 virtual ranks with and without it, the 2^26 rank rehearsal) and
# a same-box A/B of the F1 witness (hipCUB build abl/wit_cub.so vs in-tree).
set -o pipefail
TAG=${1:-g4}
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "=== shard tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_shard_mp.py > gpurun_out/shard_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/shard_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/shard_tests_$TAG.log
echo "=== shard phases 2^24 / 8 (split inverse)"
timeout -k 10 300 python tools/shard_phases.py 24 8 > gpurun_out/shard_phases_split_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_phases_split_$TAG.txt; exit 1; }
tail -4 gpurun_out/shard_phases_split_$TAG.txt
echo "=== shard phases 2^24 / 8 (redundant inverse)"
LSP_SHARD_SPLIT_INTT=0 timeout -k 10 300 python tools/shard_phases.py 24 8 > gpurun_out/shard_phases_nosplit_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_phases_nosplit_$TAG.txt; exit 1; }
tail -4 gpurun_out/shard_phases_nosplit_$TAG.txt
echo "=== witness A/B"
for i in 1 2 3; do
  for lib in abl/wit_cub.so linea_stark_prover_amd/_lib/liblsp_hip.so; do
    r=$(LSP_LIB=$lib timeout -k 10 200 python tools/time_witness.py 20 --gpu-only 2>&1 | grep "GPU witness") || exit 1
    echo "$(basename $lib) $r" | tee -a gpurun_out/witness_ab_$TAG.txt
  done
done
echo "=== rank rehearsal 2^26 (split inverse)"
timeout -k 10 600 python tools/rank_rehearsal.py --log-n 26 --ranks 0,7 --steps 2 > gpurun_out/rehearsal_$TAG.jsonl 2> gpurun_out/rehearsal_$TAG.err || { tail -20 gpurun_out/rehearsal_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/rehearsal_$TAG.jsonl
echo done
