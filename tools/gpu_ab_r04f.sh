#!/bin/bash
# r04f: parity of the host-side changes (parallel query assembly/serialization,
# per-thread host subtrees) and their same-box A/B against the previous build
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh r04f tests:test_gpu_parity.py,test_gpu_fullsize.py,test_gpu_shard.py || exit 1
timeout -k 10 300 python tools/ab_inproc.py _ab/base.so _ab/new.so --pairs 40 > gpurun_out/ab_r04f.txt 2>&1 || { tail -20 gpurun_out/ab_r04f.txt; exit 1; }
cat gpurun_out/ab_r04f.txt
timeout -k 10 300 python tools/ab_inproc.py _ab/new.so _ab/new.so --pairs 60 --swap --env-b LSP_HOST_TREE_TOP=2048 > gpurun_out/ab_top2048_r04f.txt 2>&1 || { tail -20 gpurun_out/ab_top2048_r04f.txt; exit 1; }
cat gpurun_out/ab_top2048_r04f.txt
