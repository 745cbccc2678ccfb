#!/bin/bash
# The one GPU-box driver script (replaces round 3's single-use gpu_r03*.sh):
#
#   bash tools/gpu.sh TAG STEP [STEP ...]
#
# Steps run in order; each GPU step has its own time limit and the script
# stops at the first failure (nothing more touches the GPU after a fault,
# abort or timeout).  Logs and results go to gpurun_out/<step>_<TAG>.*.
#
#   tests            every GPU test (pytest -m gpu)
#   tests:<files>    the listed test files only, comma-separated (tests/ implied)
#   tests-dbg:<files> the same on the bounds-checked debug library (LSP_LIB=liblsp_hip_dbg.so)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (what the driver runs)
#   benchq           a quick bench: main leg only, no CPU baseline / extra legs
#   prof             rocprofv3 kernel trace (+ --stats) of a quick bench
#   pmc              the PMC passes bench.py's roofline reads (tools/pmc_stamp.sh)
#   rehearse         ranks 0, 5, 7 of the 2^26 proof over 8 ranks (tools/rank_rehearsal.py)
#   rehearse-red     the same with the redundant inverse forced (LSP_SHARD_SPLIT_INTT=0): the
#                    other exchange a calibrated 8-GPU run may choose
#   ub:<name>        the microbenchmark tools/ubench/<name> (built beforehand) under a 120 s limit
#   py:<script>      python <script> under a 300 s limit (tools/ implied), output to a log
#   bench8x1         the driver's N = 8 launcher path with 8 ranks sharing this one GPU
#                    (torch.distributed.run --nproc-per-node 8 bench.py --gpus 8; sharded legs at
#                    2^20 / 2^22 over gloo, since 8 ranks of 2^26 do not fit one card)
#   h2d              tools/ubench/h2d: host -> device upload modes for a 128 MiB trace (build it first)
#   tests900:<files> the listed test files with a 900 s per-test limit (the full-size oracle comparisons)
#   pmclds:<lib>     one rocprofv3 --pmc pass of the LDS counters (SQ_INSTS_LDS SQ_WAIT_INST_LDS
#                    SQ_LDS_BANK_CONFLICT) over a 2^19 prove on the library _ab/<lib>.so
#   ktrace:<lib>     rocprofv3 kernel trace (+ --stats) of 2^19 proves on _ab/<lib>.so, summarised
#                    per kernel (tools/prof_summary.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:?usage: tools/gpu.sh TAG STEP...}
shift
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=30"

fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }

for step in "$@"; do
  echo "=== $step ($(date +%T))"
  case "$step" in
    tests)
      log=gpurun_out/tests_$TAG.log
      timeout -k 10 1000 $PYT -m gpu tests > $log 2>&1 || fail "$step" $log
      tail -2 $log ;;
    tests:*)
      log=gpurun_out/tests_$TAG.log
      files=$(echo "${step#tests:}" | tr ',' '\n' | sed 's#^#tests/#' | tr '\n' ' ')
      timeout -k 10 1000 $PYT -v $files >> $log 2>&1 || fail "$step" $log
      grep -E "passed|failed" $log | tail -1 ;;
    tests-dbg:*)
      # the listed GPU test files on the bounds-checked debug library (build.py --debug-bounds)
      log=gpurun_out/tests_dbg_$TAG.log
      files=$(echo "${step#tests-dbg:}" | tr ',' '\n' | sed 's#^#tests/#' | tr '\n' ' ')
      LSP_LIB=$PWD/linea_stark_prover_amd/_lib/liblsp_hip_dbg.so timeout -k 10 1000 $PYT $files >> $log 2>&1 \
        || fail "$step" $log
      grep -E "passed|failed" $log | tail -1 ;;
    smoke)
      log=gpurun_out/smoke_$TAG.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || fail "$step" $log
      cat $log ;;
    bench)
      timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
        || fail "$step" gpurun_out/bench_$TAG.err
      cut -c1-600 gpurun_out/bench_$TAG.json ;;
    benchq)
      timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --inflight 0 --shard-leg none \
        --batch-leg none --shape-leg none --wide-leg 0 --no-host-trace-leg > gpurun_out/benchq_$TAG.json \
        2> gpurun_out/benchq_$TAG.err || fail "$step" gpurun_out/benchq_$TAG.err
      python -c "import json; d=json.load(open('gpurun_out/benchq_$TAG.json')); print(d['ms_per_step'], d['prove_time_median_s'], d['roofline']['ms'], d['roofline_valu']['ms'])" ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --inflight 0 --shard-leg none --batch-leg none \
        --shape-leg none --wide-leg 0 --no-host-trace-leg > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err \
        || fail "$step" gpurun_out/prof_$TAG.err
      echo "kernel trace in gpurun_out/prof_$TAG" ;;
    pmc)
      bash tools/pmc_stamp.sh pmc_$TAG || exit 1 ;;
    rehearse|rehearse-red)
      log=gpurun_out/${step}_$TAG.jsonl
      [ "$step" = rehearse-red ] && export LSP_SHARD_SPLIT_INTT=0
      for r in 0 5 7; do
        timeout -k 10 400 python tools/rank_rehearsal.py --log-n 26 --size 8 --ranks $r --steps 2 >> $log \
          2>> gpurun_out/${step}_$TAG.err || fail "$step" gpurun_out/${step}_$TAG.err
      done
      unset LSP_SHARD_SPLIT_INTT
      python -c "
import json
for l in open('$log'):
    if l.startswith('{'):
        d = json.loads(l); print(d['rank'], round(d['prove_s_median'], 4), d['device_used_gib'], d['proof_wire_bytes'])" ;;
    bench8x1)
      timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29561 bench.py --gpus 8 --shard-leg 20,22 --batch-leg 20 --no-cpu-baseline \
        > gpurun_out/bench8x1_$TAG.json 2> gpurun_out/bench8x1_$TAG.err || fail "$step" gpurun_out/bench8x1_$TAG.err
      grep '^{' gpurun_out/bench8x1_$TAG.json | cut -c1-400 ;;
    h2d)
      timeout -k 10 120 tools/ubench/h2d 128 9 > gpurun_out/h2d_$TAG.json 2>&1 || fail "$step" gpurun_out/h2d_$TAG.json
      cat gpurun_out/h2d_$TAG.json ;;
    tests900:*)
      log=gpurun_out/tests900_$TAG.log
      files=$(echo "${step#tests900:}" | tr ',' '\n' | sed 's#^#tests/#' | tr '\n' ' ')
      timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread $files >> $log 2>&1 \
        || fail "$step" $log
      grep -E "passed|failed" $log | tail -1 ;;
    pmclds:*)
      lib=${step#pmclds:}
      d=gpurun_out/pmclds_${lib}_$TAG
      LSP_LIB=$PWD/_ab/$lib.so LSP_LIB_OLDER=1 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
        --output-format csv -d $d -o run -- python3 tools/time_prove.py 19 > $d.log 2>&1 || fail "$step" $d.log
      python tools/pmc_lds_summary.py $d/run_counter_collection.csv | tee $d.txt ;;
    ktrace:*)
      lib=${step#ktrace:}
      d=gpurun_out/ktrace_${lib}_$TAG
      LSP_LIB=$PWD/_ab/$lib.so LSP_LIB_OLDER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $d -o run -- python3 tools/time_prove.py 19 > $d.log 2>&1 || fail "$step" $d.log
      python tools/prof_summary.py $d/run_kernel_stats.csv 4 > $d.txt 2>&1; head -25 $d.txt ;;
    ub:*)
      name=${step#ub:}
      timeout -k 10 120 tools/ubench/$name > gpurun_out/ub_${name}_$TAG.txt 2>&1 || fail "$step" gpurun_out/ub_${name}_$TAG.txt
      cat gpurun_out/ub_${name}_$TAG.txt ;;
    py:*)
      script=${step#py:}
      log=gpurun_out/$(basename ${script%% *} .py)_$TAG.log
      timeout -k 10 300 python tools/$script > $log 2>&1 || fail "$step" $log
      tail -20 $log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== done ($(date +%T))"
