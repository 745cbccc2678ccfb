# full GPU tests, bench, rocprof kernel trace of the bench (tag = $1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-g3}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['ms_per_step'], d['inflight']['ms_per_proof'], d['phases_ms'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --inflight 0 > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail -20 gpurun_out/prof_$TAG.err; exit 1; }
echo done
