set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_witness.py tests/test_gpu_shard.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/g2_tests.log 2>&1 || { tail -30 gpurun_out/g2_tests.log; exit 1; }
tail -2 gpurun_out/g2_tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline --inflight 0 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err || { tail -20 gpurun_out/bench_g2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_g2.json')); print(d['ms_per_step'], d['phases_ms'])"
