set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "inverse_denominators or open_reduce or batch_inverse" > gpurun_out/g1_tests.log 2>&1 || { tail -30 gpurun_out/g1_tests.log; exit 1; }
tail -2 gpurun_out/g1_tests.log
timeout -k 10 600 python bench.py --ncols 6 --no-cpu-baseline --inflight 0 > gpurun_out/bench_6x6.json 2> gpurun_out/bench_6x6.err || { tail -20 gpurun_out/bench_6x6.err; exit 1; }
cut -c1-1500 gpurun_out/bench_6x6.json
