#!/bin/bash
# r03z: opened values computed on the non-holder ranks' cosets -- sharded
# parity (virtual ranks and gloo processes), then ranks 0, 5, 6, 7 of the
# 2^26 proof over 8 ranks (loopback rehearsal)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_mp.py tests/test_gpu_parity.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/shard_tests_r03z.log 2>&1 || { tail -30 gpurun_out/shard_tests_r03z.log; exit 1; }
tail -3 gpurun_out/shard_tests_r03z.log
for r in 0 5 7; do
  timeout -k 10 400 python tools/rank_rehearsal.py --log-n 26 --size 8 --ranks $r --steps 2 >> gpurun_out/rehearsal_r03z.jsonl 2>> gpurun_out/rehearsal_r03z.err || { tail -5 gpurun_out/rehearsal_r03z.err; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/rehearsal_r03z.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        ph = d["phases_ms"]
        print(d["rank"], round(d["prove_s_median"], 4), ph.get("compute quotient polynomial"),
              ph.get("compute opened values with Lagrange interpolation"), ph.get("open"), d["device_used_gib"])
PY
