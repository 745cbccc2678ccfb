#!/bin/bash
# r03z2: strong-scaling rehearsal of the 2^24 proof (bench's sharded leg) -- rank 0
# and the last rank of G = 2, 4, 8 (loopback, one rank per process), plus G = 1
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/rehearsal_2e24_r03z2.jsonl
for G in 1 2 4 8; do
  R="0"; [ $G -gt 1 ] && R="0,$((G-1))"
  timeout -k 10 300 python tools/rank_rehearsal.py --log-n 24 --size $G --ranks $R --steps 3 >> $OUT 2>> gpurun_out/rehearsal_2e24_r03z2.err || { tail -5 gpurun_out/rehearsal_2e24_r03z2.err; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/rehearsal_2e24_r03z2.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["size"], d["rank"], round(d["prove_s_median"], 4), d["device_used_gib"])
PY
