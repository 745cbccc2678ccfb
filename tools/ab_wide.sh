#!/bin/bash
# same-box A/B of two library builds on the wide C3 AIR (2^20 rows): prove time and the quotient phase
# usage: tools/ab_wide.sh libA.so libB.so [rounds]
set -o pipefail
A=$1; B=$2; N=${3:-2}
for i in $(seq $N); do
  for lib in $A $B; do
    LSP_LIB=$lib timeout -k 10 300 python bench.py --air wide --log-n 20 --steps 2 --warmup 1 --no-cpu-baseline \
      --inflight 0 --no-host-trace-leg --shard-leg none --batch-leg none > gpurun_out/ab_wide_tmp.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_wide_tmp.json')); p=d['phases_ms']; print(sys.argv[1], 'prove %.1f ms' % (d['prove_time_s']*1e3), 'quotient %.2f ms' % p['compute quotient polynomial'], 'verified', d['verified'])" $(basename $lib)
  done
done
