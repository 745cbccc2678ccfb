#!/bin/bash
# Same-box A/B of two builds (abl/old.so, abl/new.so: tools/variant_lib.py) on the quotient phase:
# the wide C3 AIR at 2^20 (bench.py --air wide) and the 3x3 AIR at 2^19, alternating, twice.
set -o pipefail
for i in 1 2; do for v in old new; do
LSP_LIB=abl/$v.so timeout -k 10 300 python bench.py --air wide --log-n 20 --steps 2 --warmup 1 --no-cpu-baseline --batch-leg none --shard-leg none --inflight 0 --no-host-trace-leg > gpurun_out/bq_$v.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bq_$v.json'));print('$v', round(d['ms_per_step'],1), d['phases_ms']['compute quotient polynomial'])"
LSP_LIB=abl/$v.so timeout -k 10 300 python tools/time_prove.py 19 2>&1 | grep -E "log_n|quotient polynomial" | tr '\n' ' '; echo
done; done
