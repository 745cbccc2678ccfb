#!/bin/bash
# r03x: quotient thread order (point vs LDE row order) at 2^19, 2^22 and on
# rank 0 of a 2^26 proof over 8 ranks (loopback rehearsal)
set -o pipefail
mkdir -p gpurun_out
for o in point row point row; do
  LSP_QUOTIENT_ORDER=$o timeout -k 10 200 python tools/time_prove.py 19 22 > gpurun_out/qorder_$o.txt 2>&1 || { tail -5 gpurun_out/qorder_$o.txt; exit 1; }
  echo "== $o" >> gpurun_out/qorder_r03x.txt
  grep -E "log_n=|compute quotient" gpurun_out/qorder_$o.txt >> gpurun_out/qorder_r03x.txt
done
for o in point row; do
  echo "== rehearsal 2^26/8 rank 0 $o" >> gpurun_out/qorder_r03x.txt
  LSP_QUOTIENT_ORDER=$o timeout -k 10 400 python tools/rank_rehearsal.py --log-n 26 --size 8 --ranks 0 --steps 1 >> gpurun_out/qorder_r03x.txt 2>&1 || { tail -5 gpurun_out/qorder_r03x.txt; exit 1; }
done
cat gpurun_out/qorder_r03x.txt | cut -c1-300
