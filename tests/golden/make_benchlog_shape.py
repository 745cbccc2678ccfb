"""Extract the data-shaped spans of the reference's bench.log (its only record
of one proof's structure: the 6+6 permutation AIR, w = 14, at 2^19 rows) into
tests/golden/benchlog_shape.json.

    python tests/golden/make_benchlog_shape.py /root/reference/bench.log

Output: the span names with their `dims:` / `added_bits:` annotations, in log
order (timings dropped) -- data the reference already holds, read as text.
"""
import json
import os
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/bench.log"
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "benchlog_shape.json")
spans = []
for ln, line in enumerate(open(src, encoding="utf-8"), 1):
    m = re.search(r"[┝┕]━ (.+?) \[ [^\]]* \](.*)$", line)
    if not m or "dims:" not in m.group(2):
        continue
    spans.append({"line": ln, "span": f"{m.group(1)} {m.group(2).strip()}"})
json.dump({"source": "bench.log (reference repo root)", "log_n": 19, "width": 14, "spans": spans},
          open(out, "w"), indent=1)
print(f"{len(spans)} spans -> {out}")
