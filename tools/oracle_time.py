"""Wall time of the C oracle's whole proof (test infrastructure: the checker and
bench.py's cpu_baseline) on this host: python tools/oracle_time.py [LOG_N ...]
(3x3 permutation AIR, 16 threads; LO_TIME=1 adds the oracle's per-phase times)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cref  # noqa: E402

cref.build()
p = cref.setup()
for log_n in [int(a) for a in sys.argv[1:]] or [19]:
    tb, w = cref.gen_perm_trace(p, log_n, 3)
    t = time.perf_counter()
    cref.prove(p, tb, 1 << log_n, w, cref.perm_air(3), nthreads=16)
    print(f"log_n={log_n}: {time.perf_counter() - t:.2f} s", flush=True)
