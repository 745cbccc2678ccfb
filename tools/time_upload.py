"""Same-process A/B of the drop-in upload: one 2^19 proof
with the trace resident in HBM against the same proof from pageable host
memory, the upload through the pinned ring (LSP_H2D_STAGED=1, the default)
and through one pageable hipMemcpyAsync (LSP_H2D_STAGED=0), interleaved
round-robin so box drift hits every mode alike.
Usage: time_upload.py [LOG_N] [ROUNDS]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from linea_stark_prover_amd.air import permutation_air  # noqa: E402
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 19
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = Context(StarkConfig())
ctx.set_phase_timing(False)
a, d, _ = ctx.config.seeded()
pub = np.concatenate([a, d])
air = permutation_air(3)
tr = gen_permutation_trace(log_n, 3, a, d)
h, w = tr.shape[0], tr.shape[1]
dp = ctx.dev_alloc(tr.nbytes)
ctx.h2d(dp, tr)


def resident():
    return ctx.prove(dp, air, pub, h, w)


def host(staged):
    os.environ["LSP_H2D_STAGED"] = "1" if staged else "0"
    return ctx.prove(tr, air, pub)


modes = {"resident": resident, "host_ring": lambda: host(True), "host_pageable": lambda: host(False)}
ref = resident()
for f in modes.values():  # warm every path (pinned ring allocation, pool threads)
    assert f() == ref
ts = {k: [] for k in modes}
for r in range(rounds):
    for k, f in modes.items():
        ctx.synchronize()
        t = time.perf_counter()
        f()
        ts[k].append(time.perf_counter() - t)
med = {k: statistics.median(v) * 1e3 for k, v in ts.items()}
print(f"log_n={log_n} trace {tr.nbytes / 2**20:.0f} MiB, {rounds} interleaved rounds, median ms: "
      + ", ".join(f"{k} {v:.2f}" for k, v in med.items()))
print(f"host_ring - resident = {med['host_ring'] - med['resident']:.2f} ms; "
      f"host_pageable - resident = {med['host_pageable'] - med['resident']:.2f} ms; "
      f"upload rate through the ring {tr.nbytes / max(med['host_ring'] - med['resident'], 1e-3) / 1e6:.1f} GB/s "
      f"(of the proof's added time)")
ctx.dev_free(dp)
