"""Same-process A/B of the drop-in upload: one 2^19 proof
with the trace resident in HBM against the same proof from pageable host
memory -- the caller's buffer registered in place with the DMA queued
asynchronously (LSP_H2D_PIN=1, the default), the same on a freshly allocated
copy of the trace every step (what a caller handing over a new Vec pays:
first-time page locking), and one synchronous pageable hipMemcpyAsync
(LSP_H2D_PIN=0) -- interleaved round-robin so box drift hits every mode alike.
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


def host(pin, t=None):
    os.environ["LSP_H2D_PIN"] = "1" if pin else "0"
    return ctx.prove(tr if t is None else t, air, pub)


fresh = [None]


def host_fresh():
    return host(True, fresh[0])


modes = {"resident": resident, "host_pinned": lambda: host(True), "host_pinned_fresh": host_fresh,
         "host_pageable": lambda: host(False)}
ref = resident()
fresh[0] = tr.copy()
for f in modes.values():  # warm every path
    assert f() == ref
ts = {k: [] for k in modes}
for r in range(rounds):
    for k, f in modes.items():
        if k == "host_pinned_fresh":
            fresh[0] = None
            fresh[0] = tr.copy()  # new pages, written (outside the timed region)
        ctx.synchronize()
        t = time.perf_counter()
        f()
        ts[k].append(time.perf_counter() - t)
med = {k: statistics.median(v) * 1e3 for k, v in ts.items()}
print(f"log_n={log_n} trace {tr.nbytes / 2**20:.0f} MiB, {rounds} interleaved rounds, median ms: "
      + ", ".join(f"{k} {v:.2f}" for k, v in med.items()))
for k in ("host_pinned", "host_pinned_fresh", "host_pageable"):
    add = med[k] - med["resident"]
    print(f"{k} - resident = {add:.2f} ms ({tr.nbytes / max(add, 1e-3) / 1e6:.1f} GB/s of the proof's added time)")
ctx.dev_free(dp)
