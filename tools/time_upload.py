"""Same-process A/B of the drop-in upload, interleaved
round-robin so box drift hits every mode alike: one 2^19 proof with the trace
resident in HBM; the same proof from pageable host memory (lsp_prove, mem =
HOST); the upload alone; the upload then the resident proof of the uploaded
copy; and the GPU left idle for the upload's 2.4 ms, then the resident proof
(what an idle gap alone costs the next proof: the clock's ramp).
(profiles/r05c_time_upload.txt is the earlier form of this tool, which also
timed registering the caller's buffer in place: no faster than pageable.)
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


def host(_pin=False):
    return ctx.prove(tr, air, pub)


dp2 = ctx.dev_alloc(tr.nbytes)


def h2d_only():  # the upload alone (lsp_memcpy_h2d: one pageable hipMemcpyAsync + a stream sync)
    ctx.h2d(dp2, tr)


def h2d_then_resident():  # the same upload, then the resident proof of the uploaded copy
    ctx.h2d(dp2, tr)
    return ctx.prove(dp2, air, pub, h, w)


def idle_then_resident():  # the GPU idle for as long as the upload takes, then the resident proof
    time.sleep(0.0024)
    return ctx.prove(dp, air, pub, h, w)


modes = {"resident": resident, "host": lambda: host(False), "h2d_only": h2d_only,
         "h2d_then_resident": h2d_then_resident, "idle_then_resident": idle_then_resident}
ref = resident()
for k, f in modes.items():  # warm every path
    assert k == "h2d_only" or f() == ref
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
for k in ("host", "h2d_then_resident", "idle_then_resident"):
    add = med[k] - med["resident"]
    print(f"{k} - resident = {add:.2f} ms ({tr.nbytes / max(add, 1e-3) / 1e6:.1f} GB/s of the proof's added time)")
print(f"h2d_only: {med['h2d_only']:.2f} ms = {tr.nbytes / med['h2d_only'] / 1e6:.1f} GB/s")
ctx.dev_free(dp)
ctx.dev_free(dp2)
