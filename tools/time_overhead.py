"""Host overhead around lsp_prove (diagnostic): wall time of Context.prove
against the library's own 'prove' span, per step, at 2^log_n (device trace).
Run with LSP_TIME_TOPS=1 for the library's query-phase breakdown.
Usage: python tools/time_overhead.py [log_n] [steps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 19
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ctx = Context(StarkConfig())
a, d, _ = ctx.config.seeded()
pub = np.concatenate([a, d])
air = permutation_air(3)
h, w = 1 << lg, 8
dp = ctx.gen_permutation_trace_device(lg, 3, a, d, seed=1)
for _ in range(2):
    ctx.prove(dp, air, pub, h, w)
ctx.synchronize()
for _ in range(steps):
    t = time.perf_counter()
    pf = ctx.prove(dp, air, pub, h, w)
    wall = (time.perf_counter() - t) * 1e3
    span = dict(ctx.last_timings())["prove"]
    print(f"wall {wall:7.3f} ms  prove span {span:7.3f} ms  outside {wall - span:6.3f} ms  proof {len(pf)} B", flush=True)
