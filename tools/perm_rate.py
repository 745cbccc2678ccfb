"""Poseidon2 permutation rate (lsp_calibrate_poseidon2, best of 5 runs) and
a 2^19 prove time -- quick A/B for multiplier variants."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace
ctx = Context(StarkConfig())
print("perm rate M/s:", round(max(ctx.calibrate_poseidon2() for _ in range(5)), 1))
a, d, _ = ctx.config.seeded()
tr = gen_permutation_trace(19, 3, a, d)
pub = np.concatenate([a, d])
dp = ctx.dev_alloc(tr.nbytes); ctx.h2d(dp, tr)
ctx.prove(dp, permutation_air(3), pub, tr.shape[0], tr.shape[1])
ts = []
for _ in range(5):
    ctx.synchronize(); t = time.perf_counter()
    ctx.prove(dp, permutation_air(3), pub, tr.shape[0], tr.shape[1]); ts.append(time.perf_counter() - t)
print("prove 2^19 ms: min %.1f median %.1f" % (min(ts) * 1e3, sorted(ts)[2] * 1e3))
print(dict((k, round(v, 2)) for k, v in ctx.last_timings() if k in ("merkle tree", "commit to quotient poly chunks", "commit phase")))
