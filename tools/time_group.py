"""Sharded prove over G virtual ranks on ONE GPU (lsp_prove_group, threads):
not a multi-GPU measurement -- the ranks share the device -- but it shows the
exchange path's overhead against the single-rank prove of the same trace."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, ProverGroup, StarkConfig, gen_permutation_trace
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = StarkConfig()
a, d, _ = cfg.seeded()
tr = gen_permutation_trace(log_n, 3, a, d)
pub = np.concatenate([a, d])
air = permutation_air(3)
ctx = Context(cfg)
ref = ctx.prove(tr, air, pub)
ts = []
for _ in range(3):
    t = time.perf_counter(); ctx.prove(tr, air, pub); ts.append(time.perf_counter() - t)
print(f"2^{log_n} single rank (host trace incl. upload): {min(ts) * 1e3:.1f} ms")
for G in (2, 4, 8):
    grp = ProverGroup([Context(cfg) for _ in range(G)])
    assert grp.prove(tr, air, pub) == ref
    ts = []
    for _ in range(3):
        t = time.perf_counter(); grp.prove(tr, air, pub); ts.append(time.perf_counter() - t)
    print(f"2^{log_n} G={G} virtual ranks on one GPU: {min(ts) * 1e3:.1f} ms (proof identical)")
