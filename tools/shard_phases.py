"""Where a sharded proof's extra device time goes: per-phase times (HIP
events, lsp_last_timings) of the single-rank prove and of every rank of a
G-rank virtual group on one GPU (lsp_prove_group), same trace, same proof.
Usage: python tools/shard_phases.py [log_n] [G]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, ProverGroup, StarkConfig
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = StarkConfig()
a, d, _ = cfg.seeded()
pub = np.concatenate([a, d])
air = permutation_air(3)
ctx = Context(cfg)
din = ctx.gen_permutation_trace_device(log_n, 3, a, d)  # same seed on every rank: same trace
h, w = 1 << log_n, 8
ref = ctx.prove(din, air, pub, h, w)
t = time.perf_counter(); ctx.prove(din, air, pub, h, w); t1 = time.perf_counter() - t
single = dict(ctx.last_timings())
ctx.dev_free(din)
ctx.close()  # the group's 8 contexts need the memory (2^24: ~90 GB single-rank pool)
ctxs = [Context(cfg) for _ in range(G)]
ptrs = []
for c in ctxs:
    ptrs.append(c.gen_permutation_trace_device(log_n, 3, a, d))
grp = ProverGroup(ctxs)
assert grp.prove(ptrs, air, pub, h, w) == ref
t = time.perf_counter(); grp.prove(ptrs, air, pub, h, w); tg = time.perf_counter() - t
ranks = [dict(c.last_timings()) for c in ctxs]
print(f"2^{log_n}: single rank {t1 * 1e3:.1f} ms wall; G={G} virtual ranks {tg * 1e3:.1f} ms wall ({tg / t1:.2f}x)")
print(f"{'phase':52s} {'single':>8s} " + " ".join(f"{'r' + str(r):>7s}" for r in range(G)) + f" {'sum':>8s}")
for k in single:
    vals = [rk.get(k, 0.0) for rk in ranks]
    print(f"{k:52s} {single[k]:8.2f} " + " ".join(f"{v:7.2f}" for v in vals) + f" {sum(vals):8.2f}")
