"""C4 at scale on ONE GPU: the 2^log_n proof by a single rank, then by G virtual
ranks (lsp_prove_group, one context per rank, all on device 0), checked
byte-identical.  Virtual ranks share the device, so the group's wall time is
the sum of the ranks' work (plus exchanges), not an 8-GPU time; per-rank work
~ total / G is what one rank of a real G-GPU run would do.
usage: python tools/shard_scale.py [log_n] [G]"""
import gc, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, ProverGroup, StarkConfig, gen_permutation_trace

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 23
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = StarkConfig()
a, d, _ = cfg.seeded()
t = time.perf_counter()
tr = gen_permutation_trace(log_n, 3, a, d)
print(f"trace 2^{log_n} x {tr.shape[1]} generated in {time.perf_counter() - t:.1f} s", flush=True)
pub = np.concatenate([a, d])
air = permutation_air(3)
ctx = Context(cfg)
ref = ctx.prove(tr, air, pub)  # warm-up (pools, tables)
t = time.perf_counter()
ref = ctx.prove(tr, air, pub)
t1 = time.perf_counter() - t
assert ctx.verify(ref, air, pub)
print(f"single rank: {t1:.3f} s ({(1 << log_n) / t1 / 1e6:.2f} M rows/s), proof {len(ref)} bytes, verified", flush=True)
ctx.close()
del ctx
gc.collect()
grp = ProverGroup([Context(cfg) for _ in range(G)])
pf = grp.prove(tr, air, pub)  # warm-up
t = time.perf_counter()
pf = grp.prove(tr, air, pub)
tg = time.perf_counter() - t
print(f"G={G} virtual ranks on one GPU: {tg:.3f} s of shared-device time, proof identical: {pf == ref}", flush=True)
assert pf == ref
