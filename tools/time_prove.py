"""Quick prove timing on the GPU (diagnostic, not the bench contract).
Usage: time_prove.py [LOG_N | wLOG_N ...]   (wLOG_N: the wide C3 AIR, W = 184)"""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace, gen_wide_trace

args = sys.argv[1:] or ["16", "19"]
ctx = Context(StarkConfig())
a, d, _ = ctx.config.seeded()
pub = np.concatenate([a, d])
for arg in args:
    wide = arg.startswith("w")
    lg = int(arg[1:] if wide else arg)
    t0 = time.time()
    if wide:
        tr, air = gen_wide_trace(lg, a, d)
    else:
        tr, air = gen_permutation_trace(lg, 3, a, d), permutation_air(3)
    t1 = time.time()
    h, w = tr.shape[0], tr.shape[1]
    dp = ctx.dev_alloc(tr.nbytes); ctx.h2d(dp, tr)
    del tr
    pf = ctx.prove(dp, air, pub, h, w)  # warm
    ts = []
    for _ in range(int(os.environ.get("LSP_TP_REPS", "3"))):
        ctx.synchronize(); t = time.time(); pf = ctx.prove(dp, air, pub, h, w); ts.append(time.time() - t)
    ok = ctx.verify(pf, air, pub)
    med = sorted(ts)[len(ts) // 2]
    print(f"log_n={lg}{' wide' if wide else ''} w={w} gen={t1-t0:.2f}s prove={min(ts)*1e3:.1f}ms "
          f"median={med*1e3:.2f}ms rows/s={h/min(ts):.0f} verify={ok}", flush=True)
    for name, ms in ctx.last_timings():
        print(f"   {name:55s} {ms:9.3f} ms")
    ctx.dev_free(dp)
