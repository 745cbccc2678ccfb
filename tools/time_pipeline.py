"""Throughput of P independent 2^log_n proofs in flight on ONE GPU (P
contexts = P HIP streams, one host thread each) vs one at a time.
    python tools/time_pipeline.py [log_n] [proofs per context] [P,P,...]"""
import os, sys, threading, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 19
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
cfg = StarkConfig()
a, d, _ = cfg.seeded()
pub = np.concatenate([a, d])
air = permutation_air(3)
tr = gen_permutation_trace(log_n, 3, a, d)
for P in ([int(x) for x in sys.argv[3].split(',')] if len(sys.argv) > 3 else (1, 2, 3)):
    ctxs = [Context(cfg) for _ in range(P)]
    ptrs = []
    for c in ctxs:
        p = c.dev_alloc(tr.nbytes); c.h2d(p, tr); ptrs.append(p)
        c.prove(p, air, pub, tr.shape[0], tr.shape[1])  # warm
    def worker(i):
        for _ in range(K):
            ctxs[i].prove(ptrs[i], air, pub, tr.shape[0], tr.shape[1])
    t = time.perf_counter()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(P)]
    [x.start() for x in th]; [x.join() for x in th]
    dt = time.perf_counter() - t
    print(f"P={P}: {P * K} proofs in {dt * 1e3:.0f} ms -> {dt / (P * K) * 1e3:.1f} ms per proof, "
          f"{P * K * (1 << log_n) / dt / 1e6:.2f} M rows/s")
