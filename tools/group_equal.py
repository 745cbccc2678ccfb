"""One proof over G virtual ranks (ProverGroup: G contexts on this GPU, the
in-process transport) against the one-context proof of the same trace, byte
for byte, at sizes the GPU suite does not run (tests/test_gpu_shard.py stops at
2^22).  Usage: python tools/group_equal.py LOG_N [G] ; both inverse-NTT
exchanges (LSP_SHARD_SPLIT_INTT = 1, 0) are checked."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from linea_stark_prover_amd.air import permutation_air  # noqa: E402
from linea_stark_prover_amd.build import library_hash, source_hash  # noqa: E402
from linea_stark_prover_amd.prover import Context, ProverGroup, StarkConfig, gen_permutation_trace  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
print(f"lib_src_sha16={library_hash() or source_hash()}", flush=True)
cfg = StarkConfig()
ok = True
with Context(cfg) as ctx:
    a, d, _ = cfg.seeded()
    tr = gen_permutation_trace(log_n, 3, a, d)
    pub = np.concatenate([a, d])
    t = time.time()
    single = ctx.prove(tr, permutation_air(3), pub)
    print(f"2^{log_n}: one context {time.time() - t:.2f} s, {len(single)} bytes", flush=True)
for split in ("1", "0"):
    os.environ["LSP_SHARD_SPLIT_INTT"] = split
    ctxs = [Context(cfg) for _ in range(G)]
    grp = ProverGroup(ctxs)
    try:
        t = time.time()
        proof = grp.prove(tr, permutation_air(3), pub)
        same = proof == single
        ok &= same
        print(f"2^{log_n} over {G} virtual ranks, split inverse={split}: {time.time() - t:.2f} s, "
              f"byte-identical to one context: {same}", flush=True)
    finally:
        grp.close()
        for c in ctxs:
            c.close()
sys.exit(0 if ok else 1)
