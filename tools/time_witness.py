"""Time the GPU witness generation (F1) for the wide-AIR shape (SURVEY 8(d)
C3: 4 LogUp lookups of 3 columns over 2 tables + 8 permutation groups of
6+6) against the host C++ generator (lsp_gen_wide_trace, which also draws
the random raw columns)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_wide_trace
from linea_stark_prover_amd.trace import RawLookupTrace, RawPermutationTrace, RawTrace

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << log_n
ctx = Context(StarkConfig())
a, d, _ = ctx.config.seeded()
g = np.random.default_rng(7)
TOP = 0x12AB655E9A2CA556


def rand_col(m):
    c = g.integers(0, 2**63, size=(m, 4), dtype=np.uint64) * 2 + g.integers(0, 2, size=(m, 4), dtype=np.uint64)
    c[:, 3] %= np.uint64(TOP)
    return c


lookups = []
for _ in range(4):
    tabs = [[rand_col(n) for _ in range(3)] for _ in range(2)]
    t = g.integers(0, 2, n)
    j = g.integers(0, n, n)
    acols = [np.where(t[:, None] == 0, tabs[0][c][j], tabs[1][c][j]) for c in range(3)]
    lookups.append(RawLookupTrace(acols, tabs))
perms = []
for _ in range(8):
    acols = [rand_col(n) for _ in range(6)]
    p = g.permutation(n)
    perms.append(RawPermutationTrace(acols, [c[p] for c in acols]))
rt = RawTrace(ctx, [a, d])
rt.push_traces(perms[:1], lookups[:1])  # warm
ts = []
for _ in range(3):
    ctx.synchronize()
    t0 = time.perf_counter()
    cfgs = rt.push_traces(perms, lookups)
    ctx.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"GPU witness (incl. raw-column uploads), 2^{log_n} rows, width {rt.width}: {min(ts) * 1e3:.1f} ms")
if "--gpu-only" in sys.argv:
    sys.exit(0)
t0 = time.perf_counter()
tr, air = gen_wide_trace(log_n, a, d)
print(f"host C++ lsp_gen_wide_trace (random columns + witness), width {tr.shape[1]}: {(time.perf_counter() - t0) * 1e3:.1f} ms")
