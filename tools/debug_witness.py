"""Diagnostic: GPU lookup witness vs the oracle, column by column (reads the
device trace back even when the library's closing check fails)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import pyoracle as O
from linea_stark_prover_amd.field import to_mont, from_mont
from linea_stark_prover_amd.prover import Context, StarkConfig
from linea_stark_prover_amd.trace import RawTrace, RawLookupTrace
sys.path.insert(0, "tests")
from test_gpu_witness import _lookup_case, _mont_cols
s = O.setup_from_seed(); al, de = s.alpha, s.delta
n, nt, nbc = 8, 1, 1
a, b, af, bf = _lookup_case(n, nt, nbc, 22, 3)
cfg, cols = O.lookup_witness(a, b, af, bf, al, de)
ctx = Context(StarkConfig())
rt = RawTrace(ctx, [to_mont([al]), to_mont([de])])
try:
    rt.push_traces([], [RawLookupTrace(_mont_cols(a), [_mont_cols(t) for t in b], to_mont(af), [to_mont(f) for f in bf])])
except Exception as e:
    print("raised:", e)
got = np.zeros((rt.height, rt.width, 4), np.uint64)
ctx.d2h(got, rt.ptr)
names = ["a"] * 1 + ["b"] * nbc * nt + ["afil"] + ["bfil"] * nt + ["ainv"] + ["binv"] * nt + ["occ"] * nt + ["psum"]
for c in range(rt.width):
    g = from_mont(got[:, c, :]); e = cols[c]
    print(c, names[c], "OK" if g == e else "DIFF", g if g != e else "")
    if g != e: print("   exp", e)
