"""Time lsp_coset_lde_batch (device memory, added_bits 3) at several shapes:
ms per call (wall, after a warm-up, synchronised) and the metric's GB/s
(algorithmic bytes 32 w (h + 8h) / time).
Usage: python tools/time_lde.py [log_n,w ...] (default 19,8 19,4 22,8)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd import _lib as L
from linea_stark_prover_amd.prover import Context, StarkConfig
from linea_stark_prover_amd.field import to_mont

shapes = [tuple(int(x) for x in s.split(",")) for s in sys.argv[1:]] or [(19, 8), (19, 4), (22, 8)]
ctx = Context(StarkConfig())
shift = to_mont([22])
for log_n, w in shapes:
    h = 1 << log_n
    rng = np.random.default_rng(1)
    x = rng.integers(0, 2**62, size=(h, w, 4), dtype=np.uint64)
    x[..., 3] &= (1 << 58) - 1  # < r
    din = ctx.dev_alloc(x.nbytes); ctx.h2d(din, x)
    dout = ctx.dev_alloc(x.nbytes * 8)
    for _ in range(2):
        L.check(L.lib().lsp_coset_lde_batch(ctx.h, din, h, w, 3, shift.ctypes.data, dout, L.LSP_MEM_DEVICE), ctx.h)
    ctx.synchronize()
    reps = max(3, int(2e8 // (h * w)))
    t = time.perf_counter()
    for _ in range(reps):
        L.check(L.lib().lsp_coset_lde_batch(ctx.h, din, h, w, 3, shift.ctypes.data, dout, L.LSP_MEM_DEVICE), ctx.h)
    ctx.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    gbs = 32 * w * 9 * h / (ms * 1e-3) / 1e9
    print(f"lde 2^{log_n} x {w}: {ms:.3f} ms/call  {gbs:.1f} GB/s  ({reps} reps)", flush=True)
    ctx.dev_free(din); ctx.dev_free(dout)
