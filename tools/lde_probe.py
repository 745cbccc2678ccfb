"""Run the bench's trace coset LDE (h = 2^log_n, w = 8, added_bits 3, device
memory) `reps` times -- the command the rocprofv3 --pmc passes profile."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from linea_stark_prover_amd import _lib as L
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace
from linea_stark_prover_amd.field import to_mont

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 19
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = Context(StarkConfig())
a, d, _ = ctx.config.seeded()
tr = gen_permutation_trace(log_n, 3, a, d)
h, w = tr.shape[0], tr.shape[1]
din = ctx.dev_alloc(tr.nbytes); ctx.h2d(din, tr)
dout = ctx.dev_alloc(tr.nbytes * 8)
shift = to_mont([22])
for _ in range(reps):
    L.check(L.lib().lsp_coset_lde_batch(ctx.h, din, h, w, 3, shift.ctypes.data, dout, L.LSP_MEM_DEVICE), ctx.h)
ctx.synchronize()
print("lde probe done", h, w, reps)
