"""Host-side parts of bench.py's timed step at 2^log_n: lsp_prove alone, the
proof serialization (_take_proof) and the Python step around them, per proof.

    python tools/time_step_parts.py [log_n] [proofs]
"""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from linea_stark_prover_amd import _lib as L  # noqa: E402
from linea_stark_prover_amd.air import permutation_air  # noqa: E402
from linea_stark_prover_amd.prover import Context, StarkConfig, _fr_arr  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 19
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = StarkConfig()
ctx = Context(cfg)
ctx.set_phase_timing(True, only=("coset_lde_batch", "merkle tree"))
a, d, _ = cfg.seeded()
import numpy as np  # noqa: E402
pub = np.concatenate([a, d])
air = permutation_air(3)
h, w = 1 << log_n, 8
dtrace = ctx.gen_permutation_trace_device(log_n, 3, a, d)
for _ in range(3):
    ctx.prove(dtrace, air, pub, h, w)
ctx.synchronize()
desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
pubv = _fr_arr(pub).reshape(-1, 4)
tp, ts, tf, tstep = [], [], [], []
for _ in range(n):
    t0 = time.perf_counter()
    proof = ctypes.c_void_p()
    rc = L.lib().lsp_prove(ctx.h, dtrace, h, w, desc, len(desc), pubv.ctypes.data_as(ctypes.c_void_p), pubv.shape[0],
                           L.LSP_MEM_DEVICE, ctypes.byref(proof))
    assert rc == 0
    t1 = time.perf_counter()
    m = ctypes.c_size_t()
    L.lib().lsp_proof_serialize(proof, None, 0, ctypes.byref(m))
    buf = ctypes.create_string_buffer(m.value)
    L.lib().lsp_proof_serialize(proof, buf, m.value, ctypes.byref(m))
    raw = buf.raw[:m.value]
    t2 = time.perf_counter()
    L.lib().lsp_proof_free(proof)
    t3 = time.perf_counter()
    tp.append(t1 - t0)
    ts.append(t2 - t1)
    tf.append(t3 - t2)
for _ in range(n):
    t0 = time.perf_counter()
    ctx.prove(dtrace, air, pub, h, w)
    tstep.append(time.perf_counter() - t0)
ms = lambda v: f"{statistics.median(v) * 1e3:.3f}"  # noqa: E731
print(f"2^{log_n}: lsp_prove {ms(tp)} ms, serialize {ms(ts)} ms ({len(raw)} bytes), free {ms(tf)} ms, "
      f"Context.prove step {ms(tstep)} ms (medians of {n})")
