"""Host time around one lsp_prove call (diagnostic): Python argument prep, the
call itself against its phase span, proof serialization, the copy into
Python bytes and the handle free.  Usage: python tools/time_host_tail.py"""
import os, sys, time, ctypes
sys.path.insert(0, os.getcwd())
import numpy as np
from linea_stark_prover_amd import _lib as L
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig, _fr_arr, _ptr
ctx = Context(StarkConfig())
a, d, _ = ctx.config.seeded()
pub = np.concatenate([a, d])
air = permutation_air(3)
h, w = 1 << 19, 8
dp = ctx.gen_permutation_trace_device(19, 3, a, d, seed=1)
for _ in range(2): ctx.prove(dp, air, pub, h, w)
ctx.synchronize()
for _ in range(5):
    t0 = time.perf_counter()
    desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
    pb = _fr_arr(pub).reshape(-1, 4)
    proof = ctypes.c_void_p()
    t1 = time.perf_counter()
    L.check(L.lib().lsp_prove(ctx.h, dp, h, w, desc, len(desc), _ptr(pb), pb.shape[0], L.LSP_MEM_DEVICE, ctypes.byref(proof)))
    t2 = time.perf_counter()
    n = ctypes.c_size_t()
    L.check(L.lib().lsp_proof_serialize(proof, None, 0, ctypes.byref(n)))
    t3 = time.perf_counter()
    buf = ctypes.create_string_buffer(n.value)
    L.check(L.lib().lsp_proof_serialize(proof, buf, n.value, ctypes.byref(n)))
    raw = buf.raw[:n.value]
    t4 = time.perf_counter()
    L.lib().lsp_proof_free(proof)
    t5 = time.perf_counter()
    span = dict(ctx.last_timings())["prove"]
    us = lambda a, b: (b - a) * 1e6
    print(f"prep {us(t0,t1):6.1f} us  lsp_prove {us(t1,t2)/1e3:7.3f} ms (span {span:7.3f})  serialize {us(t2,t3):6.1f}  copy {us(t3,t4):6.1f}  free {us(t4,t5):6.1f} us", flush=True)
