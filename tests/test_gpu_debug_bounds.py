"""The bounds-checked debug build on the GPU (csrc/dbg_bounds.hpp).

Each case runs in a child process with LSP_LIB pointing at liblsp_hip_dbg.so
(built by build.py --debug-bounds; tests/test_sanitize.py builds it on CPU):
* the probe's deliberately failing check comes back as LSP_E_STATE naming its
  file and line, and the context stays usable;
* whole proofs through every prover kernel family (LDE, Merkle leaves and
  levels, quotient, open, FRI, grinding) raise no check and are
  byte-identical to the oracle's.
The product build answers the probe with "not a debug-bounds build"."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from linea_stark_prover_amd import _lib as L
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace
from oracle import cref
assert b"debug-bounds" in L.lib().lsp_version()
with Context(StarkConfig(proof_of_work_bits=6)) as ctx:
    rc = L.lib().lsp_debug_bounds_probe(ctx.h)
    msg = L.lib().lsp_last_error(ctx.h).decode()
    assert rc == L.LSP_E_STATE and "bounds check failed at k_field.hip:" in msg, (rc, msg)
    print("probe:", msg)
    p = cref.setup()
    for log_n, ncols in ((8, 3), (11, 6), (14, 3)):
        tb, w = cref.gen_perm_trace(p, log_n, ncols)
        trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4).copy()
        pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
        got = ctx.prove(trace, permutation_air(ncols), pub)
        exp = cref.prove(p, trace.ctypes.data, 1 << log_n, w, cref.perm_air(ncols),
                         fri=cref.fri_params(cref.O.FriParams(proof_of_work_bits=6)))
        assert got == exp, (log_n, ncols)
        assert ctx.verify(got, permutation_air(ncols), pub)
print("debug-bounds ok")
'''


def test_debug_build_probe_and_clean_proofs():
    from linea_stark_prover_amd import build as B
    if not os.path.exists(B.DBG_LIB):
        pytest.skip("liblsp_hip_dbg.so not built (python -m linea_stark_prover_amd.build --debug-bounds)")
    env = dict(os.environ, LSP_LIB=B.DBG_LIB)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "debug-bounds ok" in r.stdout


def test_product_build_is_not_debug(gpu_ctx):
    from linea_stark_prover_amd import _lib as L
    assert L.lib().lsp_debug_bounds_probe(gpu_ctx.h) == L.LSP_E_STATE
    assert b"not a debug-bounds build" in L.lib().lsp_last_error(gpu_ctx.h)
