"""Every tuning knob of the library ("knobs") leaves the proof
bytes unchanged.

The knobs only move work between schedules that compute the same values:
Merkle levels on the host or the GPU (LSP_HOST_TREE_TOP), FRI rounds on the
host (LSP_FRI_HOST_TAIL), when the host pool starts spinning for a tree top
(LSP_TOP_WARM), row / quad / pair / one-lane permutations for narrow
levels (LSP_ROW_MAX, LSP_COOP_MAX, LSP_PAIR_MAX), zero-copy tree tops, host subtree tasks, LDE pass
plans (LSP_NTT_KMAX, LSP_NTT_LOGCW, LSP_NTT_TWL), the host pool size and the
IFMA host batches.  Several are read once per process, so each setting runs in a
child process; the per-call knobs vary inside each child.  The default proof is
pinned to the oracle elsewhere (test_gpu_fullsize.py, test_gpu_parity.py), so
equality with it is the parity check here.  Sizes 2^12 and 2^16: the latter's
trees cross the pair (32K) and quad (16K) level limits and the 1024-digest host
top, and its FRI runs GPU rounds before the host tail."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, json, os, sys
import numpy as np
sys.path.insert(0, %r)
from linea_stark_prover_amd.air import permutation_air
from linea_stark_prover_amd.prover import Context, StarkConfig, gen_permutation_trace
ctx = Context(StarkConfig())
a, d, _ = ctx.config.seeded()
pub = np.concatenate([a, d])
air = permutation_air(3)
combos = [(None, None), ("0", "0"), ("64", "64"), ("4096", "4096")]
out = {}
for lg in (12, 16):
    tr = gen_permutation_trace(lg, 3, a, d)
    for top, tail in combos:
        for k, v in (("LSP_HOST_TREE_TOP", top), ("LSP_FRI_HOST_TAIL", tail)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        pf = ctx.prove(tr, air, pub)
        out["%%d/%%s/%%s" %% (lg, top, tail)] = hashlib.sha256(pf).hexdigest()
    assert ctx.verify(pf, air, pub)
print(json.dumps(out))
""" % ROOT

SETTINGS = {
    "default": {},
    "no_zerocopy_no_subtree_no_defer": {"LSP_TOP_ZEROCOPY": "0", "LSP_HOST_SUBTREE": "0", "LSP_NO_DEFER_TOPS": "1"},
    "one_lane_levels": {"LSP_COOP_MAX": "0", "LSP_PAIR_MAX": "0", "LSP_ROW_MAX": "0"},
    "quads_to_32k": {"LSP_COOP_MAX": "32768", "LSP_COOP_BS": "256", "LSP_ROW_MAX": "0"},
    "rows_to_16k": {"LSP_ROW_MAX": "16384"},
    "no_top_warm": {"LSP_TOP_WARM": "0"},
    "top_warm_64k": {"LSP_TOP_WARM": "65536"},
    "lde_plans": {"LSP_NTT_KMAX": "7", "LSP_NTT_LOGCW": "3", "LSP_NTT_TWL": "0"},
    "host_serial_scalar": {"LSP_HOST_THREADS": "1", "LSP_HOST_IFMA": "0"},
}


def _child(extra):
    env = dict(os.environ, **extra)
    for k in ("LSP_HOST_TREE_TOP", "LSP_FRI_HOST_TAIL"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


@pytest.fixture(scope="module")
def default_hashes():
    return _child({})


def test_per_call_knobs_keep_the_proof(default_hashes):
    for lg in (12, 16):
        ref = default_hashes[f"{lg}/None/None"]
        for key, hx in default_hashes.items():
            if key.startswith(f"{lg}/"):
                assert hx == ref, key


@pytest.mark.parametrize("name", [n for n in SETTINGS if n != "default"])
def test_process_knobs_keep_the_proof(default_hashes, name):
    got = _child(SETTINGS[name])
    for lg in (12, 16):
        ref = default_hashes[f"{lg}/None/None"]
        for key, hx in got.items():
            if key.startswith(f"{lg}/"):
                assert hx == ref, (name, key)


def test_default_proof_is_the_in_process_proof(gpu_ctx, default_hashes):
    """the child's default equals this process's proof (same seed, same trace)"""
    import numpy as np
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    pf = gpu_ctx.prove(gen_permutation_trace(12, 3, a, d), permutation_air(3), np.concatenate([a, d]))
    assert hashlib.sha256(pf).hexdigest() == default_hashes["12/None/None"]


def test_phase_timing_selection(gpu_ctx):
    """lsp_ctx_set_phase_timing: none, only the named phases, or all (the
    default); the proof bytes do not depend on it"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    import numpy as np
    a, d, _ = gpu_ctx.config.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(3)
    tr = gen_permutation_trace(10, 3, a, d)
    full = gpu_ctx.prove(tr, air, pub)
    names_all = [n for n, _ in gpu_ctx.last_timings()]
    assert "coset_lde_batch" in names_all and "merkle tree" in names_all and "prove" in names_all
    try:
        gpu_ctx.set_phase_timing(False)
        assert gpu_ctx.prove(tr, air, pub) == full
        assert gpu_ctx.last_timings() == []
        gpu_ctx.set_phase_timing(True, only=["coset_lde_batch", "merkle tree"])
        assert gpu_ctx.prove(tr, air, pub) == full
        got = gpu_ctx.last_timings()
        assert sorted(n for n, _ in got) == ["coset_lde_batch", "merkle tree"] and all(ms > 0 for _, ms in got)
    finally:
        gpu_ctx.set_phase_timing(True)
    assert gpu_ctx.prove(tr, air, pub) == full
    assert [n for n, _ in gpu_ctx.last_timings()] == names_all
