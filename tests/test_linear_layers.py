"""U2/U3: caller-set Poseidon2 linear layers and round constants.

The reference builds ONE permutation from thread_rng (bin/src/main.rs:49) and
hashes the Mmcs and the challenger with it (main.rs:50-57,78,88).  For the
unchanged p3_uni_stark::verify to accept a library proof, the library must
prove with exactly that Perm: its round constants (lsp_params.round_constants,
filled by p3_hip::Params::from_rng) and, should the fork's
Poseidon2Bls12337<3> use other layers than the default, its internal diagonal
and external matrix (lsp_params.internal_diag / external_mds).

Here a context is built with explicit non-default constants and non-default
layers; every permutation path of the library -- the host scalar and
AVX-512 IFMA tree tops, the host verifier, and on the GPU the one-lane, lane
pair and DPP-quad kernels and the whole proof -- must agree with the two
oracles set up with the same parameters (the proof byte for byte).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SEED = 0xC0FFEE  # not the library's seeded set
DIAG = (3, 5, O.P - 7)                                 # M_I = J + diag(d)
MDS = (5, 7, 1, 3, 2, 9, 4, 4, O.P - 1)              # M_E, row-major
CASES = {"diag": (DIAG, None), "mds": (None, MDS), "both": (DIAG, MDS), "default_explicit": ((1, 1, 2), None)}


def _setup(case, sbox_degree=11):
    diag, mds = CASES[case]
    s = O.setup_from_seed(SEED, sbox_degree=sbox_degree)
    s.perm.int_diag, s.perm.ext_mds = diag, mds
    return s


def _rc(s):
    from linea_stark_prover_amd.field import to_mont
    pp = s.perm
    return to_mont([x for r in pp.ext_initial for x in r] + [x for r in pp.ext_terminal for x in r] + pp.internal)


def _ctx(s, device):
    from linea_stark_prover_amd.prover import Context, StarkConfig
    cfg = StarkConfig(sbox_degree=s.perm.sbox_degree, internal_diag=s.perm.int_diag, external_mds=s.perm.ext_mds)
    return Context(cfg, device=device, round_constants=_rc(s))


def _pub(s):
    from linea_stark_prover_amd.field import to_mont
    return to_mont([s.alpha, s.delta])


def _cref_params(cref, s):
    return cref.params_from_setup(s)


def test_oracles_agree_on_generic_layers(oracle_lib):
    """C oracle (lo_poseidon2_permute) == Python oracle, and explicit default
    layers == the default path"""
    for case in CASES:
        s = _setup(case)
        p = _cref_params(oracle_lib, s)
        for st in ([0, 0, 0], [1, 2, 3], [O.P - 1, 5, O.P // 3]):
            buf = oracle_lib.fr_buf(st)
            oracle_lib.lib().lo_poseidon2_permute(ctypes.byref(p), buf)
            assert oracle_lib.buf_to_ints(buf, 3) == O.permute(st, s.perm), case
    d = O.setup_from_seed(SEED)
    e = _setup("default_explicit")
    e.perm.ext_mds = O.DEFAULT_EXT_MDS
    assert O.permute([4, 5, 6], d.perm) == O.permute([4, 5, 6], e.perm)
    # and the layers change the permutation
    assert O.permute([4, 5, 6], d.perm) != O.permute([4, 5, 6], _setup("diag").perm)


@pytest.mark.parametrize("case", ["diag", "mds", "both"])
def test_host_paths_generic_layers(product_lib, case):
    """the host tree-top paths (IFMA 8/16 lanes when the CPU has them, and the
    scalar 4 x 64-bit path in a child process with LSP_HOST_IFMA=0)"""
    from tests.test_host import _host_merkle_checks
    s = _setup(case)
    _host_merkle_checks(product_lib, _ctx(s, -1), s.perm, 5)
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from tests.test_host import _host_merkle_checks\n"
        "from tests.test_linear_layers import _setup, _ctx\n"
        "from linea_stark_prover_amd import _lib\n"
        "for d in (11, 17):\n"
        "    s = _setup(%r, d)\n"
        "    _host_merkle_checks(_lib.lib(), _ctx(s, -1), s.perm, d)\n"
    ) % (ROOT, case)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, LSP_HOST_IFMA="0"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("case", ["both"])
def test_host_verifier_generic_layers(product_lib, oracle_lib, case):
    """lsp_verify on a host-only context with the layers accepts the oracle's
    proof made with them, and a context with the default layers rejects it"""
    from linea_stark_prover_amd.air import permutation_air
    s = _setup(case)
    p = _cref_params(oracle_lib, s)
    tb, w = oracle_lib.gen_perm_trace(p, 5, 3)
    proof = oracle_lib.prove(p, tb, 1 << 5, w, oracle_lib.perm_air(3))
    assert oracle_lib.verify(p, proof, oracle_lib.perm_air(3)) == 0
    assert _ctx(s, -1).verify(proof, permutation_air(3), _pub(s))
    d = O.setup_from_seed(SEED)
    assert not _ctx(d, -1).verify(proof, permutation_air(3), _pub(s))


def test_bad_layer_values_rejected(product_lib):
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.prover import Context, StarkConfig
    from linea_stark_prover_amd.field import to_mont
    s = _setup("diag")
    rc = _rc(s)
    diag = to_mont(DIAG)
    diag[1] = np.array([~np.uint64(0)] * 4, np.uint64)  # not canonical
    p = _lib.LspParams(sbox_degree=11, rounds_f=8, rounds_p=22, round_constants=rc.ctypes.data, log_blowup=3,
                       log_final_poly_len=0, num_queries=33, proof_of_work_bits=0, public_degree=1,
                       internal_diag=diag.ctypes.data, external_mds=None)
    h = ctypes.c_void_p()
    assert product_lib.lsp_ctx_create(-1, ctypes.byref(p), ctypes.byref(h)) == _lib.LSP_E_ARG


# ------------------------------------------------------------------ GPU
def _cref_hash_rows(cref, p, vals, n, w):
    buf = cref.fr_buf(vals)
    out = (ctypes.c_uint64 * 4)()
    res = []
    for i in range(n):
        cref.lib().lo_hash_iter(ctypes.byref(p), ctypes.byref(buf, i * w * 32), ctypes.c_size_t(w), out)
        res.append(O.from_mont_bytes(bytes(out)))
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["diag", "mds", "both"])
def test_gpu_kernels_generic_layers(product_lib, oracle_lib, case):
    """k_permute, and k_hash_rows1 at widths taking every lane mode: <= 16K rows
    on DPP quads, 16K..32K on lane pairs, more one per lane"""
    from linea_stark_prover_amd.field import from_mont, to_mont
    s = _setup(case)
    p = _cref_params(oracle_lib, s)
    rng = np.random.default_rng(3)
    with _ctx(s, 0) as ctx:
        states = [[int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(3)] for _ in range(64)]
        got = from_mont(ctx.poseidon2_permute(to_mont([x for st in states for x in st]).reshape(-1, 3, 4)).reshape(-1, 4))
        assert got == [x for st in states for x in O.permute(st, s.perm)]
        for n, w in ((1000, 3), (20000, 2), (40000, 1)):
            vals = [int(x) for x in rng.integers(0, 1 << 62, n * w)]
            out = from_mont(ctx.hash_rows(to_mont(vals).reshape(n, w, 4)))
            idx = list(range(0, n, max(1, n // 97))) + [n - 1]
            exp = _cref_hash_rows(oracle_lib, p, [vals[i * w + k] for i in idx for k in range(w)], len(idx), w)
            assert [out[i] for i in idx] == exp, (case, n, w)


@pytest.mark.gpu
@pytest.mark.parametrize("case,logn,sbox", [("both", 10, 11), ("diag", 8, 17), ("mds", 14, 11)])
def test_gpu_proof_generic_layers_matches_oracle(product_lib, oracle_lib, case, logn, sbox):
    """lsp_prove with non-default round constants and linear layers is byte
    for byte the oracle's proof under the same parameters (Merkle trees down
    through the GPU quad levels and the host IFMA tops, transcript, FRI tail)"""
    from linea_stark_prover_amd.air import permutation_air
    s = _setup(case, sbox)
    p = _cref_params(oracle_lib, s)
    tb, w = oracle_lib.gen_perm_trace(p, logn, 3)
    expect = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.perm_air(3))
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << logn, w, 4).copy()
    with _ctx(s, 0) as ctx:
        proof = ctx.prove(trace, permutation_air(3), _pub(s))
        assert proof == expect
        assert ctx.verify(proof, permutation_air(3), _pub(s))


@pytest.mark.gpu
def test_gpu_sharded_proof_generic_layers(product_lib, oracle_lib):
    """the sharded prover (4 virtual ranks: subtree roots, the split inverse
    NTTs' exchanges, host tree tops per rank) with non-default constants and
    layers equals the oracle's proof"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import ProverGroup
    s = _setup("both")
    p = _cref_params(oracle_lib, s)
    logn = 12
    tb, w = oracle_lib.gen_perm_trace(p, logn, 3)
    expect = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.perm_air(3))
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << logn, w, 4).copy()
    ctxs = [_ctx(s, 0) for _ in range(4)]
    try:
        assert ProverGroup(ctxs).prove(trace, permutation_air(3), _pub(s)) == expect
    finally:
        for c in ctxs:
            c.close()
