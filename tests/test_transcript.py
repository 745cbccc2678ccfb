"""The transcript conventions U7, U8 and U12 as named switches (SURVEY 8(c),
include/lsp.h lsp_params), on the CPU: the Python and C oracles agree byte
for byte under every variant, each variant's proof verifies under its own
setting and fails under the default one, and the product's host verifier
(lsp_verify on a host-only context) follows the same switches.

The reference's HashChallenger (bin/src/config.rs:23) and the fork's
p3-uni-stark / p3-fri (bin/src/main.rs:78-96) fix one of these variants; no
reference artefact says which (parity unpinned), so every one is a switch
with SURVEY 8(c)'s choice as the default."""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as O

# (StarkConfig switch, FriParams field, value under the variant)
VARIANTS = {
    "skip_log_degree": dict(observe_log_degree=False),
    "skip_public_values": dict(observe_public_values=False),
    "observe_opened_values": dict(observe_opened_values=True),
    "sample_bits_montgomery": dict(sample_bits_montgomery=True),
    "skip_final_poly": dict(observe_final_poly=False),
    "all": dict(observe_log_degree=False, observe_public_values=False, observe_opened_values=True,
                sample_bits_montgomery=True, observe_final_poly=False),
}


def stark_switches(name):
    """the StarkConfig keyword arguments of a variant"""
    fp = VARIANTS[name]
    return dict(skip_log_degree=not fp.get("observe_log_degree", True),
                skip_public_values=not fp.get("observe_public_values", True),
                observe_opened_values=fp.get("observe_opened_values", False),
                sample_bits_montgomery=fp.get("sample_bits_montgomery", False),
                skip_final_poly=not fp.get("observe_final_poly", True))


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_oracles_agree_under_each_variant(oracle_lib, name):
    logn, ncols, pow_bits = 3, 3, 3  # a few grinding steps exercise U8 in the witness check
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    cfgs, cols = O.synthetic_perm_trace(logn, ncols, s.alpha, s.delta, O.DEFAULT_SEED)
    rows = O.columns_to_rows(cols)
    tb, w = oracle_lib.gen_perm_trace(p, logn, ncols)
    fp = O.FriParams(proof_of_work_bits=pow_bits, **VARIANTS[name])
    pf = O.prove(cfgs, rows, [s.alpha, s.delta], s.perm, fp)
    cb = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.air_desc(cfgs), fri=oracle_lib.fri_params(fp))
    assert cb == O.serialize_proof(pf)
    assert O.verify(cfgs, pf, [s.alpha, s.delta], s.perm, fp)
    assert oracle_lib.verify(p, cb, oracle_lib.air_desc(cfgs), fri=oracle_lib.fri_params(fp)) == 0
    # the default transcript rejects it, and the default proof differs
    dfp = O.FriParams(proof_of_work_bits=pow_bits)
    assert oracle_lib.verify(p, cb, oracle_lib.air_desc(cfgs), fri=oracle_lib.fri_params(dfp)) != 0
    assert not O.verify(cfgs, pf, [s.alpha, s.delta], s.perm, dfp)
    base = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.air_desc(cfgs), fri=oracle_lib.fri_params(dfp))
    assert base != cb


def test_montgomery_sample_bits_is_the_montgomery_word():
    """U8's switch reads the low bits of x * 2^256 mod r (ark-ff's in-memory limbs)"""
    s = O.setup_from_seed()
    a = O.HashChallenger(s.perm, mont_bits=False)
    b = O.HashChallenger(s.perm, mont_bits=True)
    for ch in (a, b):
        ch.observe(5)
        ch.observe(7)
    x = O.hash_iter([5, 7], s.perm)
    assert a.sample_bits(20) == x & 0xFFFFF
    assert b.sample_bits(20) == (x * O.MONT_R % O.P) & 0xFFFFF


@pytest.mark.parametrize("name", ["observe_opened_values", "sample_bits_montgomery", "all"])
def test_product_verifier_follows_the_switches(oracle_lib, product_lib, name):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    logn, ncols = 5, 3
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, logn, ncols)
    fp = O.FriParams(proof_of_work_bits=2, **VARIANTS[name])
    proof = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.perm_air(ncols), fri=oracle_lib.fri_params(fp))
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    air = permutation_air(ncols)
    with Context(StarkConfig(proof_of_work_bits=2, **stark_switches(name)), device=-1) as v:
        assert v.verify(proof, air, pub)
    with Context(StarkConfig(proof_of_work_bits=2), device=-1) as v:
        assert not v.verify(proof, air, pub)


def test_params_struct_size_and_switch_values_checked(product_lib):
    """lsp_params.struct_size guards against callers built with another
    lsp.h; switches other than 0/1 are refused"""
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.prover import StarkConfig
    _, _, rc = StarkConfig().seeded()
    base = dict(sbox_degree=11, rounds_f=8, rounds_p=22, round_constants=rc.ctypes.data, log_blowup=3,
                num_queries=33, public_degree=1)
    h = ctypes.c_void_p()
    good = _lib.LspParams(**base)
    assert good.struct_size == ctypes.sizeof(_lib.LspParams) == 88
    assert product_lib.lsp_ctx_create(-1, ctypes.byref(good), ctypes.byref(h)) == _lib.LSP_OK
    product_lib.lsp_ctx_destroy(h)
    for size in (0, 11, 17, 60, 87, 89):  # 11 / 17: an old-layout caller's first field (sbox_degree)
        bad = _lib.LspParams(**base)
        bad.struct_size = size
        assert product_lib.lsp_ctx_create(-1, ctypes.byref(bad), ctypes.byref(h)) == _lib.LSP_E_ARG
    for sw in _lib.TRANSCRIPT_SWITCHES:
        bad = _lib.LspParams(**base, **{sw: 2})
        assert product_lib.lsp_ctx_create(-1, ctypes.byref(bad), ctypes.byref(h)) == _lib.LSP_E_ARG
