"""Property tests of the library's host field arithmetic (A1, BLS12-377 Fr as
ark-ff stores it: 4 x u64 Montgomery, R = 2^256) against Python big ints,
SURVEY §4's "inverse/exp properties, using hypothesis".  Edge values (0, 1,
r - 1, r - 2, 2^252, R mod r) are drawn first; hypothesis adds random ones.
CPU only: lsp_fr_* are host functions.
"""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from oracle import pyoracle as O

P = O.P
EDGES = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, 1 << 252, (1 << 256) % P, (1 << 261) % P, 22, 0xFFFFFFFF]
elem = st.one_of(st.sampled_from(EDGES), st.integers(min_value=0, max_value=P - 1))


def mont(v):
    from linea_stark_prover_amd.field import to_mont
    return np.ascontiguousarray(to_mont([v])[0])


def val(a):
    from linea_stark_prover_amd.field import from_mont
    return from_mont(a.reshape(1, 4))[0]


@settings(max_examples=300, deadline=None)
@given(elem, elem)
def test_mul_matches_big_ints(product_lib, x, y):
    a, b, out = mont(x), mont(y), np.zeros(4, np.uint64)  # held: .ctypes.data of a temporary dangles
    product_lib.lsp_fr_mul(a.ctypes.data, b.ctypes.data, out.ctypes.data)
    assert val(out) == x * y % P


@settings(max_examples=200, deadline=None)
@given(elem.filter(lambda v: v != 0))
def test_inverse(product_lib, x):
    a, out = mont(x), np.zeros(4, np.uint64)
    product_lib.lsp_fr_inv(a.ctypes.data, out.ctypes.data)
    assert val(out) == pow(x, P - 2, P)


@settings(max_examples=200, deadline=None)
@given(elem)
def test_canonical_round_trip(product_lib, x):
    can = np.frombuffer(x.to_bytes(32, "little"), np.uint64).copy()
    m = np.zeros(4, np.uint64)
    product_lib.lsp_fr_from_canonical(can.ctypes.data, m.ctypes.data)
    assert np.array_equal(m, mont(x))  # the Montgomery words ark-ff stores
    back = np.zeros(4, np.uint64)
    product_lib.lsp_fr_to_canonical(m.ctypes.data, back.ctypes.data)
    assert np.array_equal(back, can)


@settings(max_examples=200, deadline=None)
@given(st.binary(min_size=0, max_size=80))
def test_from_be_bytes_mod_order(product_lib, b):
    """FF_Bls12_377Fr::from_be_bytes_mod_order (trace/src/permutation.rs:102-104): any length, reduced mod r"""
    out = np.zeros(4, np.uint64)
    product_lib.lsp_fr_from_be_bytes_mod_order(b, len(b), out.ctypes.data)
    assert val(out) == int.from_bytes(b, "big") % P


@pytest.mark.parametrize("bits", range(0, 48))
def test_two_adic_generator_orders(product_lib, bits):
    """w_(2^k) has order exactly 2^k, and w_(2^k)^2 = w_(2^(k-1)) (TwoAdicField)"""
    out = np.zeros(4, np.uint64)
    product_lib.lsp_two_adic_generator(bits, out.ctypes.data)
    g = val(out)
    assert g == O.two_adic_generator(bits)
    assert pow(g, 1 << bits, P) == 1
    if bits:
        assert pow(g, 1 << (bits - 1), P) == P - 1
        prev = np.zeros(4, np.uint64)
        product_lib.lsp_two_adic_generator(bits - 1, prev.ctypes.data)
        assert val(prev) == g * g % P


@settings(max_examples=100, deadline=None)
@given(elem, elem, st.integers(min_value=0, max_value=40), st.booleans())
def test_fold_row_matches_oracle(product_lib, e0, e1, log_height, flip):
    """TwoAdicFriGenericConfig::fold_row (host, the verifier side of A15)"""
    idx = (e0 ^ e1) % (1 << log_height) if log_height else 0
    beta = (e0 * 7 + e1 + int(flip)) % P
    b, a0, a1, out = mont(beta), mont(e0), mont(e1), np.zeros(4, np.uint64)
    product_lib.lsp_fri_fold_row(idx, log_height, b.ctypes.data, a0.ctypes.data, a1.ctypes.data, out.ctypes.data)
    assert val(out) == O.fold_row(idx, log_height, beta, e0, e1)
