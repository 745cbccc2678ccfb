"""Edge values through each device multiplier: 0, 1, r - 1, r - 2, (r - 1)/2,
2^252, R mod r, ... as operands of
* the NTT's 29-bit product (coset_dft_batch of 2 coefficients: c_0 + c_1 s and
  c_0 - c_1 s, every c_1 against every shift s),
* the Poseidon2 kernels' product (every state of three edge values, and
  sponge rows of them),
* the batch inverse and the LDE of constant columns.
Checker: Python big ints / pyoracle.  Bit-exact.
"""
import itertools

import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

P = O.P
EDGES = [0, 1, 2, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2, 1 << 252, (1 << 256) % P, (1 << 261) % P,
         (1 << 253) - 1 - P, 0xFFFFFFFF]


def mont(vals):
    from linea_stark_prover_amd.field import to_mont
    return to_mont(list(vals))


def ints(a):
    from linea_stark_prover_amd.field import from_mont
    return from_mont(a.reshape(-1, 4))


def test_ntt_product_edges(gpu_ctx):
    n = len(EDGES)
    # column j: c_0 = EDGES[(j + 3) % n], c_1 = EDGES[j]
    c0 = [EDGES[(j + 3) % n] for j in range(n)]
    coeffs = mont(c0 + EDGES).reshape(2, n, 4)
    for s in EDGES:
        got = ints(gpu_ctx.coset_dft_batch(coeffs, mont([s])[0]))
        exp = [(c0[j] + EDGES[j] * s) % P for j in range(n)] + [(c0[j] - EDGES[j] * s) % P for j in range(n)]
        assert got == exp, f"shift {s:#x}"


def test_poseidon2_edge_states(gpu_ctx):
    pp = O.setup_from_seed().perm
    states = list(itertools.product(EDGES[:8], repeat=3))  # 512 states
    got = ints(gpu_ctx.poseidon2_permute(mont([x for s in states for x in s]).reshape(-1, 3, 4)))
    exp = [x for s in states for x in O.permute(list(s), pp)]
    assert got == exp


def test_sponge_edge_rows(gpu_ctx):
    pp = O.setup_from_seed().perm
    rows = [[EDGES[(i + k) % len(EDGES)] for k in range(7)] for i in range(len(EDGES))]
    got = ints(gpu_ctx.hash_rows(mont([x for r in rows for x in r]).reshape(len(rows), 7, 4)))
    assert got == [O.hash_iter(r, pp) for r in rows]


def test_batch_inverse_edges(gpu_ctx):
    vals = [v for v in EDGES if v] * 37  # past one workgroup's chunk
    got = ints(gpu_ctx.batch_inverse(mont(vals)))
    assert got == [pow(v, P - 2, P) for v in vals]


@pytest.mark.parametrize("v", [0, 1, P - 1, (1 << 252)])
def test_lde_of_constant_columns(gpu_ctx, v):
    """a constant column interpolates to the constant: every LDE row equals it"""
    h, w = 1 << 10, 3
    s = mont([O.GENERATOR])[0]
    got = ints(gpu_ctx.coset_lde_batch(mont([v] * (h * w)).reshape(h, w, 4), 3, s))
    assert got == [v] * (8 * h * w)
