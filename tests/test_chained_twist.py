"""The chained coset twist of the fused LDE pass (k_ntt.hip k_ntt_rm,
prove.cpp chain_ratio), CPU only:

  * the block order: blocks k0 + bitrev_a(j), j < nk = 2^a (k0 a multiple of
    nk), of the bit-reversed LDE of 2^b blocks have the coset shifts
    s w_N^bitrev_b(k0) rho^j with rho = w_N^(2^b / nk) -- so every later block's
    twist s_j^i / h is the previous block's times rho^i;
  * the bound: the registers carry the running twisted value through nk - 1
    products by a canonical factor; starting below 8.3 r with normalised limbs
    it stays below 8.3 r (the tile invariant) with every column sum < 2^64.

The kernels themselves are checked bit for bit by the GPU LDE / proof / shard
suites (tests/test_gpu_parity.py, test_gpu_dft.py, test_gpu_shard.py)."""
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pyoracle as O  # noqa: E402

from test_f29_bounds import MASK, R, f29_mul, limbs, val  # noqa: E402


@pytest.mark.parametrize("b,a,k0", [(3, 3, 0), (3, 2, 0), (3, 2, 4), (3, 1, 6), (2, 2, 0), (6, 3, 8), (6, 6, 0)])
def test_block_shifts_form_a_geometric_run(b, a, k0):
    log_h = 5
    logN = log_h + b
    wN = O.two_adic_generator(logN)
    s = O.GENERATOR
    nk = 1 << a
    assert k0 % nk == 0
    shift = [s * pow(wN, O.bitrev(k0 + k, b), O.P) % O.P for k in range(nk)]  # lde_twist's bases
    rho = pow(wN, (1 << b) // nk, O.P)  # chain_ratio
    order = [O.bitrev(j, a) for j in range(nk)]  # the kernel's arr = bitrev(j)
    assert order[0] == 0
    for j in range(1, nk):
        assert shift[order[j]] == shift[order[j - 1]] * rho % O.P
    # hence the twist factors s_j^i / h chain by rho^i, row by row
    hinv = O.inv(1 << log_h)
    for i in (0, 1, 7, (1 << log_h) - 1):
        t = pow(shift[order[0]], i, O.P) * hinv % O.P
        for j in range(1, nk):
            t = t * pow(rho, i, O.P) % O.P
            assert t == pow(shift[order[j]], i, O.P) * hinv % O.P


def test_running_twist_stays_in_the_tile_bound():
    rng = random.Random(5)
    inv261 = pow(2, -261, R)
    bound = int(8.3 * R)
    starts = [bound - 1, bound - R // 3, R - 1, 8 * R + (1 << 200)] + [rng.randrange(bound) for _ in range(40)]
    for x0 in starts:
        x = limbs(x0)
        assert all(v <= MASK for v in x[:8])
        ref = x0
        for _ in range(7):  # 8 coset blocks: block 0 from its table, 7 chained products
            f = rng.choice([R - 1, R - 2, rng.randrange(R)])
            x, worst = f29_mul(x, limbs(f))
            ref = ref * f * inv261 % R
            assert worst < 1 << 64
            assert all(v <= MASK for v in x[:8])
            assert val(x) < bound
            assert val(x) % R == ref
