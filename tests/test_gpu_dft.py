"""The TwoAdicSubgroupDft surface beyond coset_lde_batch ([EXT p3-dft]
Radix2DitParallel, bin/src/config.rs:22): dft_batch, coset_dft_batch,
idft_batch, coset_idft_batch, lde_batch (lsp_coset_dft_batch /
lsp_coset_idft_batch / lsp_coset_lde_batch).

Checker: pyoracle's radix-2 NTT (oracle/pyoracle.py `ntt`, `idft`) at sizes
it finishes in seconds; above that, round trips and agreement with the LDE
kernels (themselves pinned to the oracle in test_gpu_parity.py).  Integer
arithmetic mod r: bit-exact equality throughout.
"""
import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

P = O.P


def rand_fr(rng, shape):
    from linea_stark_prover_amd.field import to_mont
    n = int(np.prod(shape))
    vals = [int.from_bytes(rng.bytes(32), "little") % P for _ in range(n)]
    return to_mont(vals).reshape(tuple(shape) + (4,))


def ints(a):
    from linea_stark_prover_amd.field import from_mont
    return from_mont(a)


def mont(vals):
    from linea_stark_prover_amd.field import to_mont
    return to_mont(vals)


def cols_of(mat):
    h, w = mat.shape[0], mat.shape[1]
    flat = ints(mat.reshape(-1, 4))
    return [[flat[i * w + c] for i in range(h)] for c in range(w)]


def oracle_coset_dft(col, shift):
    """p(shift w_h^j) at row bitrev(j)"""
    h = len(col)
    s, tw = 1, []
    for c in col:
        tw.append(c * s % P)
        s = s * shift % P
    return O.reverse_slice_index_bits(O.ntt(tw, O.two_adic_generator(O.log2_strict(h))))


def oracle_coset_idft(col, shift):
    c = O.idft(col)
    si, s, out = O.inv(shift), 1, []
    for x in c:
        out.append(x * s % P)
        s = s * si % P
    return out


@pytest.mark.parametrize("logh,w", [(0, 1), (0, 3), (1, 2), (2, 1), (3, 8), (5, 3), (8, 14), (10, 2), (12, 5)])
@pytest.mark.parametrize("coset", [False, True])
def test_dft_matches_oracle(gpu_ctx, logh, w, coset):
    rng = np.random.default_rng(7 * logh + w + coset)
    h = 1 << logh
    coeffs = rand_fr(rng, (h, w))
    shift = int.from_bytes(rng.bytes(32), "little") % P if coset else 1
    got = gpu_ctx.coset_dft_batch(coeffs, mont([shift])[0] if coset else None)
    exp = [oracle_coset_dft(col, shift) for col in cols_of(coeffs)]
    assert ints(got.reshape(-1, 4)) == [exp[c][i] for i in range(h) for c in range(w)]


@pytest.mark.parametrize("logh,w", [(0, 2), (1, 1), (2, 3), (4, 8), (7, 1), (9, 14), (11, 4), (12, 3)])
@pytest.mark.parametrize("coset", [False, True])
def test_idft_matches_oracle(gpu_ctx, logh, w, coset):
    rng = np.random.default_rng(11 * logh + w + coset)
    h = 1 << logh
    evals = rand_fr(rng, (h, w))
    shift = int.from_bytes(rng.bytes(32), "little") % P if coset else 1
    got = gpu_ctx.coset_idft_batch(evals, mont([shift])[0] if coset else None)
    exp = [oracle_coset_idft(col, shift) for col in cols_of(evals)]
    assert ints(got.reshape(-1, 4)) == [exp[c][i] for i in range(h) for c in range(w)]


def test_shift_one_is_the_plain_transform(gpu_ctx):
    rng = np.random.default_rng(5)
    m = rand_fr(rng, (256, 3))
    one = mont([1])[0]
    assert np.array_equal(gpu_ctx.coset_dft_batch(m), gpu_ctx.coset_dft_batch(m, one))
    assert np.array_equal(gpu_ctx.coset_idft_batch(m), gpu_ctx.coset_idft_batch(m, one))


@pytest.mark.parametrize("logh,w", [(14, 8), (16, 3), (18, 2), (19, 1)])
def test_round_trip_and_lde_agreement(gpu_ctx, logh, w):
    """at sizes past the Python oracle: idft(dft(c)) = c on a coset, and every
    coset block of lde_batch equals coset_dft of the coefficients idft_batch gives"""
    from linea_stark_prover_amd.prover import Radix2DitParallel
    dft = Radix2DitParallel(gpu_ctx)
    rng = np.random.default_rng(logh)
    h = 1 << logh
    vals = rand_fr(rng, (h, w))
    s = mont([int.from_bytes(rng.bytes(32), "little") % P])[0]
    ev = dft.coset_dft_batch(vals, s)  # bit-reversed rows
    nat = ev.reshape(h, -1)[[O.bitrev(j, logh) for j in range(h)]].reshape(h, w, 4)
    assert np.array_equal(dft.coset_idft_batch(nat, s), vals)
    added = 2
    lde = dft.lde_batch(vals, added)
    coeffs = dft.idft_batch(vals)
    wN = O.two_adic_generator(logh + added)
    for k in range(1 << added):
        blk = dft.coset_dft_batch(coeffs, mont([pow(wN, O.bitrev(k, added), P)])[0])
        assert np.array_equal(blk, lde[k * h:(k + 1) * h]), f"coset block {k}"


def test_bad_arguments(gpu_ctx):
    from linea_stark_prover_amd import _lib
    m = rand_fr(np.random.default_rng(1), (6, 2))
    with pytest.raises(_lib.LspError) as e:
        gpu_ctx.coset_dft_batch(m)  # 6 rows: not a power of two
    assert e.value.code == _lib.LSP_E_SIZE
    m = rand_fr(np.random.default_rng(1), (8, 2))
    with pytest.raises(_lib.LspError) as e:
        gpu_ctx.coset_idft_batch(m, mont([0])[0])
    assert e.value.code == _lib.LSP_E_ARG
