"""GPU parity: every hot-path stage of liblsp_hip.so against the oracle.

Checker: oracle/lsp_oracle.c (C restatement, pinned to oracle/pyoracle.py by
tests/test_oracle.py) and, at tiny sizes, pyoracle itself.  Everything here is
integer arithmetic mod r, so the bar is bit-exact equality.
"""
import ctypes

import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

P = O.P


def rand_fr(rng, shape):
    """uniform canonical Fr in Montgomery limbs"""
    n = int(np.prod(shape))
    vals = [int.from_bytes(rng.bytes(32), "little") % P for _ in range(n)]
    from linea_stark_prover_amd.field import to_mont
    return to_mont(vals).reshape(tuple(shape) + (4,))


def ints(a):
    from linea_stark_prover_amd.field import from_mont
    return from_mont(a)


def oracle_params(oracle_lib):
    return oracle_lib.setup()


def c_ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------ LDE
# pass plans (k_ntt.hip, k <= 10 per pass): one fused pass up to 2^10; [6,5] [6,6] [7,6]
# [7,7] [8,7] [8,8] [9,8] [9,9] above, with the per-pass column chunk and partial chunks;
# (the wide plan of 48+ columns: test_coset_lde_wide_plan)
@pytest.mark.parametrize("logh,w,added", [(1, 1, 1), (3, 2, 3), (5, 8, 3), (8, 14, 3), (10, 4, 2), (12, 8, 3),
                                          (13, 3, 3), (11, 1, 3), (14, 5, 3), (15, 14, 3), (16, 2, 1),
                                          (17, 1, 3), (18, 3, 2)])
def test_coset_lde_matches_oracle(gpu_ctx, oracle_lib, logh, w, added):
    rng = np.random.default_rng(logh * 100 + w)
    h = 1 << logh
    mat = rand_fr(rng, (h, w))
    shift = rand_fr(rng, (1,))
    got = gpu_ctx.coset_lde_batch(mat, added, shift)
    exp = np.zeros_like(got)
    shifts = np.repeat(shift.reshape(1, 4), w, axis=0).copy()
    oracle_lib.lib().lo_coset_lde_batch(c_ptr(mat), ctypes.c_size_t(h), ctypes.c_size_t(w), added, c_ptr(shifts),
                                        c_ptr(exp), 8)
    assert np.array_equal(got, exp)


def test_coset_lde_wide_plan(gpu_ctx, oracle_lib):
    """From 48 columns launch_lde plans 8-column chunks: 2^19 x 50 runs as
    [7,6,6] (whole 256-byte row segments, a partial last chunk of 2) instead of
    [10,9].  Columns transform independently, so the oracle checks a few of
    them, from the first chunk, a chunk boundary and the partial chunk."""
    rng = np.random.default_rng(1950)
    logh, w, added = 19, 50, 1
    h = 1 << logh
    mat = rng.integers(0, 2**64, size=(h, w, 4), dtype=np.uint64)  # canonical Montgomery words:
    mat[..., 3] &= (1 << 58) - 1                                   # every value < 2^250 < r
    shift = rand_fr(rng, (1,))
    got = gpu_ctx.coset_lde_batch(mat, added, shift)
    cols = [0, 7, 8, 48, 49]
    sub = np.ascontiguousarray(mat[:, cols])
    exp = np.zeros((h << added, len(cols), 4), dtype=np.uint64)
    shifts = np.repeat(shift.reshape(1, 4), len(cols), axis=0).copy()
    oracle_lib.lib().lo_coset_lde_batch(c_ptr(sub), ctypes.c_size_t(h), ctypes.c_size_t(len(cols)), added,
                                        c_ptr(shifts), c_ptr(exp), 16)
    assert np.array_equal(got[:, cols], exp)


def test_coset_lde_per_column_shifts(gpu_ctx, oracle_lib):
    rng = np.random.default_rng(7)
    h, w, added = 1 << 9, 4, 3
    mat = rand_fr(rng, (h, w))
    shifts = rand_fr(rng, (w,))
    got = gpu_ctx.coset_lde_batch(mat, added, shifts)
    exp = np.zeros_like(got)
    oracle_lib.lib().lo_coset_lde_batch(c_ptr(mat), ctypes.c_size_t(h), ctypes.c_size_t(w), added, c_ptr(shifts),
                                        c_ptr(exp), 8)
    assert np.array_equal(got, exp)


def test_coset_lde_tiny_vs_pyoracle(gpu_ctx):
    rng = np.random.default_rng(3)
    h, w = 8, 3
    mat = rand_fr(rng, (h, w))
    rows = [ints(mat[i]) for i in range(h)]
    exp = O.coset_lde_batch(rows, 3, O.GENERATOR)
    from linea_stark_prover_amd.field import to_mont
    got = gpu_ctx.coset_lde_batch(mat, 3, to_mont([O.GENERATOR]))
    assert [ints(got[i]) for i in range(len(exp))] == exp


# ------------------------------------------------------------- Poseidon2
def test_poseidon2_permute_matches_oracle(gpu_ctx, oracle_lib):
    rng = np.random.default_rng(11)
    n = 4099
    st = rand_fr(rng, (n, 3))
    got = gpu_ctx.poseidon2_permute(st)
    p = oracle_params(oracle_lib)
    exp = st.copy()
    for i in range(n):
        oracle_lib.lib().lo_poseidon2_permute(ctypes.byref(p), c_ptr(exp[i]))
    assert np.array_equal(got, exp)


def test_poseidon2_known_answer_vs_pyoracle(gpu_ctx):
    s = O.setup_from_seed()
    from linea_stark_prover_amd.field import to_mont
    st = to_mont([0, 1, 2]).reshape(1, 3, 4)
    got = ints(gpu_ctx.poseidon2_permute(st)[0])
    assert got == O.permute([0, 1, 2], s.perm)


@pytest.mark.parametrize("w", [1, 2, 3, 4, 7, 8, 14, 23])
def test_hash_rows_matches_sponge(gpu_ctx, oracle_lib, w):
    rng = np.random.default_rng(w)
    n = 300
    rows = rand_fr(rng, (n, w))
    got = gpu_ctx.hash_rows(rows)
    p = oracle_params(oracle_lib)
    exp = np.zeros((n, 4), np.uint64)
    for i in range(n):
        oracle_lib.lib().lo_hash_iter(ctypes.byref(p), c_ptr(rows[i]), ctypes.c_size_t(w), c_ptr(exp[i]))
    assert np.array_equal(got, exp)


# ---------------------------------------------------------------- Merkle
# heights cover every host tree-top path (prove.cpp host_levels): below one
# 16-digest subtree (2^3), one subtree (2^4), 16 subtree tasks (2^8), wide levels
# first (2^9 .. 2^13), and trees hashed wholly on the host (h <= 1024, one matrix)
@pytest.mark.parametrize("logh,widths", [(0, [3]), (1, [2]), (3, [2]), (4, [8]), (5, [1]), (8, [2]), (9, [3]),
                                         (10, [1, 1, 1, 1]), (12, [8]), (13, [2]), (11, [3, 5])])
def test_merkle_commit_open_verify(gpu_ctx, oracle_lib, logh, widths):
    from linea_stark_prover_amd.prover import MerkleTreeMmcs
    rng = np.random.default_rng(logh)
    h = 1 << logh
    mats = [rand_fr(rng, (h, w)) for w in widths]
    mmcs = MerkleTreeMmcs(gpu_ctx)
    root, tree = mmcs.commit(mats)
    cat = np.concatenate(mats, axis=1).copy()
    layers = np.zeros((2 * h - 1, 4), np.uint64)
    p = oracle_params(oracle_lib)
    oracle_lib.lib().lo_merkle_commit(ctypes.byref(p), c_ptr(cat), ctypes.c_size_t(h), ctypes.c_size_t(cat.shape[1]),
                                      c_ptr(layers), 8)
    assert np.array_equal(root.reshape(4), layers[-1])
    off = 0
    for lv in range(logh + 1):  # every layer, GPU-made and host-made
        assert np.array_equal(tree.layer(lv), layers[off:off + (h >> lv)]), f"layer {lv}"
        off += h >> lv
    for idx in sorted({0, h - 1, h // 3}):
        rows, path = mmcs.open_batch(idx, tree)
        for m, r in zip(mats, rows):
            assert np.array_equal(r, m[idx])
        assert mmcs.verify_batch(root, widths, logh, idx, rows, path)
        if logh:
            bad = path.copy()
            bad[0, 0] ^= np.uint64(1)
            assert not mmcs.verify_batch(root, widths, logh, idx, rows, bad)


# every level on the GPU (LSP_HOST_TREE_TOP=0, read per commit): the row-form
# compression (k_merkle_level_row) makes the levels of 64..1024 nodes, the quads
# above them, k_merkle_top the last 128 digests -- each layer against the oracle's
@pytest.mark.parametrize("logh,widths", [(8, [3]), (11, [1]), (12, [2, 3]), (14, [8])])
def test_merkle_layers_all_on_gpu(gpu_ctx, oracle_lib, monkeypatch, logh, widths):
    from linea_stark_prover_amd.prover import MerkleTreeMmcs
    monkeypatch.setenv("LSP_HOST_TREE_TOP", "0")
    rng = np.random.default_rng(100 + logh)
    h = 1 << logh
    mats = [rand_fr(rng, (h, w)) for w in widths]
    root, tree = MerkleTreeMmcs(gpu_ctx).commit(mats)
    cat = np.concatenate(mats, axis=1).copy()
    layers = np.zeros((2 * h - 1, 4), np.uint64)
    p = oracle_params(oracle_lib)
    oracle_lib.lib().lo_merkle_commit(ctypes.byref(p), c_ptr(cat), ctypes.c_size_t(h), ctypes.c_size_t(cat.shape[1]),
                                      c_ptr(layers), 8)
    assert np.array_equal(root.reshape(4), layers[-1])
    off = 0
    for lv in range(logh + 1):
        assert np.array_equal(tree.layer(lv), layers[off:off + (h >> lv)]), f"layer {lv}"
        off += h >> lv


# ------------------------------------------------------------------- FRI
@pytest.mark.parametrize("logn", [1, 3, 10, 14])
def test_fri_fold_matches_pyoracle_and_fold_row(gpu_ctx, logn):
    from linea_stark_prover_amd.prover import TwoAdicFriGenericConfig
    from linea_stark_prover_amd.field import to_mont
    rng = np.random.default_rng(logn)
    n = 1 << logn
    v = rand_fr(rng, (n,))
    beta = rand_fr(rng, (1,))
    g = TwoAdicFriGenericConfig(gpu_ctx)
    got = g.fold_matrix(beta, v)
    vi = ints(v)
    bi = ints(beta)[0]
    if logn <= 10:
        assert ints(got) == O.fold_vector(vi, bi)
    for i in sorted({0, n // 2 - 1, n // 5}):
        e = g.fold_row(i, logn - 1, beta, v[2 * i], v[2 * i + 1])
        assert np.array_equal(e.reshape(4), got[i])
        assert ints(to_mont([O.fold_row(i, logn - 1, bi, vi[2 * i], vi[2 * i + 1])]))[0] == ints(got[i])[0]


# ----------------------------------------------------------- batch inverse
@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 4096, 4097, 8191, 8192, 70001, (1 << 20) + 3, (1 << 24) + 4097])
def test_batch_inverse(gpu_ctx, n):
    """hierarchical Montgomery trick: one-workgroup base (n <= 4096), one and
    several up/down levels above it"""
    rng = np.random.default_rng(n)
    m = min(n, 3000)
    x = rand_fr(rng, (m,))
    if n > m:  # tile the random block (distinct values are not needed, only nonzero ones)
        x = np.concatenate([x] * (n // m + 1))[:n]
    inv = gpu_ctx.batch_inverse(x)
    idx = sorted(set(range(min(n, 1500))) | set(range(max(0, n - 1500), n)) |
                 set(rng.integers(0, n, 1000).tolist()))
    xi, ii = ints(x[idx]), ints(inv[idx])
    for a, b in zip(xi, ii):
        assert a * b % P == 1


# ---------------------------------------------------------- interpolation
def test_interpolate_coset_matches_pyoracle(gpu_ctx):
    from linea_stark_prover_amd.field import to_mont
    rng = np.random.default_rng(5)
    h, w = 16, 3
    mat = rand_fr(rng, (h, w))
    z = rand_fr(rng, (1,))
    shift = to_mont([O.GENERATOR])
    got = ints(gpu_ctx.interpolate_coset(mat, h, shift, z))
    exp = O.interpolate_coset([ints(mat[i]) for i in range(h)], O.GENERATOR, ints(z)[0])
    assert got == exp


# ------------------------------------- open: inverse denominators, reduce
@pytest.mark.parametrize("log_n", [0, 3, 7])
def test_inverse_denominators_match_pyoracle(gpu_ctx, log_n):
    from linea_stark_prover_amd.field import to_mont
    rng = np.random.default_rng(100 + log_n)
    pts = rand_fr(rng, (3,))
    got = gpu_ctx.inverse_denominators(pts, log_n, to_mont([O.GENERATOR]))
    exp = O.inverse_denominators(log_n, O.GENERATOR, ints(pts))
    assert [ints(got[p]) for p in range(3)] == exp


@pytest.mark.parametrize("n,w,npts", [(8, 3, 2), (64, 8, 2), (32, 1, 1), (1, 5, 3)])
def test_open_reduce_matches_pyoracle(gpu_ctx, n, w, npts):
    """two matrices reduced one after the other (the offset carries over), as
    TwoAdicFriPcs::open reduces trace@(zeta, zeta_next) then the quotient chunks"""
    from linea_stark_prover_amd.field import to_mont
    rng = np.random.default_rng(n * 100 + w)
    m1, m2 = rand_fr(rng, (n, w)), rand_fr(rng, (n, 2))
    inv = rand_fr(rng, (npts, n))
    y1, y2 = rand_fr(rng, (npts, w)), rand_fr(rng, (1, 2))
    alpha = rand_fr(rng, (1,))
    ro = rand_fr(rng, (n,))
    ro_exp = ints(ro)
    a = ints(alpha)[0]
    off = gpu_ctx.open_reduce(m1, inv, y1, alpha, to_mont([1]), ro)
    off = gpu_ctx.open_reduce(m2, inv[:1], y2, alpha, off, ro)
    e = O.open_reduce([ints(m1[i]) for i in range(n)], [ints(inv[p]) for p in range(npts)],
                      [ints(y1[p]) for p in range(npts)], a, 1, ro_exp)
    e = O.open_reduce([ints(m2[i]) for i in range(n)], [ints(inv[0])], [ints(y2[0])], a, e, ro_exp)
    assert ints(ro) == ro_exp
    assert ints(off.reshape(1, 4))[0] == e == pow(a, npts * w + 2, P)


# -------------------------------------------------------------- quotient
def _perm_setup(logn, ncols, oracle_lib):
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, logn, ncols)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << logn, w, 4).copy()
    return s, p, trace, w


@pytest.mark.parametrize("logn,ncols", [(3, 3), (6, 3), (5, 6), (10, 3)])
def test_quotient_matches_oracle(gpu_ctx, oracle_lib, logn, ncols):
    from linea_stark_prover_amd.air import permutation_air
    s, p, trace, w = _perm_setup(logn, ncols, oracle_lib)
    air = permutation_air(ncols)
    proof, dbg = oracle_lib.prove(p, trace.ctypes.data, 1 << logn, w, oracle_lib.perm_air(ncols), debug=True)
    N = (1 << logn) << 3
    lde = np.frombuffer(dbg["trace_lde"].raw, dtype=np.uint64).reshape(N, w, 4).copy()
    alpha = np.array(dbg["challenges"][0:4], dtype=np.uint64).reshape(1, 4)
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    got = gpu_ctx.quotient_values(lde, 1 << logn, air, pub, alpha)
    exp = np.frombuffer(dbg["quotient"].raw, dtype=np.uint64).reshape(-1, 4)
    assert np.array_equal(got, exp)


# ------------------------------------------------------------ full prove
def _pub(p):
    return np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])


@pytest.mark.parametrize("logn,ncols", [(1, 3), (2, 3), (3, 3), (4, 6), (8, 3), (11, 3), (12, 6), (13, 3)])
def test_prove_bit_exact_vs_oracle(gpu_ctx, oracle_lib, logn, ncols):
    from linea_stark_prover_amd.air import permutation_air
    s, p, trace, w = _perm_setup(logn, ncols, oracle_lib)
    air = permutation_air(ncols)
    pub = _pub(p)
    got = gpu_ctx.prove(trace, air, pub)
    exp = oracle_lib.prove(p, trace.ctypes.data, 1 << logn, w, oracle_lib.perm_air(ncols))
    assert got == exp
    assert gpu_ctx.verify(got, air, pub)
    assert oracle_lib.verify(p, got, oracle_lib.perm_air(ncols)) == 0


def test_prove_tiny_vs_pyoracle(gpu_ctx, oracle_lib):
    from linea_stark_prover_amd.air import permutation_air
    s, p, trace, w = _perm_setup(3, 3, oracle_lib)
    cfgs, cols = O.synthetic_perm_trace(3, 3, s.alpha, s.delta, O.DEFAULT_SEED)
    pf = O.prove(cfgs, O.columns_to_rows(cols), [s.alpha, s.delta], s.perm)
    assert gpu_ctx.prove(trace, permutation_air(3), _pub(p)) == O.serialize_proof(pf)


def test_prove_lookup_and_permutation_air(gpu_ctx, oracle_lib):
    """Wide-AIR shape: LogUp lookup config + permutation config in one trace."""
    from linea_stark_prover_amd.air import AirLookupConfig, AirPermutationConfig, LineaAIR
    from linea_stark_prover_amd.field import to_mont
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    rng = O.SplitMix64(99)
    n = 64
    tab = [[rng.sample_fr() for _ in range(n)] for _ in range(3)]
    tab2 = [[rng.sample_fr() for _ in range(n)] for _ in range(3)]
    a = [[0] * n for _ in range(3)]
    for i in range(n):
        j = rng.below(n)
        src = tab if i % 3 else tab2
        for c in range(3):
            a[c][i] = src[c][j]
    af = [1] * n
    af[5] = 0
    cfg, cols = O.lookup_witness(a, [tab, tab2], af, [[1] * n, [1] * n], s.alpha, s.delta)
    pc, pcols = O.synthetic_perm_trace(6, 3, s.alpha, s.delta, 5)
    cfgs = [cfg, O.shift_cfg(pc[0], len(cols))]
    rows = O.columns_to_rows(cols + pcols)
    w = len(rows[0])
    trace = to_mont([x for r in rows for x in r]).reshape(n, w, 4)
    c0, c1 = cfgs
    air = LineaAIR([AirLookupConfig(c0.a_cols, c0.b_cols, c0.a_filter, c0.b_filter, c0.a_inv, c0.b_inv, c0.occ,
                                    c0.check),
                    AirPermutationConfig(c1.a_cols, c1.b_cols, c1.b_inv, c1.check)])
    assert air.descriptor() == oracle_lib.air_desc(cfgs)
    got = gpu_ctx.prove(trace, air, _pub(p))
    exp = oracle_lib.prove(p, trace.ctypes.data, n, w, oracle_lib.air_desc(cfgs))
    assert got == exp
    assert gpu_ctx.verify(got, air, _pub(p))


def test_prove_rejects_tampering(gpu_ctx, oracle_lib):
    from linea_stark_prover_amd.air import permutation_air
    s, p, trace, w = _perm_setup(6, 3, oracle_lib)
    air = permutation_air(3)
    pf = bytearray(gpu_ctx.prove(trace, air, _pub(p)))
    for off in (8 + 24 + 5, 8 + 24 + 64 + 7, len(pf) // 2, len(pf) - 3):
        bad = bytearray(pf)
        bad[off] ^= 1
        assert not gpu_ctx.verify(bytes(bad), air, _pub(p))


def test_prove_rejects_bad_arguments(gpu_ctx, oracle_lib):
    """lsp_prove on malformed input returns an error code (the reference's
    prover panics on these) and leaves the context usable: non-power-of-two
    and one-row traces, a trace narrower than the AIR's columns, fewer than
    two public values; then a good proof on the same context"""
    import ctypes
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.air import permutation_air
    s, p, trace, w = _perm_setup(4, 3, oracle_lib)
    air = permutation_air(3)
    pub = _pub(p)

    def code(tr, pv):
        with pytest.raises(_lib.LspError) as e:
            gpu_ctx.prove(tr, air, pv)
        return e.value.code

    assert code(np.ascontiguousarray(trace[:12]), pub) == _lib.LSP_E_SIZE   # 12 rows
    assert code(np.ascontiguousarray(trace[:1]), pub) == _lib.LSP_E_SIZE    # 1 row
    assert code(np.ascontiguousarray(trace[:, : w - 1]), pub) == _lib.LSP_E_ARG  # column w-1 missing
    assert code(trace, pub[:1]) == _lib.LSP_E_ARG                          # [alpha] only
    desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
    assert _lib.lib().lsp_prove(gpu_ctx.h, trace.ctypes.data, 16, w, desc, len(desc), pub.ctypes.data, 2,
                                _lib.LSP_MEM_HOST, None) == _lib.LSP_E_ARG  # no output handle
    got = gpu_ctx.prove(trace, air, pub)
    assert got == oracle_lib.prove(p, trace.ctypes.data, 16, w, oracle_lib.perm_air(3))


def test_prove_large_self_consistency(gpu_ctx):
    """2^16 rows: no oracle at this size in the default run; the product's
    verifier must accept and the LDE must agree with the trace on the low
    coset's defining property (re-proving is deterministic)."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(16, 3, a, d)
    pub = np.concatenate([a, d])
    air = permutation_air(3)
    pf1 = gpu_ctx.prove(tr, air, pub)
    pf2 = gpu_ctx.prove(tr, air, pub)
    assert pf1 == pf2
    assert gpu_ctx.verify(pf1, air, pub)


@pytest.mark.parametrize("bits", [1, 8, 13, 20])
def test_prove_with_pow_grinding_matches_oracle(oracle_lib, bits):
    """F2: GPU grinding finds the same (smallest) witness as the oracle."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    s, p, trace, w = _perm_setup(5, 3, oracle_lib)
    cfg = StarkConfig(proof_of_work_bits=bits)
    with Context(cfg) as ctx:
        got = ctx.prove(trace, permutation_air(3), _pub(p))
        assert ctx.verify(got, permutation_air(3), _pub(p))
    fri = oracle_lib.fri_params(O.FriParams(proof_of_work_bits=bits))
    exp = oracle_lib.prove(p, trace.ctypes.data, 32, w, oracle_lib.perm_air(3), fri=fri)
    assert got == exp
    assert oracle_lib.verify(p, got, oracle_lib.perm_air(3), fri=fri) == 0


@pytest.mark.parametrize("logn,ncols", [(16, 3), (15, 6)])
def test_prove_bit_exact_vs_oracle_large(gpu_ctx, oracle_lib, logn, ncols):
    """Full proofs at 2^15-2^16 rows against the multithreaded C oracle (a few
    seconds on the host): every stage at the sizes where the GPU kernels take
    their wide (non-cooperative, multi-pass) paths."""
    from linea_stark_prover_amd.air import permutation_air
    s, p, trace, w = _perm_setup(logn, ncols, oracle_lib)
    got = gpu_ctx.prove(trace, permutation_air(ncols), _pub(p))
    exp = oracle_lib.prove(p, trace.ctypes.data, 1 << logn, w, oracle_lib.perm_air(ncols))
    assert got == exp
