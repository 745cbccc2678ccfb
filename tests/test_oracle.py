"""CPU tests of the oracle itself: known answers, uniqueness theorems, the two
restatements (Python big-int, C) agreeing byte-for-byte, golden fixtures,
witness invariants and self-verification."""
import hashlib
import json
import os

import pytest

from oracle import pyoracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


# ------------------------------------------------------------ known answers
def test_field_constants():
    P = O.P
    assert P.bit_length() == 253
    v, s = P - 1, 0
    while v % 2 == 0:
        v //= 2
        s += 1
    assert s == 47 == O.TWO_ADICITY
    assert pow(22, (P - 1) // 2, P) == P - 1  # GEN is a non-residue
    assert O.ROOT_2_47 == 0x11d4b7f60cb92cc160c69477d1a8a12f9b506ee363e3f04a476ef4a4ec2a895e
    assert O.MONT_R == 0x0d4bda322bbb9a9d16d81575512c0fee7257f50f6ffffff27d1c7ffffffffff3
    assert (-pow(P, -1, 1 << 64)) % (1 << 64) == 0x0a117fffffffffff
    assert (-pow(P, -1, 1 << 32)) % (1 << 32) == 0xffffffff
    for k in range(1, 48):
        g = O.two_adic_generator(k)
        assert pow(g, 1 << (k - 1), P) == P - 1  # w^(n/2) = -1
        assert pow(g, 1 << k, P) == 1
    import math
    assert [d for d in (3, 5, 7, 11, 13, 17) if math.gcd(d, P - 1) == 1] == [11, 17]


def test_mont_roundtrip():
    for x in (0, 1, 2, O.P - 1, 0xDEADBEEF << 200):
        assert O.from_mont_bytes(O.to_mont_bytes(x)) == x % O.P


# ------------------------------------------------------- uniqueness (A2/A13)
@pytest.mark.parametrize("logh,added", [(0, 1), (2, 3), (3, 2), (5, 3)])
def test_lde_is_polynomial_evaluation(logh, added):
    rng = O.SplitMix64(logh * 7 + added)
    h = 1 << logh
    col = [rng.sample_fr() for _ in range(h)]
    shift = rng.sample_fr()
    lde = O.coset_lde_column(col, added, shift)
    coeffs = O.idft(col)
    gh = O.two_adic_generator(logh)
    assert [O.eval_poly(coeffs, pow(gh, i, O.P)) for i in range(h)] == col
    lg = logh + added
    g = O.two_adic_generator(lg)
    for i in range(len(lde)):
        assert lde[i] == O.eval_poly(coeffs, shift * pow(g, O.bitrev(i, lg), O.P) % O.P)


def test_interpolate_coset_is_polynomial_evaluation():
    rng = O.SplitMix64(5)
    h, w = 16, 3
    rows_nat = [[rng.sample_fr() for _ in range(w)] for _ in range(h)]
    z = rng.sample_fr()
    shift = O.GENERATOR
    ys = O.interpolate_coset(O.reverse_slice_index_bits(rows_nat), shift, z)
    for c in range(w):
        col = [r[c] for r in rows_nat]  # values at shift * w_h^i
        coeffs = O.idft(col)  # p(shift*x) coefficients in x
        zz = z * O.inv(shift) % O.P
        assert ys[c] == O.eval_poly(coeffs, zz)


def test_selectors_match_definitions():
    log_h, logQ = 3, 5
    first, last, trans, inv_z = O.selectors_on_coset(log_h, logQ)
    h = 1 << log_h
    gq = O.two_adic_generator(logQ)
    wl = O.inv(O.two_adic_generator(log_h))
    for i in range(1 << logQ):
        x = O.GENERATOR * pow(gq, i, O.P) % O.P
        zh = (pow(x, h, O.P) - 1) % O.P
        assert first[i] == zh * O.inv(x - 1) % O.P
        assert last[i] == zh * O.inv(x - wl) % O.P
        assert trans[i] == (x - wl) % O.P
        assert inv_z[i] * zh % O.P == 1


def test_fold_matrix_matches_fold_row():
    rng = O.SplitMix64(9)
    for logm in (0, 1, 4):
        v = [rng.sample_fr() for _ in range(2 << logm)]
        beta = rng.sample_fr()
        f = O.fold_vector(v, beta)
        for i in range(1 << logm):
            assert f[i] == O.fold_row(i, logm, beta, v[2 * i], v[2 * i + 1])


# --------------------------------------------------------------- golden
def test_golden_setup_and_primitives():
    s = O.setup_from_seed()
    assert hex(s.alpha) == GOLDEN["setup"]["alpha"] and hex(s.delta) == GOLDEN["setup"]["delta"]
    assert [hex(x) for x in O.permute([0, 1, 2], s.perm)] == GOLDEN["poseidon2_012"]
    for w, hv in GOLDEN["hash_iter_range"].items():
        assert hex(O.hash_iter(list(range(int(w))), s.perm)) == hv
    assert hex(O.compress(1, 2, s.perm)) == GOLDEN["compress_1_2"]
    lay = GOLDEN["poseidon2_012_layers"]
    s.perm.int_diag = [int(x, 16) for x in lay["int_diag"]]
    s.perm.ext_mds = [int(x, 16) for x in lay["ext_mds"]]
    assert [hex(x) for x in O.permute([0, 1, 2], s.perm)] == lay["out"]
    s.perm.int_diag = s.perm.ext_mds = None
    col = [pow(3, i, O.P) for i in range(4)]
    assert [hex(x) for x in O.coset_lde_column(col, 3, O.GENERATOR)] == GOLDEN["lde_col_3pow_h4_b3"]


def test_golden_proofs_python_and_c(oracle_lib):
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    for key, ent in GOLDEN["proofs"].items():
        ncols = int(key.split("_")[1].split("x")[0])
        logn = int(key.split("_n")[1])
        tb, w = oracle_lib.gen_perm_trace(p, logn, ncols)
        cb = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.perm_air(ncols))
        assert hashlib.sha256(cb).hexdigest() == ent["sha256"], key
        if "hex" in ent:
            assert cb.hex() == ent["hex"]
            pf = O.deserialize_proof(cb)
            cfgs = [O.PermCfg(list(range(ncols)), list(range(ncols, 2 * ncols)), 2 * ncols, 2 * ncols + 1)]
            assert O.verify(cfgs, pf, [s.alpha, s.delta], s.perm)


# ------------------------------------------- Python vs C restatements
@pytest.mark.parametrize("logn,ncols", [(1, 3), (3, 3), (3, 6), (5, 3)])
def test_python_and_c_oracles_agree(oracle_lib, logn, ncols):
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    cfgs, cols = O.synthetic_perm_trace(logn, ncols, s.alpha, s.delta, O.DEFAULT_SEED)
    rows = O.columns_to_rows(cols)
    tb, w = oracle_lib.gen_perm_trace(p, logn, ncols)
    assert oracle_lib.buf_to_ints(tb, len(rows) * w) == [x for r in rows for x in r]
    pf = O.prove(cfgs, rows, [s.alpha, s.delta], s.perm)
    cb = oracle_lib.prove(p, tb, 1 << logn, w, oracle_lib.air_desc(cfgs))
    assert cb == O.serialize_proof(pf)
    assert oracle_lib.verify(p, cb, oracle_lib.air_desc(cfgs)) == 0


def _lookup_case(s, n=16, seed=7):
    rng = O.SplitMix64(seed)
    tab = [[rng.sample_fr() for _ in range(n)] for _ in range(2)]
    tab2 = [[rng.sample_fr() for _ in range(n)] for _ in range(2)]
    a = [[0] * n for _ in range(2)]
    for i in range(n):
        j = rng.below(n)
        src = tab if i % 2 else tab2
        a[0][i], a[1][i] = src[0][j], src[1][j]
    af = [1] * n
    af[3] = 0
    return O.lookup_witness(a, [tab, tab2], af, [[1] * n, [1] * n], s.alpha, s.delta)


def test_lookup_witness_invariant_and_proof(oracle_lib):
    s = O.setup_from_seed()
    cfg, cols = _lookup_case(s)
    assert cols[cfg.check][-1] == 0  # trace/src/lookup.rs:165-168
    pc, pcols = O.synthetic_perm_trace(4, 3, s.alpha, s.delta, 99)
    assert pcols[pc[0].check][-1] == 1  # trace/src/permutation.rs:76-79
    cfgs = [cfg, O.shift_cfg(pc[0], len(cols))]
    rows = O.columns_to_rows(cols + pcols)
    pf = O.prove(cfgs, rows, [s.alpha, s.delta], s.perm)
    assert O.verify(cfgs, pf, [s.alpha, s.delta], s.perm)
    p = oracle_lib.setup()
    cb = oracle_lib.prove(p, oracle_lib.fr_buf([x for r in rows for x in r]), 16, len(rows[0]),
                          oracle_lib.air_desc(cfgs))
    assert cb == O.serialize_proof(pf)


def test_bad_witness_is_rejected():
    s = O.setup_from_seed()
    cfgs, cols = O.synthetic_perm_trace(3, 3, s.alpha, s.delta, O.DEFAULT_SEED)
    cols[0][2] = (cols[0][2] + 1) % O.P  # break the permutation; check column now wrong
    rows = O.columns_to_rows(cols)
    pf = O.prove(cfgs, rows, [s.alpha, s.delta], s.perm)
    assert not O.verify(cfgs, pf, [s.alpha, s.delta], s.perm)


def test_tampered_proofs_rejected(oracle_lib):
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, 4, 3)
    cb = bytearray(oracle_lib.prove(p, tb, 16, w, oracle_lib.perm_air(3)))
    for off in (30, 100, 500, len(cb) // 3, len(cb) - 40):
        bad = bytearray(cb)
        bad[off] ^= 0x10
        assert oracle_lib.verify(p, bytes(bad), oracle_lib.perm_air(3)) != 0


def test_permutation_counts_match_survey_formula():
    """perms = N*ceil(w/2) + (N-1) + N*ceil(q/2) + (N-1) + sum_FRI(len-1)."""
    s = O.setup_from_seed()
    logn, ncols = 3, 3
    cfgs, cols = O.synthetic_perm_trace(logn, ncols, s.alpha, s.delta, O.DEFAULT_SEED)
    O.PERM_COUNTER[0] = 0
    O.prove(cfgs, O.columns_to_rows(cols), [s.alpha, s.delta], s.perm)
    h, w, q = 1 << logn, 2 * ncols + 2, 4
    N = 8 * h
    fri = 0
    L = N
    while L > 8:
        fri += L // 2 + L // 2 - 1
        L //= 2
    expect = N * ((w + 1) // 2) + (N - 1) + N * ((q + 1) // 2) + (N - 1) + fri
    # + transcript hashes (a handful)
    assert expect <= O.PERM_COUNTER[0] <= expect + 200


@pytest.mark.parametrize("logh,w,added", [(1, 1, 1), (4, 3, 3), (9, 2, 3)])
def test_eval_points_matches_lde(oracle_lib, logh, w, added):
    """lo_eval_points (barycentric, the full-size LDE spot check) and
    lo_lde_point agree with the oracle's NTT-based coset LDE on every row."""
    import ctypes
    import numpy as np
    L = oracle_lib.lib()
    rng = np.random.default_rng(logh)
    h, N = 1 << logh, 1 << (logh + added)
    mat = rng.integers(0, 2**63, size=(h, w, 4), dtype=np.uint64)
    mat[..., 3] &= (1 << 59) - 1  # < r (Montgomery words are any value < r)
    shift = np.array([22, 0, 0, 0], np.uint64)
    shifts = np.repeat(shift.reshape(1, 4), w, axis=0).copy()
    lde = np.zeros((N, w, 4), np.uint64)
    P = lambda a: ctypes.c_void_p(a.ctypes.data)
    L.lo_coset_lde_batch(P(mat), ctypes.c_size_t(h), ctypes.c_size_t(w), added, P(shifts), P(lde), 4)
    xs = np.zeros((N, 4), np.uint64)
    for j in range(N):
        L.lo_lde_point(ctypes.c_size_t(h), added, P(shift), ctypes.c_uint64(j), P(xs[j]))
    got = np.zeros((N, w, 4), np.uint64)
    L.lo_eval_points(P(mat), ctypes.c_size_t(h), ctypes.c_size_t(w), P(xs), ctypes.c_size_t(N), P(got), 4)
    assert np.array_equal(got, lde)


def test_background_oracle_job_matches_direct_call(oracle_lib, tmp_path):
    """tests/oracle_job.py (the GPU suite's background oracle proofs): jobs run
    in order, each proof written whole, equal to calling the oracle directly"""
    import subprocess
    import sys
    jobs = [(str(tmp_path / "a.bin"), 6, 3), (str(tmp_path / "b.bin"), 5, 6)]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run([sys.executable, os.path.join(root, "tests", "oracle_job.py"), "2"] +
                   [f"{o}:{n}:{c}" for o, n, c in jobs], check=True, timeout=300)
    p = oracle_lib.setup()
    for out, log_n, ncols in jobs:
        tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
        expect = oracle_lib.prove(p, tb, 1 << log_n, w, oracle_lib.perm_air(ncols), nthreads=2)
        with open(out, "rb") as f:
            assert f.read() == expect
        assert not os.path.exists(out + ".part")


def test_lde_thread_split_is_bit_exact(oracle_lib):
    """lo_coset_lde_batch with each NTT stage split over threads (fewer columns
    than threads, N >= 2^14) equals the column-parallel transform bit for bit,
    and sampled rows equal barycentric evaluation (lo_eval_points)"""
    import ctypes
    import numpy as np
    L = oracle_lib.lib()
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    logh, w, added = 12, 3, 3
    h, N = 1 << logh, 1 << (logh + added)
    rng = np.random.default_rng(7)
    mat = rng.integers(0, 2**63, size=(h, w, 4), dtype=np.uint64)
    mat[..., 3] &= (1 << 59) - 1  # < r
    shift = np.array([22, 0, 0, 0], np.uint64)
    shifts = np.repeat(shift.reshape(1, 4), w, axis=0).copy()
    outs = []
    for th in (1, 2, 6):  # 1: one thread; 2: columns in parallel; 6 > w: stages split
        out = np.zeros((N, w, 4), np.uint64)
        L.lo_coset_lde_batch(P(mat), ctypes.c_size_t(h), ctypes.c_size_t(w), added, P(shifts), P(out), th)
        outs.append(out)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    rows = [0, 1, 2, N // 2 + 3, N - 1, 12345]
    xs = np.zeros((len(rows), 4), np.uint64)
    for k, j in enumerate(rows):
        L.lo_lde_point(ctypes.c_size_t(h), added, P(shift), ctypes.c_uint64(j), P(xs[k]))
    got = np.zeros((len(rows), w, 4), np.uint64)
    L.lo_eval_points(P(mat), ctypes.c_size_t(h), ctypes.c_size_t(w), P(xs), ctypes.c_size_t(len(rows)), P(got), 4)
    assert np.array_equal(got, outs[2][rows])
