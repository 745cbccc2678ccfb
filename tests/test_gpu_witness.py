"""F1: witness generation on the GPU (lsp_witness_permutation / _lookup via
linea_stark_prover_amd.trace.RawTrace) against the oracle's restatement of
trace/src/permutation.rs:24-93 and trace/src/lookup.rs:46-176."""
import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


def _rand_fr(rng, n):
    return [rng.sample_fr() for _ in range(n)]


def _perm_case(n, w, seed):
    rng = O.SplitMix64(seed)
    a = [_rand_fr(rng, n) for _ in range(w)]
    order = list(range(n))
    for i in range(n - 1, 0, -1):  # Fisher-Yates
        j = rng.below(i + 1)
        order[i], order[j] = order[j], order[i]
    b = [[col[order[i]] for i in range(n)] for col in a]
    return a, b


def _lookup_case(n, nt, nbc, seed, key_range=5, p_bf=0.8, p_af=0.9):
    """tables of small values (many duplicate keys), random filters; every
    enabled A row copies an enabled B row, disabled A rows hold values no
    table has"""
    g = np.random.default_rng(seed)
    b = [[[int(v) for v in g.integers(0, key_range, n)] for _ in range(nbc)] for _ in range(nt)]
    bf = [[int(g.random() < p_bf) for _ in range(n)] for _ in range(nt)]
    bf[0][0] = 1
    enabled = [(t, i) for t in range(nt) for i in range(n) if bf[t][i]]
    a = [[0] * n for _ in range(nbc)]
    af = []
    for i in range(n):
        if g.random() < p_af:
            t, j = enabled[int(g.integers(0, len(enabled)))]
            for c in range(nbc):
                a[c][i] = b[t][c][j]
            af.append(1)
        else:
            for c in range(nbc):
                a[c][i] = 1000 + int(g.integers(0, 50))
            af.append(0)
    return a, b, af, bf


def _challenges():
    s = O.setup_from_seed()
    return s.alpha, s.delta


def _mont_cols(cols):
    from linea_stark_prover_amd.field import to_mont
    return [to_mont(c) for c in cols]


@pytest.mark.parametrize("log_n,w", [(0, 1), (3, 3), (10, 6), (13, 3)])
def test_permutation_witness_matches_oracle(gpu_ctx, log_n, w):
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.trace import RawPermutationTrace, RawTrace
    al, de = _challenges()
    a, b = _perm_case(1 << log_n, w, 11 + log_n)
    cfg, cols = O.perm_witness(a, b, al, de)
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    cfgs = rt.push_traces([RawPermutationTrace(_mont_cols(a), _mont_cols(b))], [])
    got = rt.get_trace(host=True)
    exp = np.stack(_mont_cols(cols), axis=1)
    assert np.array_equal(got, exp)
    assert (cfgs[0].a_columns_ids, cfgs[0].b_columns_ids, cfgs[0].b_inverse_id, cfgs[0].check_id) == \
        (cfg.a_cols, cfg.b_cols, cfg.b_inv, cfg.check)
    rt.close()


@pytest.mark.parametrize("log_n,nt,nbc,key_range", [(3, 1, 1, 3), (8, 2, 3, 4), (11, 3, 2, 2), (12, 2, 3, 1000)])
def test_lookup_witness_matches_oracle(gpu_ctx, log_n, nt, nbc, key_range):
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.trace import RawLookupTrace, RawTrace
    al, de = _challenges()
    n = 1 << log_n
    a, b, af, bf = _lookup_case(n, nt, nbc, 7 * log_n + nt, key_range)
    cfg, cols = O.lookup_witness(a, b, af, bf, al, de)
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    lt = RawLookupTrace(_mont_cols(a), [_mont_cols(t) for t in b], to_mont(af), [to_mont(f) for f in bf])
    rt.push_traces([], [lt])
    got = rt.get_trace(host=True)
    exp = np.stack(_mont_cols(cols), axis=1)
    assert np.array_equal(got, exp)
    rt.close()


def test_mixed_trace_pads_heights_and_proves(gpu_ctx):
    """RawTrace::push_traces with blocks of different heights (zero padding,
    filters 0) in push order; the device-assembled trace proves to the same
    bytes as the host-assembled one"""
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.trace import RawLookupTrace, RawPermutationTrace, RawTrace
    al, de = _challenges()
    n = 1 << 9
    a, b, af, bf = _lookup_case(n // 2, 2, 2, 5)
    pa, pb = _perm_case(n, 3, 6)
    # oracle: pad the lookup block to n rows, then lookups first
    pad = lambda c: list(c) + [0] * (n - len(c))  # noqa: E731
    _, lcols = O.lookup_witness([pad(c) for c in a], [[pad(c) for c in t] for t in b], pad(af),
                                [pad(f) for f in bf], al, de)
    _, pcols = O.perm_witness(pa, pb, al, de)
    exp = np.stack(_mont_cols(lcols + pcols), axis=1)
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    lt = RawLookupTrace(_mont_cols(a), [_mont_cols(t) for t in b], to_mont(af), [to_mont(f) for f in bf])
    cfgs = rt.push_traces([RawPermutationTrace(_mont_cols(pa), _mont_cols(pb))], [lt])
    assert np.array_equal(rt.get_trace(host=True), exp)
    air = rt.air(cfgs)
    pub = np.concatenate([to_mont([al]), to_mont([de])])
    ptr, h, w = rt.get_trace()
    pf_dev = gpu_ctx.prove(ptr, air, pub, h, w)
    assert pf_dev == gpu_ctx.prove(exp, air, pub)
    assert gpu_ctx.verify(pf_dev, air, pub)
    rt.close()


def test_lookup_filters_default_to_enabled(gpu_ctx):
    """read_file's padding: missing a_filter / b_filter entries are 1"""
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.trace import RawLookupTrace, RawTrace
    al, de = _challenges()
    n = 64
    a, b, _, _ = _lookup_case(n, 1, 2, 9, p_bf=1.0, p_af=1.0)
    _, cols = O.lookup_witness(a, b, [1] * n, [[1] * n], al, de)
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    rt.push_traces([], [RawLookupTrace(_mont_cols(a), [_mont_cols(t) for t in b])])
    assert np.array_equal(rt.get_trace(host=True), np.stack(_mont_cols(cols), axis=1))
    rt.close()


def test_invalid_witness_is_rejected(gpu_ctx):
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.trace import RawLookupTrace, RawPermutationTrace, RawTrace
    al, de = _challenges()
    a, b = _perm_case(32, 2, 3)
    b[0][5] = (b[0][5] + 1) % O.P  # no longer a permutation
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    with pytest.raises(_lib.LspError, match="should be 1 on the last row"):
        rt.push_traces([RawPermutationTrace(_mont_cols(a), _mont_cols(b))], [])
    la, lb, laf, lbf = _lookup_case(32, 1, 2, 4)
    la[0][3], laf[3] = 999999, 1  # an enabled A row no table holds
    with pytest.raises(_lib.LspError, match="should be 0 on the last row"):
        rt.push_traces([], [RawLookupTrace(_mont_cols(la), [_mont_cols(t) for t in lb], to_mont(laf),
                                           [to_mont(f) for f in lbf])])
    rt.close()


def test_large_lookup_self_consistent(gpu_ctx):
    """2^18 rows, 2 tables, keys from 3 values: long runs in the multiplicity
    sort; the LogUp sum must close (checked by the library) and the trace
    must prove"""
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.trace import RawLookupTrace, RawTrace
    al, de = _challenges()
    n = 1 << 18
    g = np.random.default_rng(1)
    vals = to_mont([0, 1, 2, 77])
    tab = vals[g.integers(0, 3, n)]
    tab2 = vals[g.integers(0, 4, n)]
    a = vals[g.integers(0, 3, n)]
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    cfgs = rt.push_traces([], [RawLookupTrace([a], [[tab], [tab2]])])
    got = rt.get_trace(host=True)
    from linea_stark_prover_amd.field import from_mont
    occ = np.array(from_mont(got[:, -3, :])) + np.array(from_mont(got[:, -2, :]))
    assert int(occ.sum()) == n  # every A row counted once
    ptr, h, w = rt.get_trace()
    air = rt.air(cfgs)
    pub = np.concatenate([to_mont([al]), to_mont([de])])
    assert gpu_ctx.verify(gpu_ctx.prove(ptr, air, pub, h, w), air, pub)
    rt.close()


def test_cbor_inputs_to_proof(gpu_ctx):
    """F4 -> F1 -> prove: CBOR traces parsed natively, witness generated on the
    GPU, equal to the oracle's witness; lsp_raw_trace_push gives the same block"""
    import ctypes
    import os
    import sys
    from linea_stark_prover_amd import _lib as L
    from linea_stark_prover_amd.field import to_mont
    from linea_stark_prover_amd.prover import _ptr
    from linea_stark_prover_amd.trace import RawLookupTrace, RawPermutationTrace, RawTrace
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import cbor_enc as C
    al, de = _challenges()
    n = 128
    a, b, af, bf = _lookup_case(n, 2, 2, 31)
    pa, pb = _perm_case(n, 2, 32)
    lbytes = C.enc(C.lookup_trace(a, b, af, bf))
    pbytes = C.enc(C.permutation_trace(pa, pb), words_as_bytes=True)
    _, lcols = O.lookup_witness(a, b, af, bf, al, de)
    _, pcols = O.perm_witness(pa, pb, al, de)
    exp = np.stack(_mont_cols(lcols + pcols), axis=1)
    rt = RawTrace(gpu_ctx, [to_mont([al]), to_mont([de])])
    cfgs = rt.push_traces([RawPermutationTrace.read_file(pbytes)], [RawLookupTrace.read_file(lbytes)])
    assert np.array_equal(rt.get_trace(host=True), exp)
    # the C-ABI path: parse + push the lookup block into a host trace
    h = ctypes.c_void_p()
    L.check(L.lib().lsp_raw_trace_parse(lbytes, len(lbytes), ctypes.byref(h)))
    host = np.zeros((n, exp.shape[1], 4), np.uint64)
    alm, dem = to_mont([al]), to_mont([de])
    gpu_ctx._chk(L.lib().lsp_raw_trace_push(gpu_ctx.h, h, n, _ptr(alm), _ptr(dem), _ptr(host), exp.shape[1], 0,
                                            L.LSP_MEM_HOST))
    L.lib().lsp_raw_trace_free(h)
    lw = len(lcols)
    assert np.array_equal(host[:, :lw], exp[:, :lw])
    air = rt.air(cfgs)
    pub = np.concatenate([alm, dem])
    ptr, hh, w = rt.get_trace()
    assert gpu_ctx.verify(gpu_ctx.prove(ptr, air, pub, hh, w), air, pub)
    rt.close()
